"""Freeze-Omni MI355X runtime: C-ABI binding, kernels, paged KV, replica scheduling."""
