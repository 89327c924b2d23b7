"""Event-timed fo_gemm launches at the prefill row counts of a turn (M = 8 users x 5 prefix tokens = 40,
8 x (5 + 2) = 56) on the Qwen2 shapes: python scripts/gemm_mid_probe.py (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "freeze-omni_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_sweep_util import timeit  # noqa: E402
from fo.ops import PackedLinear  # noqa: E402

dev = torch.device("cuda:0")
for name, N, K, sw in [("qwen_qkv", 4608, 3584, False), ("qwen_o", 3584, 3584, False),
                       ("qwen_gu", 18944, 3584, True), ("qwen_down", 3584, 18944, False)]:
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    lin = PackedLinear(w, swiglu_up=w if sw else None)
    r = []
    for M in (16, 24, 32, 40, 48, 56, 64):
        x = torch.randn(M, K, device=dev)
        out = torch.empty(M, N, device=dev)
        t = timeit(lambda: lin(x, out=out), reps=20)
        r.append(f"M{M}:{t:6.1f}us({lin.nbytes / t / 1e3:4.2f}TB/s)")
    print(f"{name:9s} {lin.nbytes / 1e6:7.1f}MB " + " ".join(r), flush=True)
