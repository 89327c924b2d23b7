"""Per-node floor of a replayed hipGraph on this box: a 256-element axpy captured 48 times (the smallest
kernel on the path), beside the M = 8 / 16 TTS o-projection (1.6 MB) from the same harness.
python scripts/launch_floor_probe.py (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import ops  # noqa: E402

dev = torch.device("cuda:0")
a = torch.zeros(256, device=dev)
b = torch.ones(256, device=dev)
print(f"axpy 256      {graph_time(lambda: ops.axpy_(a, b), 48):6.2f} us per node", flush=True)
lin = PackedLinear((torch.randn(896, 896, device=dev) * 0.02).to(torch.bfloat16))
for M in (1, 8, 16):
    x = torch.randn(M, 896, device=dev)
    out = torch.empty(M, 896, device=dev)
    print(f"tts_o M={M:2d}    {graph_time(lambda: lin(x, out=out, M=M), 48):6.2f} us per node", flush=True)
