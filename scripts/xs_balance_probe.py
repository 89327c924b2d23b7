"""Is the X-stationary gate/up stream (k_gemm_xs, M = 16, K = 3584) bound per CU or by the chip's HBM stream?
Times the kernel, graph-replayed over two weight copies beyond the Infinity Cache, at gate/up widths whose unit
counts land on different (workgroups x units per workgroup) grids: the dispatcher gives every workgroup
ceil(units / 256) units.  A per-CU-bound stream takes time ~ units per workgroup; an HBM-bound one ~ total bytes.
The 18,944-wide layer runs 237 workgroups x 5 units (19 CUs idle): if the per-CU model holds, balancing its units
over all 256 CUs would save up to 1 - 1184 / (256 x 5) of the launch.  python scripts/xs_balance_probe.py (GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402

dev = torch.device("cuda:0")
D = 3584
g = torch.Generator(device=dev).manual_seed(0)
M = 16
x = torch.randn(M, D, device=dev, generator=g)
for I in (10240, 12288, 16384, 18944, 20480, 24576):
    units = I // 16
    per = (units + 255) // 256
    G = (units + per - 1) // per
    copies = max(2, -(-600 * 2**20 // (2 * I * D * 2)))   # beyond the 256 MB Infinity Cache
    lins = [PackedLinear((torch.randn(I, D, device=dev, generator=g) * 0.02).to(torch.bfloat16),
                         swiglu_up=(torch.randn(I, D, device=dev, generator=g) * 0.02).to(torch.bfloat16))
            for _ in range(copies)]
    outs = [torch.empty(M, I, device=dev) for _ in range(copies)]
    it = iter(range(1 << 30))
    us = min(graph_time(lambda: (lambda i: lins[i](x, out=outs[i], M=M))(next(it) % copies), 8 * copies)
             for _ in range(2))
    nbytes = 2 * I * D * 2
    print(f"I={I:6d} units {units:5d} -> {G:3d} WGs x {per} units: {us:6.2f} us  {nbytes / us / 1e6:5.2f} TB/s  "
          f"{us / per:6.2f} us per unit-round", flush=True)
    del lins, outs
    torch.cuda.empty_cache()
