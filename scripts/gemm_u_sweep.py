"""k-steps in flight per wave (fo_gemm_set_u) of the one-row-tile fp32-X grid GEMM on the small, latency-bound
hot shapes: the Qwen2 o (N 3584, one tile per workgroup) and q|k|v (N 4608, tile pairs) projections at 16 / 8
rows and the TTS decoder's o / q|k|v.  U = 4 (policy), 7 on 16 waves (one tile: a wave's whole K range in one
round, K = 3584 = 16 x 7 x 32), 8 on 8 waves.  Graph-replayed over six weight copies; outputs compared with the
policy's.  python scripts/gemm_u_sweep.py (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
shapes = [("qwen_o", 3584, 3584, 16, 1), ("qwen_o_m8", 3584, 3584, 8, 1), ("qwen_qkv", 4608, 3584, 16, 2),
          ("qwen_qkv_m8", 4608, 3584, 8, 2), ("tts_o", 896, 896, 8, 1), ("tts_qkv", 1152, 896, 8, 2)]
for name, N, K, M, nt in shapes:
    lins = [PackedLinear((torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)) for _ in range(6)]
    x = torch.randn(M, K, device=dev, generator=g)
    ys = [torch.randn(M, N, device=dev, generator=g) for _ in range(6)]
    y0 = [y.clone() for y in ys]
    res = []
    ref = None
    for u, nw in ((0, 0), (4, 16), (4, 8), (7, 16), (8, 8)):
        if u == 7 and nt != 1:
            continue
        lib.fo_gemm_tune(nw, nt if nw else 0)
        lib.fo_gemm_set_u(u)
        it = iter(range(1 << 30))
        try:
            us = min(graph_time(lambda: (lambda i: lins[i](x, out=ys[i], M=M))(next(it) % 6), 48) for _ in range(2))
            out = lins[0](x, M=M)
            torch.cuda.synchronize()
        except RuntimeError as e:
            res.append(f"u{u} nw{nw}: failed {e}")
            continue
        if ref is None:
            ref = out.clone()
        err = (out - ref).abs().max().item()
        res.append(f"u{u} nw{nw} {us:6.2f}us {lins[0].nbytes / us / 1e6:.2f}TB/s" + ("" if err < 1e-4 else f" ERR {err:.2g}"))
    lib.fo_gemm_tune(0, 0)
    lib.fo_gemm_set_u(0)
    print(f"{name:12s} M={M:2d} {lins[0].nbytes / 1e6:5.1f}MB  " + " | ".join(res), flush=True)
    del lins, ys, y0
    torch.cuda.empty_cache()
