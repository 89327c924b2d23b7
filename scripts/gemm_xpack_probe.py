"""Does the X read of the latency-bound M = 16 projections (Qwen2 q|k|v with RoPE, o with residual) cost by its
16-row-segment access pattern?  The same GEMM, graph-replayed over six cold weight copies, with X as fp32 rows
(split into bf16 hi / lo in the kernel) and with X pre-split and packed in MFMA A-fragment order (fo_gemm_set_xpack:
each wave's X fragment one contiguous 1 KiB read per half); outputs compared.  python scripts/gemm_xpack_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)


def pack(x):   # [16, K] fp32 -> hi, lo [K/32][64][8] bf16 (lane = 16 * (col % 32 // 8) + row)
    M, K = x.shape
    xf = torch.zeros(16, K, device=x.device)
    xf[:M] = x
    hi = xf.to(torch.bfloat16)
    lo = (xf - hi.float()).to(torch.bfloat16)
    f = lambda t: t.view(16, K // 32, 4, 8).permute(1, 2, 0, 3).contiguous()  # noqa: E731
    return f(hi), f(lo)


for name, N, K, M, res in [("qwen_o", 3584, 3584, 16, True), ("qwen_qkv_plain", 4608, 3584, 16, False),
                           ("qwen_o_m8", 3584, 3584, 8, True), ("tts_o", 896, 896, 8, True),
                           ("tts_down", 896, 4864, 8, True)]:
    lins = [PackedLinear((torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)) for _ in range(6)]
    x = torch.randn(M, K, device=dev, generator=g)
    hi, lo = pack(x)
    y0 = torch.randn(M, N, device=dev, generator=g)
    ys = [y0.clone() for _ in range(6)]
    out = {}
    for mode in ("fp32", "packed", "fp32", "packed"):
        it = iter(range(1 << 30))

        def run(i):
            if mode == "packed":
                lib.fo_gemm_set_xpack(hi.data_ptr(), lo.data_ptr(), K, (M + 15) // 16)
            lins[i](x, out=ys[i], residual=res, M=M)
        us = graph_time(lambda: run(next(it) % 6), 48)
        ys[0].copy_(y0)
        run(0)
        torch.cuda.synchronize()
        out.setdefault(mode, []).append((us, ys[0].clone()))
    a, b = out["fp32"][0][1], out["packed"][0][1]
    err = float((a - b).abs().max() / a.abs().max())
    print(f"{name:15s} M={M:2d} N={N:5d} K={K:5d}  fp32 X {min(u for u, _ in out['fp32']):6.2f} us  packed X "
          f"{min(u for u, _ in out['packed']):6.2f} us  max rel diff {err:.1e}", flush=True)
    del lins, ys
    torch.cuda.empty_cache()
