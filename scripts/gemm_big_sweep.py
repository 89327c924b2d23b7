"""Tile / wave / K-split sweep of the 64-row-tile GEMM (k_gemm<NT, 4, NW, 2>) on the many-row shapes of a turn: the
AR decoder's sentence prefill (8 sessions x 32-40 sub-token rows: M 256 / 320 at D 896, FFN 4864) and the speech
encoder's 3x3 stride-2 convolutions (im2col: conv1 M 2808 K 32, conv2 M 608 K 9216, N 1024).  Each configuration is
event-timed over 20 launches (fo_gemm_tune forces waves / tiles, splitk the K split) and checked against fp64.
    python scripts/gemm_big_sweep.py (GPU only)"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "freeze-omni_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_sweep_util import timeit  # noqa: E402
from fo import _lib  # noqa: E402
from fo.ops import PackedLinear  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
SHAPES = [("tts_o", 256, 896, 896, False), ("tts_down", 256, 896, 4864, False), ("tts_qkv", 256, 2688, 896, False),
          ("tts_gu", 256, 4864, 896, True), ("tts_down320", 320, 896, 4864, False), ("tts_gu320", 320, 4864, 896, True),
          ("enc_conv2", 608, 1024, 9216, False), ("enc_conv1", 2808, 1024, 32, False)]
CONFIGS = [(0, 0, 0)] + [(nw, nt, s) for nt in (1, 2, 4, 8) for nw in (4, 8, 16) for s in (1, 2, 4, 8)
                         if not (nt == 8 and nw > 4) and not (nt == 4 and nw > 8)]
for name, M, N, K, sw in SHAPES:
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    u = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16) if sw else None
    x = torch.randn(M, K, generator=g)
    a = x.double() @ w.double().t()
    ref = (torch.nn.functional.silu(a) * (x.double() @ u.double().t())) if sw else a
    lin = PackedLinear(w.to(dev), swiglu_up=None if u is None else u.to(dev))
    xd = x.to(dev)
    out = torch.empty(M, N, device=dev)
    res = []
    for nw, nt, s in CONFIGS:
        if s and s > (K // 32):
            continue
        lib.fo_gemm_tune(nw, nt)
        try:
            fn = (lambda: lin(xd, out=out, splitk=s)) if s else (lambda: lin(xd, out=out))
            fn()
            torch.cuda.synchronize()
            err = float((out.cpu().double() - ref).abs().max() / ref.abs().max())
            t = timeit(fn, reps=20)
        except Exception as e:   # a configuration the dispatcher refuses
            lib.fo_gemm_tune(0, 0)
            continue
        finally:
            lib.fo_gemm_tune(0, 0)
        res.append((t, nw, nt, s, err))
    res.sort()
    auto = [r for r in res if r[1] == 0]
    print(f"{name:12s} M{M} N{N} K{K}{' sw' if sw else ''}: auto {auto[0][0]:7.1f}us (err {auto[0][4]:.1e}) | best "
          + " ".join(f"nw{nw}nt{nt}S{s}:{t:.1f}({e:.0e})" for t, nw, nt, s, e in res[:6]), flush=True)
