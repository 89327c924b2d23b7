"""GEMM shape/split sweep on the GPU: event-timed average per launch for the hot-path shapes."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "freeze-omni_amd"))
from fo import _lib, ops  # noqa: E402
from fo.ops import PackedLinear  # noqa: E402


def timeit(fn, reps=30):
    lib = _lib.load()
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.fo_event_create(ctypes.byref(e0))
    lib.fo_event_create(ctypes.byref(e1))
    for _ in range(3):
        fn()
    s = ops.stream()
    lib.fo_event_record(e0, s)
    for _ in range(reps):
        fn()
    lib.fo_event_record(e1, s)
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value / reps * 1e3


shapes = [("qwen_down_m8", 3584, 18944, 8, False), ("qwen_gu_m8", 18944, 3584, 8, True), ("qwen_qkv", 4608, 3584, 16, False), ("qwen_o", 3584, 3584, 16, False), ("qwen_down", 3584, 18944, 16, False),
          ("qwen_gu", 18944, 3584, 16, True), ("tts_qkv", 2688, 896, 8, False), ("tts_o", 896, 896, 8, False),
          ("tts_gu", 4864, 896, 8, True), ("tts_down", 896, 4864, 8, False), ("lm_head", 152064, 3584, 8, False)]
if len(sys.argv) > 1 and sys.argv[1] == "enc":   # speech encoder / adapter: 8 users x 4 frames (2 for the adapter)
    shapes = [("enc_qkv", 3072, 1024, 32, False), ("enc_o", 1024, 1024, 32, False), ("enc_ff1", 4096, 1024, 32, False),
              ("enc_ff2", 1024, 4096, 32, False), ("ada_conv", 2048, 5120, 16, False), ("ada_proj", 3584, 2048, 16, False),
              ("sub_out", 1024, 4864, 32, False)]
dev = torch.device("cuda:0")
lib = _lib.load()
for name, N, K, M, sw in shapes:
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    lin = PackedLinear(w, swiglu_up=w if sw else None)
    x = torch.randn(M, K, device=dev)
    out = torch.empty(M, N, device=dev)
    ref = lin(x, out=torch.empty(M, N, device=dev)).clone()
    auto = timeit(lambda: lin(x, out=out))
    res = []
    for nw in (4, 8, 16):
        for nt in ((2, 4) if sw else (1, 2, 4)):
            for S in (1, 2, 4):
                lib.fo_gemm_tune(nw, nt)
                t = timeit(lambda: lin(x, out=out, splitk=S))
                err = (out - ref).abs().max().item()
                res.append((t, f"nw{nw}nt{nt}S{S}:{t:6.1f}" + ("" if err < 1e-3 else f"(ERR {err:.2g})")))
    lib.fo_gemm_tune(0, 0)
    res.sort()
    print(f"{name:9s} M={M:2d} N={N:6d} K={K:5d} {lin.nbytes / 1e6:7.1f}MB auto {auto:6.1f}us "
          f"({lin.nbytes / auto / 1e6:4.2f} TB/s) best: " + " ".join(r for _, r in res[:6]), flush=True)
