"""Tile shape / K split sweep of the 17-64-row Qwen2 GEMMs (chunk 0 with its chat prefix M=56, the
assistant prefix M=40, duplex chunks M=32), graph-replayed over enough weight copies that no launch
finds its weights in cache (as scripts/gemm_graph_sweep.py).  python scripts/gemm_mid_sweep.py (GPU).
The (waves, tiles) forcing reached the mid-row kernels only in the 8-tile trial recorded in DESIGN.md
section 5 (profiles/r01g_gemm_mid_sweep.log); on the current library only the K split varies here."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "freeze-omni_amd"))
from fo import _lib, ops  # noqa: E402
from fo.ops import PackedLinear  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
es = ops.engine_stream(dev)
e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
lib.fo_event_create(ctypes.byref(e0))
lib.fo_event_create(ctypes.byref(e1))


def graph_time(fn, reps):
    s = es.cuda_stream
    with torch.cuda.stream(es):
        fn()
        _lib.call("fo_graph_begin", s)
        try:
            for _ in range(reps):
                fn()
        finally:
            ex = ctypes.c_void_p()
            _lib.call("fo_graph_end", s, ctypes.byref(ex))
        _lib.call("fo_graph_launch", ex, s)
        lib.fo_event_record(e0, s)
        _lib.call("fo_graph_launch", ex, s)
        lib.fo_event_record(e1, s)
        torch.cuda.synchronize()
        _lib.call("fo_graph_destroy", ex)
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value / reps * 1e3


shapes = [("gu", 18944, 3584, True), ("down", 3584, 18944, False), ("qkv", 4608, 3584, False), ("o", 3584, 3584, False)]
Ms = [int(m) for m in sys.argv[1:]] or [32, 40, 56]
for name, N, K, sw in shapes:
    copies = max(2, min(8, int(1.2e9 // (N * K * 2 * (2 if sw else 1)))))
    lins = []
    for c in range(copies):
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        lins.append(PackedLinear(w, swiglu_up=w if sw else None))
        del w
    reps = copies * max(1, 16 // copies)
    for M in Ms:
        x = torch.randn(M, K, device=dev)
        out = torch.empty(M, N, device=dev)
        res = []
        for nw, nt in ((0, 0), (4, 4), (8, 4), (2, 4), (4, 8), (2, 8), (4, 2), (8, 2)):
            if sw and nt == 1:
                continue
            for S in (0, 1, 2, 4, 8):
                lib.fo_gemm_tune(nw, nt)
                it = iter(range(1 << 30))
                t = graph_time(lambda: lins[next(it) % copies](x, out=out, splitk=S), reps)
                res.append((t, f"nw{nw}nt{nt}S{S}"))
        lib.fo_gemm_tune(0, 0)
        auto = [t for t, k in res if k == "nw0nt0S0"][0]
        res.sort()
        print(f"{name:5s} M={M:2d} {lins[0].nbytes / 1e6:6.1f}MB auto {auto:7.2f}us best: "
              + " ".join(f"{k}:{t:.2f}" for t, k in res[:6]), flush=True)
    del lins
    torch.cuda.empty_cache()
