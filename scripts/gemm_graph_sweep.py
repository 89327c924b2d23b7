"""Device-side GEMM sweep for the latency-bound shapes: each configuration is captured as a hipGraph of
`reps` launches that walk `copies` weight copies (so no launch finds its weights in cache) and replayed
once, event-timed -- no Python launch overhead in the number (scripts/gemm_sweep.py's eager timing
floors at ~8.5 us per launch on the host).  python scripts/gemm_graph_sweep.py (GPU only)."""
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
        fn()  # allocate / warm outside the capture
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


if len(sys.argv) > 1 and sys.argv[1] == "mid":   # duplex: 8 sessions x 7 encoder frames / x 4(+5) LLM rows
    shapes = [("enc_qkv56", 3072, 1024, 56, False), ("enc_o56", 1024, 1024, 56, False),
              ("enc_ff1_56", 4096, 1024, 56, False), ("enc_ff2_56", 1024, 4096, 56, False),
              ("qwen_gu32", 18944, 3584, 32, True), ("qwen_gu48", 18944, 3584, 48, True),
              ("qwen_down32", 3584, 18944, 32, False), ("qwen_qkv32", 4608, 3584, 32, False)]
elif len(sys.argv) > 1 and sys.argv[1] == "tts":   # the AR decode step's shapes only
    shapes = [("tts_qkv", 1152, 896, 8, False), ("tts_o", 896, 896, 8, False), ("tts_gu", 4864, 896, 8, True),
              ("tts_down", 896, 4864, 8, False), ("tts_out", 1028, 896, 8, False)]
else:
    shapes = None
shapes = shapes or [("tts_qkv", 2688, 896, 8, False), ("tts_o", 896, 896, 8, False), ("tts_gu", 4864, 896, 8, True),
          ("tts_down", 896, 4864, 8, False), ("tts_out", 1028, 896, 8, False),
          ("qwen_qkv", 4608, 3584, 16, False), ("qwen_o", 3584, 3584, 16, False),
          ("qwen_down", 3584, 18944, 16, False), ("qwen_gu", 18944, 3584, 16, True)]
for name, N, K, M, sw in shapes:
    copies = max(2, min(24, int(1.2e9 // (N * K * 2 * (2 if sw else 1)))))
    lins = []
    for c in range(copies):
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        lins.append(PackedLinear(w, swiglu_up=w if sw else None))
        del w
    x = torch.randn(M, K, device=dev)
    out = torch.empty(M, N, device=dev)
    reps = copies * max(1, 48 // copies)
    res = []
    for nw in (0, 4, 8, 16):
        for nt in ((0,) if nw == 0 else ((2, 4) if sw else (1, 2, 4))):
            for S in ((0,) if nw == 0 else (1, 2, 4)):
                lib.fo_gemm_tune(nw, nt)
                it = iter(range(1 << 30))
                t = graph_time(lambda: lins[next(it) % copies](x, out=out, splitk=S), reps)
                res.append((t, "auto" if nw == 0 else f"nw{nw}nt{nt}S{S}"))
    lib.fo_gemm_tune(0, 0)
    auto = [t for t, k in res if k == "auto"][0]
    res.sort()
    print(f"{name:9s} M={M:2d} {lins[0].nbytes / 1e6:7.1f}MB auto {auto:6.2f}us best: "
          + " ".join(f"{k}:{t:.2f}" for t, k in res[:6]), flush=True)
    del lins
    torch.cuda.empty_cache()
