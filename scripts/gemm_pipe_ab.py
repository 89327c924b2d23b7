"""A/B of the software-pipelined weight-stream GEMM (fo_gemm_set_pipe 0/1/2) on the M <= 16 hot shapes:
event-timed average per launch over alternating weight copies (> the 256 MB Infinity Cache), and a
bit-equality check of the outputs against the plain loop."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "freeze-omni_amd"))
from fo import _lib, ops  # noqa: E402
from fo.ops import PackedLinear  # noqa: E402

lib = _lib.load()


def timeit(fns, reps=40):
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.fo_event_create(ctypes.byref(e0))
    lib.fo_event_create(ctypes.byref(e1))
    for f in fns:
        f()
    s = ops.stream()
    lib.fo_event_record(e0, s)
    for i in range(reps):
        fns[i % len(fns)]()
    lib.fo_event_record(e1, s)
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value / reps * 1e3


shapes = [("qwen_gu", 18944, 3584, 16, True), ("qwen_gu_m8", 18944, 3584, 8, True), ("qwen_down", 3584, 18944, 16, False),
          ("qwen_qkv", 4608, 3584, 16, False), ("qwen_o", 3584, 3584, 16, False), ("lm_head", 152064, 3584, 8, False)]
if __name__ != "__main__":   # imported for timeit() by gemm_gu_sweep.py
    shapes = []
dev = torch.device("cuda:0")
for name, N, K, M, sw in shapes:
    ncp = 2 if N * K * 2 * (2 if sw else 1) > (128 << 20) else 6
    lins = []
    for c in range(ncp):
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        lins.append(PackedLinear(w, swiglu_up=w if sw else None))
        del w
    x = torch.randn(M, K, device=dev)
    outs = [torch.empty(M, N, device=dev) for _ in range(ncp)]
    res = {}
    ref = None
    for mode in (0, 1, 2, 0, 1, 2):
        lib.fo_gemm_set_pipe(mode)
        t = timeit([lambda i=i: lins[i](x, out=outs[i]) for i in range(ncp)])
        res.setdefault(mode, []).append(t)
        lins[0](x, out=outs[0])
        torch.cuda.synchronize()
        if ref is None:
            ref = outs[0].clone()
        same = torch.equal(outs[0], ref)
        if not same:
            print(f"  {name} mode {mode}: max diff {(outs[0] - ref).abs().max().item():.3g}", flush=True)
    lib.fo_gemm_set_pipe(0)
    mb = lins[0].nbytes / 1e6
    print(f"{name:10s} M={M:2d} {mb:7.1f}MB " + " ".join(
        f"pipe{m}: {min(v):6.1f}us ({lins[0].nbytes / min(v) / 1e6:4.2f}TB/s)" for m, v in res.items()), flush=True)
    del lins, outs
    torch.cuda.empty_cache()
