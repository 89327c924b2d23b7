"""Does a weight prefetch into the Infinity Cache (MALL, 256 MB) shorten the latency-bound Qwen2 GEMMs?
For each shape: one event-timed launch after a 1 GB flush (cold), and after the flush + a read of the
packed weights with default-policy loads (warm).  python scripts/mall_probe.py (GPU only)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "freeze-omni_amd"))
from fo import _lib, ops  # noqa: E402
from fo.ops import PackedLinear  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
lib.fo_event_create(ctypes.byref(e0))
lib.fo_event_create(ctypes.byref(e1))
flush = torch.zeros(256 << 20, device=dev)   # 1 GiB


def one(fn):
    s = ops.stream()
    lib.fo_event_record(e0, s)
    fn()
    lib.fo_event_record(e1, s)
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value * 1e3


for name, N, K, M, sw in [("qwen_qkv", 4608, 3584, 16, False), ("qwen_o", 3584, 3584, 16, False),
                          ("qwen_down", 3584, 18944, 16, False), ("qwen_gu", 18944, 3584, 16, True)]:
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    lin = PackedLinear(w, swiglu_up=w if sw else None)
    del w
    x = torch.randn(M, K, device=dev)
    out = torch.empty(M, N, device=dev)
    view = lin.packed.view(torch.int32)
    res = {"cold": [], "warm": [], "hot": []}
    for _ in range(10):
        flush.add_(1.0)
        res["cold"].append(one(lambda: lin(x, out=out)))
        flush.add_(1.0)
        view.sum()                     # default-policy read of the packed weights
        res["warm"].append(one(lambda: lin(x, out=out)))
        res["hot"].append(one(lambda: lin(x, out=out)))   # right after itself
    torch.cuda.synchronize()
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    print(f"{name:9s} {lin.nbytes / 1e6:7.1f}MB cold {med['cold']:6.1f}us warm(after prefetch) {med['warm']:6.1f}us "
          f"hot(replay) {med['hot']:6.1f}us", flush=True)
