"""Does a partly Infinity-Cache-resident weight stream run faster?  The Qwen2 gate/up (k_gemm_xs, 272 MB,
237 workgroups x 4-5 units of 224 KB) timed after a 1 GiB flush and a default-policy read of the first p
units of every workgroup's range (p = 0..5: 0 .. 272 MB; the MALL holds 256 MB), HIP events on the stream.
python scripts/gu_mall_probe.py (GPU only)."""
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
D, I, M = 3584, 18944, 16
g = torch.Generator(device=dev).manual_seed(0)
w = (torch.randn(I, D, device=dev, generator=g) * 0.02).to(torch.bfloat16)
u = (torch.randn(I, D, device=dev, generator=g) * 0.02).to(torch.bfloat16)
gu = PackedLinear(w, swiglu_up=u)
del w, u
x = torch.randn(M, D, device=dev, generator=g)
out = torch.empty(M, I, device=dev)
view = gu.packed.view(torch.int32)
units = gu.packed.numel() * 2 // (2 * 112 * 1024)
per = (units + 255) // 256
G = (units + per - 1) // per
unit_i32 = 2 * 112 * 1024 // 4
ranges = [(units * b // G, units * (b + 1) // G) for b in range(G)]
sink = torch.zeros(1, device=dev, dtype=torch.int64)


def one():
    s = ops.stream()
    lib.fo_event_record(e0, s)
    gu(x, out=out)
    lib.fo_event_record(e1, s)
    ms = ctypes.c_float()
    torch.cuda.synchronize()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value * 1e3


print(f"units {units} per-WG {per} grid {G} unit {unit_i32 * 4 / 1e3:.0f} KB", flush=True)
for p in range(0, per + 1):
    ts = []
    for _ in range(8):
        flush.fill_(1.0)
        if p:
            for ub, ue in ranges:
                sink += view[ub * unit_i32:min(ub + p, ue) * unit_i32].sum()
        torch.cuda.synchronize()
        ts.append(one())
    ts.sort()
    mb = sum(min(p, ue - ub) for ub, ue in ranges) * unit_i32 * 4 / 1e6
    med = ts[len(ts) // 2]
    print(f"prefetched {mb:6.1f} MB: gate/up {med:6.2f} us ({gu.nbytes / med / 1e6:.2f} TB/s)  min {ts[0]:6.2f}",
          flush=True)
