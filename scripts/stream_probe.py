"""Cold-weight GEMM timing vs the read-only stream ceiling (measurement tool, GPU only).

Every timed launch reads a different copy of the weights (copies total > 1.5 GB, beyond the 256 MB
Infinity Cache), as in a real forward where each layer's weights are read once.  Launch sequences
are captured in a graph so host launch cost stays out of the numbers.
  python scripts/stream_probe.py            # hot-path shapes
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
from fo import _lib  # noqa: E402
from fo.ops import PackedLinear  # noqa: E402

probe = ctypes.CDLL(os.path.join(ROOT, "scripts", "probe", "libprobe.so"))
probe.probe_time.restype = ctypes.c_double
probe.probe_time.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_longlong,
                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
out_u = torch.zeros(1 << 16, dtype=torch.int32, device=dev)


def read_probe(kind, bufs, bytes_, ntiles=0, KS=0, nt=0, nw=0, u=0, grid=0, reps=24):
    arr = (ctypes.c_void_p * len(bufs))(*[b.data_ptr() for b in bufs])
    return probe.probe_time(kind, arr, len(bufs), bytes_, ntiles, KS, nt, nw, u, grid, reps, out_u.data_ptr())


def graph_time(fns, reps):
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for f in fns:
            f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for r in range(reps):
            fns[r % len(fns)]()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


shapes = [("qwen_gu", 18944, 3584, 16, True), ("qwen_down", 3584, 18944, 16, False), ("qwen_qkv", 4608, 3584, 16, False),
          ("qwen_o", 3584, 3584, 16, False), ("tts_gu", 4864, 896, 8, True), ("tts_qkv", 2688, 896, 8, False),
          ("enc_ff1", 4096, 1024, 32, False), ("enc_qkv", 3072, 1024, 32, False)]
if len(sys.argv) > 1:
    shapes = [s for s in shapes if s[0] in sys.argv[1:]]
lib = _lib.load()
for name, N, K, M, sw in shapes:
    one = N * K * 2 * (2 if sw else 1)
    C = max(2, min(24, int(1.6e9 // one) + 1))
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    lins = [PackedLinear(w, swiglu_up=w if sw else None) for _ in range(C)]
    x = torch.randn(M, K, device=dev)
    out = torch.empty(M, N, device=dev)
    reps = max(C, 48)
    cold = graph_time([lambda L=L: L(x, out=out) for L in lins], reps)
    warm = graph_time([lambda: lins[0](x, out=out)], reps)
    nb = lins[0].nbytes
    line = f"{name:9s} M={M:2d} {nb / 1e6:6.1f}MB x{C:2d} gemm cold {cold:6.1f}us ({nb / cold / 1e3:4.2f}TB/s) warm {warm:6.1f}us"
    KS = lins[0].Kp // 32
    ntiles = lins[0].packed.numel() // (KS * 512)
    bufs = [L.packed for L in lins]
    res = []
    for nt, nw, u in ((1, 4, 4), (2, 4, 4), (4, 4, 4), (2, 8, 4), (4, 8, 4), (1, 16, 4), (4, 4, 2), (8, 4, 2),
                      (2, 8, 8), (1, 16, 8)):
        if ntiles % nt:
            continue
        t = read_probe(1, bufs, nb, ntiles, KS, nt, nw, u, reps=reps)
        res.append((t, f"nt{nt}nw{nw}u{u}:{t:.1f}"))
    res.sort()
    lin_t = [(read_probe(0, bufs, nb, grid=g, reps=reps), g) for g in (512, 1024, 2048, 4096)]
    lb = min(lin_t)
    print(line + f" | read frag best {res[0][1]} ({nb / res[0][0] / 1e3:4.2f}TB/s) "
          + " ".join(r for _, r in res[1:4]) + f" | read lin {lb[0]:.1f}us g{lb[1]} ({nb / lb[0] / 1e3:4.2f}TB/s)",
          flush=True)
    del lins, bufs
    torch.cuda.empty_cache()
