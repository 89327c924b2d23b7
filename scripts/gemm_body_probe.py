"""Price the parts of the GEMM main loop (measurement tool, GPU only): cold-weight launches of the
probe body (scripts/probe/probe.hip k_gemm_probe) with X loads / MFMAs toggled, next to the bare
read of the same packed weights.  python scripts/gemm_body_probe.py"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
probe = ctypes.CDLL(os.path.join(ROOT, "scripts", "probe", "libprobe.so"))
probe.probe_gemm.restype = ctypes.c_double
probe.probe_gemm.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_int]
probe.probe_time.restype = ctypes.c_double
probe.probe_time.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_longlong,
                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
XM = {0: "f32hilo", 1: "noX", 2: "bf16", 3: "presplit", 4: "f32hilo-IL"}
shapes = [("qwen_gu", 2368, 3584, [(4, 4, 4), (8, 4, 4), (8, 4, 3), (16, 4, 1), (16, 4, 2), (8, 2, 4), (4, 2, 4),
                                     (4, 4, 6), (4, 4, 8)]),
          ("qwen_down", 224, 18944, [(1, 16, 4), (2, 16, 4)]),
          ("qwen_o", 224, 3584, [(1, 16, 4), (1, 4, 4)]),
          ("qwen_qkv", 288, 3584, [(1, 16, 4), (2, 8, 4)])]
pipes = {"qwen_gu": [(4, 4, 2), (4, 4, 4), (4, 8, 2), (2, 8, 2), (2, 8, 4), (8, 4, 1), (2, 4, 4)],
         "qwen_down": [(1, 16, 2), (1, 16, 4), (2, 16, 2), (1, 8, 4)],
         "qwen_o": [(1, 16, 2), (1, 16, 4), (1, 4, 4), (1, 8, 4)],
         "qwen_qkv": [(1, 16, 2), (1, 16, 4), (2, 8, 2), (1, 8, 4), (1, 4, 4)]}
probe.probe_pipe.restype = ctypes.c_double
probe.probe_pipe.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
out = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
for name, ntiles, K, cfgs in shapes[:1] if len(sys.argv) > 1 else shapes:
    nb = ntiles * 16 * K * 2
    C = max(2, int(1.6e9 // nb) + 1)
    bufs = [torch.randint(-2000, 2000, (nb // 2,), dtype=torch.int16, device=dev) for _ in range(C)]
    arr = (ctypes.c_void_p * C)(*[b.data_ptr() for b in bufs])
    X = torch.randn(16, K, device=dev)
    Y = torch.empty(16, ntiles * 16, device=dev)
    reps = max(C, 48)
    rds = []
    for nt, nw, u in ((1, 16, 4), (4, 4, 4), (8, 4, 4), (16, 4, 2), (8, 2, 4), (4, 4, 8), (4, 4, 6), (8, 4, 2)):
        if ntiles % nt == 0:
            rds.append(f"nt{nt}nw{nw}u{u} {probe.probe_time(1, arr, C, nb, ntiles, K // 32, nt, nw, u, 0, reps, out.data_ptr()):.1f}"
                       f"/il {probe.probe_time(2, arr, C, nb, ntiles, K // 32, nt, nw, u, 0, reps, out.data_ptr()):.1f}")
    print(f"{name}: {nb / 1e6:.1f} MB, bare read " + " ".join(rds), flush=True)
    for nt, nw, u in cfgs:
        row = []
        for xm, mf in ((0, 1), (4, 1), (3, 1), (2, 1), (1, 1), (0, 0)):
            t = probe.probe_gemm(arr, C, ntiles, K, nt, nw, u, xm, mf, X.data_ptr(), Y.data_ptr(), reps)
            row.append(f"{XM[xm]}{'' if mf else '-nomfma'} {t:6.1f}")
        print(f"  nt{nt} nw{nw} u{u}: " + " | ".join(row), flush=True)
    for nt, nw, u in pipes[name] if len(sys.argv) < 2 else []:
        row = [f"spl{spl} {probe.probe_pipe(arr, C, ntiles, K, nt, nw, u, spl, X.data_ptr(), Y.data_ptr(), reps):6.1f}"
               for spl in (0, 1)]
        print(f"  PIPE nt{nt} nw{nw} u{u}: " + " | ".join(row), flush=True)
    del bufs
    torch.cuda.empty_cache()
