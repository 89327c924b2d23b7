"""Qwen2 gate/up (M = 8, 16; fused SwiGLU) over waves x tiles-per-workgroup x K split x pipelined loop,
event-timed over two alternating weight copies (> the 256 MB Infinity Cache)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib, timeit  # noqa: E402

dev = torch.device("cuda:0")
N, K = 18944, 3584
lins = []
for c in range(2):
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    lins.append(PackedLinear(w, swiglu_up=w))
    del w
for M in (16, 8):
    x = torch.randn(M, K, device=dev)
    outs = [torch.empty(M, N, device=dev) for _ in range(2)]
    res = []
    ref = lins[0](x, out=torch.empty(M, N, device=dev)).clone()
    for pipe in (0, 1, 2):
        for nw in (4, 8):
            for nt in (2, 4, 8):
                for S in (1, 2, 4):
                    lib.fo_gemm_set_pipe(pipe)
                    lib.fo_gemm_tune(nw, nt)
                    t = min(timeit([lambda i=i: lins[i](x, out=outs[i], splitk=S) for i in range(2)]) for _ in range(2))
                    err = (outs[0] - ref).abs().max().item()
                    res.append((t, f"pipe{pipe} nw{nw} nt{nt} S{S}" + ("" if err < 1e-4 else f" ERR {err:.2g}")))
    lib.fo_gemm_tune(0, 0)
    lib.fo_gemm_set_pipe(0)
    auto = min(timeit([lambda i=i: lins[i](x, out=outs[i]) for i in range(2)]) for _ in range(2))
    res.sort()
    print(f"gate/up M={M} auto {auto:.1f}us ({lins[0].nbytes / auto / 1e6:.2f} TB/s)", flush=True)
    for t, d in res[:10]:
        print(f"   {t:6.1f}us {lins[0].nbytes / t / 1e6:.2f}TB/s  {d}", flush=True)
