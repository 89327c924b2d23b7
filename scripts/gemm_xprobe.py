"""fp32 (hi/lo split) vs bf16 activations for the Qwen2 GEMM shapes (is the split a cost?)."""
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
for name, N, K, M, sw in [("qwen_qkv", 4608, 3584, 16, False), ("qwen_o", 3584, 3584, 16, False),
                          ("qwen_down", 3584, 18944, 16, False), ("qwen_gu", 18944, 3584, 16, True),
                          ("qwen_gu_m8", 18944, 3584, 8, True), ("qwen_down_m8", 3584, 18944, 8, False)]:
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    lin = PackedLinear(w, swiglu_up=w if sw else None)
    out = torch.empty(M, N, device=dev)
    r = []
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(M, K, device=dev).to(dt)
        for nw, u in ((0, 0), (4, 4), (8, 4), (16, 4)):
            lib.fo_gemm_tune(nw, 0)
            t = timeit(lambda: lin(x, out=out))
            r.append(f"{'f32' if dt == torch.float32 else 'bf16'}/nw{nw}u{u}:{t:6.1f}")
        lib.fo_gemm_tune(0, 0)
    print(f"{name:12s} {lin.nbytes / 1e6:7.1f}MB " + " ".join(r), flush=True)
