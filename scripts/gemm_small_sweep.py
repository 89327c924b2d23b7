"""The Qwen2 o projection (N 3584, K 3584) and plain q|k|v (N 4608) at 16 / 8 rows, as the layer launches them
(o: residual + next-norm statistics epilogue), over tiles per workgroup x K split across workgroups (the split
merged inside the launch by its last arriver, fo_gemm merge mode 2): with the K range split S ways every
workgroup reads 1/S of the fp32 activation rows, the re-read that sets these latency-bound launches' time.
Graph-replayed over weight copies beyond the Infinity Cache; error vs a torch fp32 reference per configuration.
python scripts/gemm_small_sweep.py (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import _lib, ops  # noqa: E402
from fo.ops import PackedLinear  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda:0")
CFGS = [(0, 0, 0), (16, 1, 1), (16, 1, 2), (8, 2, 2), (8, 2, 4), (8, 4, 4), (8, 4, 8), (8, 8, 8), (8, 7, 8),
        (16, 2, 2), (16, 4, 4), (8, 8, 4), (4, 8, 8)]
for name, N, K, stats in (("qwen_o", 3584, 3584, True), ("qwen_qkv", 4608, 3584, False)):
    copies = 24
    ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
    lins = [PackedLinear(w) for w in ws]
    gamma = torch.ones(N, device=dev)
    for M in (16, 8):
        x = torch.randn(M, K, device=dev)
        res0 = torch.randn(M, N, device=dev)
        out = res0.clone()
        st = ops.RowStats(M, dev)
        yg = torch.empty(M, N, device=dev)
        ref = (res0 if stats else 0) + x @ ws[0].float().t()
        scale = ref.abs().max().item()
        rows = []
        for nw, nt, S in CFGS:
            lib.fo_gemm_tune(nw, nt)
            it = iter(range(1 << 30))

            def f(S=S):
                i = next(it) % copies
                if stats:
                    lins[i](x, out=out, residual=True, M=M, splitk=S, stats_out=st.set(gamma, yg))
                else:
                    lins[i](x, out=out, M=M, splitk=S)
            try:
                t = graph_time(f, 48)
            except RuntimeError as e:
                rows.append((1e9, f"nw{nw} nt{nt} S{S} failed: {e}"))
                continue
            ops.Runtime.get(dev).ws.zero_()
            out.copy_(res0)
            if stats:
                lins[0](x, out=out, residual=True, M=M, splitk=S, stats_out=st.set(gamma, yg))
            else:
                lins[0](x, out=out, M=M, splitk=S)
            torch.cuda.synchronize()
            err = (out - ref).abs().max().item() / scale
            rows.append((t, f"{'auto' if nw == 0 else f'nw{nw} nt{nt} S{S}'}  err {err:.1e}"))
        lib.fo_gemm_tune(0, 0)
        rows.sort()
        print(f"{name} M={M}: " + " | ".join(f"{d} {t:.2f}us" for t, d in rows[:8]), flush=True)
    del lins, ws
    torch.cuda.empty_cache()
