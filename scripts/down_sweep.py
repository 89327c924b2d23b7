"""Qwen2 down projection (N 3584, K 18944, M = 16 listen / 8 text) over waves x tiles per workgroup x K split x
pipelined loop (fo_gemm_tune / splitk / fo_gemm_set_pipe), with the RMSNorm-statistics epilogue and residual the
layer uses, event-timed over two alternating weight copies (> the 256 MB Infinity Cache); the reduce launch of
the K split is inside the time.  python scripts/down_sweep.py (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib, timeit  # noqa: E402
from fo import ops  # noqa: E402

dev = torch.device("cuda:0")
N, K = 3584, 18944
lins = []
for c in range(2):
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    lins.append(PackedLinear(w))
    if c == 0:
        w0 = w
    del w
gamma = torch.ones(N, device=dev)
for M in (16, 8):
    x = torch.randn(M, K, device=dev)
    res0 = torch.randn(M, N, device=dev)
    outs = [res0.clone() for _ in range(2)]
    stats = ops.RowStats(M, dev)
    yg = torch.empty(M, N, device=dev)

    def run(i, S=0):
        outs[i].copy_(res0)
        return lins[i](x, out=outs[i], residual=True, M=M, splitk=S, stats_out=stats.set(gamma, yg))

    lib.fo_gemm_tune(0, 0)
    lib.fo_gemm_set_pipe(3)
    run(0)
    torch.cuda.synchronize()
    ref = res0 + x @ w0.float().t()   # torch fp32 reference of the same bf16 weights
    scale = ref.abs().max().item()
    aerr = (outs[0] - ref).abs().max().item() / scale
    auto = min(timeit([lambda i=i: run(i) for i in range(2)]) for _ in range(2))
    res = []
    # DOWN_CFGS="pipe,nw,nt,S;...": only those configurations (default: the full grid)
    cfgs = [tuple(int(v) for v in c.split(",")) for c in os.environ.get("DOWN_CFGS", "").split(";") if c] or \
        [(p, w, t, s) for p in (0, 2) for w in (8, 16) for t in (4, 8) for s in (4, 8, 16)]
    for pipe, nw, nt, S in cfgs:
                if True:
                    lib.fo_gemm_set_pipe(pipe)
                    lib.fo_gemm_tune(nw, nt)
                    try:
                        t = min(timeit([lambda i=i: run(i, S) for i in range(2)]) for _ in range(2))
                    except RuntimeError as e:
                        res.append((1e9, f"pipe{pipe} nw{nw} nt{nt} S{S} failed: {e}"))
                        continue
                    ops.Runtime.get(dev).ws.zero_()   # no stale split-K slabs from an earlier configuration
                    run(0, S)
                    torch.cuda.synchronize()
                    err = (outs[0] - ref).abs().max().item() / scale
                    bad = (outs[0] - ref).abs() > 1e-3 * scale
                    where = ""
                    if bad.any():
                        rows, cols = bad.nonzero(as_tuple=True)
                        where = (f" ERR {err:.2g} ({int(bad.sum())} elems, rows {sorted(set(rows.tolist()))[:4]},"
                                 f" cols {cols.min().item()}..{cols.max().item()})")
                    res.append((t, f"pipe{pipe} nw{nw} nt{nt} S{S}{where}"))
    lib.fo_gemm_tune(0, 0)
    lib.fo_gemm_set_pipe(3)
    res.sort()
    print(f"down M={M} auto {auto:.1f}us ({lins[0].nbytes / auto / 1e6:.2f} TB/s), rel err vs torch fp32 {aerr:.2g}",
          flush=True)
    for t, d in res:
        print(f"   {t:6.1f}us {lins[0].nbytes / t / 1e6:.2f}TB/s  {d}", flush=True)
