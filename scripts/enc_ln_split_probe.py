"""The speech encoder's LayerNorm-on-load GEMMs (q|k|v 1024 -> 3072, FFN w_1 1024 -> 4096 + ReLU; fo_gemm_ln) at the
listen chunk's 32 rows and the duplex tick's 56, with the K range split over 1 / 2 / 4 / 8 workgroups (+ the reduce
launch when split): each column tile's workgroup reads all M rows of X for its K range, so the X bytes per workgroup
fall with the split while the partial slabs and the reduce launch are added.  Graph-replayed over 4 weight copies.
python scripts/enc_ln_split_probe.py (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
D, NCP = 1024, 4
prod = ops.PackedLinear((torch.randn(D, D, device=dev, generator=g) * 0.03).to(torch.bfloat16))
lnw = 1 + 0.1 * torch.randn(D, device=dev, generator=g)
lnb = 0.1 * torch.randn(D, device=dev, generator=g)
for name, N, act in (("qkv", 3 * D, "none"), ("ff1", 4 * D, "relu")):
    ws = [ops.PackedLinear((torch.randn(N, D, device=dev, generator=g) * 0.03).to(torch.bfloat16),
                           bias=torch.randn(N, device=dev, generator=g) * 0.1) for _ in range(NCP)]
    for M in (32, 56):
        xin = torch.randn(M, D, device=dev, generator=g)
        x = torch.empty(M, D, device=dev)
        st = ops.RowStats(M, dev, with_sums=True)
        prod.rowstats(xin, x, st)
        out = torch.empty(M, N, device=dev)
        ref = ws[0].ln(x, lnw, lnb, st, out=torch.empty(M, N, device=dev), act=act).clone()
        row = []
        for S in (1, 2, 4, 8):
            it = iter(range(1 << 30))
            t = graph_time(lambda: ws[next(it) % NCP].ln(x, lnw, lnb, st, out=out, act=act, splitk=S), NCP * 10)
            o = ws[0].ln(x, lnw, lnb, st, out=torch.empty(M, N, device=dev), act=act, splitk=S)
            err = float((o - ref).abs().max() / (ref.abs().max() + 1e-30))
            row.append(f"S{S} {t:6.2f} us (rel {err:.1e})")
        print(f"{name} M={M:2d} N={N}: " + " | ".join(row), flush=True)
