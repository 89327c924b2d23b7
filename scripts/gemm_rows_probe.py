"""k_gemm_rows (65..128 rows: the waves split the rows, weight fragments shared through an LDS-DMA ring) against the
two row-half launches of k_gemm_xsk it replaces, on the Qwen2 gate/up (272 MB, SwiGLU) and down (136 MB, residual),
graph-replayed over two weight copies (> the Infinity Cache); each time includes the k_gemm_reduce launch.  Also
the 64-row k_gemm_xsk for scale, and the max |difference| of the two paths' outputs (fp32 summation order only).
python scripts/gemm_rows_probe.py [M ...] (GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402

dev = torch.device("cuda:0")
D, I = 3584, 18944
Ms = [int(m) for m in sys.argv[1:]] or [64, 72, 96, 128]
g = torch.Generator(device=dev).manual_seed(0)
copies = 2
gus = [PackedLinear((torch.randn(I, D, device=dev, generator=g) * 0.02).to(torch.bfloat16),
                    swiglu_up=(torch.randn(I, D, device=dev, generator=g) * 0.02).to(torch.bfloat16))
       for _ in range(copies)]
downs = [PackedLinear((torch.randn(D, I, device=dev, generator=g) * 0.01).to(torch.bfloat16)) for _ in range(copies)]
for M in Ms:
    xg = torch.randn(M, D, device=dev, generator=g)
    xd = torch.randn(M, I, device=dev, generator=g)
    og = [torch.empty(M, I, device=dev) for _ in range(copies)]
    od = [torch.zeros(M, D, device=dev) for _ in range(copies)]
    res = {}
    for on in ((4, 0) if M <= 64 else ((5, 6, 1) if os.environ.get('ROWS_DEPTH') else (1, 3, 2, 0))):
        lib.fo_gemm_set_rows(on)
        yg = gus[0](xg, M=M).clone()
        yd = torch.zeros(M, D, device=dev)
        downs[0](xd, out=yd, residual=True, M=M)
        torch.cuda.synchronize()
        it = iter(range(1 << 30))
        tg = min(graph_time(lambda: (lambda i: gus[i](xg, out=og[i], M=M))(next(it) % copies), 8) for _ in range(2))
        it = iter(range(1 << 30))
        td = min(graph_time(lambda: (lambda i: downs[i](xd, out=od[i], residual=True, M=M))(next(it) % copies), 8)
                 for _ in range(2))
        res[on] = (tg, td, yg, yd)
        name = {1: "k_gemm_rows", 3: "rows, split consumer map", 2: "k_gemm_wrow (probe)", 4: "k_gemm_rows (33+ rows)", 5: "PROBE W only, 7 deep", 6: "PROBE W only, 11 deep",
                0: "row halves / xsk"}[on]
        print(f"M={M:4d} {name:18s} gate/up {tg:7.2f} us ({2 * I * D * 2 / tg / 1e6:4.2f} TB/s)  "
              f"down {td:7.2f} us ({I * D * 2 / td / 1e6:4.2f} TB/s)", flush=True)
    lib.fo_gemm_set_rows(1)
    if 0 not in res:
        continue
    k1 = 4 if M <= 64 else 1
    dg = float((res[k1][2] - res[0][2]).abs().max() / res[0][2].abs().max())
    dd = float((res[k1][3] - res[0][3]).abs().max() / res[0][3].abs().max())
    print(f"M={M:4d} rows vs halves: gate/up max rel diff {dg:.2e}, down {dd:.2e}", flush=True)
