"""Where does the X-stationary gate/up stream (k_gemm_xs, M = 16, K = 3584, the dominant kernel) lose against the
lm_head's 6.4 TB/s?  Graph-replayed over weight copies beyond the Infinity Cache (as xs_balance_probe.py), the
shipped kernel against probe variants (fo_gemm_set_xs_variant): 1 = no cross-wave LDS reduction (wrong results: the
bound of removing the two barriers per unit), 2 = default-policy (not nt) weight loads, 3 = round 4's 8 waves x 14
k-steps (shipped until r05; the shipped shape is 16 x 7 since), 4 = 8 x 14 with the cross-wave reduction without
workgroup barriers (the last-arriving wave reduces; bit-identical to 8 x 14).
Also the Qwen2 lm_head (1.09 GB) for the achievable streaming rate.  python scripts/xs_variant_probe.py (GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402

dev = torch.device("cuda:0")
D, I, M = 3584, 18944, 16
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, D, device=dev, generator=g)
copies = 3
lins = [PackedLinear((torch.randn(I, D, device=dev, generator=g) * 0.02).to(torch.bfloat16),
                     swiglu_up=(torch.randn(I, D, device=dev, generator=g) * 0.02).to(torch.bfloat16))
        for _ in range(copies)]
outs = [torch.empty(M, I, device=dev) for _ in range(copies)]
nbytes = 2 * I * D * 2
ref = lins[0](x, M=M).clone()
for rnd in range(2):
    for var, name in ((0, "shipped <16,7>"), (1, "no reduction (bound)"), (2, "default-policy loads"),
                      (3, "8 waves x 14 (r04)"), (4, "8 x 14 barrier-free")):
        lib.fo_gemm_set_xs_variant(var)
        if var in (0, 2):   # (3 / 4 sum 8 wave partials: another rounding order; 1 is wrong by design)
            y = lins[0](x, M=M)
            torch.cuda.synchronize()
            assert torch.equal(y, ref), f"variant {var} differs from the shipped kernel"
        it = iter(range(1 << 30))
        us = min(graph_time(lambda: (lambda i: lins[i](x, out=outs[i], M=M))(next(it) % copies), 8 * copies)
                 for _ in range(2))
        print(f"round {rnd} {name:24s} {us:7.2f} us  {nbytes / us / 1e6:5.2f} TB/s  frac {nbytes / us / 1e6 / 8:.3f}",
              flush=True)
lib.fo_gemm_set_xs_variant(0)
del lins, outs
torch.cuda.empty_cache()
V = 152064
heads = [PackedLinear((torch.randn(V, D, device=dev, generator=g) * 0.02).to(torch.bfloat16)) for _ in range(2)]
xs8 = torch.randn(8, D, device=dev, generator=g)
lo = [torch.empty(8, V, device=dev) for _ in range(2)]
it = iter(range(1 << 30))
us = min(graph_time(lambda: (lambda i: heads[i](xs8, out=lo[i], M=8))(next(it) % 2), 8) for _ in range(2))
print(f"lm_head 8 rows {us:7.2f} us  {V * D * 2 / us / 1e6:5.2f} TB/s", flush=True)
