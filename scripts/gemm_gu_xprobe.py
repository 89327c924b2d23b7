"""Is the 16-row gate/up held back by its X rows?  Same kernel and launch shape (auto policy, M = 16),
three X contents: 16 distinct rows, rows 8-15 duplicating rows 0-7 (half the distinct X lines), and
the M = 8 launch for reference.  Two alternating weight copies (> the 256 MB Infinity Cache)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, timeit  # noqa: E402

dev = torch.device("cuda:0")
N, K = 18944, 3584
lins = []
for c in range(2):
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    lins.append(PackedLinear(w, swiglu_up=w))
    del w
x8 = torch.randn(8, K, device=dev)
cases = {"M16 distinct": torch.randn(16, K, device=dev), "M16 rows 8-15 = rows 0-7": torch.cat([x8, x8]).contiguous(),
         "M8": x8}
for name, x in cases.items():
    outs = [torch.empty(x.shape[0], N, device=dev) for _ in range(2)]
    t = min(timeit([lambda i=i: lins[i](x, out=outs[i]) for i in range(2)]) for _ in range(3))
    print(f"{name:26s} {t:6.1f} us  {lins[0].nbytes / t / 1e6:.2f} TB/s", flush=True)
