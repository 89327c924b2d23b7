"""How much of an M = 16 Qwen2 projection's time is HBM latency: the same graph-timed launch with its weights
resident in the 256 MB Infinity Cache (one weight copy re-read) against weights streamed from HBM (six
alternating copies).  python scripts/gemm_mall_probe.py (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import ops  # noqa: E402

dev = torch.device("cuda:0")
M = 16
for name, N, K, rope in (("qkv", 4608, 3584, 128), ("o", 3584, 3584, None), ("down", 3584, 18944, None),
                         ("tts_o", 896, 896, None), ("tts_down", 896, 4864, None)):
    lins = [PackedLinear((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(6)]
    x = torch.randn(M, K, device=dev)
    outs = [torch.empty(M, N, device=dev) for _ in range(6)]
    r = {}
    for ncp in (1, 6, 1, 6):
        it = iter(range(1 << 30))
        t = graph_time(lambda: (lambda i: lins[i](x, out=outs[i], M=M))(next(it) % ncp), 48)
        r.setdefault(ncp, []).append(t)
    nb = lins[0].nbytes
    print(f"{name:9s} {nb / 1e6:7.1f}MB  Infinity-Cache resident {min(r[1]):6.2f}us ({nb / min(r[1]) / 1e6:4.2f}TB/s)"
          f"  HBM {min(r[6]):6.2f}us ({nb / min(r[6]) / 1e6:4.2f}TB/s)", flush=True)
    del lins
    torch.cuda.empty_cache()
