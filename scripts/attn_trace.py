"""Where the Qwen2 paged attention's time goes (k_attn_mfma<128, 8>, 28 q / 4 kv heads, 8 sessions): per-workgroup wall
clocks (fo_attention_set_trace, 100 MHz) of one launch at the text-decode shape (1 token per session) and the listen
shape (2 tokens) for L keys, with the in-launch split merge (keys per split 128, as the stacks run it): dispatch
skew, Q / block-table staging, the K / V tile loop, the partial stores, and the arrival + merge (the last split of each
item merges).  Beside it the graph-replayed time per launch.  python scripts/attn_trace.py (GPU only)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import _lib, ops  # noqa: E402
from fo.kv import BatchMeta, KVPool, KVSeq  # noqa: E402

dev = torch.device("cuda:0")
H, KVH, hd, B, CLK = 28, 4, 128, 8, 100.0
pool = KVPool(1, KVH, hd, 8192, 16, dev)
g = torch.Generator(device=dev).manual_seed(0)
trace = torch.zeros(32 * 8192, dtype=torch.int64, device=dev)
f = lambda v: f"med {np.median(v):6.2f} max {v.max():6.2f}"  # noqa: E731
flush = torch.empty(1 << 28, device=dev)   # 1 GiB: evicts L2 and the Infinity Cache
for L in (150, 200, 500, 800):
    seqs = [KVSeq(pool) for _ in range(B)]
    for s in seqs:
        s.reserve(L)
        s.length = L
    pool.k[0].normal_(generator=g)
    pool.v[0].normal_(generator=g)
    for tok in (1, 2):
        meta = BatchMeta([(s, tok, s.length, True) for s in seqs], dev, gqa=H // KVH)
        T = B * tok
        q = torch.randn(T, H * hd, device=dev, generator=g)
        out = torch.empty(T, H * hd, device=dev)
        ns = ops.attn_nsplit(2048, meta.n_items, KVH)
        ws = {"ml": torch.empty(T * H * ns * 2, device=dev), "o": torch.empty(T * H * ns * hd, device=dev),
              "t": torch.zeros(T * KVH, dtype=torch.int32, device=dev)}

        def run():
            ops.attention(q, T, None, meta.n_items, meta.max_rows, meta.tok_nvis, meta.block_table, pool.PS,
                          pool.k[0], pool.v[0], H, KVH, hd, hd ** -0.5, ns, ws["ml"], ws["o"], out, tickets=ws["t"])
        us = graph_time(run, 50)
        trace.zero_()
        cold = os.environ.get("ATTN_TRACE_COLD") == "1"
        if cold:
            flush.fill_(1.0)
            torch.cuda.synchronize()
        with torch.cuda.stream(ops.engine_stream(dev)):
            _lib.call("fo_attention_set_trace", trace.data_ptr())
            run()
            _lib.call("fo_attention_set_trace", None)
            torch.cuda.synchronize()
        ws["t"].zero_()   # (FO_ATTN_TRACE_REPS > 1: passes of different splits interleave their tickets)
        t = trace.view(-1, 32).cpu().numpy().astype(np.int64)
        t = t[t[:, 5] != 0]   # the workgroups that ran a tile loop
        t0 = t[:, 0].min()
        rel = (t - t0) / CLK
        merge = (t[:, 4] - t[:, 3]) / CLK
        last = merge > np.median(merge) + 0.5
        print(f"{'cold' if cold else 'warm'} reps={os.environ.get('FO_ATTN_TRACE_REPS', '1')} L={L:4d} tokens/session={tok}: {us:6.2f} us/launch (graph), {len(t)} WGs, splits {int(t[0, 5]) - 1}; "
              f"start {f(rel[:, 0])} | staged +{f((t[:, 1] - t[:, 0]) / CLK)} | loads landed +{f((t[:, 6] - t[:, 1]) / CLK)} | "
              f"tiles +{f((t[:, 2] - t[:, 1]) / CLK)} [K split +{f((t[:, 7] - t[:, 1]) / CLK)}, waves at max "
              f"exchange: first +{f((t[:, 16:24].min(1) - t[:, 1]) / CLK)} last +{f((t[:, 16:24].max(1) - t[:, 1]) / CLK)}, "
              f"barrier 2 +{f((t[:, 8] - t[:, 1]) / CLK)}, barrier 3 +{f((t[:, 9] - t[:, 1]) / CLK)}, "
              f"PV done +{f((t[:, 10] - t[:, 1]) / CLK)}] | "
              f"stored +{f((t[:, 3] - t[:, 2]) / CLK)} | arrive/merge +{f(merge)} (merging WGs {int(last.sum())}) | "
              f"end {f(rel[:, 4])}", flush=True)
    for s in seqs:
        s.free()
