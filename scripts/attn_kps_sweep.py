"""Qwen2 paged attention (fo_attention -> k_attn_mfma<128>, 28 q / 4 kv heads) for 8 sessions at L keys:
device time per launch (replayed hipGraph) against the keys-per-split bound of the in-launch merge, for the
text-decode shape (1 token per session, 7 query rows per item) and the listen shape (2 tokens, 14 rows).
python scripts/attn_kps_sweep.py (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import ops  # noqa: E402
from fo.kv import BatchMeta, KVPool, KVSeq  # noqa: E402

dev = torch.device("cuda:0")
H, KVH, hd, B = 28, 4, 128, 8
pool = KVPool(1, KVH, hd, 8192, 16, dev)
g = torch.Generator(device=dev).manual_seed(0)
for L in (100, 200, 400, 800):
    seqs = [KVSeq(pool) for _ in range(B)]
    for s in seqs:   # fill L keys (values random)
        s.reserve(L)
        s.length = L
    pool.k[0].normal_(generator=g)
    pool.v[0].normal_(generator=g)
    for tok in (1, 2):
        meta = BatchMeta([(s, tok, s.length, True) for s in seqs], dev, gqa=H // KVH)
        T = B * tok
        q = torch.randn(T, H * hd, device=dev, generator=g)
        out = torch.empty(T, H * hd, device=dev)
        res = []
        # torch fp32 reference (causal over the session's keys) for the error column
        ref = torch.empty(T, H * hd, device=dev)
        for b, sq in enumerate(seqs):
            Kb = pool.k[0][sq.pages].permute(1, 0, 2, 3).reshape(KVH, -1, hd)[:, :sq.length]
            Vb = pool.v[0][sq.pages].permute(1, 0, 2, 3).reshape(KVH, -1, hd)[:, :sq.length]
            for i in range(tok):
                nv = sq.length - tok + i + 1
                qq = q[b * tok + i].view(KVH, H // KVH, hd)
                sc = torch.einsum("gjd,gkd->gjk", qq, Kb[:, :nv]) * hd ** -0.5
                ref[b * tok + i] = torch.einsum("gjk,gkd->gjd", sc.softmax(-1), Vb[:, :nv]).reshape(-1)
        kpss = [int(v) for v in os.environ.get("ATTN_KPS", "64,128,256,512").split(",")]
        uniform = os.environ.get("ATTN_UNIFORM", "1") == "1"
        for kps in kpss:
            ns = ops.attn_nsplit(2048, meta.n_items, KVH)
            ws = {"ml": torch.empty(T * H * ns * 2, device=dev), "o": torch.empty(T * H * ns * hd, device=dev),
                  "t": torch.zeros(T * KVH, dtype=torch.int32, device=dev)}
            dense = tok == 1 or uniform

            def f(kps=kps, ns=ns, ws=ws, dense=dense):
                ops.attention(q, T, None if dense else meta.items, meta.n_items, meta.max_rows, meta.tok_nvis,
                              meta.block_table, pool.PS, pool.k[0], pool.v[0], H, KVH, hd, hd ** -0.5, ns, ws["ml"],
                              ws["o"], out, tickets=ws["t"], keys_per_split=kps)
            t = graph_time(f, 50)
            f()
            torch.cuda.synchronize()
            res.append((kps, t, (out - ref).abs().max().item()))
        print(f"L={L:4d} tokens/session={tok}: " + "  ".join(f"kps {k}: {t:5.2f}us (err {e:.1e})" for k, t, e in res),
              flush=True)
        for s in seqs:
            s.length -= tok
    for s in seqs:
        s.free()
