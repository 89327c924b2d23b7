"""fo_attention (paged GQA attention, work items + split-KV) against a float64 torch reference."""
import math

import pytest
import torch

from fo import ops
from fo.kv import BatchMeta, KVPool, KVSeq

pytestmark = pytest.mark.gpu


def _reference(q, pool, seqs, meta_host, H, KVH, hd, scale):
    """q [T, H*hd]; meta_host: list of (seq, tok_nvis) per token."""
    out = torch.zeros(len(meta_host), H * hd, dtype=torch.float64)
    G = H // KVH
    k = pool.k[0].double().cpu()
    v = pool.v[0].double().cpu()
    PS = pool.PS
    for t, (s, nv) in enumerate(meta_host):
        pages = seqs[s].pages
        idx = [(pages[p // PS], p % PS) for p in range(nv)]
        for h in range(H):
            kh = h // G
            K = torch.stack([k[pg, kh, sl] for pg, sl in idx])
            V = torch.stack([v[pg, kh, sl] for pg, sl in idx])
            sc = (K @ q[t, h * hd:(h + 1) * hd].double().cpu()) * scale
            out[t, h * hd:(h + 1) * hd] = torch.softmax(sc, 0) @ V
    return out


@pytest.mark.parametrize("H,KVH,hd", [(28, 4, 128), (14, 14, 64), (4, 2, 32)])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("nsplit,kps", [(None, 0), (1, 0), (3, 0), (8, 64), (16, 256), (2, 64), (16, 32)])
@pytest.mark.parametrize("wide", [False, True])
def test_attention_matches_reference(dev, H, KVH, hd, causal, nsplit, kps, wide):
    """kps > 0: splits sized per item from its key count (<= nsplit), merged in the same launch by the
    last split to arrive (tickets must come back zeroed for the next launch / graph replay).  wide: work items
    of ops.attn_max_rows(hd) query rows (Qwen2's 28 / 4 heads at 128: 4 tokens x 7 = 28 rows in two row tiles
    sharing the K / V loads, k_attn_mfma<128, 8, 2>); else 16.  kps 32 at head dim 128 and 16 rows: the 2-wave
    32-key-tile form (k_attn_mfma<128, 2>)."""
    g = torch.Generator().manual_seed(H * 1000 + hd + causal)
    pool = KVPool(1, KVH, hd, 256, 16, dev)
    pool.k.copy_(torch.randn(pool.k.shape, generator=g))
    pool.v.copy_(torch.randn(pool.v.shape, generator=g))
    base = KVSeq(pool)
    BatchMeta([(base, 37, 0, True)], dev)  # shared prefix, partial last page
    seqs = [base.fork() for _ in range(4)]
    olds = [0, 5, 90, 300]
    for s, extra in zip(seqs, olds):
        if extra:
            BatchMeta([(s, extra, s.length, True)], dev)
    news = [1, 9, 2, 20]
    G = H // KVH
    meta = BatchMeta([(s, n, s.length, causal) for s, n in zip(seqs, news)], dev, gqa=G,
                     rows=ops.attn_max_rows(hd) if wide else 16)
    if wide and hd == 128:
        assert meta.max_rows == 28
    T = meta.T
    q = torch.randn(T, H * hd, generator=g).to(dev)
    nvis = meta.tok_nvis.cpu().tolist()
    host = [(meta.tok_seq.cpu()[t].item(), nvis[t]) for t in range(T)]
    ns = ops.attn_nsplit(meta.max_keys, meta.n_items, KVH) if nsplit is None else nsplit
    part_ml = torch.empty(T * H * ns * 2, device=dev) if ns > 1 else None
    part_o = torch.empty(T * H * ns * hd, device=dev) if ns > 1 else None
    out = torch.empty(T, H * hd, device=dev)
    scale = 1 / math.sqrt(hd)
    tickets = torch.zeros(meta.n_items * KVH, dtype=torch.int32, device=dev) if kps else None
    ref = _reference(q, pool, seqs, host, H, KVH, hd, scale)
    for _ in range(2 if kps else 1):  # twice: the second launch starts from the tickets the first left
        out.fill_(float("nan"))
        ops.attention(q, T, meta.items, meta.n_items, meta.max_rows, meta.tok_nvis, meta.block_table, pool.PS,
                      pool.k[0], pool.v[0], H, KVH, hd, scale, ns, part_ml, part_o, out, tickets=tickets,
                      keys_per_split=kps or 256)
        torch.testing.assert_close(out.cpu().double(), ref, atol=2e-5, rtol=1e-4)
        if kps:
            assert int(tickets.abs().sum()) == 0


@pytest.mark.parametrize("hd", [64, 128, 32])
def test_single_row_decode_attention(dev, hd):
    """One token per session with one query head per kv head (the AR speech decoder step) takes the
    decode kernel (fp32, one work group per session x head): vs float64, keys across page boundaries."""
    H = KVH = 14 if hd == 64 else 4
    g = torch.Generator().manual_seed(hd)
    pool = KVPool(1, KVH, hd, 256, 16, dev)
    pool.k.copy_(torch.randn(pool.k.shape, generator=g))
    pool.v.copy_(torch.randn(pool.v.shape, generator=g))
    seqs = [KVSeq(pool) for _ in range(5)]
    for s, n in zip(seqs, [1, 15, 16, 333, 1200]):
        BatchMeta([(s, n, 0, True)], dev)
    meta = BatchMeta([(s, 1, s.length, False) for s in seqs], dev, gqa=1)
    assert meta.max_rows == 1
    T = meta.T
    q = torch.randn(T, H * hd, generator=g).to(dev)
    nvis = meta.tok_nvis.cpu().tolist()
    host = [(meta.tok_seq.cpu()[t].item(), nvis[t]) for t in range(T)]
    out = torch.full((T, H * hd), float("nan"), device=dev)
    scale = 1 / math.sqrt(hd)
    ops.attention(q, T, meta.items, meta.n_items, meta.max_rows, meta.tok_nvis, meta.block_table, pool.PS, pool.k[0],
                  pool.v[0], H, KVH, hd, scale, 1, None, None, out)
    ref = _reference(q, pool, seqs, host, H, KVH, hd, scale)
    torch.testing.assert_close(out.cpu().double(), ref, atol=1e-5, rtol=1e-5)



@pytest.mark.parametrize("B,lens", [(8, [3, 40, 150, 300, 700, 1, 64, 129]), (3, [17, 2, 1000]), (16, None)])
def test_decode_attention_fused_with_o_projection(dev, B, lens):
    """fo_attention_o (the AR speech decoder's attention + o projection + residual + next-norm statistics in one
    launch, the head partials summed in head order by the last head) against a float64 torch reference of
    softmax(q K^T) V -> x + att Wo^T, yg = x * gamma, sum of squares: H = 14 heads of 64, o 896 x 896."""
    H, hd, D = 14, 64, 896
    g = torch.Generator().manual_seed(B * 7 + (lens[0] if lens else 0))
    lens = lens or [int(x) for x in torch.randint(1, 900, (B,), generator=g)]
    pool = KVPool(1, H, hd, 1024, 16, dev)
    pool.k.copy_(torch.randn(pool.k.shape, generator=g))
    pool.v.copy_(torch.randn(pool.v.shape, generator=g))
    seqs = [KVSeq(pool) for _ in range(B)]
    for s, n in zip(seqs, lens):
        BatchMeta([(s, n - 1, 0, False)], dev) if n > 1 else None
    meta = BatchMeta([(s, 1, s.length, False) for s in seqs], dev)
    q = torch.randn(B, H * hd, generator=g)
    wo = (torch.randn(D, H * hd, generator=g) / (H * hd) ** 0.5).to(torch.bfloat16)
    gamma = 1 + 0.1 * torch.randn(D, generator=g)
    x0 = torch.randn(B, D, generator=g)
    lin = ops.PackedLinear(wo.to(dev))
    x = x0.clone().to(dev)
    yg = torch.empty(B, D, device=dev)
    st = ops.RowStats(B, dev)
    part = torch.empty(B * H * D, device=dev)
    tickets = torch.zeros(B, dtype=torch.int32, device=dev)
    ops.launch_counts_reset()
    ops.attention_o(q.to(dev), B, None, meta.tok_nvis, meta.block_table, pool.PS, pool.k[0], pool.v[0], H, hd,
                    hd ** -0.5, lin, part, tickets, x, gamma.to(dev), yg, st)
    torch.cuda.synchronize()
    assert ops.launch_counts()["attn_o"] == 1 and st.groups == 1
    att = _reference(q, pool, seqs, [(b, seqs[b].length) for b in range(B)], H, H, hd, hd ** -0.5)
    ref = x0.double() + att @ wo.double().T
    tol = 2e-5 * float(ref.abs().max())
    assert (x.cpu().double() - ref).abs().max() < tol
    assert (yg.cpu().double() - ref * gamma.double()).abs().max() < tol * 2
    ss = (ref ** 2).sum(1)
    assert torch.allclose(st.buf[:B].cpu().double(), ss, rtol=1e-5)
    assert int(tickets.abs().sum()) == 0


@pytest.mark.parametrize("kps", [None, 8192])
def test_long_sequence_prefill_splits_stay_within_the_page_table(dev, kps):
    """an eager prefill of 40 work items (80 tokens at GQA 7) against a sequence of more than 4096 keys.
    The per-launch keys_per_split (ops.attn_keys_per_split: one split per item when the items fill the CUs) and a
    larger one passed directly (8192) must both keep every split within the 256-page LDS table -- the kernel never
    takes fewer than ceil(keys / 4096) splits -- and give the static-split result (no poisoned NaN rows)."""
    H, KVH, hd = 28, 4, 128
    g = torch.Generator().manual_seed(77)
    pool = KVPool(1, KVH, hd, 400, 16, dev)
    pool.k.copy_(torch.randn(pool.k.shape, generator=g))
    pool.v.copy_(torch.randn(pool.v.shape, generator=g))
    seq = KVSeq(pool)
    BatchMeta([(seq, 5000, 0, True)], dev)
    meta = BatchMeta([(seq, 80, seq.length, True)], dev, gqa=H // KVH, rows=16)
    assert meta.n_items == 40 and meta.max_keys == 5080
    T = meta.T
    q = torch.randn(T, H * hd, generator=g).to(dev)
    scale = 1 / math.sqrt(hd)
    ns = ops.attn_nsplit(meta.max_keys, meta.n_items, KVH)
    assert ns >= 2
    k_eff = ops.attn_keys_per_split(meta.max_keys, meta.n_items, KVH, hd, dev) if kps is None else kps
    assert k_eff <= 4096 or kps is not None
    part_ml = torch.empty(T * H * ns * 2, device=dev)
    part_o = torch.empty(T * H * ns * hd, device=dev)
    static = torch.empty(T, H * hd, device=dev)
    ops.attention(q, T, meta.items, meta.n_items, meta.max_rows, meta.tok_nvis, meta.block_table, pool.PS, pool.k[0],
                  pool.v[0], H, KVH, hd, scale, ns, part_ml, part_o, static)
    out = torch.full((T, H * hd), float("nan"), device=dev)
    tickets = torch.zeros(meta.n_items * KVH, dtype=torch.int32, device=dev)
    ops.attention(q, T, meta.items, meta.n_items, meta.max_rows, meta.tok_nvis, meta.block_table, pool.PS, pool.k[0],
                  pool.v[0], H, KVH, hd, scale, ns, part_ml, part_o, out, tickets=tickets, keys_per_split=k_eff)
    torch.cuda.synchronize()
    assert not torch.isnan(out).any() and not torch.isnan(static).any()
    torch.testing.assert_close(out, static, atol=2e-5, rtol=1e-4)
    assert int(tickets.abs().sum()) == 0
    # and the static result against a float64 reference on a few rows (the sequence's K / V gathered once)
    pages = torch.tensor(seq.pages, dtype=torch.long)
    K = pool.k[0].cpu().double()[pages].permute(1, 0, 2, 3).reshape(KVH, -1, hd)
    V = pool.v[0].cpu().double()[pages].permute(1, 0, 2, 3).reshape(KVH, -1, hd)
    nvis = meta.tok_nvis.cpu().tolist()
    qd = q.cpu().double()
    for t in (0, 41, T - 1):
        for h in (0, 13, 27):
            kh = h // (H // KVH)
            sc = K[kh, :nvis[t]] @ qd[t, h * hd:(h + 1) * hd] * scale
            ref = torch.softmax(sc, 0) @ V[kh, :nvis[t]]
            torch.testing.assert_close(static[t, h * hd:(h + 1) * hd].cpu().double(), ref, atol=2e-5, rtol=1e-4)
