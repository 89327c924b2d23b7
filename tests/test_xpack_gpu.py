"""Packed <= 64-row activations (ops.XPack): every producer (the split-K reduce, the unsplit GEMM epilogue, the
in-launch split merge, the multi-row and decode attention) writes exactly the bf16 hi / lo split of its fp32 output
in fragment order, and a GEMM reading the packed copy gives bit-identical results to the one splitting fp32 X."""
import math

import pytest
import torch

from fo import ops
from fo.kv import BatchMeta, KVPool, KVSeq

pytestmark = pytest.mark.gpu


def _pack(x):
    """fp32 [M <= 16, K] -> the (hi, lo) [K/32][64][8] bf16 fragment order of ops.XPack (rows >= M unchecked)."""
    M, K = x.shape
    xf = torch.zeros(16, K, dtype=torch.float32, device=x.device)
    xf[:M] = x
    hi = xf.to(torch.bfloat16)
    lo = (xf - hi.float()).to(torch.bfloat16)
    f = lambda t: t.view(16, K // 32, 4, 8).permute(1, 2, 0, 3).reshape(-1)  # noqa: E731
    return f(hi), f(lo)


def _pack_rb(x):
    """fp32 [M <= 32, K] -> (hi, lo) [K/32][ceil(M/16)][64][8] bf16 (the two-row-block layout)."""
    M, K = x.shape
    rb = (M + 15) // 16
    xf = torch.zeros(rb * 16, K, dtype=torch.float32, device=x.device)
    xf[:M] = x
    hi = xf.to(torch.bfloat16)
    lo = (xf - hi.float()).to(torch.bfloat16)
    f = lambda t: t.view(rb, 16, K // 32, 4, 8).permute(2, 0, 3, 1, 4).reshape(-1)  # noqa: E731
    return f(hi), f(lo), rb


def _rows(flat, M, K):
    """the first M rows of a packed half back in [M, K] (bit patterns as int16)."""
    return flat.view(K // 32, 4, 16, 8).permute(2, 0, 1, 3).reshape(16, K)[:M].view(torch.int16)


def _check_packed(xp, y, M):
    K = y.shape[1]
    hi, lo = _pack(y)
    assert torch.equal(_rows(xp.hi, M, K), _rows(hi, M, K))
    assert torch.equal(_rows(xp.lo, M, K), _rows(lo, M, K))


@pytest.mark.parametrize("M,N,K,splitk", [(16, 3584, 18944, 0), (12, 1024, 4096, 4), (16, 896, 896, 1), (9, 512, 256, 1),
                                           (40, 3584, 18944, 0), (48, 1024, 4096, 4)])
def test_yg_producers_write_the_packed_split(dev, M, N, K, splitk):
    """stats_out's yg also packed: k_gemm_reduce (split-K), the unsplit epilogue, the in-launch merge (small weights)."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K + splitk)
    lin = ops.PackedLinear((torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(dev))
    x = torch.randn(M, K, generator=g).to(dev)
    res = torch.randn(M, N, generator=g).to(dev)
    gamma = (1 + 0.1 * torch.randn(N, generator=g)).to(dev)
    st = ops.RowStats(M, dev)
    yg = torch.empty(M, N, device=dev)
    xp = ops.XPack(N, dev, M)
    xp.hi.fill_(0)
    xp.lo.fill_(0)
    out = res.clone()
    lin(x, out=out, residual=True, M=M, splitk=splitk, stats_out=st.set(gamma, yg), ypack=xp)
    torch.cuda.synchronize()
    hi, lo, rb = _pack_rb(yg)
    view = lambda t: t[:N * 16 * rb].view(N // 32, rb, 4, 16, 8).permute(1, 3, 0, 2, 4).reshape(rb * 16, N)[:M]  # noqa
    assert torch.equal(view(xp.hi).view(torch.int16), view(hi).view(torch.int16))
    assert torch.equal(view(xp.lo).view(torch.int16), view(lo).view(torch.int16))


@pytest.mark.parametrize("M,N,K,rope", [(16, 3584, 3584, False), (11, 896, 896, False), (16, 4608, 3584, True),
                                        (48, 3584, 3584, False), (40, 4608, 3584, True), (56, 1024, 1024, False)])
def test_packed_x_gemm_is_bit_identical(dev, M, N, K, rope):
    """The GEMM reading X packed equals the one splitting fp32 X, bit for bit (o-style residual epilogue, and the
    q|k|v RoPE + paged-KV append epilogue; one-row-tile kernels and the 17..64-row ones)."""
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(dev)
    x = torch.randn(M, K, generator=g).to(dev)
    xp = ops.XPack(K, dev, M)
    h, lo, _ = _pack_rb(x)
    xp.hi.copy_(h)
    xp.lo.copy_(lo)
    if not rope:
        lin = ops.PackedLinear(w)
        y0 = torch.randn(M, N, generator=g).to(dev)
        a, b = y0.clone(), y0.clone()
        lin(x, out=a, residual=True, M=M)
        lin(x, out=b, residual=True, M=M, xpack=xp)
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        return
    hd, H, KVH = 128, 28, 4
    lin = ops.PackedLinear(w, rope_hd=hd)
    pool = KVPool(1, KVH, hd, 64, 16, dev)
    seqs = [KVSeq(pool) for _ in range(M)]
    meta = BatchMeta([(s, 1, 0, True) for s in seqs], dev, gqa=H // KVH)
    pos = torch.arange(M, dtype=torch.int32, device=dev)
    inv = 1.0 / (1e6 ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(64, dtype=torch.float64)[:, None] * inv[None, :]
    cos, sin = ang.cos().float().to(dev), ang.sin().float().to(dev)
    outs = []
    for pk in (None, xp):
        q = torch.empty(M, H * hd, device=dev)
        pool.k.zero_()
        pool.v.zero_()
        lin.qkv_rope(x, M, pos, meta.tok_slot, cos, sin, q, pool.k[0], pool.v[0], H, KVH, pool.PS, xpack=pk)
        torch.cuda.synchronize()
        outs.append((q.clone(), pool.k.clone(), pool.v.clone()))
    for u, v in zip(*outs):
        assert torch.equal(u, v)


def _check_packed_rb(xp, y, M):
    """xp (an XPack) holds the bf16 hi / lo split of y's first M rows in the ceil(M/16)-row-block fragment order."""
    K = y.shape[1]
    hi, lo, rb = _pack_rb(y[:M])
    view = lambda t: t[:K * 16 * rb].view(K // 32, rb, 4, 16, 8).permute(1, 3, 0, 2, 4).reshape(rb * 16, K)[:M]  # noqa
    assert torch.equal(view(xp.hi).view(torch.int16), view(hi).view(torch.int16))
    assert torch.equal(view(xp.lo).view(torch.int16), view(lo).view(torch.int16))


CTX = [3, 40, 150, 300, 700, 1, 64, 65, 129, 9, 17, 33, 250, 5, 90, 400]


@pytest.mark.parametrize("H,KVH,hd,tokens,nseq", [(28, 4, 128, 2, 8), (14, 14, 64, 1, 16),
                                                  # 17..64 tokens (duplex ticks, prefills): 2..4 row blocks
                                                  (28, 4, 128, 4, 8), (28, 4, 128, 3, 16), (28, 4, 128, 4, 16),
                                                  (14, 14, 64, 1, 48)])
def test_attention_writes_the_packed_split(dev, H, KVH, hd, tokens, nseq):
    """fo_attention's packed output (multi-row kernel with the in-launch split merge; the decode kernel) equals
    the split of its fp32 output, at 1..4 row blocks (the token row index th / H against the packed layout)."""
    g = torch.Generator().manual_seed(H + hd + tokens * nseq)
    pool = KVPool(1, KVH, hd, 1024, 16, dev)
    pool.k.copy_(torch.randn(pool.k.shape, generator=g))
    pool.v.copy_(torch.randn(pool.v.shape, generator=g))
    seqs = [KVSeq(pool) for _ in range(nseq)]
    for i, s in enumerate(seqs):
        BatchMeta([(s, CTX[i % 16] + i // 16, 0, True)], dev)
    meta = BatchMeta([(s, tokens, s.length, True) for s in seqs], dev, gqa=H // KVH)
    T = meta.T
    assert T == tokens * nseq
    q = torch.randn(T, H * hd, generator=g).to(dev)
    ns = ops.attn_nsplit(meta.max_keys, meta.n_items, KVH)
    part_ml = torch.empty(T * H * ns * 2, device=dev)
    part_o = torch.empty(T * H * ns * hd, device=dev)
    tickets = torch.zeros(meta.n_items * KVH, dtype=torch.int32, device=dev)
    out = torch.empty(T, H * hd, device=dev)
    xp = ops.XPack(H * hd, dev, T)
    ops.launch_counts_reset()
    ops.attention(q, T, meta.items, meta.n_items, meta.max_rows, meta.tok_nvis, meta.block_table, pool.PS, pool.k[0],
                  pool.v[0], H, KVH, hd, 1 / math.sqrt(hd), ns, part_ml, part_o, out, tickets=tickets,
                  keys_per_split=128, opack=xp)
    torch.cuda.synchronize()
    c = ops.launch_counts()
    assert c["attn_opack"] == 1 and c["attn_decode" if tokens == 1 else "attn_mfma"] == 1, c
    _check_packed_rb(xp, out, T)
    assert int(tickets.abs().sum()) == 0   # the in-launch merge left its tickets zeroed


@pytest.mark.parametrize("tokens,nseq", [(2, 8), (4, 8), (1, 16)])
def test_attention_poison_reaches_the_packed_o_input(dev, tokens, nseq):
    """A broken host contract (a token sees more keys than its block table maps) poisons the attention output: NaN in
    the fp32 rows AND in the packed copy the o projection reads (k_gemm_xp), so the o projection's output rows are
    NaN instead of being computed from a previous layer's stale fragments; the other items stay finite and the
    merge tickets stay balanced."""
    H, KVH, hd = 28, 4, 128
    g = torch.Generator().manual_seed(7 + tokens)
    pool = KVPool(1, KVH, hd, 1024, 16, dev)
    pool.k.copy_(torch.randn(pool.k.shape, generator=g))
    pool.v.copy_(torch.randn(pool.v.shape, generator=g))
    seqs = [KVSeq(pool) for _ in range(nseq)]
    for i, s in enumerate(seqs):
        BatchMeta([(s, 200 + 37 * i, 0, True)], dev)
    meta = BatchMeta([(s, tokens, s.length, True) for s in seqs], dev, gqa=H // KVH)
    T = meta.T
    bad = 1   # session 1's tokens claim 4096 more keys than its pages hold
    rows = list(range(bad * tokens, (bad + 1) * tokens))
    nv = meta.tok_nvis.clone()
    nv[rows] += 4096
    q = torch.randn(T, H * hd, generator=g).to(dev)
    ns = ops.attn_nsplit(meta.max_keys, meta.n_items, KVH)
    part_ml = torch.empty(T * H * ns * 2, device=dev)
    part_o = torch.empty(T * H * ns * hd, device=dev)
    tickets = torch.zeros(meta.n_items * KVH, dtype=torch.int32, device=dev)
    att = torch.zeros(T, H * hd, device=dev)
    xp = ops.XPack(H * hd, dev, T)
    xp.hi.zero_()   # a stale, finite previous content
    xp.lo.zero_()
    ops.attention(q, T, meta.items, meta.n_items, meta.max_rows, nv, meta.block_table, pool.PS, pool.k[0], pool.v[0],
                  H, KVH, hd, 1 / math.sqrt(hd), ns, part_ml, part_o, att, tickets=tickets, keys_per_split=128,
                  opack=xp)
    wo = ops.PackedLinear((torch.randn(3584, H * hd, generator=g) * 0.02).to(torch.bfloat16).to(dev))
    y = torch.zeros(T, 3584, device=dev)
    wo(att, out=y, residual=True, M=T, xpack=xp if T > 8 else None)
    torch.cuda.synchronize()
    fin = torch.isfinite(y).all(dim=1).cpu()
    assert not fin[rows].any(), "poisoned rows must be NaN after the o projection"
    others = [r for r in range(T) if r not in rows]
    assert fin[others].all()
    assert int(tickets.abs().sum()) == 0


@pytest.mark.parametrize("M", [32, 27, 20])
def test_two_row_block_packing_layernorm_producer_and_rowstats_consumer(dev, M):
    """The speech encoder's 17..32-row blocks: the LayerNorm-on-load FFN-up GEMM writes its ReLU output packed
    (two row blocks), the FFN-down reads it -- bit-identical to reading fp32 rows."""
    g = torch.Generator(device="cpu").manual_seed(M)
    D, F = 256, 1024
    prod = ops.PackedLinear((torch.randn(D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(dev))
    up = ops.PackedLinear((torch.randn(F, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(dev),
                          torch.randn(F, generator=g).to(dev))
    down = ops.PackedLinear((torch.randn(D, F, generator=g) / F ** 0.5).to(torch.bfloat16).to(dev))
    x = torch.randn(M, D, generator=g).to(dev)
    st = ops.RowStats(M, dev, with_sums=True)
    xr = torch.randn(M, D, generator=g).to(dev)
    prod.rowstats(x, xr, st, residual=True)
    lnw = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    lnb = (0.1 * torch.randn(D, generator=g)).to(dev)
    fp = ops.XPack(F, dev, M)
    f = torch.empty(M, F, device=dev)
    up.ln(xr, lnw, lnb, st, out=f, act="relu", ypack=fp)
    torch.cuda.synchronize()
    hi, lo, rb = _pack_rb(f)
    n = F * 16 * rb
    view = lambda t: t[:n].view(F // 32, rb, 4, 16, 8)  # noqa: E731
    for a, b in ((fp.hi, hi), (fp.lo, lo)):   # rows < M only
        A = view(a).permute(1, 3, 0, 2, 4).reshape(rb * 16, F)[:M].view(torch.int16)
        B = view(b).permute(1, 3, 0, 2, 4).reshape(rb * 16, F)[:M].view(torch.int16)
        assert torch.equal(A, B)
    y0 = torch.randn(M, D, generator=g).to(dev)
    st2 = ops.RowStats(M, dev, with_sums=True)
    a, b = y0.clone(), y0.clone()
    down.rowstats(f, a, st2, residual=True)
    down.rowstats(f, b, st2, residual=True, xpack=fp)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("M", [32, 27, 56])
def test_fp32_fragment_copy_feeds_the_layernorm_gemm_bit_identically(dev, M):
    """The encoder's residual stream in fp32 fragment order (ops.XPack32): written by the producer GEMM beside its
    rows, read by the LayerNorm-on-load GEMM -- the same output bit for bit."""
    g = torch.Generator(device="cpu").manual_seed(M + 5)
    D, F = 256, 512
    prod = ops.PackedLinear((torch.randn(D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(dev))
    up = ops.PackedLinear((torch.randn(F, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(dev),
                          torch.randn(F, generator=g).to(dev))
    x = torch.randn(M, D, generator=g).to(dev)
    st = ops.RowStats(M, dev, with_sums=True)
    xr = torch.randn(M, D, generator=g).to(dev)
    p32 = ops.XPack32(D, dev, M)
    prod.rowstats(x, xr, st, residual=True, ypack32=p32)
    lnw = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    lnb = (0.1 * torch.randn(D, generator=g)).to(dev)
    a = up.ln(xr, lnw, lnb, st, act="relu")
    b = up.ln(xr, lnw, lnb, st, act="relu", xpack32=p32)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    rb = (M + 15) // 16
    back = p32.buf.view(D // 32, rb, 4, 16, 8).permute(1, 3, 0, 2, 4).reshape(rb * 16, D)[:M]
    assert torch.equal(back, xr)


@pytest.mark.parametrize("M", [16, 11])
def test_xstationary_gate_up_reads_packed_x_bit_identically(dev, M):
    """The Qwen2 gate/up X-stationary stream (k_gemm_xs) loading its X slice packed: the same SwiGLU output."""
    g = torch.Generator(device="cpu").manual_seed(M + 99)
    D, I = 3584, 18944
    lin = ops.PackedLinear((torch.randn(I, D, generator=g) * 0.02).to(torch.bfloat16).to(dev),
                           swiglu_up=(torch.randn(I, D, generator=g) * 0.02).to(torch.bfloat16).to(dev))
    x = torch.randn(M, D, generator=g).to(dev)
    xp = ops.XPack(D, dev, M)
    h, lo, _ = _pack_rb(x)
    xp.hi.copy_(h)
    xp.lo.copy_(lo)
    a = lin(x, M=M)
    b = lin(x, M=M, xpack=xp)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
