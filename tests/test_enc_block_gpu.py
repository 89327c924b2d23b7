"""fo_enc_attn_block (the attention half of a speech-encoder block in one launch: LayerNorm1, linear_q|k|v, the
rel-pos attention over the left-chunk ring + the chunk's rows, linear_out, residual -- models/encoder/transformer.py:
103-118, models/encoder/attention.py:407-459) against a plain torch float64 reference of the same op on the same
bf16-valued weights: ragged ring lengths and starts that wrap (per session), ring slots out of order, chunk rows 1, 4,
7 and 8, 4 and 16 heads.  Checks x (in place), the ring append, the row sums / sums of squares and that the tickets
are left zeroed.  Tolerance 2e-4 x max|x| (fp32 arithmetic, bf16 hi + lo activations against bf16 weights)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _reference(x, lnw, lnb, wqkv, bqkv, kr, vr, cap, st, ln, rg, ps, ptab, bu, bv, wout, bout, B, T, h, scale):
    d, dk = x.shape[1], 64
    x = x.double()
    xn = torch.nn.functional.layer_norm(x, (d,), lnw.double(), lnb.double(), 1e-5)
    qkv = xn @ wqkv.double().t() + bqkv.double()
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    att = torch.zeros(B * T, d, dtype=torch.float64)
    kr2, vr2 = kr.clone(), vr.clone()
    for b in range(B):
        old = [(st[b] + j) % cap for j in range(ln[b])]
        K = torch.cat([kr[rg[b], old].double(), k[b * T:(b + 1) * T]])
        V = torch.cat([vr[rg[b], old].double(), v[b * T:(b + 1) * T]])
        for t in range(T):
            kr2[rg[b], (st[b] + ln[b] + t) % cap] = k[b * T + t].float()
            vr2[rg[b], (st[b] + ln[b] + t) % cap] = v[b * T + t].float()
        P = ptab[ps[b]:ps[b] + K.shape[0]].double()
        for hh in range(h):
            sl = slice(hh * dk, (hh + 1) * dk)
            qh = q[b * T:(b + 1) * T, sl]
            s = ((qh + bu[hh].double()) @ K[:, sl].t() + (qh + bv[hh].double()) @ P[:, sl].t()) * scale
            att[b * T:(b + 1) * T, sl] = torch.softmax(s, -1) @ V[:, sl]
    y = x + att @ wout.double().t() + bout.double()
    return y, kr2, vr2


@pytest.mark.parametrize("qkv_in", [False, True])
@pytest.mark.parametrize("B,T,h,lens", [(8, 7, 16, [64, 0, 13, 64, 57, 5, 64, 1]), (3, 4, 16, [64, 33, 0]),
                                        (2, 8, 4, [64, 7]), (5, 1, 16, [0, 1, 2, 63, 64]), (1, 7, 8, [40])])
def test_enc_attn_block_matches_torch(dev, B, T, h, lens, qkv_in):
    """qkv_in: fo_enc_attn_out (q|k|v handed in, as the LayerNorm-on-load GEMM writes them) instead of
    fo_enc_attn_block computing LayerNorm1 + linear_q|k|v itself."""
    from fo import ops
    g = torch.Generator().manual_seed(B * 1000 + T * 10 + h)
    d, cap, slots, npos = 64 * h, 72, 12, 200
    x = torch.randn(B * T, d, generator=g) * 2
    lnw, lnb = 1 + 0.1 * torch.randn(d, generator=g), 0.1 * torch.randn(d, generator=g)
    wqkv = (torch.randn(3 * d, d, generator=g) / d ** 0.5).to(torch.bfloat16)
    bqkv = 0.1 * torch.randn(3 * d, generator=g)
    wout = (torch.randn(d, d, generator=g) / d ** 0.5).to(torch.bfloat16)
    bout = 0.1 * torch.randn(d, generator=g)
    kr, vr = torch.randn(slots, cap, d, generator=g), torch.randn(slots, cap, d, generator=g)
    ptab = torch.randn(npos, d, generator=g)
    bu, bv = 0.3 * torch.randn(h, 64, generator=g), 0.3 * torch.randn(h, 64, generator=g)
    st = [int(v) for v in torch.randint(0, cap, (B,), generator=g)]
    rg = [int(v) for v in torch.randperm(slots, generator=g)[:B]]
    ps = [int(v) for v in torch.randint(0, npos - cap - 8, (B,), generator=g)]
    scale = 1.0 / math.sqrt(64)
    ref, kr_ref, vr_ref = _reference(x, lnw, lnb, wqkv.float(), bqkv, kr, vr, cap, st, lens, rg, ps, ptab, bu, bv,
                                     wout.float(), bout, B, T, h, scale)
    qkv_l = ops.PackedLinear(wqkv.to(dev), bqkv.to(dev))
    out_l = ops.PackedLinear(wout.to(dev), bout.to(dev))
    xd, krd, vrd = x.to(dev), kr.to(dev), vr.to(dev)
    meta = torch.tensor(st + lens + rg + ps, dtype=torch.int32, device=dev)
    part = torch.full((B * h * T * d,), float("nan"), device=dev)
    tickets = torch.zeros(B, dtype=torch.int32, device=dev)
    stats = ops.RowStats(B * T, dev, with_sums=True)
    ops.launch_counts_reset()
    if qkv_in:
        xn = torch.nn.functional.layer_norm(x.double(), (d,), lnw.double(), lnb.double(), 1e-5)
        qkv = (xn @ wqkv.double().t() + bqkv.double()).float()
        wide = torch.full((B * T, 3 * d + 32), float("nan"))   # a row stride above 3d
        wide[:, :3 * d] = qkv
        ops.enc_attn_out(wide.to(dev), xd, B, T, h, krd, vrd, cap, meta, ptab.to(dev), bu.reshape(-1).to(dev),
                         bv.reshape(-1).to(dev), out_l, scale, part, tickets, stats)
    else:
        ops.enc_attn_block(xd, B, T, h, (lnw.to(dev), lnb.to(dev)), qkv_l, krd, vrd, cap, meta, ptab.to(dev),
                           bu.reshape(-1).to(dev), bv.reshape(-1).to(dev), out_l, scale, part, tickets, stats)
    torch.cuda.synchronize()
    assert ops.launch_counts()["enc_block"] == 1 and stats.groups == 1
    got = xd.cpu().double()
    tol = 2e-4 * ref.abs().max().item()
    assert (got - ref).abs().max().item() <= tol, (got - ref).abs().max().item()
    assert torch.allclose(krd.cpu(), kr_ref, atol=2e-4 * kr_ref.abs().max().item(), rtol=0)
    assert torch.allclose(vrd.cpu(), vr_ref, atol=2e-4 * vr_ref.abs().max().item(), rtol=0)
    n = B * T
    assert torch.allclose(stats.buf1[:n].cpu().double(), got.sum(1), rtol=1e-5, atol=1e-3 * d)
    assert torch.allclose(stats.buf[:n].cpu().double(), (got * got).sum(1), rtol=1e-5, atol=1e-3)
    assert int(tickets.abs().sum()) == 0


def test_enc_attn_block_refuses_unsupported_geometry(dev):
    """Head size != 64, more than 8 rows, or a ring that cannot be staged: a loud error, nothing launched."""
    from fo import ops
    h, d = 4, 256
    lin = ops.PackedLinear(torch.zeros(3 * d, d, dtype=torch.bfloat16, device=dev), torch.zeros(3 * d, device=dev))
    out = ops.PackedLinear(torch.zeros(d, d, dtype=torch.bfloat16, device=dev), torch.zeros(d, device=dev))
    z = lambda *s: torch.zeros(*s, device=dev)  # noqa: E731
    for T, cap in ((9, 72), (4, 93)):
        x = z(T, d)
        with pytest.raises(RuntimeError):
            ops.enc_attn_block(x, 1, T, h, (z(d), z(d)), lin, z(2, cap, d), z(2, cap, d), cap,
                               torch.zeros(4, dtype=torch.int32, device=dev), z(200, d), z(d), z(d), out, 0.125,
                               z(h * T * d), torch.zeros(1, dtype=torch.int32, device=dev),
                               ops.RowStats(T, dev, with_sums=True))


@pytest.mark.parametrize("dk,h,cap,T,C,B", [(64, 16, 72, 4, 4, 8), (8, 4, 16, 4, 4, 3), (64, 16, 72, 7, 3, 2),
                                             (8, 4, 16, 4, 2, 2)])
def test_relpos_chunks_equals_sequential_chunk_launches(dev, dk, h, cap, T, C, B):
    """fo_relpos_attention_chunks (a listen group's encoder attention: one workgroup per (user, head, chunk), earlier
    chunks' K / V from the q|k|v rows, the ring appends in a second launch) against C sequential
    fo_relpos_attention_fused launches on a copy of the ring: outputs and the final ring bit for bit, from a full ring
    (trimmed), a short one and an empty one; small rings wrap (cap 16 = C x T)."""
    import math

    import numpy as np
    import torch

    from fo import ops
    d = h * dk
    buffersize = cap - 8
    g = torch.Generator().manual_seed(dk * 100 + C)
    nb_slots = B + 2
    for L0 in (buffersize, 5, 0):
        kr = torch.randn(nb_slots, cap, d, generator=g).to(dev)
        vr = torch.randn(nb_slots, cap, d, generator=g).to(dev)
        qkv = torch.randn(C * B * T, 3 * d, generator=g).to(dev)
        ptab = torch.randn(600, d, generator=g).to(dev)
        bu, bv = torch.randn(d, generator=g).to(dev), torch.randn(d, generator=g).to(dev)
        starts = [(3 * b + 1) % cap for b in range(B)]
        lens = [min(L0, buffersize)] * B
        rings = [nb_slots - 1 - b for b in range(B)]
        pe = [40 + 4 * b for b in range(B)]
        metas = []
        for j in range(C):
            metas.append(starts + lens + rings + [max(0, p - 3 * T) for p in pe])
            for b in range(B):
                total = lens[b] + T
                keep = min(total, buffersize)
                starts[b] = (starts[b] + total - keep) % cap
                lens[b] = keep
                pe[b] += T
        meta = torch.tensor(np.concatenate(metas), dtype=torch.int32).to(dev)
        scale = 1.0 / math.sqrt(dk)
        kr1, vr1 = kr.clone(), vr.clone()
        seq = torch.empty(C * B * T, d, device=dev)
        n1 = B * T
        for j in range(C):
            mj = meta[4 * B * j:4 * B * (j + 1)]
            ops.relpos_attention_fused(qkv[j * n1:(j + 1) * n1], kr1, vr1, cap, mj[:B], mj[B:2 * B], mj[2 * B:3 * B],
                                       ptab, mj[3 * B:], bu, bv, B, T, h, dk, scale, seq[j * n1:(j + 1) * n1])
        one = torch.empty_like(seq)
        ops.relpos_attention_chunks(qkv, kr, vr, cap, meta, B, C, ptab, bu, bv, T, h, dk, scale, one)
        torch.cuda.synchronize()
        assert torch.equal(one, seq), (L0, float((one - seq).abs().max()))
        assert torch.equal(kr, kr1) and torch.equal(vr, vr1), L0
