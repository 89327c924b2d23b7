"""fo_gemm (packed-weight MFMA GEMM) vs a plain fp32 reference of the same op."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(x_bf, w_bf, bias, act, resid):
    y = x_bf.float() @ w_bf.float().t()
    if bias is not None:
        y = y + bias
    if act == "relu":
        y = torch.relu(y)
    elif act == "silu":
        y = torch.nn.functional.silu(y)
    if resid is not None:
        y = y + resid
    return y


@pytest.mark.parametrize("M,N,K", [(1, 64, 64), (3, 100, 96), (16, 4608, 3584), (17, 3584, 18944), (40, 1024, 9216),
                                   (64, 896, 896), (130, 272, 160), (7, 152, 32), (260, 1024, 288),
                                   (608, 1024, 9216)])
@pytest.mark.parametrize("act", ["none", "relu"])
def test_gemm_matches_fp32(dev, M, N, K, act):
    from fo.ops import PackedLinear
    g = torch.Generator(device="cpu").manual_seed(M * 1000 + N + K)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    lin = PackedLinear(w.to(dev), b.to(dev))
    y = lin(x.to(dev), act=act).cpu()
    ref = _ref(x, w, b, act, None)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)


def test_gemm_residual_bf16_out(dev):
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(7)
    M, N, K = 5, 300, 640
    w = (torch.randn(N, K, generator=g) / 25).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    r = torch.randn(M, N, generator=g)
    lin = PackedLinear(w.to(dev))
    out = r.clone().to(dev)
    lin(x.to(dev), out=out, residual=True)
    torch.testing.assert_close(out.cpu(), _ref(x, w, None, "none", r), rtol=1e-4, atol=1e-4)
    outb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    lin(x.to(dev), out=outb)
    torch.testing.assert_close(outb.float().cpu(), _ref(x, w, None, "none", None), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M", [1, 8, 33])
def test_gemm_swiglu(dev, M):
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(M)
    N, K = 4864, 896
    wg = (torch.randn(N, K, generator=g) / 30).to(torch.bfloat16)
    wu = (torch.randn(N, K, generator=g) / 30).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    lin = PackedLinear(wg.to(dev), swiglu_up=wu.to(dev))
    y = lin(x.to(dev)).cpu()
    ref = torch.nn.functional.silu(x.float() @ wg.float().t()) * (x.float() @ wu.float().t())
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,K", [(1, 3584, 3584), (9, 4608, 3584), (40, 1024, 9216), (100, 64, 288)])
def test_gemm_fp32_activations_split(dev, M, N, K):
    """fp32 X is split into bf16 hi+lo: error vs an fp64 reference ~1e-5 relative (not bf16's ~4e-3)."""
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(M + N)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g)
    b = torch.randn(N, generator=g)
    sc = torch.rand(N, generator=g) + 0.5
    sh = torch.randn(N, generator=g)
    lin = PackedLinear(w.to(dev), b.to(dev))
    lin.set_affine(sc, sh)
    y = lin(x.to(dev), act="relu").cpu().double()
    ref = torch.relu((x.double() @ w.double().t() + b.double()) * sc.double() + sh.double())
    err = (y - ref).abs().max().item()
    assert err < 2e-4 * ref.abs().max().item(), err


@pytest.mark.parametrize("M", [17, 32, 40, 48, 56, 64])
@pytest.mark.parametrize("N,K,sw", [(3584, 3584, False), (3584, 18944, False), (4096, 3584, True), (1024, 4096, False),
                                    (3072, 1024, False), (2304, 1856, False), (1152, 3584, True)])
def test_gemm_mid_rows(dev, M, N, K, sw):
    """17..64 fp32 rows on Qwen2-sized weights (the duplex ticks and the turn's prefills): the X-stationary
    split-K stream (k_gemm_xsk + k_gemm_reduce; K = 1856 = 58 k-steps leaves the last split 2 k-steps, the other
    waves' past-K steps predicated off) or, for K < 56 k-steps, one row tile of ceil(M/16) row blocks; vs an fp64
    reference (hi/lo split accuracy)."""
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(M * 31 + N + K)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g)
    if sw:
        u = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
        lin = PackedLinear(w.to(dev), swiglu_up=u.to(dev))
        y = lin(x.to(dev)).cpu().double()
        ref = torch.nn.functional.silu(x.double() @ w.double().t()) * (x.double() @ u.double().t())
    else:
        b = torch.randn(N, generator=g)
        r = torch.randn(M, N, generator=g)
        lin = PackedLinear(w.to(dev), b.to(dev))
        out = r.clone().to(dev)
        lin(x.to(dev), out=out, residual=True)
        y = out.cpu().double()
        ref = x.double() @ w.double().t() + b.double() + r.double()
    err = (y - ref).abs().max().item()
    assert err < 2e-4 * ref.abs().max().item(), err
    # deterministic: the split partials are summed in split order
    if sw:
        assert torch.equal(lin(x.to(dev)).cpu().double(), y)
    else:
        out2 = r.clone().to(dev)
        lin(x.to(dev), out=out2, residual=True)
        assert torch.equal(out2.cpu().double(), y)


@pytest.mark.parametrize("M", [65, 72, 100, 128])
@pytest.mark.parametrize("producer", ["down", "o"])
@pytest.mark.parametrize("rows", [1, 0])
def test_gemm_65_to_128_rows_on_qwen2_streams(dev, M, producer, rows):
    """65..128 rows on the Qwen2 down (136 MB) or o (26 MB) projection (residual + the next RMSNorm's statistics) and
    the gate/up (272 MB, SwiGLU + the RMSNorm consumer).  rows 1 (default): down and gate/up through k_gemm_rows (the
    8 waves split the rows, the weights stream once through an LDS-DMA ring; k_gemm_reduce runs the epilogue); rows 0
    (fo_gemm_set_rows): two launches on the row halves (k_gemm_xsk; o on the one-row-tile split-K kernels), whose
    statistics groups tile one [M][groups] layout; vs an fp64 residual -> RMSNorm -> SwiGLU reference."""
    from fo import _lib, ops
    from fo.ops import PackedLinear
    lib = _lib.load()
    prev = lib.fo_gemm_set_rows(rows)
    try:
        _qwen2_65_128(dev, M, producer, rows)
    finally:
        lib.fo_gemm_set_rows(prev)


def _qwen2_65_128(dev, M, producer, rows):
    from fo import ops
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(M)
    D, I = 3584, 18944 if producer == "down" else 3584
    wd = (torch.randn(D, I, generator=g) / I ** 0.5).to(torch.bfloat16)
    wg = (torch.randn(18944, D, generator=g) / D ** 0.5).to(torch.bfloat16)
    wu = (torch.randn(18944, D, generator=g) / D ** 0.5).to(torch.bfloat16)
    gamma = torch.rand(D, generator=g) + 0.5
    hin = torch.randn(M, I, generator=g)
    res = torch.randn(M, D, generator=g)
    down, gu = PackedLinear(wd.to(dev)), PackedLinear(wg.to(dev), swiglu_up=wu.to(dev))
    st = ops.RowStats(M, dev)
    x = res.clone().to(dev)
    yg = torch.empty(M, D, device=dev)
    ops.launch_counts_reset()
    down(hin.to(dev), out=x, residual=True, stats_out=st.set(gamma.to(dev), yg))
    out = gu(yg, norm=(st, 1e-6))
    torch.cuda.synchronize()
    c = ops.launch_counts()
    if rows:   # (o: 26 MB, k_gemm_rows from 16 MiB of weights)
        assert c["gemm_rows"] == 2 and c["gemm_xsk"] == 0 and c["gemm_reduce"] == 2, c
    else:
        assert c["gemm_xsk"] == (4 if producer == "down" else 2) and c["gemm_rows"] == 0, c   # two row halves each
        assert c["gemm_reduce"] == 4, c
    y = res.double() + hin.double() @ wd.double().t()
    torch.testing.assert_close(x.cpu().double(), y, rtol=1e-5, atol=1e-4)
    h = y * torch.rsqrt((y * y).mean(-1, keepdim=True) + 1e-6) * gamma.double()
    ref = torch.nn.functional.silu(h @ wg.double().t()) * (h @ wu.double().t())
    err = (out.cpu().double() - ref).abs().max().item()
    assert err < 2e-4 * ref.abs().max().item(), err


@pytest.mark.parametrize("M", [8, 16, 40, 56])
@pytest.mark.parametrize("sw", [False, True])
def test_gemm_rmsnorm_across_gemms(dev, M, sw):
    """RMSNorm fused across two GEMMs (RowStats): the producer (+residual) writes y * gamma and row
    partial sums, the consumer scales rows by rstd -- single pass or split over K (mid rows: the reduce
    launch applies rstd); vs fp64 residual -> RMSNorm -> projection."""
    from fo import ops
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(M * 5 + sw)
    D, N = 3584, 4096 if sw else 4608
    wp = (torch.randn(D, 1024, generator=g) / 32).to(torch.bfloat16)
    wc = (torch.randn(N, D, generator=g) / D ** 0.5).to(torch.bfloat16)
    wu = (torch.randn(N, D, generator=g) / D ** 0.5).to(torch.bfloat16)
    gamma = torch.rand(D, generator=g) + 0.5
    xin = torch.randn(M, 1024, generator=g)
    res = torch.randn(M, D, generator=g)
    prod = PackedLinear(wp.to(dev))
    cons = PackedLinear(wc.to(dev), swiglu_up=wu.to(dev)) if sw else PackedLinear(wc.to(dev))
    st = ops.RowStats(M, dev)
    x = res.clone().to(dev)
    yg = torch.empty(M, D, device=dev)
    prod(xin.to(dev), out=x, residual=True, stats_out=st.set(gamma.to(dev), yg))
    out = cons(yg, norm=(st, 1e-6))
    y = res.double() + xin.double() @ wp.double().t()
    h = y * torch.rsqrt((y * y).mean(-1, keepdim=True) + 1e-6) * gamma.double()
    ref = torch.nn.functional.silu(h @ wc.double().t()) * (h @ wu.double().t()) if sw else h @ wc.double().t()
    torch.testing.assert_close(x.cpu().double(), y, rtol=1e-5, atol=1e-4)
    err = (out.cpu().double() - ref).abs().max().item()
    assert err < 2e-4 * ref.abs().max().item(), err


def test_gemm_deterministic_splitk(dev):
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(3)
    M, N, K = 4, 3584, 18944
    w = (torch.randn(N, K, generator=g) / 100).to(torch.bfloat16).to(dev)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    lin = PackedLinear(w)
    ys = [lin(x).cpu() for _ in range(5)]
    for y in ys[1:]:
        assert torch.equal(y, ys[0])
    y1 = lin(x, splitk=1).cpu()
    torch.testing.assert_close(y1, ys[0], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,H,KVH,hd,K,splitk", [(1, 28, 4, 128, 3584, 0), (16, 28, 4, 128, 3584, 0),
                                                 (16, 28, 4, 128, 3584, 3), (40, 4, 2, 32, 128, 0),
                                                 (70, 14, 14, 64, 896, 0), (8, 14, 14, 64, 896, 2),
                                                 (24, 4, 4, 32, 128, 0), (40, 28, 4, 128, 3584, 0),
                                                 (56, 28, 4, 128, 3584, 0), (72, 28, 4, 128, 3584, 0),
                                                 (128, 28, 4, 128, 3584, 0)])
def test_gemm_qkv_rope(dev, M, H, KVH, hd, K, splitk):
    """Fused q|k|v projection + bias + rotate_half RoPE + paged-KV append vs an fp32 torch reference (72 / 128 rows
    at Qwen2 geometry: k_gemm_rows + the pair epilogue in k_gemm_reduce)."""
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(M * 7 + H + hd)
    N = (H + 2 * KVH) * hd
    PS, n_pages, half = 16, 24, hd // 2
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    x = torch.randn(M, K, generator=g)
    pos = torch.randint(0, 300, (M,), generator=g, dtype=torch.int32)
    slot = torch.randperm(n_pages * PS, generator=g)[:M].to(torch.int32)
    inv = 1.0 / (1e6 ** (torch.arange(0, half, dtype=torch.float64) / half))
    ang = torch.arange(512, dtype=torch.float64)[:, None] * inv[None]
    cos, sin = torch.cos(ang).float(), torch.sin(ang).float()
    lin = PackedLinear(w.to(dev), b.to(dev), rope_hd=hd)
    q = torch.full((M, H * hd), float("nan"), device=dev)
    kc = torch.zeros(n_pages, KVH, PS, hd, device=dev)
    vc = torch.zeros(n_pages, KVH, PS, hd, device=dev)
    lin.qkv_rope(x.to(dev), M, pos.to(dev), slot.to(dev), cos.to(dev), sin.to(dev), q, kc, vc, H, KVH, PS,
                 splitk=splitk)
    y = x.double() @ w.double().t() + b.double()
    heads = y.view(M, H + 2 * KVH, hd)
    c, s = cos.double()[pos.long()][:, None, :], sin.double()[pos.long()][:, None, :]
    x1, x2 = heads[..., :half], heads[..., half:]
    rot = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)
    torch.testing.assert_close(q.cpu().double(), rot[:, :H].reshape(M, -1), rtol=2e-5, atol=2e-5)
    kref = torch.zeros(n_pages, KVH, PS, hd, dtype=torch.float64)
    vref = torch.zeros_like(kref)
    for m in range(M):
        pg, off = int(slot[m]) // PS, int(slot[m]) % PS
        kref[pg, :, off] = rot[m, H:H + KVH]
        vref[pg, :, off] = heads[m, H + KVH:]
    torch.testing.assert_close(kc.cpu().double(), kref, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(vc.cpu().double(), vref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("M,N,K,act,splitk,psplit", [(32, 3072, 1024, "none", 0, 0), (32, 4096, 1024, "relu", 0, 4),
                                                     (17, 1024, 1024, "none", 2, 0), (8, 96, 32, "relu", 0, 0),
                                                     (1, 64, 64, "none", 0, 2), (32, 64, 32, "none", 0, 0),
                                                     (56, 3072, 1024, "none", 0, 0), (56, 4096, 1024, "relu", 0, 4),
                                                     (40, 1024, 1024, "none", 2, 0), (64, 64, 32, "relu", 0, 0)])
def test_gemm_layernorm_on_load(dev, M, N, K, act, splitk, psplit):
    """fo_gemm_rowstats (residual producer writing row sums / sums of squares) -> fo_gemm_ln (LayerNorm
    applied to X on load from those statistics) vs residual + LayerNorm + Linear in fp64."""
    from fo import ops
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(M + N + K)
    Kp = 96
    wp = (torch.randn(K, Kp, generator=g) / Kp ** 0.5).to(torch.bfloat16)
    xp = torch.randn(M, Kp, generator=g)
    r = torch.randn(M, K, generator=g) * 2 + 0.7
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g)
    lw, lb = torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1
    prod, lin = PackedLinear(wp.to(dev)), PackedLinear(w.to(dev), b.to(dev))
    st = ops.RowStats(M, dev, with_sums=True)
    x = r.clone().to(dev)
    prod.rowstats(xp.to(dev), x, st, residual=True, splitk=psplit)
    y = lin.ln(x, lw.to(dev), lb.to(dev), st, 1e-5, act=act, splitk=splitk).cpu()
    xr = r.double() + xp.double() @ wp.double().t()
    torch.testing.assert_close(x.cpu().double(), xr, rtol=2e-5, atol=2e-5)
    xn = torch.nn.functional.layer_norm(xr, (K,), lw.double(), lb.double(), 1e-5)
    ref = xn @ w.double().t() + b.double()
    if act == "relu":
        ref = torch.relu(ref)
    torch.testing.assert_close(y.double(), ref, rtol=5e-5, atol=5e-5)


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K,sw", [(8, 18944, 3584, True), (16, 18944, 3584, True), (16, 3584, 18944, False),
                                      (5, 4608, 3584, False)])
def test_gemm_pipelined_weight_stream(dev, mode, M, N, K, sw):
    """k_gemm_wpipe (software-pipelined weight stream, fo_gemm_set_pipe modes 1-3) vs an fp64 reference of
    the fp32-X GEMM (+ SwiGLU), next to the plain loop (mode 0): same tolerance for every mode."""
    from fo import _lib
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(M + N + K)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    u = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16) if sw else None
    x = torch.randn(M, K, generator=g)
    lin = PackedLinear(w.to(dev), swiglu_up=None if u is None else u.to(dev))
    lib = _lib.load()
    prev = lib.fo_gemm_set_pipe(mode)
    assert prev >= 0
    try:
        y = lin(x.to(dev)).cpu().double()
    finally:
        lib.fo_gemm_set_pipe(prev)
    a = x.double() @ w.double().t()
    ref = torch.nn.functional.silu(a) * (x.double() @ u.double().t()) if sw else a
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("M,N,K", [(8, 896, 4864), (16, 3584, 18944), (5, 1024, 4096)])
def test_gemm_split_merge_in_launch_bit_exact(dev, M, N, K):
    """Split-K merged inside the launch (fo_gemm_set_merge(1): write-through partials, per-tile ticket, the
    last split sums in split order and runs the epilogue) == slabs + k_gemm_reduce bit for bit: the
    residual-updated output and yg = y * gamma, launch after launch (tickets left zeroed); the RMSNorm row
    statistics agree as sums (their grouping differs: per tile group vs per 256 columns)."""
    from fo import _lib
    from fo.ops import PackedLinear, RowStats
    g = torch.Generator().manual_seed(M * N + K)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(dev)
    res0 = torch.randn(M, N, generator=g).to(dev)
    gamma = (1 + 0.1 * torch.randn(N, generator=g)).to(dev)
    lin = PackedLinear(w.to(dev))
    lib = _lib.load()

    def run():
        y = res0.clone()
        yg = torch.full_like(y, float("nan"))   # every column must be written (no stale memory passes)
        st = RowStats(M, dev).set(gamma, yg)
        lin(x, out=y, residual=True, splitk=4, stats_out=st)
        ss = st.buf[:M * st.groups].view(M, st.groups).sum(1)
        return y.cpu(), yg.cpu(), ss.cpu()

    prev = lib.fo_gemm_set_merge(0)
    assert prev in (0, 1, 2)
    try:
        y0, g0, s0 = run()
        lib.fo_gemm_set_merge(1)
        outs = [run() for _ in range(3)]
    finally:
        lib.fo_gemm_set_merge(prev)
    for y1, g1, s1 in outs:
        assert torch.equal(y1, y0) and torch.equal(g1, g0)
        torch.testing.assert_close(s1, s0, rtol=1e-5, atol=1e-3)
    ref = x.cpu().double() @ w.double().t() + res0.cpu().double()
    torch.testing.assert_close(y0.double(), ref, rtol=5e-5, atol=5e-5)
    torch.testing.assert_close(s0.double(), (ref ** 2).sum(1), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(g0.double(), ref * gamma.cpu().double(), rtol=5e-5, atol=5e-5)


@pytest.mark.parametrize("M,N,K,sw", [(97, 2320, 4096, False), (128, 4624, 2048, False), (66, 2208, 3584, True),
                                      (113, 3056, 4096, True)])
def test_gemm_rows_ragged_tile_groups(dev, M, N, K, sw):
    """k_gemm_rows on shapes whose tile count is no multiple of its tiles per workgroup (the last group ragged, its
    padding weight loads and tiles never stored) and whose K splits are uneven, plain (bias + residual) and SwiGLU;
    vs an fp64 reference (hi / lo accuracy), and the launch counter shows the kernel ran."""
    from fo import ops
    from fo.ops import PackedLinear
    g = torch.Generator().manual_seed(M * 7 + N + K)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g)
    ops.launch_counts_reset()
    if sw:
        u = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
        lin = PackedLinear(w.to(dev), swiglu_up=u.to(dev))
        y = lin(x.to(dev)).cpu().double()
        ref = torch.nn.functional.silu(x.double() @ w.double().t()) * (x.double() @ u.double().t())
    else:
        b = torch.randn(N, generator=g)
        r = torch.randn(M, N, generator=g)
        lin = PackedLinear(w.to(dev), b.to(dev))
        out = r.clone().to(dev)
        lin(x.to(dev), out=out, residual=True)
        y = out.cpu().double()
        ref = x.double() @ w.double().t() + b.double() + r.double()
    torch.cuda.synchronize()
    assert ops.launch_counts()["gemm_rows"] == 1
    err = (y - ref).abs().max().item()
    assert err < 2e-4 * ref.abs().max().item(), err
