"""A/B of the X-stationary persistent weight stream (k_gemm_xs, fo_gemm_set_xs 1) against the fo_gemm grid
kernels (0) on the Qwen2 M <= 16 shapes: per-launch device time from one replayed hipGraph of launches
that walk alternating weight copies (> the 256 MB Infinity Cache), with the epilogues the layer uses (SwiGLU + RMSNorm consumer, o-proj
residual + RMSNorm statistics, q|k|v + RoPE + paged-KV append, plain lm_head), and an output check of
XS against the grid kernel (max |diff| relative to the output scale)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import ops  # noqa: E402

dev = torch.device("cuda:0")
D, I, V, hd, H, KVH = 3584, 18944, 152064, 128, 28, 4
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*s, scale=0.02):
    return torch.randn(*s, device=dev, generator=g) * scale


def ab(name, make, ncp, M, nbytes):
    res = {0: [], 1: []}
    outs = {}
    for mode in (0, 1, 0, 1):
        lib.fo_gemm_set_xs(mode)
        fns = [make(i, M) for i in range(ncp)]
        it = iter(range(1 << 30))
        res[mode].append(graph_time(lambda: fns[next(it) % ncp](), ncp * max(1, 48 // ncp)))
        o = fns[0](check=True)
        torch.cuda.synchronize()
        outs[mode] = o.clone() if torch.is_tensor(o) else [t.clone() for t in o]
    a, b = outs[0], outs[1]
    if torch.is_tensor(a):
        a, b = [a], [b]
    err = max(float((x - y).abs().max() / (x.abs().max() + 1e-30)) for x, y in zip(a, b))
    t0, t1 = min(res[0]), min(res[1])
    print(f"{name:12s} M={M:2d} {nbytes / 1e6:7.1f}MB  grid {t0:6.1f}us ({nbytes / t0 / 1e6:4.2f}TB/s)  "
          f"xs {t1:6.1f}us ({nbytes / t1 / 1e6:4.2f}TB/s)  rel diff {err:.2e}", flush=True)


# gate/up with the RMSNorm consumer (x = yg of a producer, rows scaled by its statistics)
gus = [PackedLinear(rnd(I, D).to(torch.bfloat16), swiglu_up=rnd(I, D).to(torch.bfloat16)) for _ in range(2)]
os_ = [PackedLinear(rnd(D, D).to(torch.bfloat16)) for _ in range(6)]
stats = ops.RowStats(16, dev)
for M in (16, 8):
    xg = rnd(M, D, scale=1.0)
    res0 = rnd(M, D, scale=1.0)
    yg = torch.empty(M, D, device=dev)
    # producer statistics for the consumer (an o-proj with stats_out)
    os_[0](rnd(M, D, scale=1.0), out=res0.clone(), residual=True, M=M, stats_out=stats.set(torch.ones(D, device=dev), yg))
    outs = [torch.empty(M, I, device=dev) for _ in range(2)]

    def mk_gu(i, M, outs=outs, xg=xg):
        def f(check=False):
            return gus[i](xg, out=outs[i], M=M, norm=(stats, 1e-6))
        return f
    ab("gate/up+rms", mk_gu, 2, M, gus[0].nbytes)

    xo = rnd(M, D, scale=1.0)
    ys = [res0.clone() for _ in range(6)]
    ygs = [torch.empty(M, D, device=dev) for _ in range(6)]
    st = [ops.RowStats(16, dev) for _ in range(6)]
    gam = torch.rand(D, device=dev, generator=g) + 0.5

    def mk_o(i, M, xo=xo):
        def f(check=False):
            ys[i].copy_(res0) if check else None
            os_[i](xo, out=ys[i], residual=True, M=M, stats_out=st[i].set(gam, ygs[i]))
            return [ys[i], ygs[i]]
        return f
    ab("o+res+stats", mk_o, 6, M, os_[0].nbytes)

# q|k|v + RoPE + KV append (rope-packed), with the RMSNorm consumer
qkvs = [PackedLinear(rnd(H * hd + 2 * KVH * hd, D).to(torch.bfloat16), rnd(H * hd + 2 * KVH * hd), rope_hd=hd)
        for _ in range(6)]
cos = torch.rand(4096, hd // 2, device=dev, generator=g)
sin = torch.rand(4096, hd // 2, device=dev, generator=g)
PS, pages = 16, 64
kc = torch.zeros(pages, KVH, PS, hd, device=dev)
vc = torch.zeros_like(kc)
for M in (16, 8):
    xq = rnd(M, D, scale=1.0)
    pos = torch.arange(100, 100 + M, dtype=torch.int32, device=dev)
    slot = torch.arange(5, 5 + M, dtype=torch.int32, device=dev)
    q = torch.empty(M, H * hd, device=dev)

    def mk_q(i, M, xq=xq, pos=pos, slot=slot, q=q):
        def f(check=False):
            qkvs[i].qkv_rope(xq, M, pos, slot, cos, sin, q, kc, vc, H, KVH, PS, norm=(stats, 1e-6))
            return [q, kc[:2].clone(), vc[:2].clone()]
        return f
    ab("qkv+rope", mk_q, 6, M, qkvs[0].nbytes)

del gus, os_, qkvs
torch.cuda.empty_cache()
lms = [PackedLinear(rnd(V, D).to(torch.bfloat16)) for _ in range(2)]
for M in (8,):
    xl = rnd(M, D, scale=1.0)
    outs = [torch.empty(M, V, device=dev) for _ in range(2)]

    def mk_l(i, M, xl=xl, outs=outs):
        def f(check=False):
            return lms[i](xl, out=outs[i], M=M)
        return f
    ab("lm_head", mk_l, 2, M, lms[0].nbytes)
lib.fo_gemm_set_xs(1)
