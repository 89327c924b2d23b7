"""Where a persistent Qwen2 layer would win or lose (round-4 verdict item 4), measured on one seam: the o projection
(+ residual + the next RMSNorm's statistics) followed by the SwiGLU gate/up that consumes it, at 8 (text step) and
16 (listen chunk) rows, K = 3584.

  A  the product: two launches (o: fo_gemm with statistics out; gate/up: k_gemm_xs with the RMSNorm consumer)
  B  one launch (fo_probe_seam mode 0, k_seam_o_gu): o workgroups publish through an agent-scope release counter,
     the gate/up workgroups issue their first weights, poll the counter, then load X and stream on
  B1 / B2  the seam kernel's o workgroups alone / its gate/up workgroups alone (mode 1 / 2)

Per-launch device time from one replayed hipGraph over weight copies beyond the 256 MB Infinity Cache (a zeroing
node before every launch in both forms), then per-workgroup wall clocks (100 MHz) of one seam launch: when the o
workgroups publish, when the gate/up workgroups see the counter, how long they stream after it.  Outputs of B are
checked against A (relative to each output's scale).

python scripts/seam_probe.py (GPU only)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
D, I, EPS, NCP = 3584, 18944, 1e-6, 4
CLK = 100.0
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*s, scale=0.02):
    return torch.randn(*s, device=dev, generator=g) * scale


wo = [PackedLinear(rnd(D, D).to(torch.bfloat16)) for _ in range(NCP)]
gu = [PackedLinear(rnd(I, D).to(torch.bfloat16), swiglu_up=rnd(I, D).to(torch.bfloat16)) for _ in range(NCP)]
gamma = 1 + 0.1 * rnd(D, scale=1.0)
ready = torch.zeros(1, dtype=torch.int32, device=dev)
timeout = torch.zeros(1, dtype=torch.int32, device=dev)
n_o = D // 32
trace = torch.zeros(4 * 2048, dtype=torch.int64, device=dev)
for M in (8, 16):
    xo = rnd(M, D, scale=1.0)
    x0 = rnd(M, D, scale=1.0)
    xa, xb = x0.clone(), x0.clone()
    yga, ygb = torch.empty(M, D, device=dev), torch.empty(M, D, device=dev)
    ha, hb = torch.empty(M, I, device=dev), torch.empty(M, I, device=dev)
    stats = ops.RowStats(M, dev)
    sout = torch.zeros(M * n_o, device=dev)

    def prod(i, x=None, yg=None, h=None):
        x = xa if x is None else x
        ready.zero_()   # (the same zeroing node as the seam form)
        wo[i](xo, out=x, residual=True, M=M, stats_out=stats.set(gamma, yga if yg is None else yg))
        gu[i](yga if yg is None else yg, out=ha if h is None else h, M=M, norm=(stats, EPS))

    def seam(i, mode=0, tr=None, x=None):
        ready.zero_()
        if mode == 2:
            ready.fill_(n_o)
        _lib.call("fo_probe_seam", xo.data_ptr(), M, wo[i].packed.data_ptr(), None, (xb if x is None else x).data_ptr(),
                  gamma.data_ptr(), ygb.data_ptr(), sout.data_ptr(), gu[i].packed.data_ptr(), I, hb.data_ptr(), EPS,
                  ready.data_ptr(), timeout.data_ptr(), tr, mode, ops.stream(dev))

    reps = NCP * 12
    it = iter(range(1 << 30))
    t_a = graph_time(lambda: prod(next(it) % NCP), reps)
    t_b = graph_time(lambda: seam(next(it) % NCP), reps)
    t_b1 = graph_time(lambda: seam(next(it) % NCP, 1), reps)
    t_b2 = graph_time(lambda: seam(next(it) % NCP, 2), reps)
    t_a2 = graph_time(lambda: prod(next(it) % NCP), reps)
    t_b3 = graph_time(lambda: seam(next(it) % NCP), reps)
    t_z = graph_time(lambda: ready.zero_(), reps)
    # outputs: one launch each from the same inputs
    xa.copy_(x0)
    xb.copy_(x0)
    prod(0)
    seam(0)
    torch.cuda.synchronize()
    assert int(timeout.item()) == 0, "seam probe: the bounded poll timed out"
    rel = lambda p, q: float((p - q).abs().max() / (p.abs().max() + 1e-30))  # noqa: E731
    print(f"M={M:2d}  A two launches {min(t_a, t_a2) - t_z:6.2f} us   B seam {min(t_b, t_b3) - t_z:6.2f} us   "
          f"B1 o alone {t_b1 - t_z:6.2f}   B2 gate/up alone {t_b2 - t_z:6.2f}   (zeroing node {t_z:4.2f} us subtracted)",
          flush=True)
    print(f"      B vs A: x {rel(xa, xb):.1e}  yg {rel(yga, ygb):.1e}  h {rel(ha, hb):.1e}", flush=True)
    # per-workgroup clocks of one seam launch after warm launches over the other copies
    trace.zero_()

    def seq():
        for i in range(1, NCP):
            seam(i)
        seam(0, 0, trace.data_ptr())
    graph_time(seq, 1)
    t = trace.view(-1, 4).cpu().numpy()
    n_wg = int((t[:, 0] != 0).sum())
    t = t[:n_wg].astype(np.int64)
    t0 = t[:, 0].min()
    o, u = t[:n_o], t[n_o:]
    f = lambda v: f"med {np.median(v) / CLK:6.2f} max {v.max() / CLK:6.2f}"  # noqa: E731
    pub = o[:, 2] - t0
    print(f"      o WGs {len(o)}: start {f(o[:, 0] - t0)} | reduced {f(o[:, 1] - t0)} | published {f(pub)}", flush=True)
    print(f"      gate/up WGs {len(u)}: start {f(u[:, 0] - t0)} | ready seen {f(u[:, 2] - t0)} "
          f"(last publish {pub.max() / CLK:6.2f}) | end {f(u[:, 3] - t0)} | after ready {f(u[:, 3] - u[:, 2])}",
          flush=True)
    print(f"      span {(t[:, 3].max() - t0) / CLK:6.2f} us", flush=True)
