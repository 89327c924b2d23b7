"""Where a vocoder ResBlock convolution launch spends its time: per-workgroup clocks of k_conv_cl (fo_conv_set_trace:
wall start / end, and the cycles of the chunk staging -- window loads, LDS-DMA weights, barriers -- against the MFMA
k-step loops) for the three k_conv_cl stages of the real TiCodec generator at 8 users x 60 tokens: a ResBlock c1
launch of the stage's three chains side by side (K 3 / 7 / 11, dilation 1).  python scripts/vocoder_trace.py (GPU)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fo import _lib, ops  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402

dev = torch.device("cuda:0")
B, CLK = 8, 100.0
g = torch.Generator(device=dev).manual_seed(0)
trace = torch.zeros(4 * 8192, dtype=torch.int64, device=dev)
for C, L in ((256, 300), (128, 1500), (64, 6000)):
    x = torch.randn(B, L, C, device=dev, generator=g)
    pcs = [ops.PackedConv((torch.randn(C, C, k, device=dev, generator=g) / (C * k) ** 0.5).to(torch.bfloat16),
                          torch.zeros(C, device=dev)) for k in (3, 7, 11)]
    outs = [torch.empty(B, L, C, device=dev) for _ in pcs]

    def launch():
        ops.conv_cl_multi([ops.conv_desc(x, L, pc, 1, (pc.K - 1) // 2, o, pre_leaky=0.1) for pc, o in zip(pcs, outs)],
                          B, C, C, dev)
    us = graph_time(launch, 20)
    flops = sum(2 * C * C * pc.K * L * B for pc in pcs)
    trace.zero_()
    with torch.cuda.stream(ops.engine_stream(dev)):
        _lib.call("fo_conv_set_trace", trace.data_ptr())
        launch()
        _lib.call("fo_conv_set_trace", None)
        torch.cuda.synchronize()
    t = trace.view(-1, 4).cpu().numpy().astype(np.int64)
    t = t[t[:, 0] != 0]
    t0 = t[:, 0].min()
    span = (t[:, 3] - t[:, 0]) / CLK
    stage, comp = t[:, 1].astype(float), t[:, 2].astype(float)
    frac = stage / np.maximum(stage + comp, 1)
    f = lambda v: f"med {np.median(v):7.2f} max {v.max():7.2f}"  # noqa: E731
    print(f"C={C:3d} L={L:5d}: {us:7.2f} us/launch ({flops / us / 1e6:6.1f} TFLOP/s algorithmic), {len(t)} WGs; "
          f"WG span us {f(span)}; start skew us {f((t[:, 0] - t0) / CLK)}; end us {f((t[:, 3] - t0) / CLK)}; "
          f"staging share of the chunk loop {f(frac)}; stage Mcyc {f(stage / 1e6)} comp Mcyc {f(comp / 1e6)}",
          flush=True)
