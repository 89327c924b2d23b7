"""Where the 17..64-row split-K weight stream's time goes (k_gemm_xsk, the duplex tick's Qwen2 gate/up and down):
per-workgroup clocks from the probe library (make -C freeze-omni_amd/csrc probe; loaded here through FO_LIB_PATH) --
dispatch skew, the X-slice staging (bf16 hi in VGPRs, lo in LDS), the unit loop, and inside it the cycles of the
MFMA k-steps against those of each unit's cross-wave LDS reduction and partial-slab stores -- beside the
graph-replayed time per launch (4 weight copies beyond the Infinity Cache).  python scripts/xsk_trace.py (GPU only)."""
import os
import sys

import numpy as np
import torch

os.environ.setdefault("FO_LIB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "freeze-omni_amd", "fo", "libfo_hip_probe.so"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "freeze-omni_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
D, I, NCP, CLK = 3584, 18944, 4, 100.0
trace = torch.zeros(8 * 4096, dtype=torch.int64, device=dev)
f = lambda v: f"med {np.median(v):6.2f} max {v.max():6.2f}"  # noqa: E731
for name, N, K, sw in (("gate/up", I, D, True), ("down", D, I, False)):
    lins = [ops.PackedLinear((torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16),
                             swiglu_up=(torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16) if sw
                             else None) for _ in range(NCP)]
    for M in (32, 40, 48, 56):
        x = torch.randn(M, K, device=dev, generator=g)
        y = torch.empty(M, N, device=dev)
        it = iter(range(1 << 30))
        us = graph_time(lambda: lins[next(it) % NCP](x, out=y, M=M), NCP * 8)
        trace.zero_()
        for i in range(1, NCP):
            lins[i](x, out=y, M=M)
        with torch.cuda.stream(ops.engine_stream(dev)):
            _lib.call("fo_gemm_set_trace", trace.data_ptr())
            lins[0](x, out=y, M=M)
            _lib.call("fo_gemm_set_trace", None)
        torch.cuda.synchronize()
        t = trace.view(-1, 8).cpu().numpy().astype(np.int64)
        t = t[t[:, 0] != 0]
        if len(t) == 0:
            print(f"{name} M={M}: no traced workgroups (not the split-K kernel at this shape?)", flush=True)
            continue
        t0 = t[:, 0].min()
        comp, red = t[:, 3].astype(float), t[:, 4].astype(float)
        print(f"{name:7s} M={M:2d}: {us:6.2f} us/launch incl. reduce (graph), {len(t)} WGs, units {f(t[:, 5])}; "
              f"start {f((t[:, 0] - t0) / CLK)} | X staged +{f((t[:, 1] - t[:, 0]) / CLK)} | unit loop "
              f"+{f((t[:, 2] - t[:, 1]) / CLK)} | end {f((t[:, 2] - t0) / CLK)} us; loop cycles in the LDS reduction "
              f"+ slab stores {f(red / np.maximum(comp + red, 1))} (share)", flush=True)
