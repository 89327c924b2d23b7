"""Where the time of a small weight-stream GEMM goes: per-workgroup wall clocks (fo_gemm_set_trace) of the
last launch of a graph-replayed sequence over six weight copies (beyond the Infinity Cache), for the M <= 16
hot shapes below 64 MB (Qwen2 o and q|k|v, the TTS decoder's).  Prints, over the workgroups: dispatch skew
(start - first start), weight-stream time (start -> last wave's loop end), K reduce, epilogue, and the
kernel span (first start -> last epilogue issue) beside the graph-timed per-launch time.
python scripts/gemm_trace.py (GPU only; needs the probe library: make -C freeze-omni_amd/csrc probe)."""
import os
import sys

import numpy as np
import torch

# the clock hook lives in the probe library only (freeze-omni_amd/csrc: make probe)
os.environ.setdefault("FO_LIB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "freeze-omni_amd", "fo", "libfo_hip_probe.so"))

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pipe_ab import PackedLinear, lib  # noqa: E402
from gemm_graph_sweep_util import graph_time  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
shapes = [("qwen_o", 3584, 3584, 16, True), ("qwen_qkv", 4608, 3584, 16, False), ("qwen_o_m8", 3584, 3584, 8, True),
          ("tts_o", 896, 896, 8, True), ("tts_qkv", 1152, 896, 8, False), ("tts_down", 896, 4864, 8, True)]
CLK = 100.0  # wall clock, MHz
trace = torch.zeros(4096 * 24, dtype=torch.int64, device=dev)
for name, N, K, M, res in shapes:
    lins = [PackedLinear((torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)) for _ in range(6)]
    x = torch.randn(M, K, device=dev, generator=g)
    ys = [torch.randn(M, N, device=dev, generator=g) for _ in range(6)]
    it = iter(range(1 << 30))
    us = graph_time(lambda: (lambda i: lins[i](x, out=ys[i], residual=res, M=M))(next(it) % 6), 48)
    trace.zero_()

    def seq():
        for i in range(11):
            lins[i % 6](x, out=ys[i % 6], residual=res, M=M)
        lib.fo_gemm_set_trace(trace.data_ptr())
        lins[5](x, out=ys[5], residual=res, M=M)
        lib.fo_gemm_set_trace(None)
    graph_time(seq, 1)
    t = trace.view(-1, 24).cpu().numpy()
    t = t[t[:, 0] != 0]
    nwg = len(t)
    st = t[:, 0]
    loop = t[:, 1:17]
    loop_end = np.where(loop > 0, loop, 0).max(1)
    loop_first = np.where(loop > 0, loop, np.iinfo(np.int64).max).min(1)
    t0 = st.min()
    q = lambda v: f"med {np.median(v) / CLK:5.2f} max {v.max() / CLK:5.2f}"  # noqa: E731
    print(f"{name:10s} M={M:2d} N={N:5d} K={K:5d} WGs {nwg:4d}  graph {us:6.2f} us/launch  span "
          f"{(t[:, 18].max() - t0) / CLK:6.2f} us", flush=True)
    print(f"   dispatch skew {q(st - t0)} | stream first wave {q(loop_first - st)} last wave {q(loop_end - st)}"
          f" | reduce {q(t[:, 17] - loop_end)} | epilogue {q(t[:, 18] - t[:, 17])}", flush=True)
    del lins, ys
    torch.cuda.empty_cache()
