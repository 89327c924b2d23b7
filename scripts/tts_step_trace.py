"""Phase timeline of the fused AR decode step (fo_tts_step) at real geometry, 8 sessions: per barrier, the
median over workgroups of the work time before arrival and of the wait at the barrier, and the last
arrival (wall clock of the 100 MHz counter, 10 ns).  python scripts/tts_step_trace.py (GPU only)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
sys.path.insert(0, ROOT)
from fo import ops  # noqa: E402
from fo.tts import TTSEngine  # noqa: E402
from fo.weights import SynthSource  # noqa: E402
from oracle import configs  # noqa: E402
from oracle.params import tts_shapes  # noqa: E402

dev = torch.device("cuda:0")
B = 8
cfg = configs.get("real")
src = SynthSource(cfg["seed"], tts_shapes(cfg), dev, cfg["overrides"])
tts = TTSEngine(src, cfg["decoder_json"], dev, kv_tokens=1 << 15)
tts.fused = True
gen = torch.Generator().manual_seed(0)
ncu = torch.cuda.get_device_properties(dev).multi_processor_count
names = []
for l in range(4):
    names += [f"L{l} qkv", f"L{l} attn", f"L{l} o", f"L{l} gu", f"L{l} down"]
names += ["out"]
es = ops.engine_stream(dev)
with torch.cuda.stream(es):
    items = [((torch.randn(40, 896, generator=gen) * 0.5).to(dev), (torch.randn(24, 896, generator=gen) * 0.5).to(dev))
             for _ in range(B)]
    seqs = tts.start(items)
    g = tts.decode_graph(B, tts.vocab + 4, 1, 0, 2048, 512, None, capture=False)
    tr = torch.zeros(ncu * 64, dtype=torch.int64, device=dev)
    g.fused.trace = tr.data_ptr()
    g.ids.fill_(tts.sos)
    g.prime()
    for st in range(30):
        g.launch(seqs, list(range(B)), st, st)
    torch.cuda.synchronize()
    t = tr.view(ncu, 64).cpu().numpy().astype(np.int64)
t0 = t[:, 0].min()
print(f"kernel: first start -> last end {(t[:, 63].max() - t0) / 100:.1f} us; start skew {(t[:, 0].max() - t0) / 100:.1f} us")
prev = t[:, 0]
for e, n in enumerate(names):
    arr, ext = t[:, 1 + 2 * e], t[:, 2 + 2 * e]
    work = np.median(arr - prev) / 100
    print(f"{n:10s} work med {work:6.2f} us max {(arr - prev).max() / 100:6.2f}  last arrival +{(arr.max() - prev.min()) / 100:6.2f}"
          f"  exit spread {(ext.max() - ext.min()) / 100:5.2f}  wait med {np.median(ext - arr) / 100:6.2f} us", flush=True)
    prev = ext
print(f"draw + exit: {(t[:, 63].max() - prev.min()) / 100:.1f} us")
# layer-1 sub-phases (workgroups that had the job), from the exit of the barrier before the phase
q0 = t[:84, 2 + 2 * 4]
print("L1 qkv: stage %.2f  mma %.2f  reduce %.2f  epilogue %.2f us (median over its 84 WGs)" % tuple(
    np.median(np.diff(np.stack([q0, t[:84, 50], t[:84, 51], t[:84, 52], t[:84, 53]]), axis=0), axis=1) / 100))
g0 = t[:, 2 + 2 * 7]
print("L1 gu: stage %.2f  first pair %.2f  rest %.2f us (median over WGs)" % tuple(
    np.median(np.diff(np.stack([g0, t[:, 54], t[:, 55], t[:, 56]]), axis=0), axis=1) / 100))
