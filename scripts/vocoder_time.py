"""Device time and MFMA throughput of one batched TiCodec vocoder call at real geometry (users x 60 tokens ->
36146 samples each, upsample_initial_channel 512), the bench's per-40-token call, event-timed over
replays.  python scripts/vocoder_time.py [users] [reps] (GPU only)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
sys.path.insert(0, ROOT)
from fo import _lib, ops  # noqa: E402
from fo.codec import CodecEngine  # noqa: E402
from fo.weights import SynthSource  # noqa: E402
from oracle import configs  # noqa: E402
from oracle.params import codec_shapes  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = configs.get("real")
src = SynthSource(cfg["seed"], codec_shapes(cfg), dev, cfg["overrides"])
eng = CodecEngine(src, cfg["codec_json"], dev)
ids = torch.from_numpy(np.random.default_rng(0).integers(0, 1024, size=(B, 60))).to(dev, torch.int32)
lib = _lib.load()
with torch.cuda.stream(ops.engine_stream(dev)):
    eng(ids)
    torch.cuda.synchronize()
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.fo_event_create(ctypes.byref(e0))
    lib.fo_event_create(ctypes.byref(e1))
    s = ops.stream(dev)
    lib.fo_event_record(e0, s)
    for _ in range(reps):
        eng(ids)
    lib.fo_event_record(e1, s)
    torch.cuda.synchronize()
ms = ctypes.c_float()
lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
t = ms.value / reps * 1e-3
fl = eng.flops(60) * B
print(f"vocoder: {B} users x 60 tokens: {t * 1e3:.3f} ms per call, {fl / 1e9:.1f} GFLOP "
      f"({fl / t / 1e12:.1f} TFLOP/s algorithmic; hi/lo split doubles the MFMA work) vs 2500 TFLOP/s bf16 dense",
      flush=True)
