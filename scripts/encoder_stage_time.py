"""Device time of one listen chunk's ENCODER stage at real geometry (24 blocks, d 1024, 8 users x 19 frames ->
speech encoder -> adapter), captured as one hipGraph and replayed (the ListenGraph encoder stage without the
LLM stage beside it), plus each kernel's share from a second replay under HIP events per launch.
python scripts/encoder_stage_time.py [users] (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gemm_graph_sweep_util import graph_time  # noqa: E402
from fo import ops  # noqa: E402
from fo.speech import AdapterEngine, SpeechEncoderEngine  # noqa: E402
from fo.weights import SynthSource  # noqa: E402
from oracle import configs  # noqa: E402
from oracle.params import adapter_shapes, encoder_shapes  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
cfg = configs.get("real")
src = SynthSource(cfg["seed"], {**encoder_shapes(cfg, "user"), **adapter_shapes(cfg, "user")}, dev, cfg["overrides"])
enc = SpeechEncoderEngine(src, cfg, "user", dev, max_sessions=2 * B)
ada = AdapterEngine(src, cfg, "user", dev, max_sessions=2 * B)
for R, name in ((19, "framing A"), (32, "framing B")):
    with torch.cuda.stream(ops.engine_stream(dev)):
        eb = enc.buffers(B, R)
        T = enc.dims(R)[2]
        ab = ada.buffers(B, T)
        caches = [enc.new_cache() for _ in range(B)]
        acs = [ada.new_cache() for _ in range(B)]
        meta, _ = enc.host_meta(caches, [0] * B)
        eb["meta"].copy_(torch.from_numpy(meta))
        ab["slots"].copy_(torch.tensor([c.slot for c in acs], dtype=torch.int32))
        feats = torch.randn(B, R, 80, device=dev) * 3 + 8
    enc.buffersize = enc.buffersize  # ring never advanced: every replay sees the same empty context

    def stage():
        x, T_ = enc.run(feats, B, R, eb)
        ada.run(x, B, T_, ab)

    t = graph_time(stage, 20)
    print(f"encoder stage, {B} users, {name} (R={R}): {t:8.1f} us per chunk "
          f"({(enc.weight_bytes + ada.weight_bytes) / 1e6:.0f} MB of weights -> "
          f"{(enc.weight_bytes + ada.weight_bytes) / t / 1e6:.2f} TB/s)", flush=True)
