"""Device time of one AR speech-decoder step at real geometry (896 / 14 heads / 4864, 4 layers, 8 sessions,
~300 cached keys): the multi-kernel step replayed as
the decode graph the benchmark uses, event-timed over 200 steps (host meta preparation included: the
number is the step rate the speak loop can reach).  python scripts/tts_step_time.py [B] (GPU only)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
sys.path.insert(0, ROOT)
from fo import _lib, ops  # noqa: E402
from fo.tts import TTSEngine  # noqa: E402
from fo.weights import SynthSource  # noqa: E402
from oracle import configs  # noqa: E402
from oracle.params import tts_shapes  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8   # argv[2] == "multi": the multi-kernel step only
cfg = configs.get("real")
src = SynthSource(cfg["seed"], tts_shapes(cfg), dev, cfg["overrides"])
tts = TTSEngine(src, cfg["decoder_json"], dev, kv_tokens=1 << 15)
lib = _lib.load()
e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
lib.fo_event_create(ctypes.byref(e0))
lib.fo_event_create(ctypes.byref(e1))
gen = torch.Generator().manual_seed(0)
for fused in (False, False):
    es = ops.engine_stream(dev)
    with torch.cuda.stream(es):
        items = [((torch.randn(40, 896, generator=gen) * 0.5).to(dev), (torch.randn(24, 896, generator=gen) * 0.5).to(dev))
                 for _ in range(B)]
        seqs = tts.start(items)
        g = tts.decode_graph(B, tts.vocab + 4, 1, 0, 2048, 512, None)
        g.ids.fill_(tts.sos)
        g.prime()
        for st in range(20):
            g.launch(seqs, list(range(B)), st, st)
        torch.cuda.synchronize()
        s = es.cuda_stream
        n = 200
        lib.fo_event_record(e0, s)
        for st in range(20, 20 + n):
            g.launch(seqs, list(range(B)), st, st)
        lib.fo_event_record(e1, s)
        torch.cuda.synchronize()
        g.check()
        ms = ctypes.c_float()
        lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
        print(f"multi step, {B} sessions, keys {seqs[0].kv.length}: "
              f"{ms.value / n * 1e3:7.1f} us per step", flush=True)
        if g.exec is not None:
            # the same graph replayed with no host work at all (the captured step advances its own metadata;
            # the pages of the n positions are reserved and uploaded first by one regular launch)
            for q in seqs:
                q.kv.reserve(q.kv.length + n + 32)
            g.launch(seqs, list(range(B)), 20 + n, 20 + n)
            lib.fo_event_record(e0, s)
            for st in range(n):
                _lib.call("fo_graph_launch", g.exec, s)
            lib.fo_event_record(e1, s)
            torch.cuda.synchronize()
            lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
            print(f"multi step, graph replay only (no host work): {ms.value / n * 1e3:7.1f} us per step", flush=True)
        tts.free(seqs)
