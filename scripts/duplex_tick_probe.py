"""Per-tick host timing of the config-5 duplex loop (bench.run_duplex, 8 sessions, 20 s): the slow ticks, and for
each the split between pump (VAD, framing), the batched fbank + delivery, and the batched prefill.
python scripts/duplex_tick_probe.py [seconds] (GPU only; FO_DUPLEX_BATCH_FBANK selects the gating form)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
import bench  # noqa: E402
from fo import duplex  # noqa: E402

rec = []
orig_tick = duplex.DuplexScheduler.tick


def tick(self):
    t0 = time.perf_counter()
    defer = [] if duplex.BATCH_FBANK else None
    for s in self.sessions:
        s.pump(defer)
    t1 = time.perf_counter()
    duplex.deliver_deferred(defer)
    t2 = time.perf_counter()
    work = []
    for s in self.sessions:
        d = s.next_feature()
        if d is not None:
            work.append((s, d))
    if not work:
        rec.append((t1 - t0, t2 - t1, 0.0, 0, len(defer or [])))
        return []
    import torch
    with torch.no_grad():
        results = self.pipeline.speech_dialogue_batch([s.request(d) for s, d in work])
    out = [(s, d, s.apply(d, r)) for (s, d), r in zip(work, results)]
    rec.append((t1 - t0, t2 - t1, time.perf_counter() - t2, len(work), len(defer or [])))
    return out


duplex.DuplexScheduler.tick = tick
if os.environ.get("PROBE_NOGC") == "1":   # hypothesis checks for slow ticks: no cyclic GC
    import gc
    gc.disable()
if os.environ.get("PROBE_CLONE") == "1":  # ... or each chunk's rows as their own tensor, not a view of the batch
    import models.AudioFeatureGating as afg
    _fb = afg.fbank_batch
    afg.fbank_batch = lambda g, r: [f.clone() for f in _fb(g, r)]
secs = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
sys.argv = [sys.argv[0], "--scenario", "duplex"]
args = bench.parse()
import torch  # noqa: E402
from fo.engine import FreezeOmniEngine  # noqa: E402
dev = torch.device("cuda", 0)
eng = FreezeOmniEngine(os.path.join(ROOT, "configs", args.config), device=dev, max_sessions=max(8, args.users))
sync = torch.cuda.synchronize
bench.run_duplex(eng, args, 6.0, sync)
for rep in range(2):
    rec.clear()
    r = bench.run_duplex(eng, args, secs, sync)
    ticks = np.array(r["ticks"]) * 1e3
    print(f"run {rep} batched_fbank={duplex.BATCH_FBANK}: wall {r['wall']:.2f} s, {len(ticks)} ticks, p50 "
          f"{np.percentile(ticks, 50):.2f} p90 {np.percentile(ticks, 90):.2f} max {ticks.max():.2f} ms", flush=True)
    a = np.array([x[:3] for x in rec]) * 1e3
    slow = [i for i, x in enumerate(rec) if sum(x[:3]) > 0.02]
    print(f"  per tick() call: pump p50 {np.median(a[:, 0]):.3f} ms, fbank+deliver p50 {np.median(a[:, 1]):.3f}, "
          f"prefill p50 {np.median(a[:, 2]):.3f}; {len(rec)} calls, {len(slow)} over 20 ms", flush=True)
    for i in slow[:12]:
        x = rec[i]
        print(f"  call {i}: pump {x[0] * 1e3:.2f} fbank+deliver {x[1] * 1e3:.2f} prefill {x[2] * 1e3:.2f} ms, "
              f"items {x[3]}, deferred chunks {x[4]}", flush=True)
