"""Receive-only replica on the device (bench.py N > 1): an engine built from shapes only
(ReceiveSource: uninitialised weights) and filled by fo.replica.broadcast_frozen from a fully built
engine gives the same results bit for bit -- listen (state probabilities), the AR codec ids and the
vocoder PCM -- so every weight the path reads is covered by the broadcast (packed layouts, derived tables
and views included).  One process: the broadcast is replayed through a recording stand-in of
torch.distributed (the gloo world-2 form is tests/test_dist_cpu.py)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "configs", "tiny")


class _Record:
    def __init__(self):
        self.flats = []

    def broadcast(self, t, src):
        self.flats.append(t.clone())


class _Play:
    def __init__(self, flats):
        self.flats, self.i = flats, 0

    def broadcast(self, t, src):
        f = self.flats[self.i]
        assert f.shape == t.shape and f.dtype == t.dtype
        t.copy_(f)
        self.i += 1


def _run(eng, dev):
    from fo.speak import speak
    from fo.speech import Framer
    rng = np.random.default_rng(5)
    pcm = (rng.standard_normal(2560 * 3) * 0.05).astype(np.float32)
    kv = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
    fr, fb = Framer("A"), eng.fbank("A")
    ec = ac = None
    pe = 0
    probs = []
    for c in range(3):
        w, first = fr.push(pcm[c * 2560:(c + 1) * 2560])
        feats = fb(w[None], [first])
        r = eng.listen([dict(identity="user", status="ipu_sl" if c == 0 else "ipu_cl", feats=feats[0], kv=kv,
                             enc_cache=ec, ada_cache=ac, pe_index=pe)])[0]
        ec, ac, pe = r["enc_cache"], r["ada_cache"], r["pe_index"]
        probs.append((r["probs"]["state_1"], r["probs"]["state_2"]))
    kv.free()
    g = torch.Generator().manual_seed(3)
    D = eng.cfg["decoder_json"][0]
    items = [((torch.randn(8, D, generator=g) * 0.5).to(dev), (torch.randn(12, D, generator=g) * 0.5).to(dev))]
    states, pcm_out = [], []
    for _, seg in speak(eng, items, top_k=1, min_tokens=45, max_tokens=45, states_out=states):
        pcm_out.append(seg.reshape(-1).float().cpu())
    return probs, list(states[0].all_ids), torch.cat(pcm_out)


def test_receive_only_replica_matches_after_broadcast(dev):
    from fo.engine import FreezeOmniEngine
    from fo.replica import broadcast_frozen, frozen_checksum
    a = FreezeOmniEngine(TINY, device=dev, max_sessions=4)
    b = FreezeOmniEngine(TINY, device=dev, max_sessions=4, receive_weights=True)
    rec = _Record()
    n_a, bytes_a = broadcast_frozen(a, rec)
    play = _Play(rec.flats)
    n_b, bytes_b = broadcast_frozen(b, play)
    assert (n_a, bytes_a) == (n_b, bytes_b) and play.i == len(rec.flats)
    assert frozen_checksum(a) == frozen_checksum(b)
    pa, ia, wa = _run(a, dev)
    pb, ib, wb = _run(b, dev)
    assert pa == pb
    assert ia == ib and len(ia) >= 45
    assert torch.equal(wa, wb)


def test_pool_devices_replicas_copy_the_first_replicas_weights(dev):
    """bin/pool.py's `devices` mode: the first replica loads, the others are receive-only and filled by
    fo.replica.copy_frozen (device-to-device; here both on cuda:0), checksum-verified, and serve the same
    results; a warm-up run on the source before the copy (graph caches filled) does not change the walk."""
    from bin.pool import pipelineObjectPool
    from fo.replica import copy_frozen, frozen_checksum
    from fo.engine import FreezeOmniEngine
    a = FreezeOmniEngine(TINY, device=dev, max_sessions=4)
    pa, ia, wa = _run(a, dev)                       # warm: decode / listen / vocoder graphs exist now
    b = FreezeOmniEngine(TINY, device=dev, max_sessions=4, receive_weights=True)
    assert copy_frozen(a, b) > 0 and frozen_checksum(a) == frozen_checksum(b)
    pb, ib, wb = _run(b, dev)
    assert (pa, ia) == (pb, ib) and torch.equal(wa, wb)
    pool = pipelineObjectPool(2, {"model_path": TINY, "llm_path": os.path.join(TINY, "llm"),
                                  "devices": [str(dev), str(dev)], "top_k": 1})
    e0, e1 = (o.pipeline_proc.model.engine for o in pool.pool)
    assert frozen_checksum(e0) == frozen_checksum(e1)
    assert _run(e0, dev)[:2] == _run(e1, dev)[:2]
    assert pool.acquire() is not pool.acquire()   # least-loaded: the two sessions land on different replicas
