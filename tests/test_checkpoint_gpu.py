"""An engine built from the reference's checkpoint files (fo.checkpoint; tests/refdir.py writes the
tiny configuration's weights in those formats) runs the same path as the synthetic-weight engine:
identical state probabilities and greedy codec ids, codec PCM within the weight-norm fold's rounding."""
import os

import numpy as np
import pytest
import torch

from refdir import ROOT, make_reference_dir

pytestmark = pytest.mark.gpu


def _run(eng, dev, pcm):
    from fo.speech import Framer
    from fo import ops
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
    rng = np.random.default_rng(3)
    hid = torch.from_numpy(rng.standard_normal((8, 128)).astype(np.float32) * 0.5).to(dev)
    pre = torch.from_numpy(rng.standard_normal((12, 128)).astype(np.float32) * 0.5).to(dev)
    seqs = eng.tts.start([(hid, pre)])
    cur = torch.full((1,), eng.tts.sos, dtype=torch.int32, device=dev)
    ids = []
    for _ in range(20):
        cur = ops.sample(eng.tts.step(seqs, cur), eng.tts.vocab + 4, torch.empty(1, dtype=torch.int32, device=dev))
        ids.append(int(cur.item()))
    eng.tts.free(seqs)
    codes = torch.tensor([[i % eng.cfg["codec_json"]["n_codes"] for i in ids]], dtype=torch.int32, device=dev)
    return probs, ids, eng.codec(codes)[0].cpu().numpy()


def test_reference_checkpoint_engine_matches_synthetic(dev, tmp_path):
    from fo.engine import FreezeOmniEngine
    d = str(tmp_path / "model")
    make_reference_dir(d)
    pcm = (np.random.default_rng(0).standard_normal(2560 * 3) * 0.05).astype(np.float32)
    a = _run(FreezeOmniEngine(os.path.join(ROOT, "configs", "tiny"), device=dev, max_sessions=4), dev, pcm)
    b = _run(FreezeOmniEngine(d, device=dev, max_sessions=4), dev, pcm)
    assert a[0] == b[0]
    assert a[1] == b[1]
    np.testing.assert_allclose(b[2], a[2], rtol=1e-4, atol=5e-5)
