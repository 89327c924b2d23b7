"""The fused AR speech-decoder step (fo_tts_step: the whole decode step as one persistent kernel with
device-wide barriers) against the multi-kernel step it replaces (fo/stack.py + fo_sample_embed), on the
same sessions, weights and RNG streams: logits every step within fp32-accumulation tolerance (the two
paths sum the bf16 hi/lo MFMA partials in different orders: 1e-4 relative to the row's scale), drawn
ids equal (40 steps: the KV caches the later steps attend over agree too).  The reference-golden checks
of the fused path are test_parity_r02_gpu.py::test_real_geometry_tts_ids_match_reference[True] (real geometry, 48
greedy ids) and test_engines_gpu.py's speak tests (tiny geometry, graph and eager both fused)."""
import os

import numpy as np
import pytest
import torch

from oracle import configs
from oracle.params import all_shapes

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
CFG = configs.get("tiny")


@pytest.fixture(scope="module")
def tts(dev):
    from fo.tts import TTSEngine
    from fo.weights import SynthSource
    src = SynthSource(CFG["seed"], all_shapes(CFG), dev, CFG["overrides"])
    return TTSEngine(src, CFG["decoder_json"], dev, kv_tokens=16384)


def _items(dev, n, seed):
    g = torch.Generator().manual_seed(seed)
    t = np.load(os.path.join(G, "tts_tiny.npz"))
    out = []
    for u in range(n):
        h = torch.from_numpy(t["hidden"]) + 0.05 * u * torch.randn(t["hidden"].shape, generator=g)
        p = torch.from_numpy(t["prefix"])[: 24 - 4 * (u % 3)]
        out.append((h.to(dev).contiguous(), p.to(dev).contiguous()))
    return out


def _run(tts, dev, items, fused, steps, top_k, pen=None, max_keys=4096):
    from fo import ops
    tts.fused = fused
    es = ops.engine_stream(dev)
    with torch.cuda.stream(es):
        seqs = tts.start(items)
        B = len(seqs)
        g = tts.decode_graph(B, tts.vocab + 4, top_k, 7, max_keys, steps + 1, pen, capture=False)
        assert (g.fused is not None) == fused
        g.ids.fill_(tts.sos)
        g.set_window([[tts.sos]] * B)
        g.prime()
        logits, ids = [], []
        for st in range(steps):
            ev = g.launch(seqs, list(range(B)), st, st)
            torch.cuda.synchronize()
            g.check()
            logits.append(g.logits[:B].clone())
            ids.append(g.ids[:B].clone())
        tts.free(seqs)
    tts.fused = False
    return torch.stack(logits), torch.stack(ids)


@pytest.mark.parametrize("top_k,pen", [(1, None), (4, None), (4, (16, 1.3))])
def test_fused_step_matches_multikernel(dev, tts, top_k, pen):
    items = _items(dev, 5, 3)
    lf, idf = _run(tts, dev, items, True, 40, top_k, pen)
    lm, idm = _run(tts, dev, items, False, 40, top_k, pen)
    scale = lm.abs().amax(dim=-1, keepdim=True)
    err = ((lf - lm).abs() / scale).max().item()
    assert err < 1e-4, err
    assert torch.equal(idf, idm)


def test_fused_step_full_batch_of_sixteen(dev, tts):
    """B = 16 sessions (the MFMA row tile), greedy: every row's ids equal the multi-kernel step's."""
    items = _items(dev, 16, 5)
    lf, idf = _run(tts, dev, items, True, 12, 1)
    lm, idm = _run(tts, dev, items, False, 12, 1)
    assert torch.equal(idf, idm)
    assert ((lf - lm).abs() / lm.abs().amax(dim=-1, keepdim=True)).max().item() < 1e-4


def test_fused_step_one_session_one_key_split(dev, tts):
    """B = 1 and a 1024-key bound (one attention key split, S = 1): ids and logits as the multi-kernel step."""
    items = _items(dev, 1, 7)
    lf, idf = _run(tts, dev, items, True, 30, 4, None, max_keys=1024)
    lm, idm = _run(tts, dev, items, False, 30, 4, None, max_keys=1024)
    assert torch.equal(idf, idm)
    assert ((lf - lm).abs() / lm.abs().amax(dim=-1, keepdim=True)).max().item() < 1e-4


def test_fused_step_contract_falls_back(dev, tts):
    """Steps outside the fused kernel's contract (top-k > 64 here) keep the multi-kernel body."""
    from fo import ops
    with torch.cuda.stream(ops.engine_stream(dev)):
        g = tts.decode_graph(2, tts.vocab + 4, 65, 1, 1024, 8, None, capture=False)
    assert g.fused is None
