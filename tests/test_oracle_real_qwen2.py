"""The numpy oracle (oracle/nets.py Qwen2) pinned at REAL Qwen2-7B geometry against the reference's own
outputs (tests/golden/real_qwen2_t2.npz, make_golden.py real_qwen2): 2 of the 28 layers at hidden 3584,
28 q / 4 kv heads of 128 (7:1 GQA), intermediate 18944, rope_theta 1e6, eight ragged sessions (prefill,
two 2-row chunks, three text steps fed the reference's greedy tokens).  Checks hidden rows, state probs
and the lm_head logits at the reference's top-32 ids and 1024 fixed indices (lm_head / embedding rows are
hashed per row: oracle.weights.synth_rows).  CPU only; tolerances 1e-4 (both sides fp32, same weights).
"""
import os

import numpy as np
import pytest

from oracle import configs, nets
from oracle.params import all_shapes
from oracle.weights import SynthCheckpoint, synth_rows

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.slow
def test_oracle_qwen2_real_geometry_matches_reference():
    g = np.load(os.path.join(G, "real_qwen2_t2.npz"))
    cfg = configs.get("real")
    cfg["llm"]["num_hidden_layers"] = 2
    shapes = all_shapes(cfg)
    W = SynthCheckpoint(cfg["seed"], shapes, cfg["overrides"])
    q = nets.Qwen2(W, cfg)
    rows0 = g["rows0"].tolist()
    B = len(rows0)
    emb_shape = shapes["model.embed_tokens.weight"]
    head_shape = shapes["lm_head.weight"]
    off = {0: 0, 1: 0, 2: 0}
    for b in range(B):
        kv = nets.KV(2)
        for s in range(6):
            if s == 0:
                x = g["emb0"][off[0]:off[0] + rows0[b]].astype(np.float32)
                off[0] += rows0[b]
            elif s < 3:
                x = g[f"emb{s}"][2 * b:2 * b + 2].astype(np.float32)
            else:
                x = synth_rows(cfg["seed"], "model.embed_tokens.weight", emb_shape, [int(g["toks"][s - 3, b])])
            h = q.forward(x, kv)
            want = g["hid0"][b:b + 1] if s == 0 else (g[f"hid{s}"][2 * b:2 * b + 2] if s < 3 else g[f"hid{s}"][b:b + 1])
            got = h[-1:] if s == 0 else h
            np.testing.assert_allclose(got, want, atol=1e-4, rtol=1e-4, err_msg=f"session {b} step {s}")
            s1, s2 = nets.state_probs(W, h)
            np.testing.assert_allclose([s1, s2], g["probs"][s, b, 1:], atol=1e-5)
            if s >= 2:
                r = 4 * b + (s - 2)
                ids = np.concatenate([g["dec_top_ids"][r], g["fixed_idx"]])
                w = synth_rows(cfg["seed"], "lm_head.weight", head_shape, ids, cfg["overrides"])
                lg = h[-1] @ w.T
                np.testing.assert_allclose(lg[:32], g["dec_top_vals"][r], atol=1e-4, rtol=1e-4)
                np.testing.assert_allclose(lg[32:], g["dec_fixed"][r], atol=1e-4, rtol=1e-4)
                assert int(g["dec_top_ids"][r][0]) == int(g["toks"][s - 2, b])
