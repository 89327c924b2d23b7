"""Qwen2-7B geometry on the GPU vs the CPU oracle: hidden 3584, 28 q / 4 kv heads of 128, intermediate
18944 (one of the 28 layers, so the oracle's counter-hash weights take seconds to regenerate on the host).

The weight-stream GEMMs (k_gemm_wstream for gate/up at 9-16 rows, the software-pipelined k_gemm_wpipe
for down at 16 rows and gate/up at <= 8 rows) only run at this size, so this is their parity check at
the shapes the bench times: 8 sessions x 2 rows (a listen chunk, M = 16) and 8 x 1 (a text step,
M = 8), after ragged prefills (M = 124, the many-row-tile path).  Tolerance: fp32 activations with
bf16 weights vs the fp32 oracle, relative to the hidden state's scale.
"""
import numpy as np
import pytest
import torch

from oracle import configs, nets
from oracle.params import all_shapes
from oracle.weights import SynthCheckpoint

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfg():
    c = configs.get("real")
    c["llm"]["num_hidden_layers"] = 1
    return c


@pytest.fixture(scope="module")
def W(cfg):
    return SynthCheckpoint(cfg["seed"], all_shapes(cfg), cfg["overrides"])


def _close(a, b, rel=2e-3):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    scale = float(np.abs(b).max())
    np.testing.assert_allclose(a, b, rtol=rel, atol=rel * scale)


def test_qwen2_layer_real_geometry_matches_oracle(dev, cfg, W):
    from fo import _lib
    from fo.llm import LLMEngine
    from fo.weights import SynthSource
    src = SynthSource(cfg["seed"], all_shapes(cfg), dev, cfg["overrides"])
    D = cfg["llm"]["hidden_size"]
    assert D == 3584 and cfg["llm"]["intermediate_size"] == 18944
    llm = LLMEngine(src, cfg["llm"], dev, kv_tokens=4096, page_size=16)
    q = nets.Qwen2(W, cfg)
    rng = np.random.default_rng(7)
    n = 8
    seqs = [llm.new_seq() for _ in range(n)]
    okv = [nets.KV(1) for _ in range(n)]
    assert _lib.load().fo_gemm_set_pipe(3) == 0   # the default policy (pipelined down / <= 8-row gate/up)
    # ragged prefills (9..23 rows), then a listen chunk (2 rows each, M = 16), then a text step (M = 8)
    for rows in ([9 + 2 * i for i in range(n)], [2] * n, [1] * n):
        xs = [(rng.standard_normal((r, D)) * 0.5).astype(np.float16).astype(np.float32) for r in rows]
        x = torch.from_numpy(np.concatenate(xs)).to(dev)
        h, _ = llm.forward(x, [(s, r) for s, r in zip(seqs, rows)])
        want = np.concatenate([q.forward(xi, kv) for xi, kv in zip(xs, okv)])
        _close(h, want)
        last = np.cumsum(rows) - 1
        p = llm.state_probs(h, last.tolist()).cpu().numpy()
        o = 0
        for i, r in enumerate(rows):
            s1, s2 = nets.state_probs(W, want[o:o + r])
            assert abs(p[i][1] - s1) < 2e-3 and abs(p[i][2] - s2) < 2e-3, (i, p[i], s1, s2)
            o += r
    for s in seqs:
        s.free()
    assert llm.pool.pages_in_use() == 0
