"""Qwen2-7B geometry on the GPU vs the CPU oracle: hidden 3584, 28 q / 4 kv heads of 128, intermediate
18944 (one of the 28 layers, so the oracle's counter-hash weights take seconds to regenerate on the host).

The weight-stream GEMMs (k_gemm_wstream for gate/up at 9-16 rows, the software-pipelined k_gemm_wpipe
for down at 16 rows and gate/up at <= 8 rows) only run at this size, so this is their parity check at
the shapes the bench times: 8 sessions x 2 rows (a listen chunk, M = 16) and 8 x 1 (a text step,
M = 8), after ragged prefills (9..23 rows, M = 128, the many-row-tile path).

Compared: the layer's DELTA (residual stream after the layer minus its input, i.e. attention + MLP output)
against the oracle's delta at the delta's own scale -- the input x would otherwise dominate and hide an
error in either branch -- and the final-normed hidden and state-head probs.  Tolerance: fp32 activations
with bf16 weights vs the fp32 oracle.
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
    from fo import _lib, ops
    from fo.kv import BatchMeta
    from fo.llm import LLMEngine
    from fo.weights import SynthSource
    src = SynthSource(cfg["seed"], all_shapes(cfg), dev, cfg["overrides"])
    D = cfg["llm"]["hidden_size"]
    assert D == 3584 and cfg["llm"]["intermediate_size"] == 18944
    llm = LLMEngine(src, cfg["llm"], dev, kv_tokens=4096, page_size=16)
    q = nets.Qwen2(W, cfg)
    st = q.stack
    rng = np.random.default_rng(7)
    n = 8
    seqs = [llm.new_seq() for _ in range(n)]
    okv = [nets.KV(1) for _ in range(n)]
    lib = _lib.load()
    prev = lib.fo_gemm_set_pipe(3)   # the default policy (pipelined down / <= 8-row gate/up)
    try:
        # ragged prefills (9..23 rows, M = 128), then a listen chunk (2 rows each, M = 16), then a text step (M = 8)
        for rows in ([9 + 2 * i for i in range(n)], [2] * n, [1] * n):
            assert sum(rows) in (128, 16, 8)
            xs = [(rng.standard_normal((r, D)) * 0.5).astype(np.float16).astype(np.float32) for r in rows]
            x_in = np.concatenate(xs)
            x = torch.from_numpy(x_in).to(dev)
            meta = BatchMeta([(s, r, s.length, True) for s, r in zip(seqs, rows)], dev, gqa=llm.H // llm.KVH)
            llm.stack.forward(x, meta)               # the residual stream after the layer (no final norm)
            res = x.clone()
            ops.rmsnorm(x, llm.norm, llm.eps, out=x)  # = LLMEngine.forward's output
            want_res = []
            for xi, kv in zip(xs, okv):
                past = kv.length()
                c, s_ = nets.rope_cos_sin(np.arange(past, past + xi.shape[0]), q.inv_freq, round_fp16=True)
                want_res.append(st.layer(0, nets.f16(xi), c, s_, kv, causal_offset=past, first_fp16=True))
            want_res = np.concatenate(want_res)
            _close(res - torch.from_numpy(x_in).to(dev), want_res - x_in, rel=3e-3)
            want = nets.rmsnorm(want_res, W["model.norm.weight"], cfg["llm"]["rms_norm_eps"])
            _close(x, want)
            last = np.cumsum(rows) - 1
            p = llm.state_probs(x, last.tolist()).cpu().numpy()
            o = 0
            for i, r in enumerate(rows):
                s1, s2 = nets.state_probs(W, want[o:o + r])
                assert abs(p[i][1] - s1) < 2e-3 and abs(p[i][2] - s2) < 2e-3, (i, p[i], s1, s2)
                o += r
    finally:
        lib.fo_gemm_set_pipe(prev)
    for s in seqs:
        s.free()
    assert llm.pool.pages_in_use() == 0
