"""Pin the CPU oracle (oracle/) against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest

from oracle import audio, configs, host, nets
from oracle.params import audiollm_shapes, codec_shapes, llm_shapes, tts_shapes
from oracle.weights import SynthCheckpoint, bf16_round, hash_uniform

G = os.path.join(os.path.dirname(__file__), "golden")
CFG = configs.get("tiny")


def load(name):
    return np.load(os.path.join(G, name))


@pytest.fixture(scope="module")
def W():
    shapes = {}
    shapes.update(audiollm_shapes(CFG))
    shapes.update(llm_shapes(CFG))
    shapes.update(tts_shapes(CFG))
    shapes.update(codec_shapes(CFG))
    return SynthCheckpoint(CFG["seed"], shapes, CFG["overrides"])


def test_param_inventory_matches_reference():
    ref = json.load(open(os.path.join(G, "param_shapes_tiny.json")))
    mine = audiollm_shapes(CFG)
    ref_al = {k: v for k, v in ref["audiollm"].items() if not k.startswith("llm_decoder.")}
    assert mine == ref_al
    ref_llm = {k[len("llm_decoder."):]: v for k, v in ref["audiollm"].items() if k.startswith("llm_decoder.")}
    assert llm_shapes(CFG) == ref_llm
    assert tts_shapes(CFG) == ref["tts"]
    assert codec_shapes(CFG) == ref["codec"]


def test_hash_weights_bf16_exact():
    w = hash_uniform(1, "x", (1000,), 0.0, 0.3)
    assert np.array_equal(bf16_round(w), w)
    assert abs(float(w.mean())) < 0.05 and 0.25 < float(np.abs(w).max()) <= 0.302


def test_fbank_framing_a_matches_golden():
    g = load("fbank.npz")
    fr = audio.EncoderFraming()
    pcm = g["A_pcm"]
    for i in range(g["A_feats"].shape[0]):
        out = fr.process(pcm[i * 2560:(i + 1) * 2560])[0]
        np.testing.assert_allclose(out, g["A_feats"][i], atol=2e-3, rtol=1e-4)


def test_fbank_framing_b_matches_golden():
    g = load("fbank.npz")
    fr = audio.framing_b()
    pcm = g["B_pcm"]
    for i in range(g["B_feats"].shape[0]):
        out = fr.process(pcm[i * 3584:(i + 1) * 3584])[0]
        np.testing.assert_allclose(out, g["B_feats"][i], atol=2e-3, rtol=1e-4)


def _run_audiollm(W):
    """Replays the golden script of tests/golden/make_golden.py:gold_audiollm through the oracle."""
    meta = json.load(open(os.path.join(G, "audiollm_tiny.json")))
    g = load("audiollm_tiny.npz")
    llm = nets.Qwen2(W, CFG)
    kv = nets.KV(CFG["llm"]["num_hidden_layers"])
    h = llm.forward(llm.embed(meta["role_ids"]), kv)
    out = {"pre_hidden": h}
    enc = {i: nets.Encoder(W, CFG, i) for i in ("user", "system")}
    ada = {i: nets.Adapter(W, CFG, i) for i in ("user", "system")}
    st = {i: {"enc": nets.new_encoder_state(enc[i].nb), "ada": None} for i in ("user", "system")}
    for si, step in enumerate(meta["steps"]):
        ident, status = step["identity"], step["status"]
        e = enc[ident].infer(g["feats"][si % len(g["feats"])], st[ident]["enc"])
        a, st[ident]["ada"] = ada[ident](e, st[ident]["ada"])
        if status == "ipu_sl":
            ids = meta["user_prefix_ids"] if ident == "user" else meta["system_prefix_ids"]
            a = np.concatenate([llm.embed(ids), a], axis=0)
        hid = llm.forward(a, kv)
        probs = nets.state_probs(W, hid) if ident == "user" else None
        out[f"s{si}"] = (e, a, hid, probs, st[ident]["enc"]["pe"], kv.length())
    return meta, g, out, kv


def test_audiollm_streaming_matches_golden(W):
    meta, g, out, kv = _run_audiollm(W)
    np.testing.assert_allclose(out["pre_hidden"], g["pre_hidden"][0], atol=2e-4, rtol=1e-3)
    for si, step in enumerate(meta["steps"]):
        e, a, hid, probs, pe, kvlen = out[f"s{si}"]
        np.testing.assert_allclose(e, g[f"s{si}_enc"], atol=2e-4, rtol=1e-3)
        np.testing.assert_allclose(a, g[f"s{si}_embeds"], atol=2e-3, rtol=2e-3)
        np.testing.assert_allclose(hid, g[f"s{si}_hidden"], atol=5e-4, rtol=2e-3)
        assert pe == step["pe_index"] and kvlen == step["kv_len"]
        if step["probs"] is None:
            assert probs is None
        else:
            assert abs(probs[0] - step["probs"]["state_1"]) < 1e-4
            assert abs(probs[1] - step["probs"]["state_2"]) < 1e-4
    for li in range(CFG["llm"]["num_hidden_layers"]):
        np.testing.assert_allclose(kv.k[li], g[f"kv{li}_k"], atol=5e-4, rtol=2e-3)
        np.testing.assert_allclose(kv.v[li], g[f"kv{li}_v"], atol=5e-4, rtol=2e-3)


def test_encoder_relpe_wraparound_matches_golden(W):
    g = load("encoder_wrap_tiny.npz")
    enc = nets.Encoder(W, CFG, "user")
    assert enc.max_len == int(g["max_len"])
    st = nets.new_encoder_state(enc.nb)
    st["pe"] = int(g["pe0"])
    for i in range(g["feats"].shape[0]):
        np.testing.assert_allclose(enc.infer(g["feats"][i], st), g["out"][i], atol=2e-4, rtol=1e-3)


def test_tts_greedy_ids_match_golden(W):
    g = load("tts_tiny.npz")
    dec = nets.TTSDecoder(W, CFG)
    ids, lgs = dec.infer_greedy(g["hidden"], g["prefix"], max_tokens=150, return_logits=6)
    assert ids == g["ids"].tolist()
    np.testing.assert_allclose(np.stack(lgs), g["logits"], atol=2e-4, rtol=1e-3)


@pytest.mark.parametrize("name,window,penalty", [("w20_p1.5", 20, 1.5), ("w3_p1.1", 3, 1.1)])
def test_tts_penalty_ids_match_golden(W, name, window, penalty):
    """Repetition penalty (decoder.py:348-351) vs the reference run with it on; w3_p1.1 diverges if the
    window is de-duplicated, so it pins the per-occurrence division."""
    g = load("tts_tiny.npz")
    p = load("tts_penalty_tiny.npz")
    dec = nets.TTSDecoder(W, CFG)
    ids = dec.infer_greedy(g["hidden"], g["prefix"], max_tokens=120, penalty_window_size=window, penalty=penalty)
    assert ids == p["ids_" + name].tolist()


def test_codec_matches_golden(W):
    g = load("codec_tiny.npz")
    pcm = nets.Codec(W, CFG)(g["ids"])
    np.testing.assert_allclose(pcm, g["pcm"], atol=2e-5, rtol=1e-3)


def test_silence_cut_matches_golden():
    g = load("silence_cut.npz")
    for ci in range(4):
        b2, s2 = host.find_min_sum_index(g[f"c{ci}_buf"], g[f"c{ci}_syn"], 2401, 0.01)
        assert (s2 is None) == bool(g[f"c{ci}_none"])
        np.testing.assert_array_equal(b2, g[f"c{ci}_outbuf"])
        if s2 is not None:
            np.testing.assert_array_equal(s2, g[f"c{ci}_out"])


def test_llm2tts_run_matches_golden(W):
    g = load("llm2tts_run_tiny.npz")
    t = load("tts_tiny.npz")
    dec = nets.TTSDecoder(W, CFG)
    ids = dec.infer_greedy(t["hidden"], t["prefix"], max_tokens=130)
    codec = nets.Codec(W, CFG)
    segs = host.run_chunking(ids, codec)
    assert len(segs) == int(g["n"])
    for i, s in enumerate(segs):
        np.testing.assert_allclose(s, g[f"seg{i}"], atol=3e-5, rtol=1e-3)


def test_codec_encoder_matches_golden():
    """VQVAE.encode (Encoder + residual/global VQ) restated in numpy vs the reference run on the same
    counter-hash weights (tests/golden/codec_encoder_tiny.*): encoder output, global features, ids."""
    import json
    from oracle.weights import SynthCheckpoint
    meta = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "codec_encoder_tiny.json")))
    g = load("codec_encoder_tiny.npz")
    enc = nets.CodecEncoder(SynthCheckpoint(meta["seed"], meta["shapes"]), meta["codec_json"])
    for b in range(g["wav"].shape[0]):
        c, gf = enc.encoder(g["wav"][b])
        np.testing.assert_allclose(c, g["enc_out"][b], atol=1e-5, rtol=1e-4)
        np.testing.assert_allclose(gf, g["global_features"][b], atol=1e-5, rtol=1e-4)
        loc, gids = enc.quantize(c, gf)
        np.testing.assert_array_equal(loc, g["local_tokens"][b])
        np.testing.assert_array_equal(gids, g["global_tokens"][b, 0])
