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


def test_codec_global_style_tokens_match_golden(W):
    """embed_gst with per-row, non-default global tokens (codec_gst_tiny.npz, make_golden.py codec_gst)."""
    g = load("codec_gst_tiny.npz")
    for b in range(3):
        np.testing.assert_allclose(nets.Codec(W, CFG)(g["ids"][b], g["gst"][b, 0]), g["pcm"][b], atol=2e-5, rtol=1e-3)
    np.testing.assert_allclose(nets.Codec(W, CFG)(g["ids"][1], g["gst_b"][0, 0]), g["pcm_b"][1], atol=2e-5, rtol=1e-3)


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


# ------------------------------------------------------------------ round 2 fixtures
def _prefix_ids(ident):
    meta = json.load(open(os.path.join(G, "audiollm_tiny.json")))
    return meta["user_prefix_ids"] if ident == "user" else meta["system_prefix_ids"]


def test_audiollm_framing_b_matches_golden(W):
    """The duplex (config 5) model path at framing B: [32, 80] features -> 7 encoder frames -> 4 adapter
    rows (odd-length conv step), 'ipu_sl' prefixes on both identities (tests/golden/audiollm_b_tiny.*)."""
    meta = json.load(open(os.path.join(G, "audiollm_b_tiny.json")))
    g = load("audiollm_b_tiny.npz")
    roles = json.load(open(os.path.join(G, "audiollm_tiny.json")))["role_ids"]
    llm = nets.Qwen2(W, CFG)
    kv = nets.KV(CFG["llm"]["num_hidden_layers"])
    llm.forward(llm.embed(roles), kv)
    enc = {i: nets.Encoder(W, CFG, i) for i in ("user", "system")}
    ada = {i: nets.Adapter(W, CFG, i) for i in ("user", "system")}
    st = {i: {"enc": nets.new_encoder_state(enc[i].nb), "ada": None} for i in ("user", "system")}
    for si, step in enumerate(meta["steps"]):
        ident = step["identity"]
        e = enc[ident].infer(g["feats"][si], st[ident]["enc"])
        assert e.shape[0] == step["enc_frames"] == 7
        np.testing.assert_allclose(e, g[f"s{si}_enc"], atol=2e-4, rtol=1e-3)
        a, st[ident]["ada"] = ada[ident](e, st[ident]["ada"])
        if step["status"] == "ipu_sl":
            a = np.concatenate([llm.embed(_prefix_ids(ident)), a], axis=0)
        assert a.shape[0] == step["llm_rows"]
        np.testing.assert_allclose(a, g[f"s{si}_embeds"], atol=2e-3, rtol=2e-3)
        hid = llm.forward(a, kv)
        np.testing.assert_allclose(hid, g[f"s{si}_hidden"], atol=5e-4, rtol=2e-3)
        assert st[ident]["enc"]["pe"] == step["pe_index"] and kv.length() == step["kv_len"]
        if step["probs"] is not None:
            s1, s2 = nets.state_probs(W, hid)
            assert abs(s1 - step["probs"]["state_1"]) < 1e-4 and abs(s2 - step["probs"]["state_2"]) < 1e-4


def test_llm_logits_and_greedy_text_match_golden(W):
    """lm_head logits on the reference's hidden rows, and the reconstructed text decode (assistant prefix
    prefill + greedy tokens) against the reference pieces run end to end (tests/golden/llm_text_tiny.npz)."""
    g = load("audiollm_tiny.npz")
    t = load("llm_text_tiny.npz")
    meta = json.load(open(os.path.join(G, "audiollm_tiny.json")))
    llm = nets.Qwen2(W, CFG)
    np.testing.assert_allclose(llm.logits(g["pre_hidden"][0]), t["pre_logits"][0], atol=1e-4, rtol=1e-4)
    for si in range(len(meta["steps"])):
        np.testing.assert_allclose(llm.logits(g[f"s{si}_hidden"]), t[f"s{si}_logits"], atol=1e-4, rtol=1e-4)
    kv = nets.KV(CFG["llm"]["num_hidden_layers"])
    llm.forward(llm.embed(meta["role_ids"]), kv)
    for si in range(len(meta["steps"])):
        llm.forward(g[f"s{si}_embeds"], kv)
    ids = meta["system_prefix_ids"]
    for step, want in enumerate(t["text_ids"].tolist()):
        h = llm.forward(llm.embed(ids), kv)[-1:]
        lg = llm.logits(h)[0]
        np.testing.assert_allclose(h[0], t["text_hidden"][step], atol=5e-4, rtol=2e-3)
        np.testing.assert_allclose(lg, t["text_logits"][step], atol=1e-3, rtol=1e-3)
        tok = int(np.argmax(host.post_decode_probs(lg, 1.0, 1, 0.0)))
        assert tok == want
        ids = [tok]
    assert kv.length() == int(t["kv_len_after"])


def test_post_decode_probs_match_golden():
    """The pre-multinomial distribution of AudioLLM._post_decode for temperature / top_k (0 = off,
    k > 64) / top_p (incl. the first-entry-exceeds-top_p shift) against the reference."""
    s = load("sampler_tiny.npz")
    rows = list(s["rows_384"]) + list(s["rows_4096"])
    for ri, lg in enumerate(rows):
        for si, (T, k, p) in enumerate(s["settings"]):
            want = s["probs"][ri, si, :lg.size]
            got = host.post_decode_probs(lg, float(T), int(k), float(p))
            np.testing.assert_array_equal(got > 0, want > 0)
            np.testing.assert_allclose(got, want, atol=1e-6, rtol=1e-4)


T2 = configs.get("real")
T2["train_yaml"]["encoder_conf"]["para_conf"]["transformer"]["transformer-num-blocks"] = 2


@pytest.fixture(scope="module")
def W2():
    shapes = {}
    shapes.update(audiollm_shapes(T2))
    shapes.update(tts_shapes(T2))
    shapes.update(codec_shapes(T2))
    return SynthCheckpoint(T2["seed"], shapes, T2["overrides"])


def test_real_geometry_encoder_adapter_match_golden(W2):
    """T2: 2 blocks at d=1024 / 16 heads / left 16 + the 1024 -> 3584 adapter, framing A past the ring trim
    and framing B across the RelPE wrap, against the reference (tests/golden/real_encoder_t2.npz)."""
    g = load("real_encoder_t2.npz")
    for kind in ("A", "B"):
        enc, ada = nets.Encoder(W2, T2, "user"), nets.Adapter(W2, T2, "user")
        st, ac = nets.new_encoder_state(enc.nb), None
        st["pe"] = int(g[f"{kind}_pe0"])
        for i in range(g[f"{kind}_feats"].shape[0]):
            e = enc.infer(g[f"{kind}_feats"][i], st)
            a, ac = ada(e, ac)
            np.testing.assert_allclose(e, g[f"{kind}_enc"][i], atol=5e-4, rtol=1e-3)
            scale = float(np.abs(g[f"{kind}_ada"][i]).max())
            np.testing.assert_allclose(a, g[f"{kind}_ada"][i], atol=1e-3 * scale, rtol=1e-3)
            assert st["pe"] == int(g[f"{kind}_pe"][i])


def test_real_geometry_tts_matches_golden(W2):
    """T2: LLM2TTSCodecAR at 896 / 14 heads / 4864 with all 4 layers + pre_nn + prefix layers, greedy ids
    exact and first logits rows, against the reference (tests/golden/real_tts_t2.npz)."""
    g = load("real_tts_t2.npz")
    dec = nets.TTSDecoder(W2, T2)
    ids, lgs = dec.infer_greedy(g["hidden"], g["prefix"], max_tokens=48, return_logits=4)
    assert ids == g["ids"].tolist()
    np.testing.assert_allclose(np.stack(lgs), g["logits"], atol=2e-4, rtol=1e-3)


def test_real_geometry_codec_matches_golden(W2):
    """T2: one 60-token vocoder call at upsample_initial_channel 512 (36146 samples) vs the reference."""
    g = load("real_codec_t2.npz")
    pcm = nets.Codec(W2, T2)(g["ids"])
    np.testing.assert_allclose(pcm, g["pcm"], atol=2e-5, rtol=1e-3)


def _variant_cfg(v):
    c = configs.get("tiny")
    c["train_yaml"]["model_conf"].update(v)
    return c


def test_adapter_variants_match_golden():
    """CNNSubsampling's cnn_num == 2 branch, LayerNorm and GELU (models/adapter.py:84-150), streamed over
    chunks of 4 and 7 frames with the cache fed back, against the reference (adapter_variants_tiny.*)."""
    from oracle.params import adapter_shapes
    meta = json.load(open(os.path.join(G, "adapter_variants_tiny.json")))
    g = load("adapter_variants_tiny.npz")
    for vi, v in enumerate(meta["variants"]):
        c = _variant_cfg(v)
        Wv = SynthCheckpoint(meta["seed"], adapter_shapes(c, "user"))
        ada = nets.Adapter(Wv, c, "user")
        assert ada.cnn_num == int(g[f"v{vi}_cnn_num"])
        cache = None
        for ci in range(6):
            y, cache = ada(g[f"v{vi}_c{ci}_x"], cache)
            np.testing.assert_allclose(y, g[f"v{vi}_c{ci}_y"], atol=1e-5, rtol=1e-4)
