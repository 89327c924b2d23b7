"""HIP path vs reference-generated goldens that round 2 added (tests/golden/make_golden.py):

* framing B (the duplex path of config 5): AudioLLM.recognize on [1, 32, 80] features -- 7 encoder
  frames, the odd-length adapter step, chat prefixes on both identities (audiollm_b_tiny.*);
* the Qwen2 lm_head logits and the reconstructed text decode (assistant prefix + greedy tokens) run
  through the reference's own pieces (llm_text_tiny.npz);
* the sampler's distribution: the `probs` AudioLLM._post_decode hands to torch.multinomial for
  temperature / top_k (0, k > 64) / top_p settings (sampler_tiny.npz);
* real geometry (T2): speech encoder blocks at d=1024 + the 1024 -> 3584 adapter (framings A and B),
  the 4-layer 896-wide AR decoder (eager step and captured graph) and one 60-token vocoder call at 512
  channels (real_*_t2.npz).

Tolerances are written per test: logits 1e-3 (north_star), codec ids exact at top_k = 1.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import configs
from oracle.params import adapter_shapes, codec_shapes, encoder_shapes, tts_shapes

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "configs", "tiny")
CFG = configs.get("tiny")


def load(n):
    return np.load(os.path.join(G, n))


def close(a, b, rtol=2e-3, atol=2e-4):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


@pytest.fixture(scope="module")
def pipe(dev):
    from models.pipeline import inferencePipeline
    return inferencePipeline({"model_path": TINY, "llm_path": os.path.join(TINY, "llm"), "device": "cuda:0",
                              "top_k": 1})


# ------------------------------------------------------------------ framing B
def test_framing_b_speech_dialogue_matches_reference(pipe):
    """bin/dialog_state_pred.py:777-844's call (fork form) on the reference's framing-B features:
    state probs (2e-4), pe_index, KV length and the last hidden row of every chunk."""
    meta = json.load(open(os.path.join(G, "audiollm_b_tiny.json")))
    g = load("audiollm_b_tiny.npz")
    role = meta["role_prompt"][len("<|im_start|>system\n"):]
    _, pkv, _, _, _ = pipe.speech_dialogue(None, identity="", status="pre", role=role)
    caches = {i: {"adapter_cache": None, "encoder_cache": None, "pe_index": 0} for i in ("user", "system")}
    for si, step in enumerate(meta["steps"]):
        feats = torch.from_numpy(g["feats"][si]).unsqueeze(0)
        c = caches[step["identity"]]
        probs, pkv, ac, ec, pe = pipe.speech_dialogue(feats, identity=step["identity"], status=step["status"],
                                                      past_key_values=pkv, **c)
        caches[step["identity"]] = {"adapter_cache": ac, "encoder_cache": ec, "pe_index": pe}
        assert pe == step["pe_index"] and pkv.get_seq_length() == step["kv_len"], (si, pe, pkv.get_seq_length())
        h, row = pipe.model._last_hidden
        close(h[row], g[f"s{si}_hidden"][-1], atol=1e-3)
        if step["probs"] is None:
            assert probs is None
        else:
            assert abs(probs["state_1"] - step["probs"]["state_1"]) < 2e-4, (si, probs, step["probs"])
            assert abs(probs["state_2"] - step["probs"]["state_2"]) < 2e-4, (si, probs, step["probs"])


def test_framing_b_encoder_adapter_match_reference(dev):
    """Engine level: 7 encoder frames and 4 adapter rows per [32, 80] chunk, both identities interleaved
    as in the golden script (encoder output 2e-4, adapter rows = the LLM input embeds after the prefix)."""
    from fo.speech import AdapterEngine, SpeechEncoderEngine
    from fo.weights import SynthSource
    from oracle.params import all_shapes
    meta = json.load(open(os.path.join(G, "audiollm_b_tiny.json")))
    g = load("audiollm_b_tiny.npz")
    src = SynthSource(CFG["seed"], all_shapes(CFG), dev, CFG["overrides"])
    st = {}
    for ident in ("user", "system"):
        e, a = SpeechEncoderEngine(src, CFG, ident, dev, 2), AdapterEngine(src, CFG, ident, dev, 2)
        st[ident] = [e, a, e.new_cache(), a.new_cache(), 0]
    for si, step in enumerate(meta["steps"]):
        enc, ada, ec, ac, pe = st[step["identity"]]
        out, T, pes = enc.infer(torch.from_numpy(g["feats"][si][None]).to(dev), [ec], [pe])
        assert T == 7 and pes[0] == step["pe_index"]
        st[step["identity"]][4] = pes[0]
        close(out, g[f"s{si}_enc"])
        emb, To = ada(out, T, [ac])
        assert To == 4
        close(emb, g[f"s{si}_embeds"][-To:], atol=2e-3)


# ------------------------------------------------------------------ logits + text decode
def test_lm_head_logits_and_greedy_text_match_reference(pipe):
    """lm_head on the reference's hidden rows (1e-3), then the reconstructed dialog_ss / dialog_cs decode
    from the end of the golden session: assistant-prefix prefill (eager) and one-token steps (captured
    TextGraph) -- greedy ids exact, hidden and logits within 1e-3 of the reference pieces."""
    eng = pipe.model.engine
    dev = eng.device
    g = load("audiollm_tiny.npz")
    t = load("llm_text_tiny.npz")
    meta = json.load(open(os.path.join(G, "audiollm_tiny.json")))
    llm = eng.llm
    for si in range(len(meta["steps"])):
        h = torch.from_numpy(g[f"s{si}_hidden"]).to(dev)
        close(llm.lm_head(h), t[f"s{si}_logits"], rtol=1e-3, atol=1e-3)
    seq = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
    for si in range(len(meta["steps"])):
        x = torch.from_numpy(g[f"s{si}_embeds"]).to(dev).half().float()
        llm.forward(x, [(seq, x.shape[0])])
    assert seq.length == meta["steps"][-1]["kv_len"]
    ids = list(eng.prefix_ids["system"])
    for step, want in enumerate(t["text_ids"].tolist()):
        got, hid = eng.text_step([(seq, ids)], top_k=1)
        close(hid[0], t["text_hidden"][step], atol=1e-3)
        close(llm.lm_head(hid[:1]), t["text_logits"][step][None], rtol=1e-3, atol=1e-3)
        assert got[0] == want, (step, got, want)
        ids = [got[0]]
    assert seq.length == int(t["kv_len_after"])
    seq.free()


# ------------------------------------------------------------------ sampler distribution
@pytest.mark.parametrize("block", ["rows_384", "rows_4096"])
def test_sampler_probs_match_reference(dev, block):
    """fo_sample_probs writes the distribution it draws from; it must equal the reference's
    pre-multinomial probs for every setting (kept set exact, values 1e-6 abs / 1e-4 rel), covering
    top_k = 0 (full vocabulary), k > 64, top_p with and without the first-entry shift."""
    from fo import ops
    s = load("sampler_tiny.npz")
    rows = s[block]
    first = 0 if block == "rows_384" else 3
    B, V = rows.shape
    lg = torch.from_numpy(rows).to(dev)
    for si, (T, k, p) in enumerate(s["settings"]):
        probs = torch.empty(B, V, dtype=torch.float32, device=dev)
        ids = torch.empty(B, dtype=torch.int32, device=dev)
        ops.sample_probs(lg, V, ids, probs, torch.full((B,), int(k), dtype=torch.int32, device=dev),
                         torch.full((B,), float(T), device=dev), torch.full((B,), float(p), device=dev), seed=5,
                         step=torch.arange(B, dtype=torch.int32, device=dev))
        got = probs.cpu().numpy()
        want = s["probs"][first:first + B, si, :V]
        np.testing.assert_array_equal(got > 0, want > 0, err_msg=f"setting {si}: {(T, k, p)}")
        np.testing.assert_allclose(got, want, atol=1e-6, rtol=1e-4, err_msg=f"setting {si}: {(T, k, p)}")
        drawn = ids.cpu().numpy()
        assert all(want[b, drawn[b]] > 0 for b in range(B)), (si, drawn)


@pytest.mark.parametrize("k,p", [(0, 0.9), (0, 0.0), (8, 0.8), (100, 0.0)])
def test_sampler_draw_frequencies(dev, k, p):
    """Draws follow the kept-set distribution: 6000 independent streams of one row; grouped frequencies
    within 5 standard deviations of the kernel's (reference-pinned) distribution."""
    from fo import ops
    s = load("sampler_tiny.npz")
    row = torch.from_numpy(s["rows_4096"][1] * 2.0).to(dev)
    N, V = 6000, row.numel()
    lg = row.view(1, V).expand(N, V)
    probs = torch.empty(1, V, dtype=torch.float32, device=dev)
    one = torch.empty(1, dtype=torch.int32, device=dev)
    kk = torch.full((N,), k, dtype=torch.int32, device=dev)
    T = torch.full((N,), 1.0, device=dev)
    pp = torch.full((N,), p, device=dev)
    ops.sample_probs(lg[:1], V, one, probs, kk, T, pp, seed=3)
    ids = ops.sample(lg, V, torch.empty(N, dtype=torch.int32, device=dev), kk, T, pp, seed=9,
                     step=torch.zeros(N, dtype=torch.int32, device=dev)).cpu().numpy()
    want = probs[0].cpu().numpy().astype(np.float64)
    assert np.all(want[ids] > 0)
    emp = np.bincount(ids, minlength=V) / N
    # group the kept tokens into 10 groups of ~equal probability mass (in index order, and in
    # probability order) and compare group frequencies: each group's count is ~Binomial(N, 0.1)
    for order in (np.arange(V), np.argsort(-want, kind="stable")):
        grp = np.minimum((np.cumsum(want[order]) * 10).astype(int), 9)
        mass = np.bincount(grp, weights=want[order], minlength=10)
        freq = np.bincount(grp, weights=emp[order], minlength=10)
        sd = np.sqrt(np.maximum(mass * (1 - mass), 1e-12) / N)
        assert np.all(np.abs(freq - mass) < 5 * sd + 1e-9), (freq, mass)


def test_post_decode_facade_top_k_zero_is_full_vocabulary(pipe):
    """AudioLLM._post_decode(top_k=0) samples the whole vocabulary (models/audioLLM.py:439-440,456), not
    the argmax: over 64 streams the draws are not all the argmax."""
    m = pipe.model
    s = load("sampler_tiny.npz")
    lg = torch.from_numpy(s["rows_4096"][1]).view(1, 1, -1)
    draws = {int(m._post_decode(lg, temperature=1.0, top_k=0, top_p=0.0, seed=i)) for i in range(64)}
    assert len(draws) > 8
    assert int(m._post_decode(lg, temperature=1.0, top_k=1, top_p=0.0)) == int(lg.argmax())


# ------------------------------------------------------------------ real geometry (T2)
T2 = configs.get("real")
T2["train_yaml"]["encoder_conf"]["para_conf"]["transformer"]["transformer-num-blocks"] = 2


def _t2_source(dev, shapes):
    from fo.weights import SynthSource
    return SynthSource(T2["seed"], shapes, dev, T2["overrides"])


def test_real_geometry_encoder_adapter_match_reference(dev):
    """2 encoder blocks at d=1024 / 16 heads / ff 4096 / left 16 and the 1024 -> 3584 adapter: framing A
    for 20 chunks (the 64-frame ring fills and trims) and framing B for 8 chunks across the RelPE wrap,
    both sessions in one batch per framing step.  Tolerance relative to each output's scale."""
    from fo.speech import AdapterEngine, SpeechEncoderEngine
    g = load("real_encoder_t2.npz")
    src = _t2_source(dev, {**encoder_shapes(T2, "user"), **adapter_shapes(T2, "user")})
    enc = SpeechEncoderEngine(src, T2, "user", dev, max_sessions=4)
    ada = AdapterEngine(src, T2, "user", dev, max_sessions=4)
    for kind in ("A", "B"):
        ec, ac, pe = enc.new_cache(), ada.new_cache(), int(g[f"{kind}_pe0"])
        for i in range(g[f"{kind}_feats"].shape[0]):
            out, T, pes = enc.infer(torch.from_numpy(g[f"{kind}_feats"][i][None]).to(dev), [ec], [pe])
            pe = pes[0]
            assert pe == int(g[f"{kind}_pe"][i])
            ref = g[f"{kind}_enc"][i]
            close(out, ref, rtol=2e-3, atol=2e-3 * float(np.abs(ref).max()))
            emb, To = ada(out, T, [ac])
            ref = g[f"{kind}_ada"][i]
            close(emb, ref, rtol=2e-3, atol=2e-3 * float(np.abs(ref).max()))


@pytest.mark.parametrize("C,one_launch", [(4, True), (3, True), (4, False)])
def test_real_geometry_encoder_chunk_groups_match_reference(dev, C, one_launch, monkeypatch):
    """SpeechEncoderEngine.run(chunks=C) (the offline listen's encoder stage, fo.engine.ListenGroupGraph): C
    consecutive chunks of 2 sessions in one pass -- the front end, norms and GEMMs over all C x B x T rows, the rel-pos
    attention chunk by chunk on the ring -- against the reference's chunk-by-chunk outputs: framing A for 20 chunks
    (the 64-frame ring fills and trims inside a group), framing B for 8 chunks across the RelPE wrap (a partial last
    group); then the adapter chunk by chunk on the group's rows.  one_launch: the group's attention as one
    fo_relpos_attention_chunks launch per layer (default), else one fo_relpos_attention_fused launch per chunk."""
    import fo.speech
    from fo.speech import AdapterEngine, SpeechEncoderEngine
    monkeypatch.setattr(fo.speech, "CHUNK_ATTN", one_launch)
    g = load("real_encoder_t2.npz")
    src = _t2_source(dev, {**encoder_shapes(T2, "user"), **adapter_shapes(T2, "user")})
    enc = SpeechEncoderEngine(src, T2, "user", dev, max_sessions=8)
    ada = AdapterEngine(src, T2, "user", dev, max_sessions=8)
    B = 2
    for kind in ("A", "B"):
        feats = g[f"{kind}_feats"]
        n = feats.shape[0]
        ecs, acs, pes = [enc.new_cache() for _ in range(B)], [ada.new_cache() for _ in range(B)], [int(g[f"{kind}_pe0"])] * B
        R = feats.shape[1]
        T = enc.dims(R)[2]
        for c0 in range(0, n, C):
            m = min(C, n - c0)
            f = torch.from_numpy(np.concatenate([np.repeat(feats[c0 + j][None], B, 0) for j in range(m)])).to(dev)
            bufs = enc.buffers(m * B, R)
            metas = []
            for j in range(m):
                meta, pes = enc.host_meta(ecs, pes)
                metas.append(meta)
                enc.advance(ecs, T)
                assert pes == [int(g[f"{kind}_pe"][c0 + j])] * B
            bufs["meta"].copy_(torch.from_numpy(np.concatenate(metas)).to(dev))
            out, T2_ = enc.run(f.contiguous(), B, R, bufs, chunks=m)
            assert T2_ == T
            for j in range(m):
                ref_e, ref_a = g[f"{kind}_enc"][c0 + j], g[f"{kind}_ada"][c0 + j]
                rows = out[j * B * T:(j + 1) * B * T]
                emb, To = ada(rows, T, acs)
                for b in range(B):
                    close(rows[b * T:(b + 1) * T], ref_e, rtol=2e-3, atol=2e-3 * float(np.abs(ref_e).max()))
                    close(emb[b * To:(b + 1) * To], ref_a, rtol=2e-3, atol=2e-3 * float(np.abs(ref_a).max()))


@pytest.mark.parametrize("fused", [2, 1, 0])
def test_real_geometry_batched_framing_b_encoder_matches_reference(dev, fused):
    """The duplex tick's encoder shape at real geometry: 8 copies of real_encoder_t2's framing-B session in ONE batch
    (8 x 7 = 56 rows) for its 8 chunks across the RelPE wrap.  fused 2: the LayerNorm-on-load q|k|v GEMM
    reading the fp32 fragment-order residual stream (XPack32), then attention + linear_out + residual in one
    fo_enc_attn_out launch, the LayerNorm-on-load FFN-up GEMM at four row blocks (k_gemm_ln<*, 4, 8, *>) reading its
    row sums; fused 1: the whole attention half as one fo_enc_attn_block launch; 0: the LayerNorm-on-load q|k|v /
    FFN-up GEMMs on XPack32, the rel-pos attention writing the packed out input (the default).  All three: the packed FFN-down input, the
    subsampling output linear (19,456 x 1024) on the split-K X-stationary stream (k_gemm_xsk) -- every session's rows
    against the reference's per-session output (launch counters assert which kernels ran).  Then the same 8-session
    stage as the captured EncoderGraph the duplex tick replays, on 8 fresh sessions: bit-identical to the eager batch
    (same kernels, same order)."""
    from types import SimpleNamespace

    from fo import ops
    from fo.engine import EncoderGraph
    from fo.speech import AdapterEngine, SpeechEncoderEngine
    g = load("real_encoder_t2.npz")
    src = _t2_source(dev, {**encoder_shapes(T2, "user"), **adapter_shapes(T2, "user")})
    enc = SpeechEncoderEngine(src, T2, "user", dev, max_sessions=16)
    assert enc.block_fusable, "real geometry (d 1024, 16 heads of 64) fits fo_enc_attn_block / fo_enc_attn_out"
    enc.fused_block = fused
    ada = AdapterEngine(src, T2, "user", dev, max_sessions=16)
    B = 8
    feats = g["B_feats"]
    ecs, acs, pes = [enc.new_cache() for _ in range(B)], [ada.new_cache() for _ in range(B)], [int(g["B_pe0"])] * B
    eager = []
    for i in range(feats.shape[0]):
        f = torch.from_numpy(np.repeat(feats[i][None], B, 0)).to(dev).contiguous()
        ops.launch_counts_reset()
        out, T, pes = enc.infer(f, ecs, pes)
        emb, To = ada(out, T, acs)
        torch.cuda.synchronize()
        c = ops.launch_counts()
        assert T == 7 and To == 4 and out.shape[0] == B * T
        assert pes == [int(g["B_pe"][i])] * B
        nb = len(enc.layers)
        if fused == 2:
            assert c["enc_block"] == nb and c["gemm_ln"] == 2 * nb - 1 and c["relpos"] == 0, c
            assert c["gemm_xp32"] == nb - 1, c
        elif fused == 1:
            assert c["enc_block"] == nb and c["gemm_ln"] == nb and c["relpos"] == 0 and c["gemm_xp32"] == 0, c
        else:   # block 0's q|k|v takes the LayerNorm launch
            assert c["gemm_ln"] == 2 * nb - 1 and c["gemm_xp32"] == 2 * nb - 1, c
            assert c["relpos"] == nb and c["attn_opack"] == nb and c["enc_block"] == 0, c
        assert c["gemm_xsk"] >= 1, c
        ref_e, ref_a = g["B_enc"][i], g["B_ada"][i]
        for b in range(B):
            close(out[b * T:(b + 1) * T], ref_e, rtol=2e-3, atol=2e-3 * float(np.abs(ref_e).max()))
            close(emb[b * To:(b + 1) * To], ref_a, rtol=2e-3, atol=2e-3 * float(np.abs(ref_a).max()))
        eager.append((out.clone(), emb.clone()))
    # the captured stage (engine EncoderGraph) on fresh sessions: the same values bit for bit
    eng = SimpleNamespace(device=dev, enc={"user": enc}, ada={"user": ada})
    st = ops.engine_stream(dev)
    with torch.cuda.stream(st):
        eg = EncoderGraph(eng, "user", B, feats.shape[1], st)
        try:
            items = [{"enc_cache": enc.new_cache(), "ada_cache": ada.new_cache(), "pe_index": int(g["B_pe0"])}
                     for _ in range(B)]
            for i in range(feats.shape[0]):
                for it in items:
                    it["feats"] = torch.from_numpy(feats[i]).to(dev)
                emb, To, new_pe = eg.run(items)
                st.synchronize()
                for it, p in zip(items, new_pe):
                    it["pe_index"] = p
                assert torch.equal(emb[:B * To], eager[i][1]), f"EncoderGraph chunk {i} differs from the eager batch"
                assert torch.equal(eg.eb["x"][:B * 7], eager[i][0]), f"EncoderGraph encoder rows, chunk {i}"
        finally:
            eg.destroy()


@pytest.mark.parametrize("graph", [False, True])
def test_real_geometry_tts_ids_match_reference(dev, graph):
    """The AR speech decoder at 896 / 14 heads / 4864, 4 layers + pre_nn + prefix layers: 48 greedy
    codec ids exact against the reference, on the eager step (first logits 1e-3) and inside the
    captured decode graph the benchmark replays."""
    from types import SimpleNamespace
    from fo import ops
    from fo.codec import CodecEngine
    from fo.speak import speak
    from fo.tts import TTSEngine
    g = load("real_tts_t2.npz")
    src = _t2_source(dev, {**tts_shapes(T2), **codec_shapes(T2)})
    tts = TTSEngine(src, T2["decoder_json"], dev, kv_tokens=4096)
    items = [(torch.from_numpy(g["hidden"]).to(dev), torch.from_numpy(g["prefix"]).to(dev))]
    if not graph:
        seqs = tts.start(items)
        cur = torch.full((1,), tts.sos, dtype=torch.int32, device=dev)
        ids = []
        for i in range(48):
            lg = tts.step(seqs, cur)
            if i < 4:
                ref = g["logits"][i]
                close(lg[0, :ref.size], ref, rtol=1e-3, atol=1e-3)
            cur = ops.sample(lg, tts.vocab + 4, torch.empty(1, dtype=torch.int32, device=dev))
            ids.append(int(cur.item()))
        tts.free(seqs)
    else:
        eng = SimpleNamespace(device=dev, tts=tts, codec=CodecEngine(src, T2["codec_json"], dev))
        states = []
        for _ in speak(eng, items, top_k=1, max_tokens=48, states_out=states):
            pass
        ids = states[0].all_ids
    assert ids == g["ids"].tolist()


def test_real_geometry_vocoder_matches_reference(dev):
    """One 60-token TiCodec call at upsample_initial_channel 512 (36146 samples) on the MFMA vocoder."""
    from fo.codec import CodecEngine
    g = load("real_codec_t2.npz")
    src = _t2_source(dev, codec_shapes(T2))
    eng = CodecEngine(src, T2["codec_json"], dev)
    pcm = eng(torch.from_numpy(g["ids"][None]).to(dev, torch.int32))[0]
    assert pcm.numel() == g["pcm"].size
    close(pcm, g["pcm"], rtol=1e-3, atol=1e-4)


# ------------------------------------------------------------------ adapter branches
def test_adapter_variants_match_reference(dev):
    """CNNSubsampling's cnn_num == 2 branch (stride-1 conv + BN + ReLU first, two caches), LayerNorm(2d)
    and exact GELU (models/adapter.py:84-150) on the GPU, streamed over 4- and 7-frame chunks, against
    the reference (adapter_variants_tiny.*; 5e-4 abs)."""
    from fo.speech import AdapterEngine
    from fo.weights import SynthSource
    meta = json.load(open(os.path.join(G, "adapter_variants_tiny.json")))
    g = load("adapter_variants_tiny.npz")
    for vi, v in enumerate(meta["variants"]):
        c = configs.get("tiny")
        c["train_yaml"]["model_conf"].update(v)
        ada = AdapterEngine(SynthSource(meta["seed"], adapter_shapes(c, "user"), dev), c, "user", dev, 2)
        assert ada.cnn_num == int(g[f"v{vi}_cnn_num"])
        other = ada.new_cache()   # a second session's slot must stay independent
        ac = ada.new_cache()
        for ci in range(6):
            x = g[f"v{vi}_c{ci}_x"]
            xx = torch.from_numpy(np.concatenate([x, x[::-1].copy()])).to(dev)
            y, To = ada(xx, x.shape[0], [ac, other])
            close(y[:To], g[f"v{vi}_c{ci}_y"], atol=5e-4)


def test_load_checkpoint_binds_final_pt(pipe, tmp_path):
    """models.utils.load_checkpoint re-packs the encoder / adapter / state-head weights from a final.pt
    (upstream 'encoder.' names included) and returns final.yaml's configs: a state head of zeros with
    bias (0, 5, 0, 0) must give state_1 = e^5 / (2 + e^5) on any chunk afterwards."""
    import yaml
    from models.utils import load_checkpoint
    D = pipe.model.engine.llm.D
    sd = {"predictor_head.weight": torch.zeros(4, D), "predictor_head.bias": torch.tensor([0.0, 5.0, 0.0, 0.0]),
          "encoder.global_cmvn.mean": torch.zeros(80), "unrelated.key": torch.ones(3)}
    path = str(tmp_path / "final.pt")
    torch.save(sd, path)
    orig_src = pipe.model.engine.src
    with open(str(tmp_path / "final.yaml"), "w") as f:
        yaml.safe_dump({"note": "sidecar"}, f)
    try:
        assert load_checkpoint(pipe.model, path) == {"note": "sidecar"}
        assert torch.equal(pipe.model.engine.enc["system"].mean.cpu(), torch.zeros(80))
        g = load("audiollm_tiny.npz")
        _, pkv, _, _, _ = pipe.speech_dialogue(None, identity="", status="pre", role="hi")
        probs = pipe.speech_dialogue(torch.from_numpy(g["feats"][0]).unsqueeze(0), identity="user",
                                     status="ipu_sl", past_key_values=pkv)[0]
        want = np.exp(5.0) / (2.0 + np.exp(5.0))
        assert abs(probs["state_1"] - want) < 1e-5 and abs(probs["state_2"] - 1.0 / (2.0 + np.exp(5.0))) < 1e-5
        torch.save({"predictor_head.weight": torch.zeros(3, D)}, path)
        with pytest.raises(RuntimeError):
            load_checkpoint(pipe.model, path)
    finally:   # restore the synthetic weights for later tests of this module
        pipe.model.engine.src = orig_src
        pipe.model.engine.rebind_audiollm({})
        pipe.model.rebind()


@pytest.mark.parametrize("kind", ["tiny", "real2"])
def test_grouped_encoder_pass_equals_chunk_by_chunk(dev, kind):
    """SpeechEncoderEngine.run(chunks=m) against m one-chunk infer() calls on twin caches: full groups of 4 and a
    partial 2 of 3 sessions, from an empty ring into a trimmed one.  The grouped pass runs its GEMMs and norms over m x
    the rows (other tilings, so other fp32 summation orders) -- the rows agree to 2e-5 of the output scale, i.e. to
    fp32 rounding; a ring or metadata slip would show at the 1e-1 level."""
    from fo.speech import SpeechEncoderEngine
    from fo.weights import SynthSource
    cfg = configs.get("tiny") if kind == "tiny" else T2
    src = SynthSource(cfg["seed"], encoder_shapes(cfg, "user"), dev, cfg["overrides"])
    enc = SpeechEncoderEngine(src, cfg, "user", dev, max_sessions=8)
    B, R = 3, 19
    T = enc.dims(R)[2]
    rng = np.random.default_rng(5)
    seq, grp = [enc.new_cache() for _ in range(B)], [enc.new_cache() for _ in range(B)]
    pe_s, pe_g = [0] * B, [0] * B
    worst = 0.0
    for m in (4, 4, 2, 4):
        feats = [torch.from_numpy((rng.standard_normal((B, R, 80)) * 3).astype(np.float32)).to(dev) for _ in range(m)]
        want = []
        for j in range(m):
            out, _, pe_s = enc.infer(feats[j], seq, pe_s)
            want.append(out.clone())
        bufs = enc.buffers(m * B, R)
        metas = []
        for j in range(m):
            meta, pe_g = enc.host_meta(grp, pe_g)
            metas.append(meta)
            enc.advance(grp, T)
        bufs["meta"].copy_(torch.from_numpy(np.concatenate(metas)).to(dev))
        got, _ = enc.run(torch.cat(feats).contiguous(), B, R, bufs, chunks=m)
        torch.cuda.synchronize()
        assert pe_g == pe_s
        for j in range(m):
            g, w = got[j * B * T:(j + 1) * B * T], want[j]
            d = float((g - w).abs().max() / w.abs().max())
            worst = max(worst, d)
            assert d < 2e-5, (m, j, d)
        assert [(c.start, c.len) for c in seq] == [(c.start, c.len) for c in grp]
    print(f"[grouped encoder {kind}] worst row deviation {worst:.2e} of the output scale")
