"""HIP path (through the C-ABI) vs the CPU oracle, tiny geometry, bit-identical synthetic weights.

Tolerances: the GPU keeps fp32 activations (bf16 hi/lo split into MFMA) against bf16 weights,
so hidden states agree with the fp32 oracle to ~1e-4 relative; token ids must match exactly.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import audio, configs, host, nets
from oracle.params import all_shapes
from oracle.weights import SynthCheckpoint

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
CFG = configs.get("tiny")


@pytest.fixture(scope="module")
def W():
    return SynthCheckpoint(CFG["seed"], all_shapes(CFG), CFG["overrides"])


@pytest.fixture(scope="module")
def src(dev):
    from fo.weights import SynthSource
    return SynthSource(CFG["seed"], all_shapes(CFG), dev, CFG["overrides"])


def close(a, b, rtol=2e-3, atol=2e-4):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def test_synth_weights_bit_identical(src, W):
    for name in ["model.layers.0.self_attn.q_proj.weight", "encoder_user.global_cmvn.mean", "tts.out_fnn.weight",
                 "codec.generator.ups.1.weight", "adpter_user.bn2.running_var"]:
        g = src.get(name).cpu().numpy()
        assert np.array_equal(g, W[name]), name


@pytest.mark.parametrize("kind", ["A", "B"])
def test_fbank_gpu_matches_oracle(dev, kind):
    from fo.speech import FbankGPU, Framer
    g = np.load(os.path.join(G, "fbank.npz"))
    pcm = g[f"{kind}_pcm"]
    fr = Framer(kind)
    fb = FbankGPU(kind, dev)
    ref = audio.EncoderFraming() if kind == "A" else audio.framing_b()
    for i in range(len(pcm) // fr.chunk):
        chunk = pcm[i * fr.chunk:(i + 1) * fr.chunk]
        win, first = fr.push(chunk)
        out = fb(win[None], [first])[0]
        close(out, ref.process(chunk)[0], rtol=1e-4, atol=2e-3)
        close(out, g[f"{kind}_feats"][i], rtol=1e-4, atol=2e-3)


def test_encoder_adapter_stream_matches_oracle(dev, src, W):
    from fo.speech import AdapterEngine, SpeechEncoderEngine
    feats = np.load(os.path.join(G, "audiollm_tiny.npz"))["feats"]
    enc = SpeechEncoderEngine(src, CFG, "user", dev, max_sessions=4)
    ada = AdapterEngine(src, CFG, "user", dev, max_sessions=4)
    oe, oa = nets.Encoder(W, CFG, "user"), nets.Adapter(W, CFG, "user")
    # two interleaved users, different start positions (exercises batching, ring wrap, pe offsets)
    caches = [enc.new_cache(), enc.new_cache()]
    acs = [ada.new_cache(), ada.new_cache()]
    pes = [0, 4980]
    ost = [nets.new_encoder_state(oe.nb), nets.new_encoder_state(oe.nb)]
    ost[1]["pe"] = 4980
    oac = [None, None]
    for step in range(8):
        x = torch.from_numpy(np.stack([feats[step], feats[(step + 5) % 13]])).to(dev)
        out, T, pes = enc.infer(x, caches, pes)
        emb, To = ada(out, T, acs)
        for u in range(2):
            e = oe.infer(feats[step] if u == 0 else feats[(step + 5) % 13], ost[u])
            a, oac[u] = oa(e, oac[u])
            close(out[u * T:(u + 1) * T], e)
            close(emb[u * To:(u + 1) * To], a, atol=5e-4)
            assert pes[u] == ost[u]["pe"]


def test_llm_streaming_state_probs_match_golden(dev, src, W):
    """Replays the reference's AudioLLM golden (system role, user/system chunks) on the GPU engines."""
    from fo.llm import LLMEngine
    meta = json.load(open(os.path.join(G, "audiollm_tiny.json")))
    g = np.load(os.path.join(G, "audiollm_tiny.npz"))
    llm = LLMEngine(src, CFG["llm"], dev, kv_tokens=1024, page_size=16)
    seq = llm.new_seq()
    x = llm.embed(meta["role_ids"], round_fp16=True)
    h, _ = llm.forward(x, [(seq, x.shape[0])])
    close(h, g["pre_hidden"][0], atol=5e-4)
    for si, step in enumerate(meta["steps"]):
        emb = torch.from_numpy(g[f"s{si}_embeds"]).to(dev)  # adapter output (+prefix) from the reference
        x = emb.half().float()
        h, bm = llm.forward(x, [(seq, x.shape[0])])
        close(h, g[f"s{si}_hidden"], atol=1e-3)
        assert seq.length == step["kv_len"]
        if step["probs"] is not None:
            p = llm.state_probs(h, [x.shape[0] - 1]).cpu().numpy()[0]
            assert abs(p[1] - step["probs"]["state_1"]) < 2e-4
            assert abs(p[2] - step["probs"]["state_2"]) < 2e-4


def test_llm_batched_sequences_independent(dev, src, W):
    """Two sessions forked from one system prompt (COW pages) match the oracle run separately."""
    from fo.llm import LLMEngine
    meta = json.load(open(os.path.join(G, "audiollm_tiny.json")))
    llm = LLMEngine(src, CFG["llm"], dev, kv_tokens=2048, page_size=16)
    base = llm.new_seq()
    x = llm.embed(meta["role_ids"], round_fp16=True)
    llm.forward(x, [(base, x.shape[0])])
    a, b = base.fork(), base.fork()
    q = nets.Qwen2(W, CFG)
    okv = nets.KV(CFG["llm"]["num_hidden_layers"])
    q.forward(q.embed(meta["role_ids"]), okv)
    okv_a, okv_b = okv.copy(), okv.copy()
    rng = np.random.default_rng(0)
    for it in range(3):
        ea = rng.standard_normal((2 + it, 128)).astype(np.float32)
        eb = rng.standard_normal((7, 128)).astype(np.float32)
        xx = torch.from_numpy(np.concatenate([ea, eb])).to(dev).half().float()
        h, bm = llm.forward(xx, [(a, ea.shape[0]), (b, eb.shape[0])])
        ha, hb = q.forward(ea, okv_a), q.forward(eb, okv_b)
        close(h[:ea.shape[0]], ha, atol=1e-3)
        close(h[ea.shape[0]:], hb, atol=1e-3)
    lg = llm.logits(h, [ea.shape[0] - 1, h.shape[0] - 1]).cpu().numpy()
    np.testing.assert_allclose(lg[0], q.logits(ha[-1:])[0], rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(lg[1], q.logits(hb[-1:])[0], rtol=1e-3, atol=1e-3)
    a.free()
    b.free()
    base.free()
    assert llm.pool.pages_in_use() == 0


def test_tts_greedy_ids_match_golden(dev, src, W):
    from fo.tts import TTSEngine
    t = np.load(os.path.join(G, "tts_tiny.npz"))
    eng = TTSEngine(src, CFG["decoder_json"], dev, kv_tokens=4096)
    seqs = eng.start([(torch.from_numpy(t["hidden"]).to(dev), torch.from_numpy(t["prefix"]).to(dev))])
    cur = torch.full((1,), eng.sos, dtype=torch.int32, device=dev)
    ids = []
    from fo import ops
    for i in range(150):
        lg = eng.step(seqs, cur)
        if i < 6:
            close(lg[0], t["logits"][i], atol=5e-4)
        nxt = ops.sample(lg, eng.vocab + 4, torch.empty(1, dtype=torch.int32, device=dev))
        v = int(nxt.item())
        if v == eng.eos:
            break
        ids.append(v)
        cur = nxt
    assert ids == t["ids"].tolist()
    eng.free(seqs)


def test_codec_matches_golden(dev, src, W):
    from fo.codec import CodecEngine
    g = np.load(os.path.join(G, "codec_tiny.npz"))
    eng = CodecEngine(src, CFG["codec_json"], dev)
    ids = torch.from_numpy(np.stack([g["ids"], g["ids"][::-1].copy()])).to(dev, torch.int32)
    pcm = eng(ids)
    close(pcm[0], g["pcm"], atol=5e-5)
    close(pcm[1], nets.Codec(W, CFG)(g["ids"][::-1]), atol=5e-5)


def test_vqvae_global_style_tokens_match_reference(dev, src):
    """VQVAE.__call__ embeds the global style tokens passed on each call, per row (reference vqvae.py:37-42,
    embed_gst models.py:703-715): three rows with their own tokens, one token set broadcast over two rows, and the
    configured tokens (None, as llm2TTS.run's default) unchanged.  Golden: codec_gst_tiny.npz, the reference's own
    VQVAE.forward (make_golden.py codec_gst).  Tolerance 1e-4 abs (fp32 PCM)."""
    from fo.codec import CodecEngine
    from models.decoder.ticodec.vqvae import VQVAE
    g = np.load(os.path.join(G, "codec_gst_tiny.npz"))
    eng = CodecEngine(src, CFG["codec_json"], dev)
    vq = VQVAE(eng)
    ids = torch.from_numpy(g["ids"]).unsqueeze(-1)
    pcm = vq(ids, torch.from_numpy(g["gst"]))
    assert pcm.shape == (3, 1, g["pcm"].shape[1])
    close(pcm[:, 0], g["pcm"], atol=1e-4)
    close(vq(ids[:2], torch.from_numpy(g["gst_b"]))[:, 0], g["pcm_b"], atol=1e-4)
    # row 0 holds the configured tokens: the default path (no tokens) reproduces it, after a custom call on the
    # same cached (B, T) buffers
    close(vq(ids[:1], None)[0, 0], g["pcm"][0], atol=1e-4)
    close(vq(ids, torch.from_numpy(g["gst"]))[:, 0], g["pcm"], atol=1e-4)
    with pytest.raises(IndexError):
        vq(ids, torch.full((3, 1, g["gst"].shape[-1]), 10 ** 6))


def test_silence_cut_kernel_matches_golden(dev):
    from fo import ops
    g = np.load(os.path.join(G, "silence_cut.npz"))
    for ci in range(4):
        syn = g[f"c{ci}_syn"]
        res = ops.silence_cut(torch.from_numpy(syn).to(dev), 2401, torch.empty(2, device=dev)).cpu().numpy()
        b2, s2 = host.find_min_sum_index(g[f"c{ci}_buf"], syn, 2401, 0.01)
        assert (res[0] / 2401 < 0.01) == (s2 is not None)
        if s2 is not None:
            assert int(res[1]) == len(s2) - len(g[f"c{ci}_buf"])


def test_silence_cut_rows_match_single_rows_and_oracle(dev):
    """fo_silence_cut_rows (one launch for a vocoder call's rows, each staged in LDS when it fits) gives each row
    the single-row search's (min sum, cut) exactly; a row too long to stage (48,000 samples) takes the global-
    memory path and still matches the oracle's find_min_sum_index."""
    from fo import ops
    g = np.load(os.path.join(G, "silence_cut.npz"))
    syns = [g[f"c{ci}_syn"] for ci in range(4)]
    L = min(len(x) for x in syns)
    rng = np.random.default_rng(3)
    rows = np.stack([x[:L] for x in syns] + [rng.standard_normal(L).astype(np.float32) * 0.1 for _ in range(3)])
    buf = torch.zeros(rows.shape[0], L + 37, device=dev)   # row stride != L
    buf[:, :L] = torch.from_numpy(rows).to(dev)
    res = torch.empty(rows.shape[0], 2, device=dev)
    ops.silence_cut_rows(buf[:, :L], 2401, res)
    for r in range(rows.shape[0]):
        one = ops.silence_cut(buf[r, :L].contiguous(), 2401, torch.empty(2, device=dev))
        assert torch.equal(res[r], one), r
    long = (rng.standard_normal(48000) * 0.05).astype(np.float32)
    long[30000:33000] *= 1e-3   # a quiet stretch for the window search to find
    res = ops.silence_cut(torch.from_numpy(long).to(dev), 2401, torch.empty(2, device=dev)).cpu().numpy()
    b2, s2 = host.find_min_sum_index(np.zeros(0, np.float32), long, 2401, 0.01)
    assert (res[0] / 2401 < 0.01) == (s2 is not None)
    if s2 is not None:
        assert int(res[1]) == len(s2)


def test_sampler_topk_topp(dev):
    from fo import ops
    V = 1000
    lg = torch.randn(4, V, device=dev)
    ids = ops.sample(lg, V, torch.empty(4, dtype=torch.int32, device=dev)).cpu()
    assert torch.equal(ids.long(), lg.argmax(-1).cpu())
    k = torch.tensor([5, 5, 1, 64], dtype=torch.int32, device=dev)
    T = torch.tensor([0.7, 1.0, 1.0, 1.0], device=dev)
    p = torch.tensor([0.8, 0.0, 0.0, 0.9], device=dev)
    for step in range(20):
        st = torch.full((4,), step, dtype=torch.int32, device=dev)
        ids = ops.sample(lg, V, torch.empty(4, dtype=torch.int32, device=dev), k, T, p, seed=1, step=st).cpu()
        for r in range(4):
            topk = lg[r].topk(int(k[r])).indices.cpu()
            assert int(ids[r]) in topk.tolist()
        assert int(ids[2]) == int(lg[2].argmax())


@pytest.fixture(scope="module")
def speech_engine(dev, src):
    from types import SimpleNamespace
    from fo.codec import CodecEngine
    from fo.tts import TTSEngine
    return SimpleNamespace(device=dev, tts=TTSEngine(src, CFG["decoder_json"], dev, kv_tokens=16384),
                           codec=CodecEngine(src, CFG["codec_json"], dev))


def _speak_all(eng, items, graph, **kw):
    from fo.speak import speak
    states = []
    segs = [(i, s.cpu().numpy()) for i, s in speak(eng, items, states_out=states, graph=graph, **kw)]
    return [s.all_ids for s in states], segs


def _items(dev, n, seed):
    g = torch.Generator().manual_seed(seed)
    t = np.load(os.path.join(G, "tts_tiny.npz"))
    out = []
    for u in range(n):
        h = torch.from_numpy(t["hidden"]) + 0.05 * u * torch.randn(t["hidden"].shape, generator=g)
        p = torch.from_numpy(t["prefix"])[: 24 - 4 * (u % 3)]
        out.append((h.to(dev).contiguous(), p.to(dev).contiguous()))
    return out


@pytest.mark.parametrize("top_k,min_tokens", [(1, 0), (4, 0), (1, 60)])
def test_speak_graph_matches_eager(dev, speech_engine, top_k, min_tokens):
    """The captured decode graph with lazy id readback gives the eager loop's ids and PCM exactly."""
    items = _items(dev, 3, 5)
    kw = dict(top_k=top_k, max_tokens=130, min_tokens=min_tokens, seed=3)
    ids_e, segs_e = _speak_all(speech_engine, items, False, **kw)
    ids_g, segs_g = _speak_all(speech_engine, items, True, **kw)
    assert ids_g == ids_e
    assert [i for i, _ in segs_g] == [i for i, _ in segs_e]
    for (_, a), (_, b) in zip(segs_g, segs_e):
        np.testing.assert_array_equal(a, b)


def test_speak_graph_eos_shrinks_batch(dev, speech_engine):
    """Sessions hitting EOS at different steps: the graph path drains, shrinks the batch and still
    matches the eager loop token for token."""
    tts = speech_engine.tts
    saved = tts.out_fnn.bias.clone()
    try:
        tts.out_fnn.bias[tts.eos] += 3.0  # make EOS likely among the top-8 candidates
        items = _items(dev, 4, 9)
        kw = dict(top_k=8, max_tokens=200, seed=11)
        ids_e, segs_e = _speak_all(speech_engine, items, False, **kw)
        ids_g, segs_g = _speak_all(speech_engine, items, True, **kw)
    finally:
        tts.out_fnn.bias.copy_(saved)
    lens = [len(x) for x in ids_e]
    assert len(set(lens)) > 1 and min(lens) < 200   # sessions really ended at different steps
    assert ids_g == ids_e
    for (_, a), (_, b) in zip(segs_g, segs_e):
        np.testing.assert_array_equal(a, b)


def test_codec_mfma_matches_direct_at_real_geometry(dev):
    """Channel-last MFMA vocoder (polyphase ConvTranspose, implicit-GEMM convs) vs the channel-major
    direct-convolution kernels, at the real TiCodec geometry (512 -> 16 channels, x600 upsampling)."""
    from fo.codec import CodecEngine
    from fo.weights import SynthSource
    cfg = configs.get("real")
    shapes = {k: v for k, v in all_shapes(cfg).items() if k.startswith("codec.")}
    src = SynthSource(cfg["seed"], shapes, dev, cfg["overrides"])
    eng = CodecEngine(src, cfg["codec_json"], dev)
    rng = np.random.default_rng(5)
    ids = torch.from_numpy(rng.integers(0, 1024, size=(3, 50))).to(dev, torch.int32)
    a = eng(ids)
    b = eng.forward_ncl(ids).view(3, -1)
    assert a.shape == b.shape and a.shape[1] >= 50 * 600  # odd (k - u) stages add a few samples, as upstream
    close(a, b.cpu().numpy(), rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("name,window,penalty", [("w20_p1.5", 20, 1.5), ("w3_p1.1", 3, 1.1)])
@pytest.mark.parametrize("graph", [False, True])
def test_speak_penalty_ids_match_golden(dev, speech_engine, name, window, penalty, graph):
    """fo_penalty in the eager loop and inside the captured decode graph: greedy ids equal the reference
    run with the repetition penalty on (tests/golden/tts_penalty_tiny.npz, bit-exact)."""
    t = np.load(os.path.join(G, "tts_tiny.npz"))
    p = np.load(os.path.join(G, "tts_penalty_tiny.npz"))
    items = [(torch.from_numpy(t["hidden"]).to(dev), torch.from_numpy(t["prefix"]).to(dev))]
    ids, _ = _speak_all(speech_engine, items, graph, top_k=1, max_tokens=120, penalty_window_size=window,
                        penalty=penalty)
    assert ids[0] == p["ids_" + name].tolist()


def test_speak_penalty_graph_matches_eager_on_shrink(dev, speech_engine):
    """Penalty rings survive the batch shrinking at EOS (rings rebuilt from the host history) and the
    sampler-bound switch at min_tokens (rings adopted on the device): graph == eager, token for token."""
    tts = speech_engine.tts
    saved = tts.out_fnn.bias.clone()
    try:
        tts.out_fnn.bias[tts.eos] += 3.0
        items = _items(dev, 4, 9)
        kw = dict(top_k=8, max_tokens=200, min_tokens=20, seed=11, penalty_window_size=7, penalty=1.3)
        ids_e, segs_e = _speak_all(speech_engine, items, False, **kw)
        ids_g, segs_g = _speak_all(speech_engine, items, True, **kw)
    finally:
        tts.out_fnn.bias.copy_(saved)
    lens = [len(x) for x in ids_e]
    assert len(set(lens)) > 1
    assert ids_g == ids_e
    for (_, a), (_, b) in zip(segs_g, segs_e):
        np.testing.assert_array_equal(a, b)


def test_penalty_kernel_multiplicity(dev):
    """fo_penalty divides once per window occurrence, ring slot = step % W, ids outside [0, V) ignored."""
    from fo import ops
    V, W = 50, 4
    lg = torch.full((2, V), 2.0, device=dev)
    lg[1] = -2.0
    win = torch.tensor([[7, 7, -1, -1], [3, 9, 9, 9]], dtype=torch.int32, device=dev)
    ids = torch.tensor([7, 3], dtype=torch.int32, device=dev)
    step = torch.tensor([2, 4], dtype=torch.int32, device=dev)
    ops.penalty(lg, V, ids, win, step, 1.25)
    out = lg.cpu()
    assert torch.equal(win.cpu(), torch.tensor([[7, 7, 7, -1], [3, 9, 9, 9]], dtype=torch.int32))
    assert float(out[0, 7]) == np.float32(np.float32(np.float32(2.0) / np.float32(1.25)) / np.float32(1.25)) / np.float32(1.25)
    assert float(out[1, 9]) == np.float32(np.float32(np.float32(-2.0) / np.float32(1.25)) / np.float32(1.25)) / np.float32(1.25)
    assert float(out[1, 3]) == np.float32(-2.0) / np.float32(1.25)
    assert float(out[0, 0]) == 2.0 and float(out[1, 0]) == -2.0


@pytest.mark.parametrize("window,penalty,key", [(-1, 1.1, None), (3, 1.1, "ids_w3_p1.1")])
def test_codec_ar_facade_infer_matches_golden(dev, speech_engine, window, penalty, key):
    """models.decoder.decoder.LLM2TTSCodecAR.infer (the reference's generator form, decoder.py:314-367)
    yields the reference's greedy ids, with and without the repetition penalty."""
    from models.decoder.decoder import LLM2TTSCodecAR
    t = np.load(os.path.join(G, "tts_tiny.npz"))
    want = t["ids"][:120] if key is None else np.load(os.path.join(G, "tts_penalty_tiny.npz"))[key]
    m = LLM2TTSCodecAR(speech_engine.tts)
    h = torch.from_numpy(t["hidden"]).unsqueeze(0).to(dev)
    p = torch.from_numpy(t["prefix"]).unsqueeze(0).to(dev)
    ids = [int(x) for x in m.infer(h, 1, p, window, penalty, max_tokens=120)]
    assert ids == want.tolist()


def test_codec_graph_replay_matches_eager(dev, src):
    """The vocoder captured once per (users, tokens) and replayed on a non-default stream gives the eager
    launch sequence's PCM bit for bit, across shapes, repeated replays with new ids, and LRU eviction."""
    from fo import ops
    from fo.codec import CodecEngine
    eng = CodecEngine(src, CFG["codec_json"], dev)
    eng.MAX_GRAPHS = 2
    rng = np.random.default_rng(11)
    with torch.cuda.stream(ops.engine_stream(dev)):
        for B, T in [(1, 20), (3, 33), (1, 20), (2, 8), (3, 33)]:
            ids = torch.from_numpy(rng.integers(0, CFG["codec_json"]["n_codes"], size=(B, T))).to(dev, torch.int32)
            eng.use_graphs = True
            g = eng(ids)
            eng.use_graphs = False
            e = eng(ids)
            torch.cuda.synchronize()
            assert torch.equal(g, e), (B, T)
        assert len(eng._graphs) <= 2
    eng.destroy()


def test_speak_two_workers_side_by_side_match_sequential(dev, speech_engine):
    """Two sentences' speech decoded at the same time from two host threads on their own streams (the bench's
    --tts-workers 2: per-stream decode / vocoder graph caches, a locked KV page pool) gives, sentence by
    sentence, exactly the ids and PCM of speaking them one after the other on one stream."""
    import threading
    from fo import ops
    from fo.speak import speak
    jobs = [_items(dev, 3, 11), _items(dev, 3, 12)]
    kw = dict(top_k=4, min_tokens=50, max_tokens=50, seed=5)

    def run(items, stream=None, voc=None):
        import contextlib
        states = []
        segs = []
        for i, s in speak(speech_engine, items, states_out=states, stream=stream, voc_stream=voc, **kw):
            # the read-back goes on the worker's vocoder stream (which produced the PCM): on the legacy stream it
            # would wait on every blocking stream, including one the other worker is capturing a graph on
            # (hipErrorStreamCaptureImplicit)
            with (torch.cuda.stream(voc) if voc is not None else contextlib.nullcontext()):
                segs.append((i, s.cpu().numpy()))
        return [s.all_ids for s in states], segs

    ref = [run(j) for j in jobs]
    got, errs = [None, None], []

    def worker(w):
        try:
            torch.cuda.set_device(dev)
            sfx = "" if w == 0 else str(w)
            got[w] = run(jobs[w], ops.engine_stream(dev, name="tts" + sfx), ops.engine_stream(dev, name="voc" + sfx))
        except BaseException as e:   # noqa: BLE001 (re-raised below)
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not errs, errs
    for (ids_r, segs_r), (ids_g, segs_g) in zip(ref, got):
        assert ids_g == ids_r
        assert [i for i, _ in segs_g] == [i for i, _ in segs_r]
        for (_, a), (_, b) in zip(segs_g, segs_r):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("top_k,forced,joins,window", [(4, True, (0, 17), 8), (1, False, (0, 9), 32),
                                                        (4, True, (0, 0, 33), 8), (4, True, (0, 3, 5), 32)])
def test_speech_lane_matches_groups_spoken_alone(dev, speech_engine, top_k, forced, joins, window):
    """fo.speak.SpeechLane (the bench's --tts-lane): groups that join the continuously batched AR decode after
    different numbers of decode reads (while the rows before them still decode: the device-side carry-over of
    their ids and input rows; or into an empty lane), with different max_tokens and their prefill on a stream
    of its own, give every row exactly the ids and the PCM segments of its group spoken alone through speak()
    -- each row keeps its own RNG stream (key, own step)."""
    from fo import ops
    from fo.speak import SpeechLane
    jobs = [(_items(dev, 3, 21 + g), 40 + 7 * g) for g in range(len(joins))]

    def alone(items, n):
        kw = dict(top_k=top_k, max_tokens=n, min_tokens=n if forced else 0, seed=5)
        states = []
        segs = {}
        from fo.speak import speak
        for i, s in speak(speech_engine, items, states_out=states, **kw):
            segs.setdefault(i, []).append(s.cpu().numpy())
        return [s.all_ids for s in states], segs

    ref = [alone(items, n) for items, n in jobs]
    lane = SpeechLane(speech_engine, top_k=top_k, seed=5, window=window, stream=ops.engine_stream(dev, name="tts"),
                      voc_stream=ops.engine_stream(dev, name="voc"), prefill_stream=ops.engine_stream(dev, name="tts1"))
    segs = {}
    added, reads = 0, 0
    while added < len(jobs) or not lane.idle:
        while added < len(jobs) and reads >= joins[added]:
            items, n = jobs[added]
            lane.add(items, n, n if forced else 0, tag=added)
            added += 1
        if lane.idle:   # nothing to decode until the next group joins
            reads = joins[added]
            continue
        for i, s in lane.pump():
            st = lane.states[i]
            segs.setdefault((st.tag, st.key), []).append(s.cpu().numpy())
        reads += 1
        assert reads < 10000
    assert sorted(lane.done_groups) == list(range(len(jobs)))
    for g, (ids_r, segs_r) in enumerate(ref):
        got = [s.all_ids for s in lane.states if s.tag == g]
        assert got == ids_r, g
        for b in range(len(ids_r)):
            a, r = segs.get((g, b), []), segs_r.get(b, [])
            assert len(a) == len(r), (g, b)
            for x, y in zip(a, r):
                np.testing.assert_array_equal(x, y)
    lane.free()
