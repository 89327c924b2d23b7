#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE implementation.

This script is the only place that imports /root/reference (TheDoctor-JI/Freeze-Omni). It runs
on CPU in the build container (the reference never travels to the GPU box); its outputs are
small .npz/.json files of inputs and expected outputs.  Weights are counter-hash synthetic
weights (oracle/weights.py), so only I/O is stored and every consumer regenerates the weights.

Harness-side shims (the reference files are untouched), SURVEY.md §8(c):
  shortuuid / logger.logger / soundfile / librosa / web.* stubs; torchaudio.compliance.kaldi.fbank
  -> transformers.audio_utils kaldi restatement (torchaudio 2.2.0 is absent: parity of the kaldi
  fbank itself is therefore pinned to transformers' documented restatement, not to torchaudio);
  Tensor.to('cuda') no-op (models/encoder/transformer.py:279); DynamicCache legacy indexing
  (models/audioLLM.py:417) and from_legacy_cache(None) (models/decoder/decoder.py:321);
  LlamaDecoderLayer 4.45 call convention (past_key_value=, tuple return) with eager attention.
The reference runs in fp32 on CPU (autocast('cuda') is inert there).

Usage:  python tests/golden/make_golden.py
"""
import copy
import functools
import json
import logging
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
from oracle import configs as C  # noqa: E402
from oracle.weights import synth_param  # noqa: E402

torch.set_grad_enabled(False)
SHAPES = {}
torch.manual_seed(0)


# ----------------------------------------------------------------------------- shims
def _mod(name, **attrs):
    import importlib.machinery
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install_shims():
    # import third-party modules before any stub module exists (their availability probes)
    import transformers  # noqa: F401
    from transformers import AutoModelForCausalLM, AutoTokenizer, Qwen2ForCausalLM  # noqa: F401
    from transformers.models.llama import modeling_llama  # noqa: F401
    from transformers.models.qwen2 import modeling_qwen2  # noqa: F401
    from transformers import audio_utils  # noqa: F401
    _mod("shortuuid", uuid=lambda: "golden")
    lg = _mod("logger")
    lg.logger = _mod("logger.logger", setup_logger=lambda name, **kw: logging.getLogger(name))
    _mod("soundfile", read=None, write=None)
    _mod("librosa", load=None)
    web = _mod("web")
    web.parms = _mod("web.parms", GlobalParams=object)
    web.pool = _mod("web.pool", TTSObjectPool=object)

    from transformers.audio_utils import mel_filter_bank, spectrogram, window_function

    def kaldi_fbank(waveform, dither=0.0, frame_length=25.0, frame_shift=10.0, num_mel_bins=23,
                    sample_frequency=16000.0, **kw):
        assert dither == 0.0 and not kw
        wl = int(sample_frequency * frame_length * 0.001)
        ws = int(sample_frequency * frame_shift * 0.001)
        nfft = 1 << (wl - 1).bit_length()
        mel = mel_filter_bank(num_frequency_bins=nfft // 2 + 1, num_mel_filters=num_mel_bins, min_frequency=20.0,
                              max_frequency=sample_frequency / 2, sampling_rate=int(sample_frequency), norm=None,
                              mel_scale="kaldi", triangularize_in_mel_space=True)
        x = waveform.squeeze(0).double().numpy()
        fb = spectrogram(x, window_function(wl, "povey", periodic=False), frame_length=wl, hop_length=ws,
                         fft_length=nfft, power=2.0, center=False, preemphasis=0.97, mel_filters=mel,
                         log_mel="log", mel_floor=1.1920928955078125e-07, remove_dc_offset=True).T
        return torch.from_numpy(np.ascontiguousarray(fb)).float()

    ta = _mod("torchaudio")
    ta.compliance = _mod("torchaudio.compliance")
    ta.compliance.kaldi = _mod("torchaudio.compliance.kaldi", fbank=kaldi_fbank)
    ta.transforms = _mod("torchaudio.transforms")

    _orig_to = torch.Tensor.to

    def _to(self, *a, **k):
        if a and isinstance(a[0], str) and a[0].startswith("cuda"):
            return self
        if isinstance(k.get("device"), str) and k["device"].startswith("cuda"):
            k = dict(k)
            k.pop("device")
            if not a and not k:
                return self
        return _orig_to(self, *a, **k)

    torch.Tensor.to = _to

    from transformers import cache_utils
    from transformers.models.llama import modeling_llama

    def _getitem(self, i):
        return (self.layers[i].keys, self.layers[i].values)

    cache_utils.DynamicCache.__getitem__ = _getitem
    cache_utils.DynamicCache.from_legacy_cache = classmethod(lambda cls, x=None: cls())

    orig_fwd = modeling_llama.LlamaDecoderLayer.forward

    def layer_fwd(self, hidden_states, attention_mask=None, position_ids=None, past_key_value=None,
                  output_attentions=False, use_cache=False, cache_position=None, position_embeddings=None, **kw):
        self.self_attn.config._attn_implementation = "eager"
        h = orig_fwd(self, hidden_states, attention_mask=attention_mask, position_ids=position_ids,
                     past_key_values=past_key_value, use_cache=use_cache, position_embeddings=position_embeddings)
        return (h, past_key_value)

    modeling_llama.LlamaDecoderLayer.forward = layer_fwd
    sys.path.insert(0, REF)


# ----------------------------------------------------------------------------- helpers
def init_module(mod, seed, prefix="", overrides=None):
    """Overwrite every parameter/buffer of `mod` with counter-hash values keyed by state_dict name."""
    sd = mod.state_dict()
    new = {}
    for k, v in sd.items():
        name = prefix + k
        if v.dtype in (torch.int64, torch.long):
            new[k] = v
            continue
        new[k] = torch.from_numpy(synth_param(seed, name, tuple(v.shape), overrides))
    mod.load_state_dict(new)


def canonical_llm_name(k):
    """AudioLLM aliases llm_decoder.transformer = .model, .model.h = .layers, .model.wte = .embed_tokens
    (models/audioLLM.py:104-109); every alias of a shared parameter gets the canonical name's values."""
    if not k.startswith("llm_decoder."):
        return k
    n = k[len("llm_decoder."):]
    if n.startswith("transformer."):
        n = "model." + n[len("transformer."):]
    n = n.replace("model.h.", "model.layers.").replace("model.wte.", "model.embed_tokens.")
    return n


def wav_question():
    from scipy.io import wavfile
    sr, x = wavfile.read(os.path.join(REF, "assets/question.wav"))
    assert sr == 16000 and x.dtype == np.int16
    return x.astype(np.float64) / 32768.0


def synth_pcm(n, seed):
    """Band-limited noise x 4 Hz syllabic AM at -20 dBFS, int16-quantised."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 16000.0
    w = rng.standard_normal(n + 64)
    w = np.convolve(w, np.hanning(33), mode="same")[:n]
    w = w / (np.abs(w).max() + 1e-9)
    am = 0.5 * (1 + np.sin(2 * np.pi * 4 * t))
    x = 0.1 * w * am
    return np.round(x * 32767) / 32768.0


def tokenizer_dir():
    """Byte-level BPE tokenizer without merges + Qwen chat specials (fixture data)."""
    d = os.path.join(HERE, "tiny_tokenizer")
    if os.path.exists(os.path.join(d, "tokenizer.json")):
        return d
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    alphabet = pre_tokenizers.ByteLevel.alphabet()
    vocab = {ch: i for i, ch in enumerate(sorted(alphabet))}
    tok = Tokenizer(models.BPE(vocab=vocab, merges=[]))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    fast = PreTrainedTokenizerFast(tokenizer_object=tok)
    fast.add_special_tokens({"additional_special_tokens": ["<|im_start|>", "<|im_end|>"],
                             "eos_token": "<|endoftext|>"})
    os.makedirs(d, exist_ok=True)
    fast.save_pretrained(d)
    return d


def tiny_llm_dir(cfg, tmp):
    from transformers import Qwen2Config, Qwen2ForCausalLM
    qc = Qwen2Config(**cfg["llm"], torch_dtype="float32")
    m = Qwen2ForCausalLM(qc)
    init_module(m, cfg["seed"], "", cfg["overrides"])
    m.save_pretrained(tmp)
    import shutil
    for f in os.listdir(tokenizer_dir()):
        shutil.copy(os.path.join(tokenizer_dir(), f), tmp)
    return tmp


# ----------------------------------------------------------------------------- goldens
def gold_fbank():
    sys.argv = ["golden"]
    import bin.inference as binf  # noqa: the reference offline driver (framing A)
    from models.AudioFeatureGating import AudioFeatureGating
    import yaml
    out = {}
    x = wav_question()
    proc = binf.audioEncoderProcessor()
    CH = proc.get_chunk_size()
    n = int(np.ceil(len(x) / CH) * CH)
    xin = np.zeros(n)
    xin[:len(x)] = x
    feats = [proc.process(torch.tensor(xin[i:i + CH])).numpy()[0] for i in range(0, n, CH)]
    out["A_pcm"] = xin.astype(np.float32)
    out["A_feats"] = np.stack(feats).astype(np.float32)   # [13, 19, 80]
    ycfg = yaml.safe_load(open(os.path.join(REF, "configs/dialog_state_pred_config.yaml")))
    g = AudioFeatureGating(16000, 10, 0, ycfg["audio_feature_gating"]["fbank"])
    CB = g.expected_frames_per_audio_chunk
    pcm = synth_pcm(CB * 6, 99)
    fb = []
    for i in range(6):
        chunk = (pcm[i * CB:(i + 1) * CB] * 32767.0 / 32767.0).astype(np.float32) / np.float32(1.0)
        fb.append(g._extract_fbank(chunk).numpy()[0].copy())
    out["B_pcm"] = pcm.astype(np.float32)
    out["B_feats"] = np.stack(fb).astype(np.float32)     # [6, 32, 80]
    # gating semantics (status None -> history only; ipu_* -> forwarded)
    g2 = AudioFeatureGating(16000, 3, 2, ycfg["audio_feature_gating"]["fbank"])
    statuses = [None, None, "ipu_sl", "ipu_cl", None, "ipu_el"]
    gate = []
    for i, st in enumerate(statuses):
        r = g2.process_and_gate({"audio": pcm[i * CB:(i + 1) * CB].astype(np.float32), "status": st})
        gate.append(None if r is None else {"status": r["status"], "feature": r["feature"],
                                            "feature_last_chunk": r["feature_last_chunk"]})
    np.savez_compressed(os.path.join(HERE, "fbank.npz"), **out)
    with open(os.path.join(HERE, "gating.json"), "w") as f:
        json.dump({"statuses": statuses, "cache_history_size": 3, "onset": 2, "gate": gate}, f)
    print("fbank: A", out["A_feats"].shape, "B", out["B_feats"].shape)
    return out


def gold_audiollm(cfg, feats_a):
    import tempfile
    sys.argv = ["golden"]
    from models.utils import init_encoder_llm
    from models.encoder.cmvn import GlobalCMVN  # noqa: F401
    tmp = tempfile.mkdtemp()
    llm_dir = tiny_llm_dir(cfg, tmp)
    ty = copy.deepcopy(cfg["train_yaml"])
    ty["cmvn_file"] = None
    ty["model_conf"]["llm_path"] = llm_dir
    model = init_encoder_llm(ty, device="cpu")
    # cmvn: construct with hashed stats (json cmvn file format is exercised by the host loader tests)
    from models.encoder.cmvn import GlobalCMVN
    d = 80
    for enc in (model.encoder_user, model.encoder_system):
        enc.global_cmvn = GlobalCMVN(torch.zeros(d), torch.ones(d))
    # every parameter from the counter hash, keyed by the reference state_dict names
    sd = model.state_dict()
    new = {}
    for k, v in sd.items():
        name = canonical_llm_name(k)
        if v.dtype == torch.long:
            new[k] = v
        else:
            new[k] = torch.from_numpy(synth_param(cfg["seed"], name, tuple(v.shape), cfg["overrides"]))
    model.load_state_dict(new)
    model.eval()
    SHAPES["audiollm"] = {("llm_decoder." + canonical_llm_name(k)) if k.startswith("llm_decoder.") else k:
                          list(v.shape) for k, v in sd.items() if v.dtype != torch.long}
    model.init_template_compilation = lambda: None
    sce, scm = model.initialize_chat_template_embeds("system")
    uce, ucm = model.initialize_chat_template_embeds("user")
    model.system_chat_prefix_embeds, model.system_chat_prefix_mask = sce, scm
    model.user_chat_prefix_embeds, model.user_chat_prefix_mask = uce, ucm

    # capture intermediate tensors
    cap = {}
    orig_core = model._llm_forward_core

    def core(inputs):
        cap["embeds"] = inputs["inputs_embeds"].float().numpy().copy()
        h, pkv = orig_core(inputs)
        cap["hidden"] = h.float().numpy().copy()
        return h, pkv

    model._llm_forward_core = core
    enc_out = {}
    for ident in ("user", "system"):
        enc = getattr(model, f"encoder_{ident}")
        orig_infer = enc.infer

        def infer(*a, _o=orig_infer, _id=ident, **k):
            r = _o(*a, **k)
            cap["enc"] = r[0].float().numpy().copy()
            return r

        enc.infer = infer
    role = "You are a helpful assistant."
    extra = {"identity": "", "status": "pre", "past_key_values": None, "adapter_cache": None,
             "encoder_cache": None, "pe_index": 0, "role_prompt": "<|im_start|>system\n" + role}
    pkv = model.set_system_role(extra)
    res = {"role_ids": model.tokenizer([extra["role_prompt"]])["input_ids"][0],
           "user_prefix_ids": [int(model.tokenizer.eod_id)] +
           model.chat_template["prefix_for_user_utterance"][0].tolist(),
           "system_prefix_ids": model.chat_template["prefix_for_system_utterance"][0].tolist(),
           "eod_id": int(model.tokenizer.eod_id), "steps": []}
    pre_hidden = cap["hidden"]
    script = [("user", "ipu_sl"), ("user", "ipu_cl"), ("user", "ipu_cl"), ("user", "ipu_cl"),
              ("system", "ipu_sl"), ("system", "ipu_cl"), ("user", "ipu_sl"), ("user", "ipu_cl"),
              ("user", "ipu_cl"), ("user", "ipu_el")]
    caches = {i: {"encoder_cache": None, "adapter_cache": None, "pe_index": 0} for i in ("user", "system")}
    arrays = {"pre_hidden": pre_hidden}
    for si, (ident, status) in enumerate(script):
        x = torch.from_numpy(feats_a[si % len(feats_a)]).unsqueeze(0)
        e = {"identity": ident, "status": status, "past_key_values": pkv, **caches[ident]}
        probs, pkv, ac, ec, pe = model.recognize(x, e)
        caches[ident] = {"encoder_cache": ec, "adapter_cache": ac, "pe_index": pe}
        res["steps"].append({"identity": ident, "status": status, "probs": probs, "pe_index": pe,
                             "kv_len": int(pkv.get_seq_length())})
        arrays[f"s{si}_enc"] = cap["enc"][0]
        arrays[f"s{si}_embeds"] = cap["embeds"][0]
        arrays[f"s{si}_hidden"] = cap["hidden"][0]
    for li in range(len(pkv.layers)):
        arrays[f"kv{li}_k"] = pkv.layers[li].keys[0].float().numpy()
        arrays[f"kv{li}_v"] = pkv.layers[li].values[0].float().numpy()
    np.savez_compressed(os.path.join(HERE, "audiollm_tiny.npz"), feats=feats_a, **arrays)
    with open(os.path.join(HERE, "audiollm_tiny.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("audiollm: steps", len(script), "kv_len", res["steps"][-1]["kv_len"])

    # encoder-only run with RelPE wrap-around (pe_index near max_len)
    enc = model.encoder_user
    buf = [None] * enc.enc[1].num_blocks
    pe = enc.enc[1].pe.max_len - 2 * enc.enc[1].chunk_size + 1
    pe0 = pe
    outs = []
    for i in range(5):
        o, buf, _, _, pe = enc.infer(torch.from_numpy(feats_a[i]).unsqueeze(0), buf, 0, None, pe)
        outs.append(o[0].numpy().copy())
    np.savez_compressed(os.path.join(HERE, "encoder_wrap_tiny.npz"), feats=feats_a[:5], out=np.stack(outs),
                        pe0=np.array(pe0), max_len=np.array(enc.enc[1].pe.max_len))


def build_audiollm(cfg):
    """The reference AudioLLM (models/utils.py:init_encoder_llm) on a tiny local Qwen2, every parameter
    from the counter hash (keyed by the canonical state_dict names), chat-prefix embeds initialised."""
    import tempfile
    sys.argv = ["golden"]
    from models.utils import init_encoder_llm
    from models.encoder.cmvn import GlobalCMVN
    llm_dir = tiny_llm_dir(cfg, tempfile.mkdtemp())
    ty = copy.deepcopy(cfg["train_yaml"])
    ty["cmvn_file"] = None
    ty["model_conf"]["llm_path"] = llm_dir
    model = init_encoder_llm(ty, device="cpu")
    for enc in (model.encoder_user, model.encoder_system):
        enc.global_cmvn = GlobalCMVN(torch.zeros(80), torch.ones(80))
    sd = model.state_dict()
    model.load_state_dict({k: v if v.dtype == torch.long else
                           torch.from_numpy(synth_param(cfg["seed"], canonical_llm_name(k), tuple(v.shape),
                                                        cfg["overrides"])) for k, v in sd.items()})
    model.eval()
    model.init_template_compilation = lambda: None
    model.system_chat_prefix_embeds, model.system_chat_prefix_mask = model.initialize_chat_template_embeds("system")
    model.user_chat_prefix_embeds, model.user_chat_prefix_mask = model.initialize_chat_template_embeds("user")
    return model


def _capture_hooks(model, cap):
    """Record the LLM input embeds / last hidden and the encoder output of every recognize call."""
    orig_core = model._llm_forward_core

    def core(inputs):
        cap["embeds"] = inputs["inputs_embeds"].float().numpy().copy()
        h, pkv = orig_core(inputs)
        cap["hidden"] = h.float().numpy().copy()
        return h, pkv

    model._llm_forward_core = core
    for ident in ("user", "system"):
        enc = getattr(model, f"encoder_{ident}")

        def infer(*a, _o=enc.infer, **k):
            r = _o(*a, **k)
            cap["enc"] = r[0].float().numpy().copy()
            return r

        enc.infer = infer


def framing_b_feats(n, seed):
    """n consecutive [32, 80] framing-B features from the reference AudioFeatureGating
    (models/AudioFeatureGating.py:54-75, configs/dialog_state_pred_config.yaml) on synthetic PCM."""
    import yaml
    from models.AudioFeatureGating import AudioFeatureGating
    ycfg = yaml.safe_load(open(os.path.join(REF, "configs/dialog_state_pred_config.yaml")))
    g = AudioFeatureGating(16000, 10, 0, ycfg["audio_feature_gating"]["fbank"])
    CB = g.expected_frames_per_audio_chunk
    pcm = synth_pcm(CB * n, seed)
    feats = [g._extract_fbank(pcm[i * CB:(i + 1) * CB].astype(np.float32)).numpy()[0].copy() for i in range(n)]
    return pcm.astype(np.float32), np.stack(feats).astype(np.float32)


def gold_audiollm_b(cfg):
    """AudioLLM.recognize on FRAMING-B features ([1, 32, 80], the duplex path of config 5:
    bin/dialog_state_pred.py:777-844 -> models/pipeline.py:36-88): 7 encoder frames per chunk, the
    odd-length adapter step, 'ipu_sl' chat prefixes on both identities, system audio prefilled without
    prediction.  Captures encoder output, LLM input embeds, hidden, probs, pe_index and kv_len."""
    model = build_audiollm(cfg)
    cap = {}
    _capture_hooks(model, cap)
    pcm, feats = framing_b_feats(10, 123)
    extra = {"identity": "", "status": "pre", "past_key_values": None, "adapter_cache": None,
             "encoder_cache": None, "pe_index": 0, "role_prompt": "<|im_start|>system\nYou are a helpful assistant."}
    pkv = model.set_system_role(extra)
    script = [("user", "ipu_sl"), ("user", "ipu_cl"), ("user", "ipu_cl"), ("system", "ipu_sl"), ("system", "ipu_cl"),
              ("user", "ipu_sl"), ("system", "ipu_cl"), ("user", "ipu_cl"), ("user", "ipu_cl"), ("user", "ipu_el")]
    caches = {i: {"encoder_cache": None, "adapter_cache": None, "pe_index": 0} for i in ("user", "system")}
    res = {"role_prompt": extra["role_prompt"], "steps": []}
    arrays = {"feats": feats, "pcm": pcm}
    for si, (ident, status) in enumerate(script):
        x = torch.from_numpy(feats[si]).unsqueeze(0)
        e = {"identity": ident, "status": status, "past_key_values": pkv, **caches[ident]}
        probs, pkv, ac, ec, pe = model.recognize(x, e)
        caches[ident] = {"encoder_cache": ec, "adapter_cache": ac, "pe_index": pe}
        res["steps"].append({"identity": ident, "status": status, "probs": probs, "pe_index": pe,
                             "kv_len": int(pkv.get_seq_length()), "enc_frames": int(cap["enc"].shape[1]),
                             "llm_rows": int(cap["embeds"].shape[1])})
        arrays[f"s{si}_enc"] = cap["enc"][0]
        arrays[f"s{si}_embeds"] = cap["embeds"][0]
        arrays[f"s{si}_hidden"] = cap["hidden"][0]
    np.savez_compressed(os.path.join(HERE, "audiollm_b_tiny.npz"), **arrays)
    with open(os.path.join(HERE, "audiollm_b_tiny.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("audiollm framing B: steps", len(script), "enc frames", res["steps"][0]["enc_frames"],
          "kv_len", res["steps"][-1]["kv_len"])


SAMPLER_SETTINGS = [  # (temperature, top_k, top_p) of AudioLLM._post_decode (models/audioLLM.py:431-477)
    (1.0, 1, 0.0), (1.0, 0, 0.0), (0.7, 0, 0.0), (1.0, 0, 0.9), (1.3, 0, 0.5), (0.6, 0, 0.3), (0.8, 5, 0.0),
    (1.0, 100, 0.0), (1.2, 100, 0.8), (1.0, 20, 0.95), (1.0, 3, 0.05), (0.9, 64, 0.7), (1.0, 65, 0.0)]


def gold_llm_text(cfg):
    """LLM logits and the text decode, assembled from reference pieces on the tiny
    AudioLLM: lm_head (Qwen2ForCausalLM.lm_head, models/audioLLM.py:70-74,104-109) on the hidden rows of
    the audiollm_tiny session; then, from the end of that session, the reconstructed dialog_ss / dialog_cs
    steps of bin/inference.py:138-179: prefill prefix_for_system_utterance (.half(), full past mask),
    lm_head on the last row, _post_decode(top_k=1), feed that token's embedding, repeat.  Plus the
    pre-multinomial `probs` of _post_decode for SAMPLER_SETTINGS on those logits and on synthetic rows."""
    from models.audioLLM import AudioLLM
    model = build_audiollm(cfg)
    g = np.load(os.path.join(HERE, "audiollm_tiny.npz"))
    meta = json.load(open(os.path.join(HERE, "audiollm_tiny.json")))
    lm_head = model.llm_decoder.lm_head
    arrays = {"pre_logits": lm_head(torch.from_numpy(g["pre_hidden"])).numpy()}
    for si in range(len(meta["steps"])):
        arrays[f"s{si}_logits"] = lm_head(torch.from_numpy(g[f"s{si}_hidden"])).numpy()
    # replay the session's context through the reference (embeds from the golden = its own inputs)
    extra = {"identity": "", "status": "pre", "past_key_values": None, "adapter_cache": None,
             "encoder_cache": None, "pe_index": 0, "role_prompt": "<|im_start|>system\nYou are a helpful assistant."}
    pkv = model.set_system_role(extra)

    def forward(embeds, pkv):
        mask = torch.full([1, pkv.get_seq_length() + embeds.shape[1]], True)
        h, pkv = model._llm_forward_core({"inputs_embeds": embeds.half(), "attention_mask": mask,
                                          "past_key_values": pkv})
        return h, pkv

    for si in range(len(meta["steps"])):
        h, pkv = forward(torch.from_numpy(g[f"s{si}_embeds"]).unsqueeze(0), pkv)
        np.testing.assert_allclose(h[0].numpy(), g[f"s{si}_hidden"], atol=1e-5)
    assert pkv.get_seq_length() == meta["steps"][-1]["kv_len"]
    wte = model.llm_decoder.transformer.wte
    ids = model.chat_template["prefix_for_system_utterance"]
    text_ids, text_logits, text_hidden = [], [], []
    for step in range(10):
        h, pkv = forward(wte(ids), pkv)
        last = h[:, -1:]
        lg = lm_head(last)
        tok = int(model._post_decode(lg, temperature=1.0, top_k=1, top_p=0.0).reshape(-1)[0])
        text_ids.append(tok)
        text_logits.append(lg[0, 0].numpy().copy())
        text_hidden.append(last[0, 0].numpy().copy())
        ids = torch.tensor([[tok]])
    arrays.update(text_ids=np.array(text_ids, np.int64), text_logits=np.stack(text_logits),
                  text_hidden=np.stack(text_hidden), kv_len_after=np.array(pkv.get_seq_length()))
    np.savez_compressed(os.path.join(HERE, "llm_text_tiny.npz"), **arrays)
    print("llm text: greedy ids", text_ids, "kv", pkv.get_seq_length())

    # _post_decode probability vectors (the distribution torch.multinomial draws from)
    rng = np.random.default_rng(17)
    rows = [arrays["text_logits"][0], arrays["text_logits"][3], arrays["s0_logits"][-1],
            (rng.standard_normal(4096) * 3.0).astype(np.float32),
            (rng.standard_normal(4096) * 0.7).astype(np.float32)]
    orig = torch.multinomial
    probs = np.zeros((len(rows), len(SAMPLER_SETTINGS), 4096), np.float32)
    toks = np.zeros((len(rows), len(SAMPLER_SETTINGS)), np.int64)
    try:
        for ri, lg in enumerate(rows):
            for si, (T, k, p) in enumerate(SAMPLER_SETTINGS):
                cap = {}

                def mn(pr, n, **kw):
                    cap["p"] = pr.detach().clone()
                    return torch.argmax(pr).view(1)

                torch.multinomial = mn
                t = AudioLLM._post_decode(None, torch.from_numpy(np.ascontiguousarray(lg)).view(1, 1, -1),
                                          temperature=T, top_k=k, top_p=p)
                probs[ri, si, :lg.size] = cap["p"].numpy()
                toks[ri, si] = int(t.reshape(-1)[0])
    finally:
        torch.multinomial = orig
    np.savez_compressed(os.path.join(HERE, "sampler_tiny.npz"), rows_384=np.stack(rows[:3]),
                        rows_4096=np.stack(rows[3:]), settings=np.array(SAMPLER_SETTINGS, np.float64),
                        probs=probs, argmax_of_probs=toks)
    print("sampler: kept counts", [[int((probs[r, s] > 0).sum()) for s in range(len(SAMPLER_SETTINGS))]
                                   for r in range(len(rows))])


def gold_real_t2(seed=7):
    """Real-geometry (T2) reference runs with counter-hash weights (configs 'real'), one component at a
    time so the CPU time stays bounded; only I/O is committed and every consumer regenerates the weights:
      * speechEncoder.infer (models/encoder/encoder.py:149-155) with 2 of the 24 blocks at d=1024,
        16 heads, ff 4096, chunk 4 / left 16, framing A (20 chunks: the 64-frame ring fills and trims)
        and framing B (8 chunks starting 3 chunks before the RelPE wrap at max_len);
      * CNNSubsampling 1024 -> 3584 (models/adapter.py:112-157) streaming on those encoder outputs;
      * LLM2TTSCodecAR.infer (models/decoder/decoder.py:314-367): all 4 layers at 896 / 14 heads / 4864,
        pre_nn + layers_prefix, greedy (top_k=1) 48 tokens, first logits rows;
      * VQVAE.forward (vqvae.py:37-42): Quantizer.embed + Generator at upsample_initial_channel 512 on
        one 60-token call (36000 samples)."""
    import argparse
    sys.argv = ["golden"]
    from models.adapter import CNNSubsampling
    from models.decoder.decoder import LLM2TTSCodecAR
    from models.decoder.ticodec.models import Generator, Quantizer
    from models.decoder.ticodec.vqvae import VQVAE, AttrDict
    from models.encoder.cmvn import GlobalCMVN
    from models.encoder.encoder import speechEncoder
    cfg = C.get("real")
    assert cfg["seed"] == seed
    ec = cfg["train_yaml"]["encoder_conf"]
    ec["para_conf"]["transformer"]["transformer-num-blocks"] = 2
    enc = speechEncoder(80, ec["overview_conf"], ec["para_conf"], GlobalCMVN(torch.zeros(80), torch.ones(80)))
    init_module(enc, seed, "encoder_user.", cfg["overrides"])
    enc.eval()
    mc = cfg["train_yaml"]["model_conf"]
    ada = CNNSubsampling(mc["enc_out_dim"], mc["llm_embed_dim"], mc["kernel_size"], mc["activation_func"], mc["norm"])
    init_module(ada, seed, "adpter_user.", cfg["overrides"])
    ada.eval()
    fb = np.load(os.path.join(HERE, "fbank.npz"))
    out = {}
    tr = enc.enc[1]
    for kind, n, pe0 in (("A", 20, 0), ("B", 8, tr.pe.max_len - 3 * tr.chunk_size + 1)):
        feats = fb["A_feats"][np.arange(n) % len(fb["A_feats"])] if kind == "A" else framing_b_feats(n, 321)[1]
        buf, pe, cc = [None] * tr.num_blocks, pe0, None
        eo, ao, pes = [], [], []
        for i in range(n):
            o, buf, _, _, pe = enc.infer(torch.from_numpy(feats[i]).unsqueeze(0), buf, 0, None, pe)
            a, _, cc = ada(o, torch.full(o.shape[:2], True).unsqueeze(1), cache=cc, return_cache=True)
            eo.append(o[0].numpy().copy())
            ao.append(a[0].numpy().copy())
            pes.append(pe)
        out[f"{kind}_feats"] = feats
        out[f"{kind}_enc"] = np.stack(eo)
        out[f"{kind}_ada"] = np.stack(ao)
        out[f"{kind}_pe"] = np.array(pes)
        out[f"{kind}_pe0"] = np.array(pe0)
        print(f"T2 encoder {kind}: {n} chunks, enc {out[kind + '_enc'].shape}, adapter {out[kind + '_ada'].shape}")
    np.savez_compressed(os.path.join(HERE, "real_encoder_t2.npz"), **out)

    idim, odim, args = cfg["decoder_json"]
    m = LLM2TTSCodecAR(idim, odim, argparse.Namespace(**args))
    init_module(m, seed, "tts.", cfg["overrides"])
    m.eval()
    rng = np.random.default_rng(55)
    hidden = torch.from_numpy(rng.standard_normal((1, 12, idim)).astype(np.float32) * 0.5)
    prefix = torch.from_numpy(rng.standard_normal((1, 24, idim)).astype(np.float32) * 0.5)
    logits = []
    orig = m.out_fnn.forward

    def hook(x):
        y = orig(x)
        if len(logits) < 4:
            logits.append(y[0, -1].numpy().copy())
        return y

    m.out_fnn.forward = hook
    ids = [int(t) for t in m.infer(hidden, 1, prefix, -1, 1.1, max_tokens=48)]
    m.out_fnn.forward = orig
    np.savez_compressed(os.path.join(HERE, "real_tts_t2.npz"), hidden=hidden[0].numpy(), prefix=prefix[0].numpy(),
                        ids=np.array(ids, np.int64), logits=np.stack(logits))
    print("T2 tts: ids", len(ids), ids[:12])

    h = AttrDict(cfg["codec_json"])
    vq = VQVAE.__new__(VQVAE)
    torch.nn.Module.__init__(vq)
    vq.h = h
    vq.quantizer = Quantizer(h)
    vq.generator = Generator(h)
    vq.generator.remove_weight_norm()
    init_module(vq.quantizer, seed, "codec.quantizer.")
    init_module(vq.generator, seed, "codec.generator.")
    vq.eval()
    cids = torch.from_numpy(np.random.default_rng(66).integers(0, h.n_codes, size=(1, 60, 1)))
    gt = torch.tensor(h.global_tokens).unsqueeze(0).unsqueeze(0)
    pcm = vq(cids, gt)
    np.savez_compressed(os.path.join(HERE, "real_codec_t2.npz"), ids=cids[0, :, 0].numpy(), pcm=pcm[0, 0].numpy())
    print("T2 codec: pcm", tuple(pcm.shape))


REAL_QWEN2_SETTINGS = [(1.0, k, p) for k in (0, 1, 20, 100) for p in (0.0, 0.8)]   # (temperature, top_k, top_p)


def gold_real_qwen2(seed=7, n_layers=2, n_sess=8):
    """Qwen2-7B at REAL geometry (hidden 3584, 28 q / 4 kv heads of 128, intermediate 18944, rope_theta 1e6,
    vocab 152064, untied lm_head), n_layers of the 28 layers, counter-hash weights (configs 'real'), run
    through the reference's own AudioLLM methods on a Qwen2ForCausalLM (models/audioLLM.py:70-74):
    _llm_forward_core (:479-484, inputs_embeds.half() and the all-True [past | new] mask of recognize,
    :409-419), _prediction_head_forward (:486-493) and _post_decode (:431-477).
    n_sess ragged sessions, each its own DynamicCache (the reference serves one session per call):
      step 0   prefill of 9 + 2b rows (fp16-valued random embeds: the batched GPU prefill is M = 128),
      step 1-2 two-row chunks (a listen chunk, M = 16 batched),
      step 3-5 text steps: lm_head on the last hidden row, _post_decode(top_k=1) -> that token's
               embedding (wte(tok).half()) is the next step's input (a text step, M = 8 batched).
    Stored (I/O only, weights regenerate from the hash): the input embeds, hidden rows (last row of the
    prefill, every row of the other steps), state probs, the lm_head logits of the 4 decision rows per
    session reduced to (argmax, top-2 margin, top-32 ids / values, logsumexp, 1024 fixed-index values)
    plus 2 full 152,064-wide rows, and _post_decode's pre-multinomial probs on those 2 rows for
    top_k in {0, 1, 20, 100} x top_p in {0, 0.8}."""
    from transformers import Qwen2Config, Qwen2ForCausalLM
    sys.argv = ["golden"]
    from models.audioLLM import AudioLLM
    cfg = C.get("real")
    assert cfg["seed"] == seed
    lc = dict(cfg["llm"], num_hidden_layers=n_layers)
    qc = Qwen2Config(**lc, torch_dtype="float32")
    m = Qwen2ForCausalLM(qc)
    for k, v in m.state_dict().items():   # one tensor at a time (6 GB of fp32 weights at 2 layers)
        v.copy_(torch.from_numpy(synth_param(seed, k, tuple(v.shape), cfg["overrides"])))
    m.eval()
    D, V = lc["hidden_size"], lc["vocab_size"]
    head = torch.nn.Linear(D, 4)
    init_module(head, seed, "predictor_head.", cfg["overrides"])
    obj = types.SimpleNamespace(llm_decoder=m, predictor_head=head)
    wte = m.model.embed_tokens
    rng = np.random.default_rng(1234)
    rows0 = [9 + 2 * b for b in range(n_sess)]
    emb_in = {0: [(rng.standard_normal((r, D)) * 0.5).astype(np.float16) for r in rows0]}
    for s in (1, 2):
        emb_in[s] = [(rng.standard_normal((2, D)) * 0.5).astype(np.float16) for _ in range(n_sess)]
    fixed_idx = np.sort(np.random.default_rng(99).choice(V, 1024, replace=False))
    out = {"rows0": np.array(rows0, np.int64), "fixed_idx": fixed_idx.astype(np.int64)}
    for s in (0, 1, 2):
        out[f"emb{s}"] = np.concatenate(emb_in[s])
    hid = {s: [] for s in range(6)}
    probs = np.zeros((6, n_sess, 3), np.float32)
    toks = np.zeros((4, n_sess), np.int64)           # token fed at text steps 3..5 (toks[0..2]) + last pick
    dec = {k: [] for k in ("argmax", "margin", "top_ids", "top_vals", "lse", "fixed")}
    full = {}

    def reduce_logits(lg):
        v, i = torch.topk(lg, 32)
        dec["argmax"].append(int(i[0]))
        dec["margin"].append(float(v[0] - v[1]))
        dec["top_ids"].append(i.numpy().astype(np.int64))
        dec["top_vals"].append(v.numpy().astype(np.float32))
        dec["lse"].append(float(torch.logsumexp(lg.double(), 0)))
        dec["fixed"].append(lg.numpy()[fixed_idx].astype(np.float32))

    for b in range(n_sess):
        pkv = None
        tok = None
        for s in range(6):
            if s < 3:
                e = torch.from_numpy(emb_in[s][b].astype(np.float32)).unsqueeze(0)
            else:
                e = wte(torch.tensor([[tok]]))
            past = 0 if pkv is None else pkv.get_seq_length()
            mask = torch.full([1, past + e.shape[1]], True)
            h, pkv = AudioLLM._llm_forward_core(obj, {"inputs_embeds": e.half(), "attention_mask": mask,
                                                      "past_key_values": pkv})
            hid[s].append(h[0, -1:].numpy().copy() if s == 0 else h[0].numpy().copy())
            probs[s, b] = AudioLLM._prediction_head_forward(obj, h).numpy()
            if s >= 2:
                lg = m.lm_head(h[:, -1:])
                reduce_logits(lg[0, 0])
                if (b, s) in ((0, 2), (1, 3)):
                    full[f"full_b{b}_s{s}"] = lg[0, 0].numpy().copy()
                tok = int(AudioLLM._post_decode(None, lg, temperature=1.0, top_k=1, top_p=0.0).reshape(-1)[0])
                toks[s - 2, b] = tok
        print(f"real qwen2 session {b}: rows {rows0[b]} kv {pkv.get_seq_length()} tokens {toks[:, b].tolist()} "
              f"margins {[round(x, 4) for x in dec['margin'][-4:]]}", flush=True)
    for s in range(6):
        out[f"hid{s}"] = np.concatenate(hid[s]).astype(np.float32)
    out["probs"] = probs
    out["toks"] = toks
    for k, v in dec.items():
        out["dec_" + k] = np.array(v)
    out.update(full)
    # _post_decode's pre-multinomial probs at V = 152,064 (multinomial captured, argmax returned)
    orig = torch.multinomial
    rows = [full["full_b0_s2"], full["full_b1_s3"]]
    sp = np.zeros((len(rows), len(REAL_QWEN2_SETTINGS), V), np.float32)
    try:
        for ri, lg in enumerate(rows):
            for si, (T, k, p) in enumerate(REAL_QWEN2_SETTINGS):
                cap = {}

                def mn(pr, n, **kw):
                    cap["p"] = pr.detach().clone()
                    return torch.argmax(pr).view(1)

                torch.multinomial = mn
                AudioLLM._post_decode(None, torch.from_numpy(lg).view(1, 1, -1), temperature=T, top_k=k, top_p=p)
                sp[ri, si] = cap["p"].numpy()
    finally:
        torch.multinomial = orig
    out["sampler_probs"] = sp
    out["sampler_settings"] = np.array(REAL_QWEN2_SETTINGS, np.float64)
    np.savez_compressed(os.path.join(HERE, "real_qwen2_t2.npz"), **out)
    print("real qwen2: kept counts", [[int((sp[r, s] > 0).sum()) for s in range(len(REAL_QWEN2_SETTINGS))]
                                      for r in range(len(rows))],
          f"fixture {os.path.getsize(os.path.join(HERE, 'real_qwen2_t2.npz')) / 1e6:.2f} MB")


# rows per session of the 17..64-row steps after the 128-row prefill (batched over the 8 sessions): M = 32 (4 framing-B
# tokens each: a duplex tick), 40 (the 5-token assistant prefix), 44 (ragged: ticks with and without a 5-token chat
# prefix -> the attention item table), 48, 64 (four row blocks)
MID_ROWS = [[4] * 8, [5] * 8, [4, 9, 4, 4, 6, 4, 9, 4], [6] * 8, [8] * 8]


def mid_embeds(step, b, rows, D=3584):
    """fp16-valued input embeds of session b at mid step `step` (regenerated by tests/test_real_qwen2_mid_gpu.py)."""
    return (np.random.default_rng(4321 + 100 * step + b).standard_normal((rows, D)) * 0.5).astype(np.float16)


def gold_real_qwen2_mid(seed=7, n_layers=2, n_sess=8):
    """The 17..64-row Qwen2-7B steps at REAL geometry through the reference's own AudioLLM._llm_forward_core /
    _prediction_head_forward (models/audioLLM.py:479-493), the shapes every duplex tick and assistant prefix run
    (bin/dialog_state_pred.py:777-844, models/audioLLM.py:350-429): the same 2-layer counter-hash Qwen2 and the same
    eight sessions as gold_real_qwen2 (its 9 + 2b-row prefill, real_qwen2_t2.npz emb0), then the MID_ROWS steps, each
    session its own DynamicCache.  Stored (weights and the mid-step inputs regenerate): per step the hidden rows at
    1024 fixed columns, every row's float64 sum / sum of squares over all 3584 columns, each session's full last row,
    the state probs, and the lm_head logits of each session's last row reduced as in gold_real_qwen2."""
    from transformers import Qwen2Config, Qwen2ForCausalLM
    sys.argv = ["golden"]
    from models.audioLLM import AudioLLM
    cfg = C.get("real")
    assert cfg["seed"] == seed
    lc = dict(cfg["llm"], num_hidden_layers=n_layers)
    m = Qwen2ForCausalLM(Qwen2Config(**lc, torch_dtype="float32"))
    for k, v in m.state_dict().items():
        v.copy_(torch.from_numpy(synth_param(seed, k, tuple(v.shape), cfg["overrides"])))
    m.eval()
    D, V = lc["hidden_size"], lc["vocab_size"]
    head = torch.nn.Linear(D, 4)
    init_module(head, seed, "predictor_head.", cfg["overrides"])
    obj = types.SimpleNamespace(llm_decoder=m, predictor_head=head)
    base = np.load(os.path.join(HERE, "real_qwen2_t2.npz"))
    rows0 = base["rows0"].tolist()
    emb0 = base["emb0"]
    cols = np.sort(np.random.default_rng(77).choice(D, 1024, replace=False))
    fixed_idx = base["fixed_idx"]
    out = {"cols": cols.astype(np.int64), "n_steps": np.array(len(MID_ROWS))}
    insum = 0.0
    for s, rows in enumerate(MID_ROWS):
        out[f"rows{s}"] = np.array(rows, np.int64)
    acc = {k: [[] for _ in MID_ROWS] for k in ("hcols", "hsum", "hsq", "hlast", "probs", "argmax", "margin", "top_ids",
                                               "top_vals", "lse", "fixed")}
    off = np.cumsum([0] + rows0)
    for b in range(n_sess):
        e = torch.from_numpy(emb0[off[b]:off[b + 1]].astype(np.float32)).unsqueeze(0)
        mask = torch.full([1, e.shape[1]], True)
        h, pkv = AudioLLM._llm_forward_core(obj, {"inputs_embeds": e.half(), "attention_mask": mask, "past_key_values": None})
        assert np.abs(h[0, -1].numpy() - base["hid0"][b]).max() < 1e-4   # the same prefill as real_qwen2_t2.npz
        for s, rows in enumerate(MID_ROWS):
            x = mid_embeds(s, b, rows[b], D)
            insum += float(x.astype(np.float64).sum())
            past = pkv.get_seq_length()
            mask = torch.full([1, past + rows[b]], True)
            h, pkv = AudioLLM._llm_forward_core(obj, {"inputs_embeds": torch.from_numpy(x.astype(np.float32)).unsqueeze(0).half(),
                                                      "attention_mask": mask, "past_key_values": pkv})
            hv = h[0].numpy().astype(np.float32)
            acc["hcols"][s].append(hv[:, cols])
            acc["hsum"][s].append(hv.astype(np.float64).sum(1))
            acc["hsq"][s].append((hv.astype(np.float64) ** 2).sum(1))
            acc["hlast"][s].append(hv[-1])
            acc["probs"][s].append(AudioLLM._prediction_head_forward(obj, h).numpy())
            lg = m.lm_head(h[:, -1:])[0, 0]
            v, i = torch.topk(lg, 32)
            acc["argmax"][s].append(int(i[0]))
            acc["margin"][s].append(float(v[0] - v[1]))
            acc["top_ids"][s].append(i.numpy().astype(np.int64))
            acc["top_vals"][s].append(v.detach().numpy().astype(np.float32))
            acc["lse"][s].append(float(torch.logsumexp(lg.double(), 0)))
            acc["fixed"][s].append(lg.detach().numpy()[fixed_idx].astype(np.float32))
        print(f"real qwen2 mid session {b}: kv {pkv.get_seq_length()} margins {[round(x[-1], 4) for x in acc['margin']]}",
              flush=True)
    for k, per in acc.items():
        for s in range(len(MID_ROWS)):
            v = per[s]
            out[f"{k}{s}"] = np.concatenate(v) if k in ("hcols", "hsum", "hsq") else np.array(v)
    out["input_sum"] = np.array(insum)
    np.savez_compressed(os.path.join(HERE, "real_qwen2_mid_t2.npz"), **out)
    print(f"real qwen2 mid: fixture {os.path.getsize(os.path.join(HERE, 'real_qwen2_mid_t2.npz')) / 1e6:.2f} MB, "
          f"input sum {insum:.6f}")


ADAPTER_VARIANTS = [  # CNNSubsampling(enc_out_dim, llm_embed_dim, kernel_size, activation_func, norm)
    {"enc_out_dim": 16, "llm_embed_dim": 128, "kernel_size": 5, "activation_func": "relu", "norm": "batch"},
    {"enc_out_dim": 32, "llm_embed_dim": 128, "kernel_size": 5, "activation_func": "gelu", "norm": "layer"},
    {"enc_out_dim": 32, "llm_embed_dim": 96, "kernel_size": 3, "activation_func": "relu", "norm": "layer"},
    {"enc_out_dim": 32, "llm_embed_dim": 128, "kernel_size": 5, "activation_func": "gelu", "norm": "batch"}]


def gold_adapter_variants(seed):
    """CNNSubsampling's other branches (models/adapter.py:84-110,123-150): cnn_num == 2 (4*d < L: a
    stride-1 conv + BN + ReLU before the stride-2 conv, two caches), LayerNorm(2d, eps 1e-3) over
    channels, exact GELU; streamed over chunks of 4 and 7 encoder frames (framings A and B) with the
    returned cache fed back, as AudioLLM.recognize does (models/audioLLM.py:386-387)."""
    from models.adapter import CNNSubsampling
    out = {}
    rng = np.random.default_rng(31)
    for vi, v in enumerate(ADAPTER_VARIANTS):
        m = CNNSubsampling(v["enc_out_dim"], v["llm_embed_dim"], v["kernel_size"], v["activation_func"], v["norm"])
        init_module(m, seed, "adpter_user.")
        m.eval()
        cache = None
        for c in range(6):
            T = 4 if c % 2 == 0 else 7
            x = torch.from_numpy(rng.standard_normal((1, T, v["enc_out_dim"])).astype(np.float32))
            y, _, cache = m(x, torch.full((1, 1, T), True), cache=cache, return_cache=True)
            out[f"v{vi}_c{c}_x"] = x[0].numpy()
            out[f"v{vi}_c{c}_y"] = y[0].detach().numpy().copy()
        out[f"v{vi}_cnn_num"] = np.array(m.cnn_num)
    np.savez_compressed(os.path.join(HERE, "adapter_variants_tiny.npz"), **out)
    with open(os.path.join(HERE, "adapter_variants_tiny.json"), "w") as f:
        json.dump({"seed": seed, "variants": ADAPTER_VARIANTS}, f, indent=1)
    print("adapter variants: cnn_num", [int(out[f"v{i}_cnn_num"]) for i in range(len(ADAPTER_VARIANTS))])


def gold_tts(cfg):
    import argparse
    from models.decoder.decoder import LLM2TTSCodecAR
    idim, odim, args = cfg["decoder_json"]
    m = LLM2TTSCodecAR(idim, odim, argparse.Namespace(**args))
    init_module(m, cfg["seed"], "tts.", cfg["overrides"])
    m.eval()
    SHAPES["tts"] = {"tts." + k: list(v.shape) for k, v in m.state_dict().items()}
    rng = np.random.default_rng(5)
    T1, T2 = 9, 24   # text embeds rows (4 per text token at real geometry), LLM hidden rows
    hidden = torch.from_numpy(rng.standard_normal((1, T1, idim)).astype(np.float32) * 0.5)
    prefix = torch.from_numpy(rng.standard_normal((1, T2, idim)).astype(np.float32) * 0.5)
    logits = []
    orig = m.out_fnn.forward

    def hook(x):
        y = orig(x)
        if len(logits) < 6:
            logits.append(y[0, -1].numpy().copy())
        return y

    m.out_fnn.forward = hook
    ids = [int(t) for t in m.infer(hidden, 1, prefix, -1, 1.1, max_tokens=150)]
    m.out_fnn.forward = orig
    np.savez_compressed(os.path.join(HERE, "tts_tiny.npz"), hidden=hidden[0].numpy(), prefix=prefix[0].numpy(),
                        ids=np.array(ids, dtype=np.int64), logits=np.stack(logits))
    print("tts: ids", len(ids), ids[:12])
    return m


def gold_tts_penalty(cfg):
    """LLM2TTSCodecAR.infer with the repetition penalty on (decoder.py:348-351), greedy, same inputs as
    gold_tts: pins the per-occurrence division of set(generated_tokens[0][-W:]) over 0-d tensors."""
    import argparse
    from models.decoder.decoder import LLM2TTSCodecAR
    idim, odim, args = cfg["decoder_json"]
    m = LLM2TTSCodecAR(idim, odim, argparse.Namespace(**args))
    init_module(m, cfg["seed"], "tts.", cfg["overrides"])
    m.eval()
    rng = np.random.default_rng(5)
    T1, T2 = 9, 24
    hidden = torch.from_numpy(rng.standard_normal((1, T1, idim)).astype(np.float32) * 0.5)
    prefix = torch.from_numpy(rng.standard_normal((1, T2, idim)).astype(np.float32) * 0.5)
    out = {}
    for name, W, pen in (("w20_p1.5", 20, 1.5), ("w3_p1.1", 3, 1.1)):
        ids = [int(t) for t in m.infer(hidden, 1, prefix, W, pen, max_tokens=120)]
        out["ids_" + name] = np.array(ids, dtype=np.int64)
        print("tts penalty", name, len(ids), ids[:12])
    np.savez_compressed(os.path.join(HERE, "tts_penalty_tiny.npz"), **out)


CODEC_ENC_JSON = {"resblock": "1", "upsample_rates": [5, 3, 2, 2], "upsample_kernel_sizes": [10, 6, 4, 4],
                  "upsample_initial_channel": 256, "resblock_kernel_sizes": [3, 5],
                  "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5]], "n_codes": 60, "n_code_groups": 1,
                  "residul_layer": 2, "global_code_num": 8, "codebook_loss_lambda": 1.0,
                  "commitment_loss_lambda": 0.25, "global_feature_conv": [128, 64, 128, 3, 2]}


def gold_codec_encoder(seed):
    """VQVAE.encode (models/decoder/ticodec/vqvae.py:44-57): Encoder (models.py:429-522, weight norm
    removed) + Quantizer.forward (models.py:531-659, residual VQ over 2 layers + global tokens) on
    2400 samples of synthetic 24 kHz audio.  The Encoder's 32*2^i channel ladder ends in conv_post(512,
    512), so it needs 4 stages; this config (60x down, GlobalTokenEncoder after stage 1) provides them."""
    from models.decoder.ticodec.models import Encoder, Quantizer
    from models.decoder.ticodec.vqvae import VQVAE, AttrDict
    h = AttrDict(CODEC_ENC_JSON)
    vq = VQVAE.__new__(VQVAE)
    torch.nn.Module.__init__(vq)
    vq.h = h
    vq.quantizer = Quantizer(h)
    vq.encoder = Encoder(h)
    vq.encoder.remove_weight_norm()
    init_module(vq.quantizer, seed, "codec.quantizer.")
    init_module(vq.encoder, seed, "codec.encoder.")
    vq.eval()
    shapes = {**{"codec.quantizer." + k: list(v.shape) for k, v in vq.quantizer.state_dict().items()},
              **{"codec.encoder." + k: list(v.shape) for k, v in vq.encoder.state_dict().items()}}
    r = np.random.default_rng(21)
    n = np.arange(2 * 2400)
    wav = (0.3 * np.sin(2 * np.pi * 180 * n / 24000) * (1 + 0.5 * np.sin(2 * np.pi * 3 * n / 24000))
           + 0.05 * r.standard_normal(n.size)).astype(np.float32).reshape(2, 2400)
    wav[1] *= 0.5
    with torch.no_grad():
        c, gfeat = vq.encoder(torch.from_numpy(wav).unsqueeze(1))
        local, gst = vq.encode(torch.from_numpy(wav))
    np.savez_compressed(os.path.join(HERE, "codec_encoder_tiny.npz"), wav=wav, enc_out=c.numpy(),
                        global_features=gfeat.numpy(), local_tokens=local.numpy(), global_tokens=gst.numpy())
    with open(os.path.join(HERE, "codec_encoder_tiny.json"), "w") as f:
        json.dump({"codec_json": CODEC_ENC_JSON, "seed": seed, "shapes": shapes}, f)
    print("codec encoder: c", tuple(c.shape), "local", tuple(local.shape), local[0, :8, :].tolist(),
          "global", gst.tolist())


def gold_codec(cfg, tts_model):
    from models.decoder.ticodec.models import Generator, Quantizer
    from models.decoder.ticodec.vqvae import VQVAE, AttrDict
    from models.decoder.llm2tts import llm2TTS
    h = AttrDict(cfg["codec_json"])
    vq = VQVAE.__new__(VQVAE)
    torch.nn.Module.__init__(vq)
    vq.h = h
    vq.quantizer = Quantizer(h)
    vq.generator = Generator(h)
    vq.generator.remove_weight_norm()
    init_module(vq.quantizer, cfg["seed"], "codec.quantizer.")
    init_module(vq.generator, cfg["seed"], "codec.generator.")
    vq.eval()
    SHAPES["codec"] = {**{"codec.quantizer." + k: list(v.shape) for k, v in vq.quantizer.state_dict().items()},
                       **{"codec.generator." + k: list(v.shape) for k, v in vq.generator.state_dict().items()}}
    rng = np.random.default_rng(11)
    ids = torch.from_numpy(rng.integers(0, h.n_codes, size=(1, 60, 1)))
    gt = torch.tensor(h.global_tokens).unsqueeze(0).unsqueeze(0)
    pcm = vq(ids, gt)
    np.savez_compressed(os.path.join(HERE, "codec_tiny.npz"), ids=ids[0, :, 0].numpy(), pcm=pcm[0, 0].numpy())
    print("codec: pcm", tuple(pcm.shape))

    # llm2TTS.run end to end (AR decode + 40/10 codec chunking + silence cut)
    fake = llm2TTS.__new__(llm2TTS)
    fake.model = tts_model
    fake.infer = functools.partial(tts_model.infer, max_tokens=130)
    fake.codec_model = types.SimpleNamespace(vqvae=vq)
    t = np.load(os.path.join(HERE, "tts_tiny.npz"))
    hidden = torch.from_numpy(t["hidden"]).unsqueeze(0)
    prefix = torch.from_numpy(t["prefix"]).unsqueeze(0)
    segs = [s[0, 0].float().numpy().copy() for s in fake.run(hidden, 1, prefix, 40, 10, -1, 1.1, 2401, 0.01)]
    out = {f"seg{i}": s for i, s in enumerate(segs)}
    np.savez_compressed(os.path.join(HERE, "llm2tts_run_tiny.npz"), n=np.array(len(segs)), **out)
    print("llm2tts.run: segments", [len(s) for s in segs])

    # find_min_sum_index on synthetic audio (quiet gaps force both branches)
    cases = {}
    r = np.random.default_rng(3)
    for ci in range(4):
        syn = r.standard_normal(24000).astype(np.float32) * (0.2 if ci % 2 == 0 else 0.002)
        if ci == 2:
            syn[15000:19000] *= 0.001
        buf = r.standard_normal(1000 * ci).astype(np.float32) * 0.1
        b2, s2 = llm2TTS.find_min_sum_index(None, torch.from_numpy(buf).view(1, 1, -1),
                                            torch.from_numpy(syn).view(1, 1, -1), 2401, 0.01)
        cases[f"c{ci}_syn"] = syn
        cases[f"c{ci}_buf"] = buf
        cases[f"c{ci}_outbuf"] = b2[0, 0].numpy()
        cases[f"c{ci}_out"] = np.zeros(0, np.float32) if s2 is None else s2[0, 0].numpy()
        cases[f"c{ci}_none"] = np.array(s2 is None)
    np.savez_compressed(os.path.join(HERE, "silence_cut.npz"), **cases)


def gold_codec_gst(cfg):
    """VQVAE.forward with NON-default global style tokens (models/decoder/ticodec/vqvae.py:37-42, embed_gst
    models.py:703-715): three rows each with its own global tokens ([3, 1, n], as VQVAE.encode returns them), and a
    [1, 1, n] token broadcast over two rows.  Same tiny codec weights as codec_tiny.npz (the config seed)."""
    from models.decoder.ticodec.models import Generator, Quantizer
    from models.decoder.ticodec.vqvae import VQVAE, AttrDict
    h = AttrDict(cfg["codec_json"])
    vq = VQVAE.__new__(VQVAE)
    torch.nn.Module.__init__(vq)
    vq.h = h
    vq.quantizer = Quantizer(h)
    vq.generator = Generator(h)
    vq.generator.remove_weight_norm()
    init_module(vq.quantizer, cfg["seed"], "codec.quantizer.")
    init_module(vq.generator, cfg["seed"], "codec.generator.")
    vq.eval()
    rng = np.random.default_rng(23)
    n = h.global_code_num
    ids = torch.from_numpy(rng.integers(0, h.n_codes, size=(3, 24, 1)))
    gst = torch.from_numpy(rng.integers(0, h.n_codes, size=(3, 1, n)))
    gst[0, 0] = torch.tensor(h.global_tokens)          # row 0: the default tokens
    with torch.no_grad():
        pcm = vq(ids, gst)
        gst1 = torch.from_numpy(rng.integers(0, h.n_codes, size=(1, 1, n)))
        pcm_b = vq(ids[:2], gst1)                      # one token set broadcast over the batch
    np.savez_compressed(os.path.join(HERE, "codec_gst_tiny.npz"), ids=ids[..., 0].numpy(), gst=gst.numpy(),
                        pcm=pcm[:, 0].numpy(), gst_b=gst1.numpy(), pcm_b=pcm_b[:, 0].numpy())
    print("codec gst: pcm", tuple(pcm.shape), "gst", gst[:, 0].tolist(), "broadcast", gst1[0, 0].tolist())


def gold_text():
    sys.argv = ["golden"]
    from models.pipeline import inferencePipeline
    texts = ["Hello world", "1. First item 2. second", "你好、世界（测试）", "Use *bold* and `code`~",
             "Numbers: 3.14 are fine.", "Ends with comma,", "问题：\n是什么", "Line\tbreak\r\nhere;", ""]
    outs = [inferencePipeline.post_process(None, t) for t in texts]
    from models.ContextSerializer import ContextSerializer
    cs = ContextSerializer()
    events = [(0.00, "user", "ipu_sl"), (0.05, "system", "ipu_sl"), (0.10, "user", "ipu_cl"),
              (0.12, "system", "ipu_cl"), (0.20, "user", "ipu_el"), (0.25, "system", "ipu_cl"),
              (0.30, "system", "ipu_cl"), (0.35, "user", "ipu_sl"), (0.36, "system", "ipu_el"),
              (0.40, "user", "ipu_el"), (0.45, "system", "ipu_sl")]
    for i, (ts, ident, st) in enumerate(events):
        cs.add_feature_chunk({"time_stamp": ts, "identity": ident, "status": st, "feature": [i], "ipu_id": i})
    sent = []
    while True:
        if not cs.feature_queue:
            break
        sent.append(cs.get_next_feature())
    with open(os.path.join(HERE, "text_and_serializer.json"), "w") as f:
        json.dump({"texts": texts, "post_process": outs, "events": events, "serialized": sent}, f,
                  ensure_ascii=False, indent=1)


def main():
    install_shims()
    cfg = C.get("tiny")
    fb = gold_fbank()
    gold_audiollm(cfg, fb["A_feats"])
    m = gold_tts(cfg)
    gold_codec(cfg, m)
    gold_tts_penalty(cfg)
    gold_codec_encoder(cfg["seed"])
    gold_text()
    gold_audiollm_b(cfg)
    gold_llm_text(cfg)
    gold_real_t2()
    gold_real_qwen2()
    gold_real_qwen2_mid()
    gold_adapter_variants(cfg["seed"])
    gold_codec_gst(cfg)
    with open(os.path.join(HERE, "param_shapes_tiny.json"), "w") as f:
        json.dump(SHAPES, f)
    total = sum(os.path.getsize(os.path.join(HERE, f)) for f in os.listdir(HERE) if f.endswith((".npz", ".json")))
    print(f"fixtures: {total / 1e6:.2f} MB")


if __name__ == "__main__":
    if sys.argv[1:] == ["tts_penalty"]:   # regenerate only that fixture
        install_shims()
        gold_tts_penalty(C.get("tiny"))
    elif sys.argv[1:] == ["codec_encoder"]:
        install_shims()
        gold_codec_encoder(C.get("tiny")["seed"])
    elif sys.argv[1:] == ["framing_b"]:
        install_shims()
        gold_audiollm_b(C.get("tiny"))
    elif sys.argv[1:] == ["llm_text"]:
        install_shims()
        gold_llm_text(C.get("tiny"))
    elif sys.argv[1:] == ["adapter_variants"]:
        install_shims()
        gold_adapter_variants(C.get("tiny")["seed"])
    elif sys.argv[1:] == ["real_t2"]:
        install_shims()
        gold_real_t2()
    elif sys.argv[1:] == ["codec_gst"]:
        install_shims()
        gold_codec_gst(C.get("tiny"))
    elif sys.argv[1:] == ["real_qwen2"]:
        install_shims()
        gold_real_qwen2()
    elif sys.argv[1:] == ["real_qwen2_mid"]:
        install_shims()
        gold_real_qwen2_mid()
    else:
        main()
