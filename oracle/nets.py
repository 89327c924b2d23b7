"""Oracle (TEST INFRASTRUCTURE): numpy fp32 restatement of the Freeze-Omni model math.

Checker only: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by
the product path (freeze-omni_amd/).  Pinned against tests/golden/*.npz produced by the reference
(tests/golden/make_golden.py).  Numerics mirror the reference's CPU/fp32 run, including its fp16
roundings: inputs_embeds.half() (models/audioLLM.py:338,410), rotary cos/sin cast to the fp16
embeds dtype and the first RMSNorm's cast back to its fp16 input dtype (transformers Qwen2).
Weights are a dict name -> np.float32 array keyed by reference state_dict names.
"""
import math

import numpy as np

F32 = np.float32


def f16(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def linear(x, w, b=None):
    y = np.asarray(x, F32) @ np.asarray(w, F32).T
    if b is not None:
        y = y + b
    return y.astype(F32)


def layernorm(x, w, b, eps=1e-5):
    m = x.mean(-1, keepdims=True)
    v = ((x - m) ** 2).mean(-1, keepdims=True)
    return ((x - m) / np.sqrt(v + F32(eps)) * w + b).astype(F32)


def rmsnorm(x, w, eps, round_input_fp16=False):
    """Qwen2RMSNorm / LlamaRMSNorm: w * (x * rsqrt(mean(x^2)+eps)).to(input_dtype)."""
    x = np.asarray(x, F32)
    v = (x * x).mean(-1, keepdims=True)
    h = x / np.sqrt(v + F32(eps))
    if round_input_fp16:
        h = f16(h)
    return (w * h).astype(F32)


def softmax(x, axis=-1):
    x = np.asarray(x, F32)
    e = np.exp(x - x.max(axis=axis, keepdims=True))
    return (e / e.sum(axis=axis, keepdims=True)).astype(F32)


def silu(x):
    return (x / (1.0 + np.exp(-x))).astype(F32)


def leaky(x, s=0.1):
    return np.where(x >= 0, x, x * F32(s)).astype(F32)


# ============================================================ encoder (models/encoder/*)
def rel_pe_table(positions, d):
    """models/encoder/attention.py:105-121 RelPositionalEncoding.infer sin/cos rows (fp32 as torch)."""
    div = np.exp(np.arange(0, d, 2, dtype=F32) * F32(-(math.log(10000.0) / d))).astype(F32)
    pos = np.asarray(positions, F32)[:, None]
    pe = np.zeros((len(positions), d), F32)
    pe[:, 0::2] = np.sin(pos * div)
    pe[:, 1::2] = np.cos(pos * div)
    return pe


def conv2d_s2(x, w, b):
    """3x3 stride-2 valid conv. x [Cin, H, W], w [Cout, Cin, 3, 3]."""
    Cin, H, W = x.shape
    Ho, Wo = (H - 3) // 2 + 1, (W - 3) // 2 + 1
    cols = np.empty((Cin, 3, 3, Ho, Wo), F32)
    for i in range(3):
        for j in range(3):
            cols[:, i, j] = x[:, i:i + 2 * Ho:2, j:j + 2 * Wo:2]
    y = w.reshape(w.shape[0], -1) @ cols.reshape(Cin * 9, Ho * Wo)
    return (y.reshape(-1, Ho, Wo) + b[:, None, None]).astype(F32)


class Encoder:
    """speechEncoder.infer (models/encoder/encoder.py:149-155): CMVN -> Conv2dSubsampling4.infer
    (subsampling.py:67-73) -> Transformer.infer (transformer.py:267-285)."""

    def __init__(self, W, cfg, ident="user"):
        self.W = W
        self.p = f"encoder_{ident}."
        tr = cfg["train_yaml"]["encoder_conf"]["para_conf"]["transformer"]
        self.d = tr["transformer-attention-dim"]
        self.h = tr["transformer-attention-heads"]
        self.nb = tr["transformer-num-blocks"]
        self.chunk = tr["transformer-chunk_size"]
        self.left = tr["transformer-left_chunks"]
        self.buffersize = self.chunk * self.left
        self.full_chunk = (self.left + 1) * self.chunk
        self.max_len = self.chunk * (5000 // self.chunk) - self.full_chunk

    def w(self, n):
        return self.W[self.p + n]

    def subsample(self, feats):
        x = (feats - self.w("global_cmvn.mean")) * self.w("global_cmvn.istd")
        x = x.astype(F32)[None]  # [1, T, 80]
        y = np.maximum(conv2d_s2(x, self.w("enc.0.core.conv.0.weight"), self.w("enc.0.core.conv.0.bias")), 0)
        y = np.maximum(conv2d_s2(y, self.w("enc.0.core.conv.2.weight"), self.w("enc.0.core.conv.2.bias")), 0)
        C, t, f = y.shape
        y = y.transpose(1, 0, 2).reshape(t, C * f)
        return linear(y, self.w("enc.0.core.out.0.weight"), self.w("enc.0.core.out.0.bias"))

    def infer(self, feats, state):
        """feats [T, 80]; state = {'buf': [None | (K [h, L, dk], V)] * nb, 'pe': int} (mutated)."""
        x = self.subsample(feats)
        x = linear(x, self.w("enc.1.embed.0.weight"), self.w("enc.1.embed.0.bias"))
        x = np.maximum(layernorm(x, self.w("enc.1.embed.1.weight"), self.w("enc.1.embed.1.bias")), 0)
        buf = state["buf"]
        pe_len = x.shape[0] if buf[0] is None else buf[0][0].shape[1] + x.shape[0]
        pe_index = state["pe"] % self.max_len
        x = (x * F32(math.sqrt(self.d))).astype(F32)
        start = max(0, pe_index - self.full_chunk)
        pos = rel_pe_table(np.arange(start, start + pe_len), self.d)
        state["pe"] = pe_index + self.chunk
        dk = self.d // self.h
        for i in range(self.nb):
            q = f"enc.1.encoders.{i}."
            res = x
            hN = layernorm(x, self.w(q + "norm1.weight"), self.w(q + "norm1.bias"))
            Q = linear(hN, self.w(q + "self_attn.linear_q.weight"), self.w(q + "self_attn.linear_q.bias"))
            K = linear(hN, self.w(q + "self_attn.linear_k.weight"), self.w(q + "self_attn.linear_k.bias"))
            V = linear(hN, self.w(q + "self_attn.linear_v.weight"), self.w(q + "self_attn.linear_v.bias"))
            T = x.shape[0]
            Q = Q.reshape(T, self.h, dk).transpose(1, 0, 2)
            K = K.reshape(T, self.h, dk).transpose(1, 0, 2)
            V = V.reshape(T, self.h, dk).transpose(1, 0, 2)
            if buf[i] is None:
                KB, VB = K, V
            else:
                KB = np.concatenate([buf[i][0], K], axis=1)
                VB = np.concatenate([buf[i][1], V], axis=1)
            buf[i] = (KB[:, -self.buffersize:], VB[:, -self.buffersize:]) if KB.shape[1] > self.buffersize \
                else (KB, VB)
            P = linear(pos, self.w(q + "self_attn.linear_pos.weight")).reshape(-1, self.h, dk).transpose(1, 0, 2)
            qu = Q + self.w(q + "self_attn.pos_bias_u")[:, None, :]
            qv = Q + self.w(q + "self_attn.pos_bias_v")[:, None, :]
            sc = (qu @ KB.transpose(0, 2, 1) + qv @ P.transpose(0, 2, 1)) / F32(math.sqrt(dk))
            a = softmax(sc) @ VB
            a = a.transpose(1, 0, 2).reshape(T, self.d)
            x = res + linear(a, self.w(q + "self_attn.linear_out.weight"), self.w(q + "self_attn.linear_out.bias"))
            res = x
            hN = layernorm(x, self.w(q + "norm2.weight"), self.w(q + "norm2.bias"))
            f = np.maximum(linear(hN, self.w(q + "feed_forward.w_1.weight"), self.w(q + "feed_forward.w_1.bias")), 0)
            x = res + linear(f, self.w(q + "feed_forward.w_2.weight"), self.w(q + "feed_forward.w_2.bias"))
        return layernorm(x, self.w("enc.1.after_norm.weight"), self.w("enc.1.after_norm.bias"))


def new_encoder_state(nb):
    return {"buf": [None] * nb, "pe": 0}


class Adapter:
    """CNNSubsampling.forward(x, mask, cache, return_cache=True) (models/adapter.py:72-157):
    cnn_num == 1 (4*d >= L): causal conv1d(d->2d, k, stride 2) + BatchNorm(eval, eps 1e-3) or
    LayerNorm(2d, eps 1e-3) over channels + ReLU or exact GELU + Linear(2d -> L);
    cnn_num == 2 (4*d < L): causal conv1d(d->2d, k, stride 1) + BN + ReLU, then conv1d(2d->4d, k,
    stride 2) + BN + ReLU + Linear(4d -> L).  cache = [last k-1 inputs of the stride-2 conv,
    last k-1 inputs of the stride-1 conv] (zeros on the first call, :124-143)."""

    def __init__(self, W, cfg, ident="user"):
        mc = cfg["train_yaml"]["model_conf"]
        self.W = W
        self.p = f"adpter_{ident}."
        self.k = mc["kernel_size"]
        self.cnn_num = 2 if 4 * mc["enc_out_dim"] < mc["llm_embed_dim"] else 1
        self.norm = "batch" if self.cnn_num == 2 else mc.get("norm", "batch")
        self.act = "relu" if self.cnn_num == 2 else mc.get("activation_func", "relu")

    def _conv(self, xt, cache, name, stride):
        """xt [C, T] -> (y [T', Cout] incl. bias, new cache [C, k-1])."""
        left = np.zeros((xt.shape[0], self.k - 1), F32) if cache is None else cache
        xt = np.concatenate([left, xt], axis=1)
        new_cache = xt[:, 1 - self.k:].copy()
        w = self.W[self.p + name + ".weight"]
        To = (xt.shape[1] - self.k) // stride + 1
        cols = np.stack([xt[:, t * stride:t * stride + self.k].reshape(-1) for t in range(To)])
        return linear(cols, w.reshape(w.shape[0], -1), self.W[self.p + name + ".bias"]), new_cache

    def _bn(self, y, name):
        g, b = self.W[self.p + name + ".weight"], self.W[self.p + name + ".bias"]
        rm, rv = self.W[self.p + name + ".running_mean"], self.W[self.p + name + ".running_var"]
        return ((y - rm) / np.sqrt(rv + F32(1e-3)) * g + b).astype(F32)

    def __call__(self, x, cache):
        """x [T, d]; cache None or the list above.  Returns (out [T', L], new_cache)."""
        xt = x.T
        c0 = c1 = None
        if cache is not None:
            c0 = cache[0]
            c1 = cache[1] if len(cache) > 1 else None
        if self.cnn_num == 2:
            y1, c1 = self._conv(xt, c1, "conv1d1", 1)
            xt = np.maximum(self._bn(y1, "bn1"), 0).T
        y, c0 = self._conv(xt, c0, "conv1d2", 2)
        if self.norm == "batch":
            y = self._bn(y, "bn2")
        else:
            y = layernorm(y, self.W[self.p + "bn2.weight"], self.W[self.p + "bn2.bias"], eps=1e-3)
        if self.act == "gelu":
            from scipy.special import erf
            y = (0.5 * y * (1.0 + erf(y.astype(np.float64) / np.sqrt(2.0)))).astype(F32)
        else:
            y = np.maximum(y, 0)
        out = linear(y, self.W[self.p + "project.weight"], self.W[self.p + "project.bias"])
        return out, ([c0, c1] if self.cnn_num == 2 else [c0])


# ============================================================ decoder-only transformers
def rope_inv_freq(theta, hd):
    """transformers default rope: 1 / theta ** (arange(0, hd, 2) / hd) in fp32."""
    return (F32(1.0) / (F32(theta) ** (np.arange(0, hd, 2, dtype=np.int64).astype(F32) / F32(hd)))).astype(F32)


def rope_cos_sin(positions, inv_freq, round_fp16):
    fr = (np.asarray(positions, F32)[:, None] * inv_freq[None, :]).astype(F32)
    emb = np.concatenate([fr, fr], axis=-1)
    c, s = np.cos(emb).astype(F32), np.sin(emb).astype(F32)
    if round_fp16:
        c, s = f16(c), f16(s)
    return c, s


def apply_rope(x, c, s):
    """x [n_heads, T, hd]; rotate_half convention (transformers apply_rotary_pos_emb)."""
    h = x.shape[-1] // 2
    rot = np.concatenate([-x[..., h:], x[..., :h]], axis=-1)
    return (x * c[None] + rot * s[None]).astype(F32)


class KV:
    """Per-sequence key/value cache: list over layers of (K [n_kv, L, hd], V)."""

    def __init__(self, n_layers):
        self.k = [None] * n_layers
        self.v = [None] * n_layers

    def append(self, i, k, v):
        self.k[i] = k if self.k[i] is None else np.concatenate([self.k[i], k], axis=1)
        self.v[i] = v if self.v[i] is None else np.concatenate([self.v[i], v], axis=1)
        return self.k[i], self.v[i]

    def length(self, i=0):
        return 0 if self.k[i] is None else self.k[i].shape[1]

    def copy(self):
        n = KV(len(self.k))
        n.k = [None if a is None else a.copy() for a in self.k]
        n.v = [None if a is None else a.copy() for a in self.v]
        return n


def attention(q, k, v, scale, causal_offset=None):
    """q [H, T, hd], k/v [KVH, L, hd] (GQA repeat); causal_offset: query i sees keys <= offset + i."""
    H, KVH = q.shape[0], k.shape[0]
    rep = H // KVH
    k = np.repeat(k, rep, axis=0)
    v = np.repeat(v, rep, axis=0)
    sc = (q @ k.transpose(0, 2, 1)) * F32(scale)
    if causal_offset is not None:
        T, L = q.shape[1], k.shape[1]
        mask = np.arange(L)[None, :] > (causal_offset + np.arange(T))[:, None]
        sc = np.where(mask[None], -np.inf, sc)
    return (softmax(sc) @ v).astype(F32)


class DecoderStack:
    """A stack of Qwen2/Llama decoder layers (transformers Qwen2DecoderLayer / LlamaDecoderLayer)."""

    def __init__(self, W, prefix, n_layers, hidden, heads, kv_heads, eps, bias):
        self.W, self.p = W, prefix
        self.n, self.D, self.H, self.KVH, self.eps, self.bias = n_layers, hidden, heads, kv_heads, eps, bias
        self.hd = hidden // heads

    def layer(self, i, x, c, s, kv, causal_offset, first_fp16=False, kv_layer=None):
        q = f"{self.p}{i}."
        W = self.W
        T = x.shape[0]
        h = rmsnorm(x, W[q + "input_layernorm.weight"], self.eps, round_input_fp16=first_fp16)
        b = (lambda n: W[q + f"self_attn.{n}.bias"]) if self.bias else (lambda n: None)
        Q = linear(h, W[q + "self_attn.q_proj.weight"], b("q_proj")).reshape(T, self.H, self.hd).transpose(1, 0, 2)
        K = linear(h, W[q + "self_attn.k_proj.weight"], b("k_proj")).reshape(T, self.KVH, self.hd).transpose(1, 0, 2)
        V = linear(h, W[q + "self_attn.v_proj.weight"], b("v_proj")).reshape(T, self.KVH, self.hd).transpose(1, 0, 2)
        Q, K = apply_rope(Q, c, s), apply_rope(K, c, s)
        if kv is not None:
            Ka, Va = kv.append(i if kv_layer is None else kv_layer, K, V)
        else:
            Ka, Va = K, V
        a = attention(Q, Ka, Va, self.hd ** -0.5, causal_offset)
        a = a.transpose(1, 0, 2).reshape(T, self.H * self.hd)
        x = x + linear(a, W[q + "self_attn.o_proj.weight"])
        h = rmsnorm(x, W[q + "post_attention_layernorm.weight"], self.eps)
        m = silu(linear(h, W[q + "mlp.gate_proj.weight"])) * linear(h, W[q + "mlp.up_proj.weight"])
        return (x + linear(m, W[q + "mlp.down_proj.weight"])).astype(F32)


class Qwen2:
    """Qwen2Model.forward with a per-sequence cache, as reached through AudioLLM._llm_forward_core
    (models/audioLLM.py:479-484) with the fp16 input embeds of models/audioLLM.py:338,410."""

    def __init__(self, W, cfg):
        c = cfg["llm"]
        self.W = W
        self.cfg = c
        self.stack = DecoderStack(W, "model.layers.", c["num_hidden_layers"], c["hidden_size"],
                                  c["num_attention_heads"], c["num_key_value_heads"], c["rms_norm_eps"], True)
        self.inv_freq = rope_inv_freq(c["rope_theta"], self.stack.hd)

    def embed(self, ids):
        return self.W["model.embed_tokens.weight"][np.asarray(ids)]

    def forward(self, embeds, kv):
        """embeds [T, D] (rounded to fp16 as .half()); kv: KV (mutated).  Returns final-normed hidden."""
        x = f16(embeds)
        past = kv.length()
        pos = np.arange(past, past + x.shape[0])
        c, s = rope_cos_sin(pos, self.inv_freq, round_fp16=True)
        for i in range(self.stack.n):
            x = self.stack.layer(i, x, c, s, kv, causal_offset=past, first_fp16=(i == 0))
        return rmsnorm(x, self.W["model.norm.weight"], self.cfg["rms_norm_eps"])

    def logits(self, h):
        return linear(h, self.W["lm_head.weight"])


def state_probs(W, hidden):
    """AudioLLM._prediction_head_forward (models/audioLLM.py:486-493): softmax over the first 3 of 4
    head logits of the LAST position -> (state_1, state_2) (models/audioLLM.py:521-524)."""
    lg = linear(hidden, W["predictor_head.weight"], W["predictor_head.bias"])
    p = softmax(lg[:, :-1])[-1]
    return float(p[1]), float(p[2])


# ============================================================ speech decoder (models/decoder/decoder.py)
class TTSDecoder:
    """LLM2TTSCodecAR.infer (models/decoder/decoder.py:314-367) with eager attention semantics."""

    def __init__(self, W, cfg):
        idim, odim, a = cfg["decoder_json"]
        self.W, self.vocab = W, odim
        D, H = a["transformer_attention_dim"], a["transformer_attention_heads"]
        nb = a["transformer_num_blocks"]
        eps = 1e-6
        self.pre = DecoderStack(W, "tts.layers_pre_nn.", nb // 2, D, H, H, eps, False)
        self.main = DecoderStack(W, "tts.layers.", nb, D, H, H, eps, False)
        self.prefix = DecoderStack(W, "tts.layers_prefix.", nb, D, H, H, eps, False) \
            if a.get("kv_cache_prefix_finetune", 0) else None
        self.inv_freq = rope_inv_freq(10000.0, D // H)
        self.eps = eps

    def cos_sin(self, pos):
        return rope_cos_sin(pos, self.inv_freq, round_fp16=False)

    def prefill(self, hidden, prefix):
        """pre_nn + BOS + prefix KV + bidirectional prefill.  Returns the KV cache and P."""
        T = hidden.shape[0]
        c, s = self.cos_sin(np.arange(T))
        x = hidden.astype(F32)
        for i in range(self.pre.n):
            x = self.pre.layer(i, x, c, s, None, None)
        x = np.concatenate([self.W["tts.embedding.weight"][self.vocab][None], x], axis=0)
        kv = KV(self.main.n)
        P = 0
        if prefix is not None and self.prefix is not None:
            P = prefix.shape[0]
            c2, s2 = self.cos_sin(np.arange(P))
            y = prefix.astype(F32)
            for i in range(self.prefix.n):
                y = self.prefix.layer(i, y, c2, s2, kv, None)
        c, s = self.cos_sin(np.arange(x.shape[0]))
        for i in range(self.main.n):
            x = self.main.layer(i, x, c, s, kv, None)
        return kv, P

    def step(self, tok, kv, P):
        x = self.W["tts.embedding.weight"][tok][None]
        pos = kv.length() - P
        c, s = self.cos_sin(np.array([pos]))
        for i in range(self.main.n):
            x = self.main.layer(i, x, c, s, kv, None)
        x = rmsnorm(x, self.W["tts.norm.weight"], self.eps)
        return linear(x, self.W["tts.out_fnn.weight"], self.W["tts.out_fnn.bias"])[0]

    def infer_greedy(self, hidden, prefix, max_tokens=1000, return_logits=0, penalty_window_size=-1, penalty=1.1):
        kv, P = self.prefill(hidden, prefix)
        cur = self.vocab + 1
        ids, lgs = [], []
        for _ in range(max_tokens):
            lg = self.step(cur, kv, P)
            if penalty_window_size > 0:
                apply_penalty(lg, [self.vocab + 1] + ids, penalty_window_size, penalty)
            if len(lgs) < return_logits:
                lgs.append(lg)
            nxt = int(np.argmax(lg))  # top_k=1: softmax/topk/multinomial collapse to argmax
            if nxt == self.vocab + 2:
                break
            ids.append(nxt)
            cur = nxt
        return (ids, lgs) if return_logits else ids


def apply_penalty(lg, generated, W, penalty):
    """models/decoder/decoder.py:348-351: `for token in set(generated_tokens[0][-W:])` iterates 0-d tensors,
    whose hash is their identity, so the set keeps duplicates and a token seen k times in the window has
    its logit divided k times (in place, x / penalty each time, fp32)."""
    p = np.float32(penalty)
    for t in generated[-W:]:
        lg[t] = np.float32(lg[t] / p)
    return lg


# ============================================================ codec (models/decoder/ticodec/*)
def conv1d(x, w, b, dilation=1, padding=0, stride=1):
    """x [Cin, T], w [Cout, Cin, k] -> [Cout, T'] (b may be None)."""
    Cin, T = x.shape
    Cout, _, k = w.shape
    xp = np.pad(x, ((0, 0), (padding, padding)))
    To = (xp.shape[1] - dilation * (k - 1) - 1) // stride + 1
    cols = np.stack([xp[:, j * dilation:j * dilation + (To - 1) * stride + 1:stride] for j in range(k)], axis=1)
    y = w.reshape(Cout, Cin * k) @ cols.reshape(Cin * k, To)
    return (y if b is None else y + b[:, None]).astype(F32)


def conv_transpose1d(x, w, b, stride, padding):
    """torch ConvTranspose1d: x [Cin, T], w [Cin, Cout, k]."""
    Cin, T = x.shape
    _, Cout, k = w.shape
    full = (T - 1) * stride + k
    y = np.zeros((Cout, full), F32)
    for j in range(k):
        y[:, j:j + (T - 1) * stride + 1:stride] += w[:, :, j].T @ x
    y = y[:, padding:full - padding]
    return (y + b[:, None]).astype(F32)


class Codec:
    """VQVAE.forward = Quantizer.embed + embed_gst + Generator (vqvae.py:37-42, models.py:211-242,661-715)."""

    def __init__(self, W, cfg):
        self.W, self.h = W, cfg["codec_json"]

    def embed(self, ids):
        assert self.h["residul_layer"] == 1 and self.h["n_code_groups"] == 1
        return self.W["codec.quantizer.quantizer_modules.0.embedding.weight"][np.asarray(ids)].T.astype(F32)

    def global_features(self, gt=None):
        gt = self.h["global_tokens"] if gt is None else gt
        return np.concatenate([self.W[f"codec.quantizer.quantizer_modules_globaltokens.{j}.embedding.weight"][t]
                               for j, t in enumerate(gt)]).astype(F32)

    def generate(self, x, g):
        h, W, p = self.h, self.W, "codec.generator."
        x = conv1d(x, W[p + "conv_pre.weight"], W[p + "conv_pre.bias"], padding=3)
        nk = len(h["resblock_kernel_sizes"])
        for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
            x = leaky(x)
            x = conv_transpose1d(x, W[p + f"ups.{i}.weight"], W[p + f"ups.{i}.bias"], u, (k - u) // 2)
            xs = None
            for j, (kk, dil) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
                r = f"{p}resblocks.{i * nk + j}."
                y = x
                for m, d in enumerate(dil):
                    t = conv1d(leaky(y), W[r + f"convs1.{m}.weight"], W[r + f"convs1.{m}.bias"], d,
                               (kk * d - d) // 2)
                    t = conv1d(leaky(t), W[r + f"convs2.{m}.weight"], W[r + f"convs2.{m}.bias"], 1, (kk - 1) // 2)
                    y = t + y
                xs = y if xs is None else xs + y
            x = (xs / F32(nk)).astype(F32)
            if x.shape[0] == g.shape[0]:
                x = x + g[:, None]
        x = leaky(x)
        x = conv1d(x, W[p + "conv_post.weight"], W[p + "conv_post.bias"], padding=3)
        return np.tanh(x[0]).astype(F32)

    def __call__(self, ids, gt=None):
        return self.generate(self.embed(ids), self.global_features(gt))


# ============================================================ codec encoder (VQVAE.encode)
def group_norm(x, G, w, b, eps=1e-6):
    """torch GroupNorm over x [C, T]: statistics per group of C/G channels x T, then the affine."""
    C, T = x.shape
    g = x.reshape(G, -1).astype(np.float64)
    mu = g.mean(1, keepdims=True)
    var = g.var(1, keepdims=True)
    y = ((g - mu) / np.sqrt(var + eps)).reshape(C, T)
    return (y * w[:, None] + b[:, None]).astype(F32)


def vq_nearest(x, E):
    """Quantizer_module.forward (models/decoder/ticodec/models.py:531-537): rows of x [N, D] to the
    nearest codebook row by d = |x|^2 + |e|^2 - 2 x.e (argmin, first on ties) -> (ids, E[ids])."""
    d = (x * x).sum(1, keepdims=True) + (E * E).sum(1)[None] - 2 * (x @ E.T)
    ids = np.argmin(d, 1)
    return ids, E[ids]


class CodecEncoder:
    """VQVAE.encode (models/decoder/ticodec/vqvae.py:44-57) = Encoder.forward (models.py:429-522, weight
    norm removed) + Quantizer.forward (models.py:639-659: residual VQ over `residul_layer` layers of
    `n_code_groups` groups, then the global-token VQ).  Returns (local ids [T', layers*groups],
    global ids [global_code_num]) for one waveform [T]."""

    def __init__(self, W, h):
        self.W, self.h = W, h

    def resblock(self, x, r, k, dil):
        """ResBlock1 (models.py:59-131): y = conv2(leaky(conv1(leaky(y)))) + y per dilation."""
        W = self.W
        for m, d in enumerate(dil):
            t = conv1d(leaky(x), W[r + f"convs1.{m}.weight"], W[r + f"convs1.{m}.bias"], d, (k * d - d) // 2)
            t = conv1d(leaky(t), W[r + f"convs2.{m}.weight"], W[r + f"convs2.{m}.bias"], 1, (k - 1) // 2)
            x = (t + x).astype(F32)
        return x

    def gte(self, x):
        """GlobalTokenEncoder (models.py:22-57): 3 x (conv, stride s, no bias, leaky 0.1), mean over
        time, Linear + leaky 0.1, BatchNorm1d (eval)."""
        W, p = self.W, "codec.encoder.GlobalTokenEncoder."
        _, _, _, k, st = self.h["global_feature_conv"]
        for i in (0, 2, 4):
            x = leaky(conv1d(x, W[p + f"conv.{i}.weight"], None, 1, (k - st) // 2, st))
        v = x.mean(1).astype(F32)
        v = leaky(linear(v[None], W[p + "fn.0.weight"], W[p + "fn.0.bias"])[0])
        rm, rv = W[p + "fn.2.running_mean"], W[p + "fn.2.running_var"]
        return ((v - rm) / np.sqrt(rv + F32(1e-5)) * W[p + "fn.2.weight"] + W[p + "fn.2.bias"]).astype(F32)

    def encoder(self, wav):
        h, W, p = self.h, self.W, "codec.encoder."
        x = conv1d(np.asarray(wav, F32)[None], W[p + "conv_pre.weight"], W[p + "conv_pre.bias"], 1, 3)
        nk = len(h["resblock_kernel_sizes"])
        stages = list(reversed(list(zip(h["upsample_rates"], h["upsample_kernel_sizes"]))))
        ks = list(reversed(h["resblock_kernel_sizes"]))
        ds = list(reversed(h["resblock_dilation_sizes"]))
        gfeat = None
        for i, (u, k) in enumerate(stages):
            x = leaky(x)
            x = conv1d(x, W[p + f"ups.{i}.weight"], W[p + f"ups.{i}.bias"], 1, (k - u) // 2, u)
            C = x.shape[0]
            xs = None
            for j in range(nk):
                r = f"{p}resblocks.{i * nk + j}."
                y = self.resblock(x, r, ks[j], ds[j])
                xs = y if xs is None else (xs + y).astype(F32)
                n = f"{p}normalize.{i * nk + j}."
                xs = group_norm(xs, C // 16, W[n + "weight"], W[n + "bias"])
            x = (xs / F32(nk)).astype(F32)
            if i == len(stages) // 2 - 1:
                gfeat = self.gte(x)
        x = leaky(x, 0.01)   # F.leaky_relu default slope (models.py:496)
        return conv1d(x, W[p + "conv_post.weight"], W[p + "conv_post.bias"], 1, 1), gfeat

    def quantize(self, c, gfeat):
        h, W, q = self.h, self.W, "codec.quantizer."
        G = h["n_code_groups"]
        names = ["quantizer_modules", "quantizer_modules2", "quantizer_modules3", "quantizer_modules4"]
        res = c.T.astype(F32)                     # [T', 512]
        local = []
        for li in range(h["residul_layer"]):
            parts = np.split(res, G, axis=1)
            zq = []
            for g, xg in enumerate(parts):
                ids, z = vq_nearest(xg, W[q + f"{names[li]}.{g}.embedding.weight"])
                local.append(ids)
                zq.append(z)
            z = np.concatenate(zq, 1)
            quant = (res + (z - res)).astype(F32)  # straight-through form, rounded as the reference's
            res = (res - quant).astype(F32)
        gn = h["global_code_num"]
        gids = []
        for g, xg in enumerate(np.split(gfeat[None], gn, axis=1)):
            ids, _ = vq_nearest(xg, W[q + f"quantizer_modules_globaltokens.{g}.embedding.weight"])
            gids.append(int(ids[0]))
        return np.stack(local, -1), np.array(gids)

    def __call__(self, wav):
        c, g = self.encoder(wav)
        return self.quantize(c, g)
