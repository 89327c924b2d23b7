"""Parameter name/shape inventories (reference state_dict keys) for a config (TEST INFRASTRUCTURE).

Names follow the reference modules: models/audioLLM.py (encoder_user/system, adpter_user/system,
predictor_head, llm_decoder.*), models/decoder/decoder.py (LLM2TTSCodecAR, prefixed 'tts.'),
models/decoder/ticodec/models.py Generator/Quantizer (prefixed 'codec.generator.' / 'codec.quantizer.').
tests/test_oracle_golden.py checks them against the names the reference itself produced.
"""


def encoder_shapes(cfg, ident):
    ty = cfg["train_yaml"]
    sub = ty["encoder_conf"]["para_conf"]["subsampling"]
    tr = ty["encoder_conf"]["para_conf"]["transformer"]
    C = sub["subsampling-output-dim"]
    idim = sub["subsampling-input-dim"]
    f = ((idim - 1) // 2 - 1) // 2
    d = tr["transformer-attention-dim"]
    h = tr["transformer-attention-heads"]
    ff = tr["transformer-linear-units"]
    p = f"encoder_{ident}."
    s = {p + "global_cmvn.mean": [idim], p + "global_cmvn.istd": [idim],
         p + "enc.0.core.conv.0.weight": [C, 1, 3, 3], p + "enc.0.core.conv.0.bias": [C],
         p + "enc.0.core.conv.2.weight": [C, C, 3, 3], p + "enc.0.core.conv.2.bias": [C],
         p + "enc.0.core.out.0.weight": [C, C * f], p + "enc.0.core.out.0.bias": [C],
         p + "enc.1.embed.0.weight": [d, tr["transformer-input-dim"]], p + "enc.1.embed.0.bias": [d],
         p + "enc.1.embed.1.weight": [d], p + "enc.1.embed.1.bias": [d],
         p + "enc.1.after_norm.weight": [d], p + "enc.1.after_norm.bias": [d]}
    for i in range(tr["transformer-num-blocks"]):
        q = f"{p}enc.1.encoders.{i}."
        s[q + "self_attn.pos_bias_u"] = [h, d // h]
        s[q + "self_attn.pos_bias_v"] = [h, d // h]
        for n in ("linear_q", "linear_k", "linear_v", "linear_out"):
            s[q + f"self_attn.{n}.weight"] = [d, d]
            s[q + f"self_attn.{n}.bias"] = [d]
        s[q + "self_attn.linear_pos.weight"] = [d, d]
        s[q + "feed_forward.w_1.weight"] = [ff, d]
        s[q + "feed_forward.w_1.bias"] = [ff]
        s[q + "feed_forward.w_2.weight"] = [d, ff]
        s[q + "feed_forward.w_2.bias"] = [d]
        for n in ("norm1", "norm2"):
            s[q + f"{n}.weight"] = [d]
            s[q + f"{n}.bias"] = [d]
    return s


def adapter_shapes(cfg, ident):
    """CNNSubsampling (models/adapter.py:72-110): one stride-2 conv when 4*d >= L (BatchNorm or
    LayerNorm(2d) per `norm`), else a stride-1 conv d->2d + BatchNorm first and the stride-2 conv
    2d->4d + BatchNorm (cnn_num == 2)."""
    mc = cfg["train_yaml"]["model_conf"]
    d, L, k = mc["enc_out_dim"], mc["llm_embed_dim"], mc["kernel_size"]
    p = f"adpter_{ident}."
    bn = ("weight", "bias", "running_mean", "running_var")
    if 4 * d < L:
        s = {p + "conv1d1.weight": [2 * d, d, k], p + "conv1d1.bias": [2 * d],
             p + "conv1d2.weight": [4 * d, 2 * d, k], p + "conv1d2.bias": [4 * d],
             p + "project.weight": [L, 4 * d], p + "project.bias": [L]}
        for n in bn:
            s[p + f"bn1.{n}"] = [2 * d]
            s[p + f"bn2.{n}"] = [4 * d]
        return s
    s = {p + "conv1d2.weight": [2 * d, d, k], p + "conv1d2.bias": [2 * d], p + "project.weight": [L, 2 * d],
         p + "project.bias": [L]}
    for n in (bn if mc.get("norm", "batch") == "batch" else ("weight", "bias")):
        s[p + f"bn2.{n}"] = [2 * d]
    return s


def audiollm_shapes(cfg):
    mc = cfg["train_yaml"]["model_conf"]
    s = {}
    for ident in ("user", "system"):
        s.update(encoder_shapes(cfg, ident))
        s.update(adapter_shapes(cfg, ident))
    s["task_embeddings.weight"] = [10, mc["llm_embed_dim"]]
    s["predictor_head.weight"] = [4, mc["llm_embed_dim"]]
    s["predictor_head.bias"] = [4]
    return s


def llm_shapes(cfg, prefix=""):
    c = cfg["llm"]
    D, H, KV, I, V = (c["hidden_size"], c["num_attention_heads"], c["num_key_value_heads"],
                      c["intermediate_size"], c["vocab_size"])
    hd = D // H
    s = {prefix + "model.embed_tokens.weight": [V, D], prefix + "model.norm.weight": [D],
         prefix + "lm_head.weight": [V, D]}
    for i in range(c["num_hidden_layers"]):
        q = f"{prefix}model.layers.{i}."
        s[q + "self_attn.q_proj.weight"] = [H * hd, D]
        s[q + "self_attn.q_proj.bias"] = [H * hd]
        s[q + "self_attn.k_proj.weight"] = [KV * hd, D]
        s[q + "self_attn.k_proj.bias"] = [KV * hd]
        s[q + "self_attn.v_proj.weight"] = [KV * hd, D]
        s[q + "self_attn.v_proj.bias"] = [KV * hd]
        s[q + "self_attn.o_proj.weight"] = [D, H * hd]
        s[q + "mlp.gate_proj.weight"] = [I, D]
        s[q + "mlp.up_proj.weight"] = [I, D]
        s[q + "mlp.down_proj.weight"] = [D, I]
        s[q + "input_layernorm.weight"] = [D]
        s[q + "post_attention_layernorm.weight"] = [D]
    return s


def _llama_layer(s, q, D, I):
    for n in ("q_proj", "k_proj", "v_proj", "o_proj"):
        s[q + f"self_attn.{n}.weight"] = [D, D]
    s[q + "mlp.gate_proj.weight"] = [I, D]
    s[q + "mlp.up_proj.weight"] = [I, D]
    s[q + "mlp.down_proj.weight"] = [D, I]
    s[q + "input_layernorm.weight"] = [D]
    s[q + "post_attention_layernorm.weight"] = [D]


def tts_shapes(cfg):
    idim, odim, a = cfg["decoder_json"]
    D, I, nb = a["transformer_attention_dim"], a["transformer_linear_units"], a["transformer_num_blocks"]
    s = {"tts.embedding.weight": [odim + 4, idim], "tts.norm.weight": [D],
         "tts.out_fnn.weight": [odim + 4, a["encoder_output_dim"]], "tts.out_fnn.bias": [odim + 4]}
    for i in range(nb // 2):
        _llama_layer(s, f"tts.layers_pre_nn.{i}.", D, I)
    for i in range(nb):
        _llama_layer(s, f"tts.layers.{i}.", D, I)
    if a.get("kv_cache_prefix_finetune", 0):
        for i in range(nb):
            _llama_layer(s, f"tts.layers_prefix.{i}.", D, I)
    return s


def codec_shapes(cfg):
    h = cfg["codec_json"]
    s = {}
    g = 512 // h["n_code_groups"]
    for j in range(h["n_code_groups"]):
        s[f"codec.quantizer.quantizer_modules.{j}.embedding.weight"] = [h["n_codes"], g]
    for j in range(h["global_code_num"]):
        s[f"codec.quantizer.quantizer_modules_globaltokens.{j}.embedding.weight"] = [h["n_codes"],
                                                                                    128 // h["global_code_num"]]
    U = h["upsample_initial_channel"]
    s["codec.generator.conv_pre.weight"] = [U, 512, 7]
    s["codec.generator.conv_pre.bias"] = [U]
    ch = U
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        s[f"codec.generator.ups.{i}.weight"] = [U // 2 ** i, U // 2 ** (i + 1), k]
        s[f"codec.generator.ups.{i}.bias"] = [U // 2 ** (i + 1)]
    nk = len(h["resblock_kernel_sizes"])
    for i in range(len(h["upsample_rates"])):
        ch = U // 2 ** (i + 1)
        for j, (k, dil) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
            r = f"codec.generator.resblocks.{i * nk + j}."
            if h["resblock"] == "1":
                for c in ("convs1", "convs2"):
                    for m in range(len(dil)):
                        s[r + f"{c}.{m}.weight"] = [ch, ch, k]
                        s[r + f"{c}.{m}.bias"] = [ch]
            else:
                for m in range(len(dil)):
                    s[r + f"convs.{m}.weight"] = [ch, ch, k]
                    s[r + f"convs.{m}.bias"] = [ch]
    s["codec.generator.conv_post.weight"] = [1, ch, 7]
    s["codec.generator.conv_post.bias"] = [1]
    return s


def all_shapes(cfg):
    s = audiollm_shapes(cfg)
    s.update(llm_shapes(cfg))
    s.update(tts_shapes(cfg))
    s.update(codec_shapes(cfg))
    return s
