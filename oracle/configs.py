"""Model geometries used by goldens, oracle, tests and bench (TEST INFRASTRUCTURE + bench config).

Each config is written in the reference's own on-disk formats so the same loaders parse
them and real checkpoints:
  * `train_yaml`  - <model_path>/audiollm/train.yaml   (models/pipeline.py:21-24, models/utils.py:30-49)
  * `llm`         - Qwen2 config.json fields             (models/audioLLM.py:70-74)
  * `decoder_json`- <model_path>/decoder/model.json = [idim, odim, args] (models/decoder/llm2tts.py:32-39)
  * `codec_json`  - <model_path>/codec/model.json        (models/decoder/ticodec/vqvae.py:22-25)

TINY: small enough for the reference to run on CPU in seconds (goldens).
REAL: the geometry the benchmark runs.  Qwen2-7B-Instruct dims are public; the encoder,
speech decoder and codec dims are not in the reference snapshot (checkpoints absent), so
REAL uses the paper's stated sizes (24-block, ~350M-param encoder at 12.5 Hz; 4-layer
896-wide AR decoder) and HiFi-GAN-style codec settings with a 600x upsampling product
(models/decoder/llm2tts.py:132).  These assumptions are listed in DESIGN.md.
"""
import copy

CHAT_TEMPLATE = ("<|im_start|>system\nYou are a helpful assistant.<|im_end|>\n<|im_start|>user\n<audio>"
                 "<|im_end|>\n<|im_start|>assistant\n")


def _encoder_conf(d_sub, d, heads, ff, blocks, chunk, left):
    return {
        "overview_conf": {"encoder-input-dim": 80, "encoder-output-dim": d,
                          "encoder-layer-config": "subsampling-transformer"},
        "para_conf": {
            "subsampling": {"subsampling-rate": 4, "subsampling-input-dim": 80,
                            "subsampling-output-dim": d_sub, "subsampling-dropout-rate": 0.1},
            "transformer": {"transformer-input-dim": d_sub, "transformer-output-dim": d,
                            "transformer-attention-dim": d, "transformer-attention-heads": heads,
                            "transformer-linear-units": ff, "transformer-num-blocks": blocks,
                            "transformer-dropout-rate": 0.1, "transformer-attention-dropout-rate": 0.0,
                            "transformer-positional-dropout-rate": 0.1, "transformer-input-layer": "linear",
                            "transformer-pos-enc-class": "rel-enc", "transformer-normalize-before": True,
                            "transformer-concat-after": False, "transformer-positionwise-layer-type": "linear",
                            "transformer-chunk_size": chunk, "transformer-left_chunks": left,
                            "transformer-dynamic-chunks": True},
        },
    }


def _model_conf(d_enc, d_llm, heads, kv_heads, kernel):
    return {"enc_out_dim": d_enc, "llm_embed_dim": d_llm, "kernel_size": kernel, "adpter_type": "subsampling",
            "activation_func": "relu", "norm": "batch", "llm_head_num": heads, "num_key_value_heads": kv_heads,
            "task_type": "prompt", "freeze_llm": True, "freeze_encoder": True, "freeze_adpter": True,
            "chat_template": CHAT_TEMPLATE, "predict_usr_state": 4, "chunk_size": 2}


def _decoder_args(d, heads, ff, blocks, odim):
    return {"idim": d, "odim": odim, "encoder_pre_norm_type": "ln", "encoder_drop_rate": 0.1,
            "encoder_criterion": "ce", "encoder_upsample_rate": 1, "kv_cache_prefix_finetune": 1,
            "transformer_attention_dim": d, "transformer_linear_units": ff, "transformer_num_blocks": blocks,
            "transformer_attention_heads": heads, "transformer_dropout_rate": 0.1, "encoder_output_dim": d}


TINY = {
    "name": "tiny",
    "seed": 20250824,
    "train_yaml": {"input_dim": 80, "output_dim": 384, "is_json_cmvn": True,
                   "encoder_conf": _encoder_conf(32, 32, 4, 64, 2, 4, 2),
                   "model_conf": _model_conf(32, 128, 4, 2, 5)},
    "llm": {"hidden_size": 128, "intermediate_size": 256, "num_hidden_layers": 2, "num_attention_heads": 4,
            "num_key_value_heads": 2, "vocab_size": 384, "rms_norm_eps": 1e-6, "rope_theta": 1000000.0,
            "max_position_embeddings": 4096, "tie_word_embeddings": False},
    "decoder_json": [128, 60, _decoder_args(128, 4, 256, 4, 60)],
    "codec_json": {"resblock": "1", "upsample_rates": [10, 6, 10], "upsample_kernel_sizes": [20, 12, 20],
                   "upsample_initial_channel": 256, "resblock_kernel_sizes": [3, 5],
                   "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5]], "n_codes": 60, "n_code_groups": 1,
                   "residul_layer": 1, "global_code_num": 8, "codebook_loss_lambda": 1.0,
                   "commitment_loss_lambda": 0.25, "global_tokens": [3, 17, 41, 8, 22, 59, 0, 33]},
    # TTS out_fnn and the state head are scaled up so greedy decisions are well separated
    "overrides": {"out_fnn.weight": (0.0, 0.35), "predictor_head.weight": (0.0, 0.2), "lm_head.weight": (0.0, 0.3)},
}

REAL = {
    "name": "real",
    "seed": 7,
    "train_yaml": {"input_dim": 80, "output_dim": 152064, "is_json_cmvn": True,
                   "encoder_conf": _encoder_conf(1024, 1024, 16, 4096, 24, 4, 16),
                   "model_conf": _model_conf(1024, 3584, 28, 4, 5)},
    "llm": {"hidden_size": 3584, "intermediate_size": 18944, "num_hidden_layers": 28, "num_attention_heads": 28,
            "num_key_value_heads": 4, "vocab_size": 152064, "rms_norm_eps": 1e-6, "rope_theta": 1000000.0,
            "max_position_embeddings": 32768, "tie_word_embeddings": False},
    "decoder_json": [896, 1024, _decoder_args(896, 14, 4864, 4, 1024)],
    "codec_json": {"resblock": "1", "upsample_rates": [5, 5, 4, 3, 2], "upsample_kernel_sizes": [10, 10, 8, 6, 4],
                   "upsample_initial_channel": 512, "resblock_kernel_sizes": [3, 7, 11],
                   "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]], "n_codes": 1024,
                   "n_code_groups": 1, "residul_layer": 1, "global_code_num": 8, "codebook_loss_lambda": 1.0,
                   "commitment_loss_lambda": 0.25, "global_tokens": [473, 975, 120, 10, 344, 655, 12, 888]},
    "overrides": {"out_fnn.weight": (0.0, 0.1), "lm_head.weight": (0.0, 0.05)},
}


def get(name):
    return copy.deepcopy({"tiny": TINY, "real": REAL}[name])


# Qwen2 special-token ids used when no tokenizer files are present (bench on synthetic weights).
QWEN2_IDS = {"<|im_start|>": 151644, "<|im_end|>": 151645, "\n": 198, "system": 8948, "user": 872,
             "assistant": 77091}


def write_model_dirs(cfg, root):
    """Write a reference-layout model directory for `cfg` (what freeze-omni_amd loads):
    <root>/audiollm/train.yaml, decoder/model.json, codec/model.json, synthetic.json, llm/config.json."""
    import json
    import os

    import yaml
    os.makedirs(os.path.join(root, "audiollm"), exist_ok=True)
    os.makedirs(os.path.join(root, "decoder"), exist_ok=True)
    os.makedirs(os.path.join(root, "codec"), exist_ok=True)
    os.makedirs(os.path.join(root, "llm"), exist_ok=True)
    with open(os.path.join(root, "audiollm", "train.yaml"), "w") as f:
        yaml.safe_dump(cfg["train_yaml"], f, sort_keys=True)
    with open(os.path.join(root, "decoder", "model.json"), "w") as f:
        json.dump(cfg["decoder_json"], f, indent=1)
    with open(os.path.join(root, "codec", "model.json"), "w") as f:
        json.dump(cfg["codec_json"], f, indent=1)
    with open(os.path.join(root, "synthetic.json"), "w") as f:
        json.dump({"seed": cfg["seed"], "overrides": cfg["overrides"], "name": cfg["name"]}, f, indent=1)
    llm = dict(cfg["llm"], architectures=["Qwen2ForCausalLM"], model_type="qwen2", torch_dtype="bfloat16")
    with open(os.path.join(root, "llm", "config.json"), "w") as f:
        json.dump(llm, f, indent=1)


if __name__ == "__main__":
    import os
    import shutil
    import sys
    out = sys.argv[1] if len(sys.argv) > 1 else "configs"
    for n in ("tiny", "real"):
        write_model_dirs(get(n), os.path.join(out, n))
    tok = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "tiny_tokenizer")
    for f in os.listdir(tok):
        shutil.copy(os.path.join(tok, f), os.path.join(out, "tiny", "llm", f))
