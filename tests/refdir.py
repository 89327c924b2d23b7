"""Builds a model directory in the reference's on-disk layout (test infrastructure).

The real Freeze-Omni / Qwen2-7B checkpoints are not available offline, so the ingestion path
(fo.checkpoint) is exercised on the reference's FILE FORMATS filled with the tiny configuration's
counter-hash weights (oracle/weights.py):
  audiollm/train.yaml, audiollm/final.pt (fork or upstream 'encoder.' / 'adpter.' names),
  audiollm/global_cmvn (json stats), llm/config.json + tokenizer + sharded safetensors + index,
  decoder/model.json + decoder/final.pt ({'model': ...}), codec/model.json + codec/final.pt
  ({'generator': weight-normed convs (weight_g / weight_v), 'quantizer': ..., 'encoder': {}}).
"""
import json
import os
import shutil

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def tiny_weights():
    from oracle import configs
    from oracle.params import all_shapes
    from oracle.weights import SynthCheckpoint
    cfg = configs.get("tiny")
    return cfg, SynthCheckpoint(cfg["seed"], all_shapes(cfg), cfg["overrides"])


def _t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dtype)


def make_reference_dir(dst, upstream_names=False, cmvn_in_ckpt=True, llm_in_final=False):
    from safetensors.torch import save_file
    cfg, W = tiny_weights()
    src = os.path.join(ROOT, "configs", "tiny")
    for sub in ("audiollm", "decoder", "codec", "llm"):
        os.makedirs(os.path.join(dst, sub), exist_ok=True)
    shutil.copy(os.path.join(src, "audiollm", "train.yaml"), os.path.join(dst, "audiollm", "train.yaml"))
    shutil.copy(os.path.join(src, "decoder", "model.json"), os.path.join(dst, "decoder", "model.json"))
    shutil.copy(os.path.join(src, "codec", "model.json"), os.path.join(dst, "codec", "model.json"))
    for f in os.listdir(os.path.join(src, "llm")):
        shutil.copy(os.path.join(src, "llm", f), os.path.join(dst, "llm", f))
    names = list(W.keys())
    # audiollm/final.pt
    final = {}
    for k in names:
        if k.startswith(("encoder_", "adpter_", "predictor_head.", "task_embeddings.")):
            if "global_cmvn" in k and not cmvn_in_ckpt:
                continue
            if upstream_names and k.startswith(("encoder_", "adpter_")):
                head, rest = k.split(".", 1)
                if head.endswith("_user"):
                    final[head[:-len("_user")] + "." + rest] = _t(W[k])
                continue
            final[k] = _t(W[k])
    llm = {k: _t(W[k], torch.bfloat16) for k in names if k.startswith(("model.", "lm_head."))}
    if llm_in_final:
        for k, v in llm.items():
            final["llm_decoder." + k] = v
    torch.save(final, os.path.join(dst, "audiollm", "final.pt"))
    # global_cmvn json stats whose (mean, istd) differ from the checkpoint buffers
    d = len(W["encoder_user.global_cmvn.mean"])
    n = 1000.0
    mean = np.linspace(-1, 1, d)
    var = np.linspace(0.5, 2.0, d)
    with open(os.path.join(dst, "audiollm", "global_cmvn"), "w") as f:
        json.dump({"mean_stat": list(mean * n), "var_stat": list((var + mean ** 2) * n), "frame_num": n}, f)
    # llm: two safetensors shards + index
    keys = sorted(llm)
    half = len(keys) // 2
    shards = {"model-00001-of-00002.safetensors": keys[:half], "model-00002-of-00002.safetensors": keys[half:]}
    wmap = {}
    for fn, ks in shards.items():
        save_file({k: llm[k] for k in ks}, os.path.join(dst, "llm", fn))
        wmap.update({k: fn for k in ks})
    with open(os.path.join(dst, "llm", "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {}, "weight_map": wmap}, f)
    # decoder/final.pt
    torch.save({"model": {k[len("tts."):]: _t(W[k]) for k in names if k.startswith("tts.")}},
               os.path.join(dst, "decoder", "final.pt"))
    # codec/final.pt with weight-normed generator convs
    gen, quant = {}, {}
    for k in names:
        if k.startswith("codec.generator."):
            kk = k[len("codec.generator."):]
            v = W[k]
            if kk.endswith(".weight"):  # weight_norm(dim=0): weight = g * v / ||v||, g = ||v|| folds back to v
                g = np.sqrt((v.reshape(v.shape[0], -1).astype(np.float64) ** 2).sum(1)).reshape(
                    [-1] + [1] * (v.ndim - 1))
                gen[kk + "_g"] = _t(g)
                gen[kk + "_v"] = _t(v)
            else:
                gen[kk] = _t(v)
        elif k.startswith("codec.quantizer."):
            quant[k[len("codec.quantizer."):]] = _t(W[k])
    torch.save({"generator": gen, "quantizer": quant, "encoder": {}}, os.path.join(dst, "codec", "final.pt"))
    return cfg, W, (mean, 1.0 / np.sqrt(var))


def make_reference_dir_real(dst, device, llm_layers=2, enc_blocks=2):
    """configs/real at reduced depth (llm_layers Qwen2 layers with the real 152,064-row embedding and lm_head,
    enc_blocks speech-encoder blocks, the full 4-layer AR decoder and the 512-channel codec) in the reference's
    file formats, filled with the counter-hash weights the T2 goldens were made with (tests/golden/real_*_t2.npz).
    The weights are generated on `device` (fo.weights.SynthSource, k_fill_hash) and written as:
      llm/: config.json + three bf16 safetensors shards + model.safetensors.index.json (HF from_pretrained layout)
      audiollm/: train.yaml + final.pt under the UPSTREAM names 'encoder.*' / 'adpter.*' (one encoder, fanned out
                 to both identities by fo.checkpoint, as the fork's deepcopy does), fp32
      decoder/final.pt {'model': ...}, codec/final.pt {'generator': weight-normed (weight_g, weight_v),
      'quantizer': ..., 'encoder': {}}.
    Returns the configuration dict."""
    import yaml
    from safetensors.torch import save_file

    from fo.weights import SynthSource
    from oracle import configs
    from oracle.params import all_shapes
    cfg = configs.get("real")
    cfg["llm"]["num_hidden_layers"] = llm_layers
    cfg["train_yaml"]["encoder_conf"]["para_conf"]["transformer"]["transformer-num-blocks"] = enc_blocks
    src = os.path.join(ROOT, "configs", "real")
    for sub in ("audiollm", "decoder", "codec", "llm"):
        os.makedirs(os.path.join(dst, sub), exist_ok=True)
    with open(os.path.join(dst, "audiollm", "train.yaml"), "w") as f:
        yaml.safe_dump(cfg["train_yaml"], f)
    with open(os.path.join(dst, "llm", "config.json"), "w") as f:
        json.dump(cfg["llm"], f)
    for f in os.listdir(os.path.join(src, "llm")):
        if f != "config.json":
            shutil.copy(os.path.join(src, "llm", f), os.path.join(dst, "llm", f))
    shutil.copy(os.path.join(src, "decoder", "model.json"), os.path.join(dst, "decoder", "model.json"))
    shutil.copy(os.path.join(src, "codec", "model.json"), os.path.join(dst, "codec", "model.json"))
    shapes = all_shapes(cfg)
    W = SynthSource(cfg["seed"], shapes, device, cfg["overrides"])

    def host(k, dtype=torch.float32):
        return W.get(k, torch.float32).to(dtype).cpu().contiguous()

    names = sorted(shapes)
    # llm: three bf16 shards (layers 0, layers 1.., embed / norm / lm_head) + the index
    wmap = {}
    llm_names = [k for k in names if k.startswith(("model.", "lm_head."))]
    groups = {"model-00001-of-00003.safetensors": [k for k in llm_names if k.startswith("model.layers.0.")],
              "model-00002-of-00003.safetensors": [k for k in llm_names if k.startswith("model.layers.")
                                                   and not k.startswith("model.layers.0.")],
              "model-00003-of-00003.safetensors": [k for k in llm_names if not k.startswith("model.layers.")]}
    for fn, ks in groups.items():
        save_file({k: host(k, torch.bfloat16) for k in ks}, os.path.join(dst, "llm", fn))
        wmap.update({k: fn for k in ks})
    with open(os.path.join(dst, "llm", "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": 0}, "weight_map": wmap}, f)
    # audiollm/final.pt with the upstream single-encoder names
    final = {}
    for k in names:
        if k.startswith(("encoder_user.", "adpter_user.")):
            head, rest = k.split(".", 1)
            final[head[:-len("_user")] + "." + rest] = host(k)
        elif k.startswith(("predictor_head.", "task_embeddings.")):
            final[k] = host(k)
    torch.save(final, os.path.join(dst, "audiollm", "final.pt"))
    torch.save({"model": {k[len("tts."):]: host(k) for k in names if k.startswith("tts.")}},
               os.path.join(dst, "decoder", "final.pt"))
    gen, quant = {}, {}
    for k in names:
        if k.startswith("codec.generator."):
            kk, v = k[len("codec.generator."):], host(k)
            if kk.endswith(".weight"):   # weight_norm(dim=0) with g = ||v||: folds back to v (up to rounding)
                gen[kk + "_g"] = v.double().reshape(v.shape[0], -1).norm(dim=1).reshape(
                    [-1] + [1] * (v.dim() - 1)).float()
                gen[kk + "_v"] = v
            else:
                gen[kk] = v
        elif k.startswith("codec.quantizer."):
            quant[k[len("codec.quantizer."):]] = host(k)
    torch.save({"generator": gen, "quantizer": quant, "encoder": {}}, os.path.join(dst, "codec", "final.pt"))
    del W
    torch.cuda.empty_cache()
    return cfg
