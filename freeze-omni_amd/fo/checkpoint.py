"""Real-checkpoint ingestion: the reference's model directory -> the engine's weight source.

Reads exactly the files the reference loads, with loaders that execute nothing from the files
(torch.load(weights_only=True), safetensors, JSON / text):

  <model_path>/audiollm/final.pt      AudioLLM state dict        models/pipeline.py:21-30, models/utils.py:11-28
  <model_path>/audiollm/global_cmvn   CMVN stats (json / kaldi)  models/utils.py:31-38, models/encoder/cmvn.py:36-100
  <llm_path>/config.json + *.safetensors (or pytorch_model*.bin)  models/audioLLM.py:70-74 (from_pretrained)
  <model_path>/decoder/final.pt       LLM2TTSCodecAR snapshot    models/decoder/llm2tts.py:41-68
  <model_path>/codec/final.pt         {generator, quantizer, ...} models/decoder/ticodec/vqvae.py:16-35

and serves them under the engine's parameter names (fo/params.py, the fork's state_dict keys, with
'tts.' / 'codec.generator.' / 'codec.quantizer.' prefixes for the speech decoder and codec).

Reference behaviours kept or neutralised:
  * load_checkpoint uses load_state_dict(strict=False) (models/utils.py:20), so a final.pt saved with
    the upstream names 'encoder.*' / 'adpter.*' would silently leave the fork's encoder_user /
    encoder_system / adpter_user / adpter_system random (SURVEY §8(c) latent bug i).  Here upstream
    names are mapped onto BOTH identities (the fork builds encoder_system = deepcopy(encoder),
    models/audioLLM.py:66-67, adpter_system likewise :157), and every parameter the path needs must be
    present with its shape (strict): a missing or mis-shaped tensor raises with the full list.
  * 'llm_decoder.*' entries of final.pt override the HF weights (load_state_dict runs after
    from_pretrained, so the reference behaves the same way).
  * GlobalCMVN comes from the cmvn file, then final.pt's buffers override it if present (the module
    is built from the file and load_state_dict runs afterwards).
  * The codec generator's weight_norm is folded (remove_weight_norm, models/decoder/llm2tts.py:28):
    weight = g * v / ||v||, the norm taken over every dim but 0 (torch weight_norm default dim=0).
"""
import glob
import json
import math
import os

import torch

from .params import all_shapes
from .weights import CheckpointSource


def _torch_load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def load_cmvn(path, is_json):
    """models/encoder/cmvn.py:36-100 (_load_json_cmvn / _load_kaldi_cmvn): (mean, istd) float32."""
    if is_json:
        with open(path) as f:
            st = json.load(f)
        means, var, count = list(st["mean_stat"]), list(st["var_stat"]), st["frame_num"]
    else:
        with open(path) as f:
            head = f.read(2)
            if head == "\0B":
                raise ValueError("kaldi binary cmvn is not supported (recompute with --binary=false)")
            f.seek(0)
            arr = f.read().split()
        if arr[0] != "[" or arr[-2] != "0" or arr[-1] != "]":
            raise ValueError(f"{path}: not a kaldi text cmvn stats file")
        dim = (len(arr) - 4) // 2
        means = [float(v) for v in arr[1:dim + 1]]
        count = float(arr[dim + 1])
        var = [float(v) for v in arr[dim + 2:2 * dim + 2]]
    istd = []
    for i in range(len(means)):
        means[i] /= count
        v = var[i] / count - means[i] * means[i]
        istd.append(1.0 / math.sqrt(max(v, 1.0e-20)))
    return torch.tensor(means, dtype=torch.float32), torch.tensor(istd, dtype=torch.float32)


class _LazyTensors:
    """name -> tensor over safetensors shards, read on first use (the 15 GB Qwen2 never sits in host
    RAM at once); plain dict entries win."""

    def __init__(self):
        self.eager = {}
        self.files = {}   # name -> safetensors file

    def add_safetensors(self, path):
        from safetensors import safe_open
        with safe_open(path, framework="pt") as f:
            for k in f.keys():
                self.files.setdefault(k, path)

    def __contains__(self, k):
        return k in self.eager or k in self.files

    def __getitem__(self, k):
        if k in self.eager:
            return self.eager[k]
        from safetensors import safe_open
        with safe_open(self.files[k], framework="pt") as f:
            return f.get_tensor(k)

    def __setitem__(self, k, v):
        self.eager[k] = v

    def keys(self):
        return set(self.eager) | set(self.files)

    def shape(self, k):
        if k in self.eager:
            return tuple(self.eager[k].shape)
        from safetensors import safe_open
        with safe_open(self.files[k], framework="pt") as f:
            return tuple(f.get_slice(k).get_shape())


def _load_llm(llm_path, state):
    idx = os.path.join(llm_path, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            shards = sorted(set(json.load(f)["weight_map"].values()))
        for s in shards:
            state.add_safetensors(os.path.join(llm_path, s))
        return
    st = sorted(glob.glob(os.path.join(llm_path, "*.safetensors")))
    if st:
        for s in st:
            state.add_safetensors(s)
        return
    bins = sorted(glob.glob(os.path.join(llm_path, "pytorch_model*.bin")))
    if not bins:
        raise FileNotFoundError(f"{llm_path}: no *.safetensors or pytorch_model*.bin")
    for b in bins:
        for k, v in _torch_load(b).items():
            state[k] = v


def _fold_weight_norm(sd):
    """{..., 'x.weight_g', 'x.weight_v'} -> {..., 'x.weight'} (torch remove_weight_norm, dim=0)."""
    out = {}
    for k, v in sd.items():
        if k.endswith(".weight_g"):
            continue
        if k.endswith(".weight_v"):
            base = k[:-len("_v")]
            g = sd[base + "_g"].float()
            v = v.float()
            norm = v.reshape(v.shape[0], -1).norm(dim=1).reshape([-1] + [1] * (v.dim() - 1))
            out[base] = g * v / norm
            continue
        out[k] = v
    return out


def audiollm_state(path):
    """audiollm/final.pt (models/utils.py:11-20) under the engine's names: 'llm_decoder.*' -> the Qwen2
    names, upstream 'encoder.*' / 'adpter.*' -> both identities unless the fork's own key is present."""
    sd = _torch_load(path)
    if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    fork = {k for k in sd if k.startswith(("encoder_user.", "encoder_system.", "adpter_user.", "adpter_system."))}
    state = {}
    for k, v in sd.items():
        if k.startswith("llm_decoder."):
            state[k[len("llm_decoder."):]] = v
        elif k.startswith(("encoder.", "adpter.")):
            head, rest = k.split(".", 1)
            for ident in ("user", "system"):
                nk = f"{head}_{ident}.{rest}"
                if nk not in fork:
                    state[nk] = v
        else:
            state[k] = v
    return state


def reference_state(model_path, llm_path=None, cfg=None):
    """All tensors under the engine's names (lazy for the LLM shards)."""
    llm_path = llm_path or os.path.join(model_path, "llm")
    state = _LazyTensors()
    _load_llm(llm_path, state)
    # ---- audiollm/final.pt (+ global_cmvn)
    ty = (cfg or {}).get("train_yaml", {})
    cmvn_path = os.path.join(model_path, "audiollm", "global_cmvn")
    if os.path.exists(cmvn_path):
        mean, istd = load_cmvn(cmvn_path, bool(ty.get("is_json_cmvn", True)))
        for ident in ("user", "system"):
            state[f"encoder_{ident}.global_cmvn.mean"] = mean
            state[f"encoder_{ident}.global_cmvn.istd"] = istd
    for k, v in audiollm_state(os.path.join(model_path, "audiollm", "final.pt")).items():
        state[k] = v
    # ---- decoder/final.pt
    snap = _torch_load(os.path.join(model_path, "decoder", "final.pt"))
    if isinstance(snap, dict) and "model" in snap:
        snap = snap["model"]
    for k, v in snap.items():
        state["tts." + k] = v
    # ---- codec/final.pt
    ck = _torch_load(os.path.join(model_path, "codec", "final.pt"))
    for part in ("generator", "quantizer"):
        if part not in ck:
            raise KeyError(f"codec/final.pt has no '{part}' entry")
        for k, v in _fold_weight_norm(ck[part]).items():
            state[f"codec.{part}.{k}"] = v
    if "encoder" in ck:  # VQVAE(with_encoder=True) (vqvae.py:33-35): weight norm folded as the generator's
        for k, v in _fold_weight_norm(ck["encoder"]).items():
            state[f"codec.encoder.{k}"] = v
    return state


def load_reference_checkpoints(cfg, model_path, llm_path, device):
    """CheckpointSource over the reference's checkpoint files; strict check of every parameter the
    MI355X path reads (names and shapes from fo/params.py)."""
    state = reference_state(model_path, llm_path, cfg)
    need = all_shapes(cfg)
    if "lm_head.weight" not in state and cfg["llm"].get("tie_word_embeddings", False) \
            and "model.embed_tokens.weight" in state:
        state["lm_head.weight"] = state["model.embed_tokens.weight"]
    missing = [k for k in need if k not in state and not k.startswith("task_embeddings.")]
    bad = [f"{k}: {state.shape(k)} != {tuple(need[k])}" for k in need
           if k in state and state.shape(k) != tuple(need[k])]
    if missing or bad:
        raise RuntimeError("reference checkpoints do not match the model configuration:\n  missing: "
                           + ", ".join(missing[:40]) + (" ..." if len(missing) > 40 else "")
                           + "\n  shape mismatch: " + "; ".join(bad[:40]))
    return CheckpointSource(state, device)

