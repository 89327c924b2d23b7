"""Weight sources for the MI355X path.

The reference loads final.pt / Qwen2 safetensors / decoder & codec checkpoints
(models/utils.py:11-28, models/audioLLM.py:70-74, models/decoder/llm2tts.py:41-68,
models/decoder/ticodec/vqvae.py:16-35).  Those checkpoints are not available offline, so the
benchmark and tests use counter-hash synthetic weights generated ON THE DEVICE (fo_fill_hash),
keyed by the same reference state_dict names; the values are bit-identical to the CPU oracle's
(oracle/weights.py), which lets parity tests regenerate any subset on the host.

CheckpointSource serves real tensors from a name -> tensor mapping (torch.load(weights_only=True)
or safetensors) with the same interface.
"""
import zlib

import torch

from . import ops

_M64 = 0xFFFFFFFFFFFFFFFF


def _splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & _M64
    z = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def tensor_key(seed, name):
    return _splitmix64(((int(seed) * 0x100000001B3) ^ zlib.crc32(name.encode())) & _M64)


def init_spec(name, shape, overrides=None):
    """(center, scale) of the synthetic uniform for a parameter (same rule table as the oracle)."""
    if overrides:
        for pat, cs in overrides.items():
            if pat in name:
                return tuple(cs)
    last = name.rsplit(".", 1)[-1]
    rules = [
        ("global_cmvn.mean" in name, (8.0, 2.0)),
        ("global_cmvn.istd" in name, (0.25, 0.05)),
        (last == "running_var", (1.0, 0.3)),
        (last == "running_mean", (0.0, 0.1)),
        (last == "num_batches_tracked", (0.0, 0.0)),
        ("pos_bias" in name, (0.0, 0.1)),
        (last == "bias", (0.0, 0.05)),
        (len(shape) == 1, (1.0, 0.1)),
        ("embed" in name or "embedding" in name, (0.0, 0.5)),
    ]
    for cond, cs in rules:
        if cond:
            return cs
    if ".ups." in name:
        return (0.0, float(1.0 / (shape[0] ** 0.5)))
    fan_in = 1
    for s in shape[1:]:
        fan_in *= int(s)
    return (0.0, float(1.0 / fan_in ** 0.5))


class SynthSource:
    """Synthetic weights materialised on the device by fo_fill_hash."""

    def __init__(self, seed, shapes, device, overrides=None):
        self.seed, self.shapes, self.device = seed, dict(shapes), torch.device(device)
        self.overrides = overrides or {}

    def __contains__(self, name):
        return name in self.shapes

    def get(self, name, dtype=torch.float32):
        shape = tuple(self.shapes[name])
        c, s = init_spec(name, shape, self.overrides)
        t = torch.empty(shape, dtype=dtype, device=self.device)
        if s == 0.0:
            return t.fill_(c)
        return ops.fill_hash(t, tensor_key(self.seed, name), c, s)


class CheckpointSource:
    """Real weights from a mapping name -> tensor (CPU); values are moved to the device on demand."""

    def __init__(self, state, device):
        self.state, self.device = state, torch.device(device)

    def __contains__(self, name):
        return name in self.state

    def get(self, name, dtype=torch.float32):
        return self.state[name].to(device=self.device, dtype=dtype)


class OverlaySource:
    """`primary` wins where it has the name, `fallback` serves the rest (a checkpoint loaded over an
    engine that was built from another source: models/utils.py:load_checkpoint)."""

    def __init__(self, primary, fallback):
        self.primary, self.fallback = primary, fallback

    def __contains__(self, name):
        return name in self.primary or name in self.fallback

    def get(self, name, dtype=torch.float32):
        return (self.primary if name in self.primary else self.fallback).get(name, dtype)


class ReceiveSource:
    """Shapes only: every get() returns an UNINITIALISED tensor of the parameter's shape.  A replica that
    receives its frozen weights from rank 0 (fo.replica.broadcast_frozen) builds its packed layouts from
    this source: no checkpoint read, no hash fill -- the broadcast then overwrites every frozen tensor
    (derived ones such as packed GEMM weights and folded BatchNorm affines included)."""

    def __init__(self, shapes, device):
        self.shapes, self.device = dict(shapes), torch.device(device)

    def __contains__(self, name):
        return name in self.shapes

    def get(self, name, dtype=torch.float32):
        return torch.empty(tuple(self.shapes[name]), dtype=dtype, device=self.device)
