"""Counter-hash synthetic weights (TEST INFRASTRUCTURE - oracle side).

Real Freeze-Omni / Qwen2-7B checkpoints are not available offline, so every weight used by
the goldens, the oracle and the GPU benchmark is a pure function of (seed, parameter name,
element index):

    key   = splitmix64(seed * 0x100000001B3 ^ crc32(name))
    u_i   = (splitmix64(key + i) >> 40) / 2**24                in [0, 1), exact in fp32
    w_i   = bf16_rne( center + scale * (2*u_i - 1) )           fp32 ops, one rounding each

The GPU fill kernel (fo_fill_hash in freeze-omni_amd/csrc/fo_misc.hip) evaluates exactly
the same expression, so CPU oracle and MI355X path see bit-identical weights and the
reference run in tests/golden/make_golden.py is initialised from the same values.
Parameter names are the reference's state_dict keys.
"""
import zlib

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_G = 0x9E3779B97F4A7C15
_M1 = 0xBF58476D1CE4E5B9
_M2 = 0x94D049BB133111EB


def _splitmix64_int(x):
    x = (x + _G) & 0xFFFFFFFFFFFFFFFF
    z = x
    z = ((z ^ (z >> 30)) * _M1) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * _M2) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def tensor_key(seed, name):
    return _splitmix64_int(((int(seed) * 0x100000001B3) ^ zlib.crc32(name.encode())) & 0xFFFFFFFFFFFFFFFF)


def _splitmix64_np(x):
    with np.errstate(over="ignore"):
        x = x + np.uint64(_G)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_M2)
        return z ^ (z >> np.uint64(31))


def bf16_round(a):
    """Round-to-nearest-even fp32 -> bf16 -> fp32 (NaN-free inputs)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    u = (u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)
    return (u.astype(np.uint32) << np.uint32(16)).view(np.float32).reshape(a.shape)


def hash_uniform(seed, name, shape, center=0.0, scale=1.0, out_bf16=True, chunk=1 << 24):
    """Elementwise, so it is evaluated in chunks of `chunk` elements: a 545M-element Qwen2-7B embedding
    table then needs ~0.3 GB of uint64 temporaries instead of ~15 GB."""
    n = int(np.prod(shape)) if len(shape) else 1
    key = np.uint64(tensor_key(seed, name))
    out = np.empty(n, dtype=np.float32)
    for i0 in range(0, n, chunk):
        idx = np.arange(i0, min(n, i0 + chunk), dtype=np.uint64)
        with np.errstate(over="ignore"):
            v = _splitmix64_np(key + idx)
        u = (v >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        w = (np.float32(2.0) * u - np.float32(1.0)) * np.float32(scale) + np.float32(center)
        w = w.astype(np.float32)
        out[i0:i0 + len(w)] = bf16_round(w) if out_bf16 else w
    return out.reshape(shape)


def synth_rows(seed, name, shape, rows, overrides=None):
    """Rows `rows` of the 2-D parameter synth_param(seed, name, shape) without materialising the rest
    (e.g. a few embedding rows or lm_head rows of the 152,064 x 3584 Qwen2 tables)."""
    c, s = init_spec(name, tuple(shape), overrides)
    rows = np.asarray(rows, dtype=np.int64)
    K = int(shape[1])
    if s == 0.0:
        return np.full((len(rows), K), c, dtype=np.float32)
    key = np.uint64(tensor_key(seed, name))
    idx = (rows[:, None] * K + np.arange(K)[None, :]).astype(np.uint64)
    with np.errstate(over="ignore"):
        v = _splitmix64_np(key + idx)
    u = (v >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    w = ((np.float32(2.0) * u - np.float32(1.0)) * np.float32(s) + np.float32(c)).astype(np.float32)
    return bf16_round(w).reshape(len(rows), K)


def init_spec(name, shape, overrides=None):
    """(center, scale) used for parameter `name` of a given shape (shared with the GPU path)."""
    if overrides:
        for pat, cs in overrides.items():
            if pat in name:
                return cs
    last = name.rsplit(".", 1)[-1]
    if "global_cmvn.mean" in name:
        return (8.0, 2.0)
    if "global_cmvn.istd" in name:
        return (0.25, 0.05)
    if last == "running_var":
        return (1.0, 0.3)
    if last == "running_mean":
        return (0.0, 0.1)
    if last == "num_batches_tracked":
        return (0.0, 0.0)
    if "pos_bias" in name:
        return (0.0, 0.1)
    if last == "bias":
        return (0.0, 0.05)
    if len(shape) == 1:  # LayerNorm / RMSNorm / BN gains
        return (1.0, 0.1)
    if "embed" in name or "embedding" in name:
        return (0.0, 0.5)
    if ".ups." in name:  # ConvTranspose1d weight [C_in, C_out, k]
        return (0.0, float(1.0 / np.sqrt(shape[0])))
    fan_in = int(np.prod(shape[1:]))
    return (0.0, float(1.0 / np.sqrt(fan_in)))


def synth_param(seed, name, shape, overrides=None):
    c, s = init_spec(name, tuple(shape), overrides)
    if s == 0.0:
        return np.full(shape, c, dtype=np.float32)
    return hash_uniform(seed, name, tuple(shape), c, s)


class SynthCheckpoint(dict):
    """Lazily materialised name -> np.float32 array mapping for a list of (name, shape)."""

    def __init__(self, seed, shapes, overrides=None):
        super().__init__()
        self.seed = seed
        self.shapes = dict(shapes)
        self.overrides = overrides or {}

    def __missing__(self, name):
        if name not in self.shapes:
            raise KeyError(name)
        v = synth_param(self.seed, name, self.shapes[name], self.overrides)
        self[name] = v
        return v

    def keys(self):  # noqa: D401
        return self.shapes.keys()

    def __contains__(self, name):
        return name in self.shapes
