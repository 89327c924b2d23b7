"""CNNSubsampling (reference: models/adapter.py:72-157) over fo.speech.AdapterEngine.

Constructed the reference's way -- CNNSubsampling(enc_out_dim, llm_embed_dim, kernel_size, activation_func,
norm) -- it builds its own engine (every branch the reference builds: cnn_num 1 / 2, BatchNorm / LayerNorm,
ReLU / GELU) with counter-hash synthetic weights under the reference's parameter names, and
load_state_dict(sd) re-packs it from a reference state dict (conv1d1/bn1/conv1d2/bn2/project keys), as
the reference's module would be loaded.  The engine-sharing form CNNSubsampling(engine) is what AudioLLM
uses (the adapter of one replica's engine).
"""
import collections

import torch

_Keys = collections.namedtuple("IncompatibleKeys", ["missing_keys", "unexpected_keys"])


class CNNSubsampling:
    """forward(x, mask_pad, cache=None, return_cache=False) with the reference's semantics; x is
    [B, T, enc_out_dim] on the device, the cache an opaque carried-frame handle."""

    IDENT = "user"   # the engine's parameter prefix: adpter_user.*

    def __init__(self, enc_out_dim=512, llm_embed_dim=4096, kernel_size=5, activation_func="relu", norm="batch",
                 *, device="cuda:0", seed=0, max_sessions=64):
        from fo.speech import AdapterEngine
        if isinstance(enc_out_dim, AdapterEngine):   # the adapter of an existing engine (AudioLLM)
            self._conf = None
            self._set_engine(enc_out_dim)
            return
        if not torch.cuda.is_available():
            raise RuntimeError("CNNSubsampling needs an MI355X (gfx950) device: there is no CPU fallback")
        self._conf = {"enc_out_dim": int(enc_out_dim), "llm_embed_dim": int(llm_embed_dim),
                      "kernel_size": int(kernel_size), "activation_func": activation_func, "norm": norm,
                      "adpter_type": "subsampling"}
        self._device, self._max_sessions = torch.device(device), max_sessions
        from fo.params import adapter_shapes
        from fo.weights import SynthSource
        self._shapes = adapter_shapes(self._cfg(), self.IDENT)
        self._synth = SynthSource(seed, self._shapes, self._device)
        self._set_engine(self._build(self._synth))

    def _cfg(self):
        return {"train_yaml": {"model_conf": self._conf}}

    def _build(self, src):
        from fo.speech import AdapterEngine
        return AdapterEngine(src, self._cfg(), self.IDENT, self._device, self._max_sessions)

    def _set_engine(self, engine):
        self.engine = engine
        self.kernel_size = engine.k
        self.cnn_num = engine.cnn_num

    def state_dict_shapes(self):
        """The reference module's state-dict keys and shapes (models/adapter.py:72-110)."""
        if self._conf is None:
            raise RuntimeError("CNNSubsampling(engine): the weights belong to the engine (load them through it)")
        p = f"adpter_{self.IDENT}."
        return {k[len(p):]: tuple(v) for k, v in self._shapes.items()}

    def load_state_dict(self, state_dict, strict=True):
        """Re-pack the adapter from a reference state dict (tensors or arrays keyed like the reference
        module).  strict: every key must be known with its shape, and none missing (torch semantics)."""
        from fo.weights import CheckpointSource, OverlaySource
        shapes = self.state_dict_shapes()
        unexpected = [k for k in state_dict if k not in shapes]
        missing = [k for k in shapes if k not in state_dict and not k.endswith("num_batches_tracked")]
        bad = [f"{k}: {tuple(torch.as_tensor(v).shape)} != {shapes[k]}" for k, v in state_dict.items()
               if k in shapes and tuple(torch.as_tensor(v).shape) != shapes[k]]
        if bad:
            raise RuntimeError("CNNSubsampling.load_state_dict: size mismatch: " + "; ".join(bad))
        if strict and (unexpected or missing):
            raise RuntimeError(f"CNNSubsampling.load_state_dict: missing {missing}, unexpected {unexpected}")
        p = f"adpter_{self.IDENT}."
        state = {p + k: torch.as_tensor(v).detach().float().cpu() for k, v in state_dict.items() if k in shapes}
        self._set_engine(self._build(OverlaySource(CheckpointSource(state, self._device), self._synth)))
        return _Keys(missing, unexpected)

    def __call__(self, x, mask_pad, cache=None, return_cache=False):
        B, T, D = x.shape
        caches = cache if isinstance(cache, list) and cache and not torch.is_tensor(cache[0]) else None
        if caches is None:
            caches = [self.engine.new_cache() for _ in range(B)] if cache is None else [cache]
        y, To = self.engine(x.reshape(B * T, D).contiguous(), T, caches)
        y = y.view(B, To, -1)
        m = mask_pad[:, :, 0::2]
        if return_cache:
            return y, m, (caches if B > 1 else caches[0])
        return y, m

    forward = __call__
