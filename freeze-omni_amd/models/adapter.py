"""CNNSubsampling facade (reference: models/adapter.py:72-157) over fo.speech.AdapterEngine."""
import torch


class CNNSubsampling:
    """forward(x, mask_pad, cache=None, return_cache=False) with the reference's semantics; x is
    [B, T, enc_out_dim] on the device, the cache an opaque carried-frame handle."""

    def __init__(self, engine):
        self.engine = engine
        self.kernel_size = engine.k
        self.cnn_num = 1

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
