"""VQVAE facade (reference: models/decoder/ticodec/vqvae.py:37-42): forward(codes [B, T, 1], global
tokens) -> [B, 1, T*600] PCM through fo.codec.CodecEngine (the engine's configured global tokens)."""
import torch


class VQVAE:
    def __init__(self, codec_engine):
        self.engine = codec_engine
        self.h = type("H", (), dict(codec_engine.h))()

    def __call__(self, x, global_style_token=None):
        ids = torch.as_tensor(x).reshape(x.shape[0], -1).to(self.engine.device, torch.int32)
        return self.engine(ids).unsqueeze(1)
