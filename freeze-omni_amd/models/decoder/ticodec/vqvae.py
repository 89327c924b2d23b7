"""VQVAE facade (reference: models/decoder/ticodec/vqvae.py:37-57): forward(codes [B, T, 1], global
tokens) -> [B, 1, T*600] PCM through fo.codec.CodecEngine (the engine's configured global tokens);
encode(wav [B, T]) -> (local tokens [B, T', L*G], global tokens [B, 1, n]) through
fo.codec.CodecEncoderEngine when the facade was built with one (the reference's with_encoder=True)."""
import torch


class VQVAE:
    def __init__(self, codec_engine, encoder_engine=None):
        self.engine = codec_engine
        self.encoder = encoder_engine
        self.h = type("H", (), dict((codec_engine or encoder_engine).h))()

    def __call__(self, x, global_style_token=None):
        ids = torch.as_tensor(x).reshape(x.shape[0], -1).to(self.engine.device, torch.int32)
        return self.engine(ids).unsqueeze(1)

    def encode(self, x):
        if self.encoder is None:
            raise RuntimeError("VQVAE built without an encoder (reference: with_encoder=False)")
        local, gst = self.encoder.encode(x)
        return local.long(), gst.long()
