"""VQVAE facade (reference: models/decoder/ticodec/vqvae.py:37-57): forward(codes [B, T, 1], global
tokens [B or 1, 1, n]) -> [B, 1, T*600] PCM through fo.codec.CodecEngine, the global tokens embedded per call and
per row (embed_gst, models.py:703-715) -- the configured h.global_tokens when the caller passes None;
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
        g = None
        if global_style_token is not None:
            gt = torch.as_tensor(global_style_token)
            if gt.reshape(-1).tolist() != list(self.h.global_tokens):   # the configured voice: the engine's default
                g = self.engine.global_feature(gt, ids.shape[0])
        return self.engine(ids, g).unsqueeze(1)

    def encode(self, x):
        if self.encoder is None:
            raise RuntimeError("VQVAE built without an encoder (reference: with_encoder=False)")
        local, gst = self.encoder.encode(x)
        return local.long(), gst.long()
