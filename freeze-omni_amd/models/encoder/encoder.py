"""speechEncoder facade (reference: models/encoder/encoder.py:45-155) over fo.speech.SpeechEncoderEngine.

infer(xs_pad, buffer, buffer_index, buffer_out, pe_index) keeps the reference signature; `buffer` is an
opaque fo.speech.EncoderCache (pass None / the reference's [None]*num_blocks list to start)."""


class speechEncoder:
    def __init__(self, engine):
        self.engine = engine
        self.enc = [None, type("TransformerView", (), {"num_blocks": engine.nb})()]

    def output_size(self):
        return self.engine.d

    def infer(self, xs_pad, buffer, buffer_index=0, buffer_out=None, pe_index=0):
        cache = buffer if hasattr(buffer, "slot") else self.engine.new_cache()
        feats = xs_pad.reshape(-1, xs_pad.shape[-2], xs_pad.shape[-1]).contiguous()
        out, T, pes = self.engine.infer(feats, [cache], [pe_index])
        return out.view(1, T, -1), cache, buffer_index, buffer_out, pes[0]
