"""LLM2TTSCodecAR facade (reference: models/decoder/decoder.py:314-367): infer() generator of codec ids."""
import torch

from fo import ops


class LLM2TTSCodecAR:
    def __init__(self, tts_engine):
        self.engine = tts_engine
        self.vocab_size = tts_engine.vocab

    def infer(self, hidden, top_k, prefix, penalty_window_size=-1, penalty=1.1, max_tokens=1000):
        if penalty_window_size > 0:
            raise NotImplementedError("repetition penalty is not on the MI355X path")
        e = self.engine
        dev = e.device
        h = hidden.reshape(-1, hidden.shape[-1]).to(dev, torch.float32).contiguous()
        p = None if prefix is None else prefix.reshape(-1, hidden.shape[-1]).to(dev, torch.float32).contiguous()
        seqs = e.start([(h, p)])
        cur = torch.full((1,), e.sos, dtype=torch.int32, device=dev)
        k = torch.tensor([top_k], dtype=torch.int32).to(dev)
        out = torch.empty(1, dtype=torch.int32, device=dev)
        try:
            for i in range(max_tokens):
                ops.sample(e.step(seqs, cur), e.vocab + 4, out, k,
                           step=torch.full((1,), i, dtype=torch.int32, device=dev))
                t = int(out.item())
                if t == e.eos:
                    break
                yield torch.tensor([[t]], device=dev)
                cur = out.clone()
        finally:
            e.free(seqs)
