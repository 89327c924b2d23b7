"""LLM2TTSCodecAR facade (reference: models/decoder/decoder.py:314-367): infer() generator of codec ids."""
import torch

from fo import ops
from fo.tts import penalty_ring


class LLM2TTSCodecAR:
    def __init__(self, tts_engine):
        self.engine = tts_engine
        self.vocab_size = tts_engine.vocab

    def infer(self, hidden, top_k, prefix, penalty_window_size=-1, penalty=1.1, max_tokens=1000):
        e = self.engine
        dev = e.device
        h = hidden.reshape(-1, hidden.shape[-1]).to(dev, torch.float32).contiguous()
        p = None if prefix is None else prefix.reshape(-1, hidden.shape[-1]).to(dev, torch.float32).contiguous()
        seqs = e.start([(h, p)])
        cur = torch.full((1,), e.sos, dtype=torch.int32, device=dev)
        k = torch.tensor([top_k], dtype=torch.int32).to(dev)
        out = torch.empty(1, dtype=torch.int32, device=dev)
        generated = [e.sos]
        try:
            for i in range(max_tokens):
                step = torch.full((1,), i, dtype=torch.int32, device=dev)
                lg = e.step(seqs, cur)
                if penalty_window_size > 0:   # decoder.py:348-351
                    win = torch.tensor([penalty_ring(generated, penalty_window_size)], dtype=torch.int32).to(dev)
                    ops.penalty(lg, e.vocab + 4, cur, win, step, penalty)
                chk = ops.sample_check(dev)
                ops.sample(lg, e.vocab + 4, out, k, step=step, err=chk)
                t = int(out.item())
                chk.check("LLM2TTSCodecAR.infer")   # decoder.py:355-359: multinomial raises on NaN / inf
                if t == e.eos:
                    break
                generated.append(t)
                yield torch.tensor([[t]], device=dev)
                cur = out.clone()
        finally:
            e.free(seqs)
