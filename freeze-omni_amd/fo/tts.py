"""AR single-codebook speech decoder (LLM2TTSCodecAR.infer) on the MI355X kernels.

Reference: models/decoder/decoder.py:127-188 (pre_nn / kv_cache_prefix), :294-367 (prefill + AR loop,
eager attention with attention_mask=None, i.e. unmasked), top-k multinomial sampler, EOS = vocab+2.
Positions: the prefix KV occupies cache rows 0..P-1 with its own RoPE positions 0..P-1; the
bidirectional prefill then uses RoPE positions 0..T while writing rows P..P+T; decode tokens use
position cache_len - P (decoder.py:337-340).  Many sessions decode in one batched step.
"""
import torch

from . import ops, tables
from .kv import BatchMeta, KVPool, KVSeq
from .ops import F32, I32, PackedLinear
from .stack import DecoderStack


class TTSSeq:
    def __init__(self, kv, P):
        self.kv, self.P = kv, P
        self.generated = 0


class TTSEngine:
    def __init__(self, src, decoder_json, device, kv_tokens=1 << 16, page_size=16):
        idim, odim, a = decoder_json
        self.device = torch.device(device)
        self.vocab = odim
        self.D, self.H = a["transformer_attention_dim"], a["transformer_attention_heads"]
        self.hd = self.D // self.H
        self.nb = a["transformer_num_blocks"]
        self.eps = 1e-6
        cos, sin = tables.rope_tables(10000.0, self.hd, 4096, round_fp16=False)
        rope = (cos.to(self.device), sin.to(self.device))
        self.pool = KVPool(self.nb, self.H, self.hd, (kv_tokens + page_size - 1) // page_size, page_size,
                           self.device)
        mk = lambda pre, n: DecoderStack(src, pre, n, self.D, self.H, self.H, self.eps, False, rope, self.pool)  # noqa
        self.pre = mk("tts.layers_pre_nn.", self.nb // 2)
        self.main = mk("tts.layers.", self.nb)
        self.prefix = mk("tts.layers_prefix.", self.nb) if a.get("kv_cache_prefix_finetune", 0) else None
        self.embedding = src.get("tts.embedding.weight", torch.bfloat16)
        self.norm = src.get("tts.norm.weight")
        self.out_fnn = PackedLinear(src.get("tts.out_fnn.weight", torch.bfloat16), src.get("tts.out_fnn.bias"))
        self.bos, self.sos, self.eos = odim, odim + 1, odim + 2

    @property
    def weight_bytes_per_step(self):
        return self.main.weight_bytes + self.out_fnn.nbytes

    def start(self, items):
        """items: list of (hidden [T1, D] device fp32, prefix [T2, D] device fp32 or None).
        Runs pre_nn, the prefix KV fill and the bidirectional prefill for every session."""
        dev = self.device
        # pre_nn on a temporary sequence per session (no cache in the reference, full mask)
        tmp = [KVSeq(self.pool) for _ in items]
        x = torch.cat([h for h, _ in items], 0).contiguous()
        meta = BatchMeta([(s, h.shape[0], 0, False) for s, (h, _) in zip(tmp, items)], dev)
        self.pre.forward(x, meta)
        for s in tmp:
            s.free()
        seqs = []
        pre_rows = []
        r = 0
        for h, p in items:
            pre_rows.append((r, h.shape[0]))
            r += h.shape[0]
        # prefix layers write KV rows 0..P-1 (decoder.py:127-154)
        kvs = [KVSeq(self.pool) for _ in items]
        if self.prefix is not None and any(p is not None for _, p in items):
            ent, xs = [], []
            for s, (_, p) in zip(kvs, items):
                if p is not None:
                    ent.append((s, p.shape[0], 0, False))
                    xs.append(p)
            xp = torch.cat(xs, 0).contiguous()
            self.prefix.forward(xp, BatchMeta(ent, dev))
        Ps = [s.length for s in kvs]
        # BOS + pre_nn output, prefill with positions 0..T
        bos = ops.gather_rows(self.embedding, torch.full((len(items),), self.bos, dtype=I32, device=dev))
        rows = []
        for i, (r0, n) in enumerate(pre_rows):
            rows.append(bos[i:i + 1])
            rows.append(x[r0:r0 + n])
        x0 = torch.cat(rows, 0).contiguous()
        self.main.forward(x0, BatchMeta([(s, n + 1, 0, False) for s, (_, n) in zip(kvs, pre_rows)], dev))
        for s, P in zip(kvs, Ps):
            seqs.append(TTSSeq(s, P))
        return seqs

    def step(self, seqs, tokens):
        """tokens: device int32 [B] (current input ids).  Returns logits [B, vocab+4] (fp32)."""
        dev = self.device
        x = ops.gather_rows(self.embedding, tokens)
        meta = BatchMeta([(s.kv, 1, s.kv.length - s.P, False) for s in seqs], dev)
        self.main.forward(x, meta)
        ops.rmsnorm(x, self.norm, self.eps, out=x)
        for s in seqs:
            s.generated += 1
        return self.out_fnn(x)

    def free(self, seqs):
        for s in seqs:
            s.kv.free()
