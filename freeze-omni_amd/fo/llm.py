"""Qwen2 backbone of AudioLLM on the MI355X kernels (frozen LLM, per-session paged KV).

Reference: AudioLLM._llm_forward_core -> Qwen2Model (models/audioLLM.py:479-484), the dialog-state
head (models/audioLLM.py:486-527) and the sampler _post_decode (models/audioLLM.py:431-477).
"""
import numpy as np
import torch

from . import ops, tables
from .kv import BatchMeta, KVPool, KVSeq
from .ops import F32, I32, PackedLinear
from .stack import DecoderStack


class LLMEngine:
    def __init__(self, src, llm_cfg, device, head_src=None, kv_tokens=65536, page_size=16, max_pos=None):
        c = llm_cfg
        self.device = torch.device(device)
        self.D, self.V = c["hidden_size"], c["vocab_size"]
        self.H, self.KVH = c["num_attention_heads"], c["num_key_value_heads"]
        self.hd = self.D // self.H
        self.eps = c["rms_norm_eps"]
        max_pos = max_pos or min(c.get("max_position_embeddings", 32768), 32768)
        cos, sin = tables.rope_tables(c["rope_theta"], self.hd, max_pos, round_fp16=True)
        self.rope = (cos.to(self.device), sin.to(self.device))
        n_pages = (kv_tokens + page_size - 1) // page_size
        self.pool = KVPool(c["num_hidden_layers"], self.KVH, self.hd, n_pages, page_size, self.device)
        self.stack = DecoderStack(src, "model.layers.", c["num_hidden_layers"], self.D, self.H, self.KVH, self.eps,
                                  True, self.rope, self.pool, first_fp16=True)
        self.embed_tokens = src.get("model.embed_tokens.weight", torch.bfloat16)
        self.norm = src.get("model.norm.weight")
        self.lm_head = PackedLinear(src.get("lm_head.weight", torch.bfloat16))
        hs = head_src or src
        self.head_w = hs.get("predictor_head.weight") if "predictor_head.weight" in hs else None
        self.head_b = hs.get("predictor_head.bias") if self.head_w is not None else None

    @property
    def weight_bytes(self):
        return self.stack.weight_bytes

    def new_seq(self):
        return KVSeq(self.pool)

    def embed(self, ids, out=None, round_fp16=False):
        if torch.is_tensor(ids):
            ids_d = ids.to(device=self.device, dtype=I32)
        else:
            ids_d = ops.h2d(np.asarray(list(ids), np.int32), self.device)
        return ops.gather_rows(self.embed_tokens, ids_d, out=out, round_fp16=round_fp16)

    def forward(self, x, entries):
        """x: fp32 [T, D] input embeds (already rounded to fp16 values, models/audioLLM.py:338,410);
        entries: list of (KVSeq, n_tokens).  Returns (final-normed hidden [T, D], BatchMeta)."""
        meta = BatchMeta([(s, n, s.length, True) for s, n in entries], self.device, gqa=self.H // self.KVH,
                         rows=ops.attn_item_rows(self.hd))
        self.stack.forward(x, meta)
        ops.rmsnorm(x, self.norm, self.eps, out=x)
        return x, meta

    def state_probs(self, hidden, rows):
        """softmax over the first 3 predictor-head logits at the given rows -> device [S, 3]."""
        rows_d = rows if torch.is_tensor(rows) else ops.h2d(np.asarray(list(rows), np.int32), self.device)
        out = torch.empty(rows_d.numel(), 3, dtype=F32, device=self.device)
        return ops.state_head(hidden, rows_d, self.head_w, self.head_b, out)

    def logits(self, hidden, rows):
        rows_d = rows if torch.is_tensor(rows) else torch.tensor(list(rows), dtype=I32).to(self.device)
        h = ops.gather_rows(hidden, rows_d)
        return self.lm_head(h)
