"""Decoder-layer stacks on the MI355X kernels: Qwen2 (AudioLLM backbone) and the Llama layers of
the AR speech decoder (pre_nn / layers_prefix / layers).

Per layer (transformers Qwen2DecoderLayer / LlamaDecoderLayer, the call sites are
models/audioLLM.py:479-484 and models/decoder/decoder.py:127-188,294-312):
  rmsnorm -> fused QKV GEMM (+bias, RoPE and the paged-KV append in its epilogue) -> split-KV attention ->
  O GEMM (+residual, in place) -> rmsnorm -> fused gate/up GEMM with SiLU*up epilogue ->
  down GEMM (+residual, in place).
The residual stream is fp32; GEMMs read it as fp32 (bf16 hi/lo split) against bf16 weights.
"""
import os

import torch

from . import ops
from .kv import BatchMeta
from .ops import F32, PackedLinear

# FO_ATTN_DENSE=0 passes the item table even for one-token-per-sequence batches (A/B against a
# library older than fo_attention's items == NULL form)
ATTN_DENSE = os.environ.get("FO_ATTN_DENSE", "1") == "1"
# FO_ATTN_O=1 (opt-in, A/B only): the decode attention fused with the o projection (k_attn_decode_o); the default (0)
# runs them as two launches, which measured faster
ATTN_O = os.environ.get("FO_ATTN_O", "0") == "1"
# FO_XPACK_SMALL=1: packed q|k|v / o inputs also at <= 8 rows for wide stacks (the Qwen2 text step; A/B)
XPACK_SMALL = os.environ.get("FO_XPACK_SMALL", "0") == "1"


class Layer:
    __slots__ = ("ln1", "ln2", "qkv", "o", "gu", "down")


class DecoderStack:
    def __init__(self, src, prefix, n_layers, D, H, KVH, eps, bias, rope, pool, kv_layer0=0, first_fp16=False,
                 attn_keys_per_split=ops.ATTN_KEYS_PER_SPLIT):
        self.n, self.D, self.H, self.KVH, self.hd, self.eps = n_layers, D, H, KVH, D // H, eps
        self.attn_kps = attn_keys_per_split
        self.cos, self.sin = rope
        self.pool, self.kv_layer0, self.first_fp16 = pool, kv_layer0, first_fp16
        self.layers = []
        for i in range(n_layers):
            q = f"{prefix}{i}."
            L = Layer()
            L.ln1 = src.get(q + "input_layernorm.weight")
            L.ln2 = src.get(q + "post_attention_layernorm.weight")
            wq = src.get(q + "self_attn.q_proj.weight", torch.bfloat16)
            wk = src.get(q + "self_attn.k_proj.weight", torch.bfloat16)
            wv = src.get(q + "self_attn.v_proj.weight", torch.bfloat16)
            b = None
            if bias:
                b = torch.cat([src.get(q + "self_attn.q_proj.bias"), src.get(q + "self_attn.k_proj.bias"),
                               src.get(q + "self_attn.v_proj.bias")])
            L.qkv = PackedLinear(torch.cat([wq, wk, wv]), b, rope_hd=self.hd)
            del wq, wk, wv
            L.o = PackedLinear(src.get(q + "self_attn.o_proj.weight", torch.bfloat16))
            L.gu = PackedLinear(src.get(q + "mlp.gate_proj.weight", torch.bfloat16),
                                swiglu_up=src.get(q + "mlp.up_proj.weight", torch.bfloat16))
            L.down = PackedLinear(src.get(q + "mlp.down_proj.weight", torch.bfloat16))
            self.layers.append(L)
        # decode steps (one token per sequence) of an MHA stack with a small o projection -- the AR speech decoder, 14
        # heads of 64, o 896 x 896 -- fuse the attention with the o projection (fo_attention_o: each (session, head)
        # workgroup multiplies its attention row by its head's o slice; the last head sums the partials)
        self.attn_o = ATTN_O and H == KVH and self.hd == 64 and D <= 1024 and n_layers > 0

    def _packs(self, T):
        """Whether a T-row forward writes / reads packed activations (9..64 rows; <= 8 rows too for wide stacks under
        FO_XPACK_SMALL)."""
        return 8 < T <= 64 or (XPACK_SMALL and T <= 8 and self.D >= 2048)

    @property
    def weight_bytes(self):
        return sum(L.qkv.nbytes + L.o.nbytes + L.gu.nbytes + L.down.nbytes for L in self.layers)

    def workspace(self, T, nsplit, device):
        """Preallocated per-forward buffers for T tokens (graph capture must not allocate)."""
        H, KVH, hd = self.H, self.KVH, self.hd
        ws = {"h": torch.empty(T, self.D, dtype=F32, device=device),
              "q": torch.empty(T, H * hd, dtype=F32, device=device),
              "att": torch.empty(T, H * hd, dtype=F32, device=device),
              "m": torch.empty(T, self.layers[0].gu.N, dtype=F32, device=device),
              "nsplit": nsplit, "part_ml": None, "part_o": None,
              "sA": ops.RowStats(T, device), "sB": ops.RowStats(T, device),
              "xg": torch.empty(T, self.D, dtype=F32, device=device),
              "tickets": torch.zeros(max(T, 2) * KVH, dtype=torch.int32, device=device)}
        if self._packs(T) and ops.XPACK:   # packed activations for the q|k|v and o inputs (ops.XPack)
            ws["xgp"] = ops.XPack(self.D, device, T)
            ws["attp"] = ops.XPack(H * hd, device, T)
        if self.attn_o:
            ws["o_part"] = torch.empty(T * H * self.D, dtype=F32, device=device)
            ws["o_tickets"] = torch.zeros(max(T, 1), dtype=torch.int32, device=device)
        if nsplit > 1:
            ws["part_ml"] = torch.empty(T * H * nsplit * 2, dtype=F32, device=device)
            ws["part_o"] = torch.empty(T * H * nsplit * hd, dtype=F32, device=device)
        return ws

    def forward(self, x, meta: BatchMeta, ws=None, pre_normed=False, final_norm=None):
        """x: fp32 [T, D] residual stream, updated in place; KV for meta's tokens is appended.
        ws: optional workspace() of at least meta.T tokens (then nothing is allocated here).
        pre_normed: ws["h"] already holds the first layer's input RMSNorm of x (written by the
        previous decode step's sampler, fo_sample_embed).
        final_norm: gamma of the norm after the stack; the last down projection then also writes
        ws["xg"] = x * gamma and ws["sA"] row statistics, so the consumer GEMM (the output head) applies
        that RMSNorm on load instead of a separate norm launch."""
        T = meta.T
        H, KVH, hd = self.H, self.KVH, self.hd
        if ws is None:
            ws = self.workspace(T, ops.attn_nsplit(meta.max_keys, meta.n_items, KVH), x.device)
        h, q, att, m = ws["h"][:T], ws["q"][:T], ws["att"][:T], ws["m"][:T]
        nsplit, part_ml, part_o = ws["nsplit"], ws["part_ml"], ws["part_o"]
        scale = hd ** -0.5
        sA, sB, xg = ws["sA"], ws["sB"], ws["xg"][:T]
        last = len(self.layers) - 1
        # one token per sequence (decode) or the same count for every sequence, one work item each (a listen
        # chunk): the attention needs no item table (fo_attention items NULL)
        dense = ATTN_DENSE and (meta.n_items == T == meta.S or getattr(meta, "uniform", False))
        # 9..64 rows (a listen chunk, a duplex tick, a prefill): the q|k|v input (the previous down projection's
        # x*gamma) and the o input (the attention output) are also written packed by their producers and read packed
        # (ops.XPack; layer 0's q|k|v input comes from the gather and stays fp32).  At <= 8 rows (text and AR decode
        # steps) the X re-read is half as large and the extra stores cost more than the reads save (AR step 172.4 ->
        # 177.1 us, r04zf)
        xgp, attp = ws.get("xgp"), ws.get("attp")
        if not self._packs(T) or xgp is None or xgp.rows < T:
            xgp = attp = None
        # a decode batch takes the fused attention + o projection (the decode attention's form: one row per item)
        fuse_o = (self.attn_o and "o_part" in ws and meta.n_items == T == meta.S and meta.max_rows == 1 and
                  meta.block_table.shape[1] * self.pool.PS <= 4096)
        if fuse_o:
            xgp = attp = None
        # (a captured graph's meta carries its capacity, not the replay's keys: graphs keep 128-key splits, which fill
        # the chip at the listen / text shapes, r03c; eager launches -- duplex ticks, prefills -- size them per launch)
        eager = x.is_cuda and not torch.cuda.is_current_stream_capturing()
        kps = self.attn_kps or (ops.attn_keys_per_split(meta.max_keys, meta.n_items, KVH, hd, x.device) if eager else 128)
        for i, L in enumerate(self.layers):
            li = self.kv_layer0 + i
            rope = (meta.tok_pos, meta.tok_slot, self.cos, self.sin, q, self.pool.k[li], self.pool.v[li], H, KVH,
                    self.pool.PS)
            # (the first layer's rows come from a gather: no producer statistics yet; later layers apply the input
            # RMSNorm from the previous down projection's x*gamma and row sums)
            xin, norm = (h, None) if i == 0 else (xg, (sA, self.eps))
            if i == 0 and not pre_normed:
                ops.rmsnorm(x, L.ln1, self.eps, out=h, round_fp16=self.first_fp16, M=T)
            L.qkv.qkv_rope(xin, T, *rope, norm=norm, xpack=xgp if i > 0 else None)
            if fuse_o:
                ops.attention_o(q, T, None if dense else meta.items, meta.tok_nvis, meta.block_table, self.pool.PS,
                                self.pool.k[li], self.pool.v[li], H, hd, scale, L.o, ws["o_part"], ws["o_tickets"], x,
                                L.ln2, xg, sB)
            else:
                ops.attention(q, T, None if dense else meta.items, meta.n_items, meta.max_rows, meta.tok_nvis,
                              meta.block_table, self.pool.PS, self.pool.k[li], self.pool.v[li], H, KVH, hd, scale,
                              nsplit, part_ml, part_o, att, tickets=ws["tickets"], keys_per_split=kps,
                              opack=attp)
                L.o(att, out=x, residual=True, M=T, stats_out=sB.set(L.ln2, xg), xpack=attp, ypack=xgp)
            L.gu(xg, out=m, M=T, norm=(sB, self.eps), xpack=xgp)
            if i == last and final_norm is None:
                L.down(m, out=x, residual=True, M=T)
            elif i == last:
                L.down(m, out=x, residual=True, M=T, stats_out=sA.set(final_norm, xg))
            else:
                L.down(m, out=x, residual=True, M=T, stats_out=sA.set(self.layers[i + 1].ln1, xg), ypack=xgp)
        return x
