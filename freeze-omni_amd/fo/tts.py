"""AR single-codebook speech decoder (LLM2TTSCodecAR.infer) on the MI355X kernels.

Reference: models/decoder/decoder.py:127-188 (pre_nn / kv_cache_prefix), :294-367 (prefill + AR loop,
eager attention with attention_mask=None, i.e. unmasked), top-k multinomial sampler, EOS = vocab+2.
Positions: the prefix KV occupies cache rows 0..P-1 with its own RoPE positions 0..P-1; the
bidirectional prefill then uses RoPE positions 0..T while writing rows P..P+T; decode tokens use
position cache_len - P (decoder.py:337-340).  Many sessions decode in one batched step.
"""
import ctypes
import os
from types import SimpleNamespace

import numpy as np
import torch

from . import _lib, ops, tables
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
        self.vocab, self.idim = odim, idim
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
        B = len(seqs)
        meta = BatchMeta([(s.kv, 1, s.kv.length - s.P, False) for s in seqs], dev)
        ws = self.main.workspace(B, ops.attn_nsplit(meta.max_keys, meta.n_items, self.H), dev)
        x = self.embed_input(tokens, ws, B)
        self.main.forward(x, meta, ws, pre_normed=True, final_norm=self.norm)
        for s in seqs:
            s.generated += 1
        return self.out_fnn(ws["xg"][:B], norm=(ws["sA"], self.eps))

    def embed_input(self, tokens, ws, B, x=None):
        """x = embedding[tokens] (fp32) and ws["h"] = the first layer's RMSNorm of it: the decode step's
        input, as fo_sample_embed writes it for the next step inside the captured graph."""
        x = ops.gather_rows(self.embedding, tokens, out=x, M=B)
        ops.rmsnorm(x, self.main.layers[0].ln1, self.eps, out=ws["h"], M=B)
        return x

    def decode_graph(self, B, V_sample, top_k, seed, max_keys, hist_rows, pen=None, capture=True):
        """Captured decode step for a batch of B sessions (cached; rebuilt when a bound grows).
        pen = (window, penalty) adds the repetition penalty before the draw (None: off).
        capture=False: the same step body launched directly each step (no graph)."""
        # per stream: a graph's static buffers belong to the stream it was captured on and replays on (two
        # sentences' speech may decode side by side on their own streams)
        key = (B, V_sample, top_k, seed, pen, capture, ops.stream(self.device))
        g = self._graphs.get(key) if hasattr(self, "_graphs") else None
        if g is None or g.max_keys < max_keys or g.hist_rows < hist_rows:
            if not hasattr(self, "_graphs"):
                self._graphs = {}
            if g is not None:
                g.destroy()
            g = DecodeGraph(self, B, V_sample, top_k, seed, max(max_keys, 1024), max(hist_rows, 1024), pen, capture)
            self._graphs[key] = g
        return g

    def free(self, seqs):
        for s in seqs:
            s.kv.free()


def penalty_ring(generated, W):
    """Ring image of the penalty window for one session: generated = [SOS] + ids drawn so far; the id
    with generation index k sits at slot k % W (what fo_penalty writes step by step); empty slots -1."""
    ring = [-1] * W
    n = len(generated)
    for k in range(max(0, n - W), n):
        ring[k % W] = generated[k]
    return ring


class DecodeGraph:
    """One AR decode step (decoder.py:341-367: embed -> layers -> norm -> out_fnn -> sample) for a fixed
    batch of B sessions, captured once as a hipGraph and replayed per token.

    Everything the step reads is in static device buffers: the current ids (written by the previous
    replay's sampler, so ids never round-trip through the host), and a per-step metadata block
    (positions, cache slots, visible keys, RNG step, history row, block tables) uploaded with one
    async copy from a ring of pinned host buffers.  The sampled ids are also recorded into a pinned,
    host-mapped history [hist_rows, B] at the step's row, so the host reads them lazily, behind the
    GPU, after an event instead of synchronising every token.
    """

    RING = 64
    AHEAD = 128   # KV positions reserved ahead of the decode, so a session's page list changes every ~7 pages

    def __init__(self, tts, B, V_sample, top_k, seed, max_keys, hist_rows, pen=None, capture=True):
        dev = tts.device
        self.pen = pen
        # the captured step advances its own metadata for the next step (inside the sampler launch); the host
        # uploads a fresh block only when the batch, its RNG keys or a session's page list changed
        self.advance = capture
        self._uploaded = None
        self.win = torch.full((B, pen[0]), -1, dtype=I32, device=dev) if pen else None
        PS = tts.pool.PS
        self.tts, self.B, self.V_sample, self.seed = tts, B, V_sample, seed
        self.max_keys, self.hist_rows = max_keys, hist_rows
        self.maxb = (max_keys + PS - 1) // PS
        self.n_meta = 5 * B + 1 + B * self.maxb
        self.host = [torch.empty(self.n_meta, dtype=I32).pin_memory() for _ in range(self.RING)]
        self.host_np = [h.numpy() for h in self.host]
        self.meta_d = torch.zeros(self.n_meta, dtype=I32, device=dev)
        m = self.meta_d
        items = torch.tensor([[b, b, 1] for b in range(B)], dtype=I32).reshape(-1).to(dev)
        self.meta = SimpleNamespace(T=B, S=B, tok_pos=m[0:B], tok_slot=m[B:2 * B], tok_nvis=m[2 * B:3 * B],
                                    step=m[3 * B:4 * B], key=m[4 * B:5 * B], hist_row=m[5 * B:5 * B + 1],
                                    block_table=m[5 * B + 1:].view(B, self.maxb), items=items, n_items=B,
                                    max_rows=1, max_keys=max_keys)
        self.ids = torch.full((B,), tts.sos, dtype=I32, device=dev)
        self.hist = ops.HostBuffer(hist_rows, B)
        self.x = torch.empty(B, tts.D, dtype=F32, device=dev)
        self.logits = torch.empty(B, tts.vocab + 4, dtype=F32, device=dev)
        self.topk = torch.tensor([top_k] * B, dtype=I32).to(dev)
        self.ws = tts.main.workspace(B, ops.attn_nsplit(max_keys, B, tts.H), dev)
        self.err = ops.SampleCheck()   # NaN / inf logits rows (the reference's multinomial raises on them)
        self.events = []
        for _ in range(self.RING):
            e = ctypes.c_void_p()
            _lib.call("fo_event_create", ctypes.byref(e))
            self.events.append(e)
        self.exec = None
        if capture:
            self._capture()

    def _body(self):
        # x / ws["h"] hold this step's input (prime() or the previous replay's sampler); the sampler
        # records the drawn ids and writes the next step's input rows (fo_sample_embed)
        t = self.tts
        t.main.forward(self.x, self.meta, self.ws, pre_normed=True, final_norm=t.norm)
        t.out_fnn(self.ws["xg"], out=self.logits, norm=(self.ws["sA"], t.eps))
        if self.pen:
            ops.penalty(self.logits, t.vocab + 4, self.ids, self.win, self.meta.step, self.pen[1], B=self.B)
        ops.sample_embed(self.logits, self.V_sample, self.ids, t.embedding, self.x, t.main.layers[0].ln1, t.eps,
                         self.ws["h"], top_k=self.topk, seed=self.seed, step=self.meta.step, B=self.B,
                         key=self.meta.key, hist_ptr=self.hist.dev, hist_row=self.meta.hist_row, hist_ld=self.B,
                         err=self.err, **(dict(meta=self.meta_d, maxb=self.maxb, PS=t.pool.PS) if self.advance else {}))

    def prime(self):
        """Input rows of the next replay from self.ids (first step of a batch, or after the batch changed)."""
        self._uploaded = None
        self.tts.embed_input(self.ids, self.ws, self.B, x=self.x)

    def adopt(self, other):
        """Continue another graph's batch (same sessions, other sampler bound): take its ids and input rows."""
        self._uploaded = None
        self.ids.copy_(other.ids)
        if self.pen:
            self.win.copy_(other.win)
        self.x.copy_(other.x)
        self.ws["h"].copy_(other.ws["h"])

    def check(self):
        """After a step's event: raise if a logits row was NaN / inf (the reference's torch.multinomial raises,
        decoder.py:355-359)."""
        self.err.check("speech decode step")

    def _capture(self):
        s = ops.stream(self.tts.device)
        if s == 0 or s is None:
            raise RuntimeError("DecodeGraph must be captured on a non-default stream (ops.engine_stream)")
        _lib.call("fo_graph_begin", s)
        try:
            self._body()
        finally:
            ex = ctypes.c_void_p()
            _lib.call("fo_graph_end", s, ctypes.byref(ex))
        self.exec = ex

    def set_window(self, generated_lists):
        """Penalty rings of a new batch from the host-side id history ([SOS] + ids per session)."""
        if self.pen:
            rings = [penalty_ring(g, self.pen[0]) for g in generated_lists]
            self.win.copy_(torch.tensor(rings, dtype=I32).to(self.win.device))

    def set_ids(self, ids_dev):
        self._uploaded = None
        self.ids.copy_(ids_dev[:self.B])

    def launch(self, seqs, keys, step, slot):
        """Replay one step for seqs (len B, batch order) with RNG stream ids `keys` at step `step` (an int, or
        one step per row: a continuously batched lane whose rows joined at different times), history row
        `slot` (with the device-advanced metadata each row's id lands in history row = its own step); appends
        one KV position to every sequence.  Returns the step's event."""
        B, maxb, PS = self.B, self.maxb, self.tts.pool.PS
        steps = tuple(int(v) for v in step) if isinstance(step, (list, tuple)) else (int(step),) * B
        for s in seqs:
            kv = s.kv
            L = kv.length
            if len(kv.pages) * PS < L + 1 + 16:   # reserve a run of pages ahead (bounded by the block table)
                kv.reserve(min(L + 1 + self.AHEAD, maxb * PS))
            kv.reserve(L + 1)
            if len(kv.pages) > maxb:
                raise RuntimeError("decode graph block table too small")
        if self.advance and not isinstance(step, (list, tuple)) and slot != step:
            raise ValueError("decode graph: the history row is the step when the step advances its own metadata")
        # the device-advanced block is current only for the same sequences, RNG keys and block lists (version:
        # any page added, copied on write or dropped) and lengths exactly one step on
        sig = (tuple(id(s) for s in seqs), tuple(int(k) for k in keys), tuple(s.kv.version for s in seqs))
        lens = tuple(s.kv.length for s in seqs)
        up = self._uploaded
        if not (self.advance and up is not None and up[0] == sig and steps == tuple(v + 1 for v in up[1])
                and slot == up[2] + 1 and lens == tuple(n + 1 for n in up[3])):
            # the device-advanced block is not this step's: upload it from the host
            h = self.host_np[slot % self.RING]
            h[4 * B:5 * B] = keys
            h[5 * B] = slot
            bt = h[5 * B + 1:].reshape(B, maxb)
            for b, s in enumerate(seqs):
                kv = s.kv
                L = kv.length
                h[b] = L - s.P
                h[B + b] = kv.slot(L)
                h[2 * B + b] = L + 1
                h[3 * B + b] = steps[b]
                bt[b, :len(kv.pages)] = kv.pages
                bt[b, len(kv.pages):] = kv.pages[-1]   # defensive: never a foreign page past the list
            self.meta_d.copy_(self.host[slot % self.RING], non_blocking=True)
        self._uploaded = (sig, steps, slot, lens)
        for s in seqs:
            s.kv.length += 1
            s.generated += 1
        st = ops.stream(self.tts.device)
        if self.exec is None:
            self._body()
        else:
            _lib.call("fo_graph_launch", self.exec, st)
        ev = self.events[slot % self.RING]
        _lib.call("fo_event_record", ev, st)
        return ev

    def destroy(self):
        if self.exec is not None:
            _lib.call("fo_graph_destroy", self.exec)
            self.exec = None
        for e in self.events:
            _lib.call("fo_event_destroy", e)
        self.events = []
        self.hist.free()
        self.err.free()
