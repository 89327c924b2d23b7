"""Streaming speech front end on the MI355X kernels: kaldi fbank framing, speech encoder, adapter.

* Framer: the reference keeps a sample ring and a 3-frame feature carry per user
  (bin/inference.py:43-80 framing A; models/AudioFeatureGating.py:33-75 framing B).  Here the host
  keeps only the recent samples; the GPU recomputes the carried frames from them (identical values)
  so no device feature state exists; the first chunk after reset carries zero frames, as the
  reference's zero-initialised input_chunk does.
* SpeechEncoderEngine: speechEncoder.infer (models/encoder/encoder.py:149-155) = GlobalCMVN +
  Conv2dSubsampling4 (im2col + MFMA GEMMs) + rel-pos Transformer with a left-chunk KV ring per user
  (models/encoder/transformer.py:266-285, attention.py:407-459).  linear_pos(sinusoid(p)) is
  precomputed for every position at load (memory for compute: ~0.5 GB per encoder at REAL size).
* AdapterEngine: CNNSubsampling with carried frames (models/adapter.py:72-157), both conv branches,
  eval BatchNorm as a per-column affine GEMM epilogue, or LayerNorm; ReLU or GELU.
Batched: one launch sequence serves all users of a replica; per-user state lives in slot pools.
"""
import math
import os

import threading

import numpy as np
import torch

from . import ops, tables
from .ops import F32, I32, PackedLinear

# the encoder block's attention half: FO_ENC_BLOCK=0 three launches (LayerNorm-on-load q|k|v GEMM, rel-pos attention,
# out GEMM + reduce; the default); 1 one launch (fo_enc_attn_block: LayerNorm1 + q|k|v + attention + out + residual); 2
# the q|k|v GEMM, then attention + out + residual in one launch (fo_enc_attn_out)
ENC_BLOCK = int(os.environ.get("FO_ENC_BLOCK", "0") or 0)

FRAMINGS = {
    # name: (chunk_frames, carried_frames, win, shift, nfft, scale)
    "A": (16, 3, 400, 160, 512, 32768.0),   # bin/inference.py:44-52, x32768 (:74)
    "B": (28, 4, 256, 128, 256, 32767.0),   # configs/dialog_state_pred_config.yaml:24-29, x32767 (AudioFeatureGating.py:58)
}


class Framer:
    """Per-user host sample history for one framing."""

    def __init__(self, kind="A"):
        self.kind = kind
        nf, ov, wl, ws, nfft, scale = FRAMINGS[kind]
        self.chunk = nf * ws
        self.R = nf + ov
        self.window_len = (self.R - 1) * ws + wl
        self.scale = np.float32(scale)
        self.reset()

    def reset(self):
        self.hist = np.zeros(self.window_len, np.float32)
        self.first = True

    def push(self, pcm):
        """pcm: one chunk of float samples in [-1, 1) (len == chunk).  Returns (window, first)."""
        x = np.asarray(pcm, dtype=np.float32).reshape(-1)
        if x.shape[0] != self.chunk:
            raise ValueError(f"framing {self.kind}: expected {self.chunk} samples, got {x.shape[0]}")
        self.hist = np.concatenate([self.hist[self.chunk:], x * self.scale])
        first = self.first
        self.first = False
        return self.hist, first


class FbankGPU:
    def __init__(self, kind, device):
        nf, ov, wl, ws, nfft, _ = FRAMINGS[kind]
        self.nf, self.ov, self.wl, self.ws, self.nfft = nf, ov, wl, ws, nfft
        self.R = nf + ov
        self.n_samples = (self.R - 1) * ws + wl
        w, c, s, m = tables.kaldi_tables(wl, nfft)
        self.device = torch.device(device)
        self.window, self.tw_cos, self.tw_sin, self.mel = (t.to(self.device) for t in (w, c, s, m))
        # pinned staging of the calls: a ring of 4 slots (grown on demand), each reused once its copy has run
        self._pins, self._evs, self._k = [None] * 4, [None] * 4, 0
        # the reference gates every session's audio in a thread of its own (bin/dialog_state_pred.py:240-288) and the
        # gaters of one engine share this object: one caller at a time in the staging ring
        self._lock = threading.Lock()

    def _stage(self, host):
        """host float32 [n] -> a new device tensor: through this object's own pinned ring and one async copy on the
        current stream.  The batched duplex gating (one call for every session's chunk, ~0.25-0.5 MB) through
        ops.h2d's per-call pinned blocks, copied by torch's OpenMP-parallel copy_, stalled a tick for ~60 ms every
        few ticks (scripts/duplex_tick_probe.py).  A slot is rewritten four calls later, after its copy's event (long done: the listen pipelines keep at
        most one chunk's fbank queued ahead)."""
        n = host.shape[0]
        if self.device.type != "cuda" or torch.cuda.is_current_stream_capturing():
            return ops.h2d(host, self.device)
        k = self._k
        self._k = (k + 1) % len(self._pins)
        if self._evs[k] is not None:
            self._evs[k].synchronize()
        if self._pins[k] is None or self._pins[k].numel() < n:
            self._pins[k] = torch.empty(max(n, 2 * (0 if self._pins[k] is None else self._pins[k].numel())),
                                        dtype=F32, pin_memory=True)
        pin = self._pins[k]
        pin[:n].numpy()[:] = host   # (a numpy copy: torch's copy_ of >= 32K elements fans out over the OpenMP pool)
        dev = torch.empty(n, dtype=F32, device=self.device)
        dev.copy_(pin[:n], non_blocking=True)
        if self._evs[k] is None:
            self._evs[k] = torch.cuda.Event()
        self._evs[k].record(torch.cuda.current_stream(self.device))
        return dev

    def __call__(self, windows, firsts):
        """windows: np.float32 [B][n_samples]; firsts: list[bool] -> device feats [B, R, 80]."""
        with self._lock:
            return self._call(windows, firsts)

    def _call(self, windows, firsts):
        B = len(firsts)
        host = np.concatenate([np.ascontiguousarray(windows, np.float32).reshape(-1),
                               np.asarray([self.ov if f else 0 for f in firsts], np.int32).view(np.float32)])
        dev = self._stage(host)   # samples + the per-row zero-row counts (int32 bits), one async copy
        samples = dev[:B * self.n_samples].view(B, self.n_samples)
        zero_rows = dev[B * self.n_samples:].view(I32)
        out = torch.empty(B, self.R * 80, dtype=F32, device=self.device)
        ops.fbank(samples, B, self.n_samples, self.wl, self.ws, self.nfft, self.window, self.tw_cos, self.tw_sin,
                  self.mel, out, 0, zero_rows)
        return out.view(B, self.R, 80)


class SlotPool:
    def __init__(self, n):
        self.free = list(range(n - 1, -1, -1))
        self.n = n

    def get(self):
        if not self.free:
            raise RuntimeError(f"session slot pool exhausted ({self.n})")
        return self.free.pop()

    def put(self, s):
        self.free.append(s)


class EncoderCache:
    """Caller-owned encoder state (the reference's `encoder_cache` buffer list): a ring slot."""

    def __init__(self, engine):
        self.engine, self.slot = engine, engine.slots.get()
        self.start, self.len = 0, 0

    def __del__(self):
        try:
            self.engine.slots.put(self.slot)
        except Exception:
            pass


# a listen group's encoder attention: every chunk in one launch (fo_relpos_attention_chunks); FO_ENC_CHUNK_ATTN=0: one
# fo_relpos_attention_fused launch per chunk (A/B)
CHUNK_ATTN = os.environ.get("FO_ENC_CHUNK_ATTN", "1") != "0"


class SpeechEncoderEngine:
    def __init__(self, src, cfg, ident, device, max_sessions=64):
        ty = cfg["train_yaml"]
        sub = ty["encoder_conf"]["para_conf"]["subsampling"]
        tr = ty["encoder_conf"]["para_conf"]["transformer"]
        p = f"encoder_{ident}."
        self.device = torch.device(device)
        self.C = sub["subsampling-output-dim"]
        self.F = ((sub["subsampling-input-dim"] - 1) // 2 - 1) // 2
        self.d = tr["transformer-attention-dim"]
        self.h = tr["transformer-attention-heads"]
        self.dk = self.d // self.h
        self.nb = tr["transformer-num-blocks"]
        self.chunk = tr["transformer-chunk_size"]
        self.left = tr["transformer-left_chunks"]
        self.buffersize = self.chunk * self.left
        self.full_chunk = (self.left + 1) * self.chunk
        self.max_len = self.chunk * (5000 // self.chunk) - self.full_chunk
        self.cap = self.buffersize + 8
        g = lambda n, dt=F32: src.get(p + n, dt)  # noqa: E731
        self.mean, self.istd = g("global_cmvn.mean"), g("global_cmvn.istd")
        # Conv2dSubsampling4 (fo_subsample): conv1 as a 9-tap fp32 stencil (bf16-valued weights, as the GEMMs see them),
        # conv2 as an implicit GEMM with K tap-major: its weight packed from [C][C][3][3] permuted to [C][3][3][C]
        if self.C % 32:
            raise ValueError(f"subsampling-output-dim {self.C}: the implicit conv2 needs a multiple of 32")
        self.conv1_w = g("enc.0.core.conv.0.weight", torch.bfloat16).float().reshape(self.C, 9).contiguous()
        self.conv1_b = g("enc.0.core.conv.0.bias")
        self.conv2 = PackedLinear(g("enc.0.core.conv.2.weight", torch.bfloat16).permute(0, 2, 3, 1)
                                  .reshape(self.C, 9 * self.C), g("enc.0.core.conv.2.bias"))
        self.out = PackedLinear(g("enc.0.core.out.0.weight", torch.bfloat16), g("enc.0.core.out.0.bias"))
        self.embed = PackedLinear(g("enc.1.embed.0.weight", torch.bfloat16), g("enc.1.embed.0.bias"))
        self.embed_ln = (g("enc.1.embed.1.weight"), g("enc.1.embed.1.bias"))
        self.after = (g("enc.1.after_norm.weight"), g("enc.1.after_norm.bias"))
        sinus = tables.relpos_sinusoid(self.max_len, self.d).to(self.device)
        self.ptab = torch.empty(self.nb, self.max_len, self.d, dtype=F32, device=self.device)
        self.layers = []
        for i in range(self.nb):
            q = f"enc.1.encoders.{i}."
            L = {
                "ln1": (g(q + "norm1.weight"), g(q + "norm1.bias")),
                "ln2": (g(q + "norm2.weight"), g(q + "norm2.bias")),
                "qkv": PackedLinear(torch.cat([g(q + f"self_attn.linear_{n}.weight", torch.bfloat16)
                                               for n in "qkv"]),
                                    torch.cat([g(q + f"self_attn.linear_{n}.bias") for n in "qkv"])),
                "out": PackedLinear(g(q + "self_attn.linear_out.weight", torch.bfloat16),
                                    g(q + "self_attn.linear_out.bias")),
                "bu": g(q + "self_attn.pos_bias_u"), "bv": g(q + "self_attn.pos_bias_v"),
                "ff1": PackedLinear(g(q + "feed_forward.w_1.weight", torch.bfloat16), g(q + "feed_forward.w_1.bias")),
                "ff2": PackedLinear(g(q + "feed_forward.w_2.weight", torch.bfloat16), g(q + "feed_forward.w_2.bias")),
            }
            PackedLinear(g(q + "self_attn.linear_pos.weight", torch.bfloat16))(sinus, out=self.ptab[i])
            self.layers.append(L)
        del sinus
        self.kr = torch.zeros(self.nb, max_sessions, self.cap, self.d, dtype=F32, device=self.device)
        self.vr = torch.zeros_like(self.kr)
        self.slots = SlotPool(max_sessions)
        # the attention half of each block as one launch (fo_enc_attn_block) where the geometry fits it
        self.block_fusable = self.dk == 64 and self.d % 256 == 0 and self.d <= 1024 and self.cap + 8 <= 96
        self.fused_block = ENC_BLOCK if self.block_fusable else 0

    @property
    def weight_bytes(self):
        n = self.conv1_w.numel() * 2 + self.conv2.nbytes + self.out.nbytes + self.embed.nbytes
        for L in self.layers:
            n += L["qkv"].nbytes + L["out"].nbytes + L["ff1"].nbytes + L["ff2"].nbytes
        return n

    def new_cache(self):
        return EncoderCache(self)

    def dims(self, R):
        H1, W1 = (R - 3) // 2 + 1, (80 - 3) // 2 + 1
        H2, W2 = (H1 - 3) // 2 + 1, (W1 - 3) // 2 + 1
        assert W2 == self.F and H2 <= 8
        return H1, W1, H2, W2

    def buffers(self, B, R):
        """Every intermediate of one infer() for B users x R frames (graph capture allocates nothing)."""
        H1, W1, H2, W2 = self.dims(R)
        T, C, dev = H2, self.C, self.device
        e = lambda *shape: torch.empty(*shape, dtype=F32, device=dev)  # noqa: E731
        return {"y1": e(B * H1 * W1, C), "z": e(B * T, C * self.F), "o": e(B * T, self.out.N),
                "x": e(B * T, self.d), "h": e(B * T, self.d), "qkv": e(B * T, 3 * self.d),
                "att": e(B * T, self.d), "f": e(B * T, self.layers[0]["ff1"].N),
                "sA": ops.RowStats(B * T, dev, with_sums=True), "sB": ops.RowStats(B * T, dev, with_sums=True),
                "meta": torch.empty(4 * B, dtype=I32, device=dev),
                # <= 64 rows: the out and FFN-down inputs also written packed by their producers (ops.XPack)
                "attp": ops.XPack(self.d, dev, B * T) if B * T <= 64 and ops.XPACK else None,
                "fp": ops.XPack(self.layers[0]["ff1"].N, dev, B * T) if B * T <= 64 and ops.XPACK else None,
                "xp32": ops.XPack32(self.d, dev, B * T) if B * T <= 64 and ops.XPACK else None,
                "part": e(B * self.h * T * self.d) if self.fused_block and T <= 8 else None,
                "tickets": torch.zeros(B, dtype=I32, device=dev)}

    def host_meta(self, caches, pe_indices):
        """Per-user ring / position metadata [starts | lens | rings | pos starts] and the next pe_index."""
        starts, lens, rings, pstarts, new_pe = [], [], [], [], []
        for c, pe in zip(caches, pe_indices):
            pe = pe % self.max_len
            starts.append(c.start)
            lens.append(c.len)
            rings.append(c.slot)
            pstarts.append(max(0, pe - self.full_chunk))
            new_pe.append(pe + self.chunk)
        return np.asarray(starts + lens + rings + pstarts, np.int32), new_pe

    def advance(self, caches, T):
        """Ring bookkeeping after a chunk: keep the last buffersize frames (attention.py:415-428)."""
        for c in caches:
            total = c.len + T
            keep = min(total, self.buffersize)
            c.start = (c.start + total - keep) % self.cap
            c.len = keep

    def run(self, feats, B, R, bufs, chunks=1):
        """The device part of infer(): bufs from buffers(B, R) with bufs['meta'] already uploaded.
        chunks > 1: `chunks` consecutive chunks of the same B sessions in one pass (an offline input's listen,
        fo.engine.ListenGroupGraph): feats [chunks * B, R, 80] chunk-major, bufs from buffers(chunks * B, R), meta
        [chunks][4 B] (each chunk's ring / position metadata, host_meta after the chunks before it).  Every row-wise
        step (the Conv2dSubsampling4 front end -- each chunk's window carries its own context frames --, the embed,
        the norms, q|k|v, linear_out, the FFN) runs once over all the rows; the rel-pos attention runs chunk by chunk
        in order, each launch appending its chunk's K / V to the ring the next one reads (attention.py:407-459), so
        chunk j sees exactly the left context the sequential order gives it."""
        H1, W1, H2, W2 = self.dims(R)
        T, C = H2, self.C
        N = B * chunks
        ops.subsample(feats, N, R, 80, self.mean, self.istd, self.conv1_w, self.conv1_b, C, bufs["y1"],
                      self.conv2.packed, self.conv2.bias, bufs["z"])
        self.out(bufs["z"], out=bufs["o"], M=N * T)
        x = self.embed(bufs["o"], out=bufs["x"], M=N * T)
        ops.layernorm(x, *self.embed_ln, out=x, relu=True, M=N * T)
        ops.scale_(x[:N * T], math.sqrt(self.d))
        meta = bufs["meta"]
        h, qkv, att, f = bufs["h"], bufs["qkv"], bufs["att"], bufs["f"]
        scale = 1.0 / math.sqrt(self.dk)
        if chunks > 1:
            return self._run_chunks(x, B, T, chunks, bufs, meta, scale)
        st, ln, rg, ps = meta[:B], meta[B:2 * B], meta[2 * B:3 * B], meta[3 * B:]
        # pre-norms applied by the GEMMs on load (fo_gemm_ln) from the residual producers' row sums
        fuse_ln = B * T <= 64 and os.environ.get("FO_ENC_LN_ON_LOAD", "1") != "0"
        sA, sB = bufs["sA"], bufs["sB"]
        attp, fp, xp32 = (bufs.get("attp"), bufs.get("fp"), bufs.get("xp32")) if fuse_ln else (None, None, None)
        last = len(self.layers) - 1
        if fuse_ln and bufs.get("part") is not None and self.fused_block == 1:
            # a launch for the attention half (LayerNorm1 .. residual, + the row sums ff1's norm reads), then
            # feed_forward as two GEMMs
            for i, L in enumerate(self.layers):
                ops.enc_attn_block(x, B, T, self.h, L["ln1"], L["qkv"], self.kr[i], self.vr[i], self.cap, meta,
                                   self.ptab[i], L["bu"], L["bv"], L["out"], scale, bufs["part"], bufs["tickets"], sB)
                L["ff1"].ln(x, *L["ln2"], sB, out=f, act="relu", ypack=fp)
                L["ff2"](f, out=x, residual=True, xpack=fp)
            ops.layernorm(x, *self.after, out=x)
            return x, T
        if fuse_ln and bufs.get("part") is not None and self.fused_block == 2:
            # q|k|v by the LayerNorm-on-load GEMM, then attention + linear_out + residual (+ the row sums ff1's norm
            # reads) in one launch, then feed_forward as two GEMMs (w_2 also writes the next block's statistics and
            # its fp32 packed residual)
            for i, L in enumerate(self.layers):
                if i > 0:
                    L["qkv"].ln(x, *L["ln1"], sA, out=qkv, xpack32=xp32)
                else:
                    ops.layernorm(x, *L["ln1"], out=h)
                    L["qkv"](h, out=qkv)
                ops.enc_attn_out(qkv, x, B, T, self.h, self.kr[i], self.vr[i], self.cap, meta, self.ptab[i], L["bu"],
                                 L["bv"], L["out"], scale, bufs["part"], bufs["tickets"], sB)
                L["ff1"].ln(x, *L["ln2"], sB, out=f, act="relu", ypack=fp)
                if i < last:
                    L["ff2"].rowstats(f, x, sA, residual=True, xpack=fp, ypack32=xp32)
                else:
                    L["ff2"](f, out=x, residual=True, xpack=fp)
            ops.layernorm(x, *self.after, out=x)
            return x, T
        for i, L in enumerate(self.layers):
            if fuse_ln and i > 0:
                L["qkv"].ln(x, *L["ln1"], sA, out=qkv, xpack32=xp32)
            else:
                ops.layernorm(x, *L["ln1"], out=h)
                L["qkv"](h, out=qkv)
            ops.relpos_attention_fused(qkv, self.kr[i], self.vr[i], self.cap, st, ln, rg, self.ptab[i], ps,
                                       L["bu"], L["bv"], B, T, self.h, self.dk, scale, att, opack=attp)
            if fuse_ln:
                L["out"].rowstats(att, x, sB, residual=True, xpack=attp, ypack32=xp32)
                L["ff1"].ln(x, *L["ln2"], sB, out=f, act="relu", ypack=fp, xpack32=xp32)
            else:
                L["out"](att, out=x, residual=True)
                ops.layernorm(x, *L["ln2"], out=h)
                L["ff1"](h, out=f, act="relu")
            if fuse_ln and i < last:
                L["ff2"].rowstats(f, x, sA, residual=True, xpack=fp, ypack32=xp32)
            else:
                L["ff2"](f, out=x, residual=True, xpack=fp)
        ops.layernorm(x, *self.after, out=x)
        return x, T

    def _run_chunks(self, x, B, T, chunks, bufs, meta, scale):
        """run(chunks > 1): the blocks over chunks * B * T rows, the attention chunk by chunk (rows chunk-major)."""
        N = B * chunks
        M = N * T
        n1 = B * T
        h, qkv, att, f = bufs["h"][:M], bufs["qkv"][:M], bufs["att"][:M], bufs["f"][:M]
        fuse_ln = M <= 64 and os.environ.get("FO_ENC_LN_ON_LOAD", "1") != "0"
        sA, sB = bufs["sA"], bufs["sB"]
        # (the attention output is written per chunk, so it is not packed for linear_out: the packed image's rows are
        # the launch's own)
        fp, xp32 = (bufs.get("fp"), bufs.get("xp32")) if fuse_ln else (None, None)
        last = len(self.layers) - 1
        x = x[:M]
        for i, L in enumerate(self.layers):
            if fuse_ln and i > 0:
                L["qkv"].ln(x, *L["ln1"], sA, out=qkv, xpack32=xp32)
            else:
                ops.layernorm(x, *L["ln1"], out=h)
                L["qkv"](h, out=qkv)
            if CHUNK_ATTN:   # the chunks in order inside one launch per (user, head)
                ops.relpos_attention_chunks(qkv, self.kr[i], self.vr[i], self.cap, meta, B, chunks, self.ptab[i],
                                            L["bu"], L["bv"], T, self.h, self.dk, scale, att)
            else:            # one launch per chunk (A/B)
                for j in range(chunks):
                    mj = meta[4 * B * j:4 * B * (j + 1)]
                    ops.relpos_attention_fused(qkv[j * n1:(j + 1) * n1], self.kr[i], self.vr[i], self.cap, mj[:B],
                                               mj[B:2 * B], mj[2 * B:3 * B], self.ptab[i], mj[3 * B:], L["bu"],
                                               L["bv"], B, T, self.h, self.dk, scale, att[j * n1:(j + 1) * n1])
            if fuse_ln:
                L["out"].rowstats(att, x, sB, residual=True, ypack32=xp32)
                L["ff1"].ln(x, *L["ln2"], sB, out=f, act="relu", ypack=fp, xpack32=xp32)
            else:
                L["out"](att, out=x, residual=True)
                ops.layernorm(x, *L["ln2"], out=h)
                L["ff1"](h, out=f, act="relu")
            if fuse_ln and i < last:
                L["ff2"].rowstats(f, x, sA, residual=True, xpack=fp, ypack32=xp32)
            else:
                L["ff2"](f, out=x, residual=True, xpack=fp)
        ops.layernorm(x, *self.after, out=x)
        return x, T

    def infer(self, feats, caches, pe_indices):
        """feats: device [B, R, 80]; caches: list[EncoderCache]; pe_indices: list[int].
        Returns (out [B*T, d] device fp32, T, new pe_indices)."""
        B, R, _ = feats.shape
        bufs = self.buffers(B, R)
        meta, new_pe = self.host_meta(caches, pe_indices)
        bufs["meta"].copy_(ops.h2d(meta, self.device))
        x, T = self.run(feats, B, R, bufs)
        self.advance(caches, T)
        return x, T, new_pe


class AdapterCache:
    """Caller-owned adapter state (the reference's `adapter_cache`): carried conv input frames."""

    def __init__(self, engine):
        self.engine, self.slot = engine, engine.slots.get()
        for c in engine.caches:
            c[self.slot].zero_()

    def __del__(self):
        try:
            self.engine.slots.put(self.slot)
        except Exception:
            pass


class AdapterEngine:
    """CNNSubsampling (models/adapter.py:72-157), every branch the reference builds:
    cnn_num == 1 (4*d >= L): causal conv1d(d -> 2d, k, stride 2) + eval BatchNorm (a per-column affine
    in the GEMM epilogue) or LayerNorm(2d, eps 1e-3) + ReLU / exact GELU, then Linear(2d -> L);
    cnn_num == 2 (4*d < L): conv1d(d -> 2d, k, stride 1) + BN + ReLU first, then the stride-2 conv
    2d -> 4d + BN + ReLU and Linear(4d -> L), each conv with its own carried k-1 input frames.
    adpter_type 'cnn' / 'linear' (CNNAdapter / LinearAdapter) are rejected at load: their forward takes no
    cache, so the reference's recognize (models/audioLLM.py:386-387) cannot call them either."""

    def __init__(self, src, cfg, ident, device, max_sessions=64):
        mc = cfg["train_yaml"]["model_conf"]
        atype = mc.get("adpter_type", "subsampling")
        if atype != "subsampling":
            raise ValueError(f"adpter_type {atype!r}: only 'subsampling' (CNNSubsampling) streams with a cache "
                             "(models/audioLLM.py:159-165,386-387)")
        self.d, self.L, self.k = mc["enc_out_dim"], mc["llm_embed_dim"], mc["kernel_size"]
        self.cnn_num = 2 if 4 * self.d < self.L else 1
        self.norm = mc.get("norm", "batch") if self.cnn_num == 1 else "batch"
        if self.norm not in ("batch", "layer"):
            raise ValueError(f"adapter norm {self.norm!r}: CNNSubsampling builds bn2 only for 'batch' or 'layer' "
                             "(models/adapter.py:100-103)")
        self.act = "gelu" if (self.cnn_num == 1 and mc.get("activation_func", "relu") == "gelu") else "relu"
        p = f"adpter_{ident}."
        self.device = torch.device(device)
        d, k = self.d, self.k

        def bn_affine(lin, name):
            g, b = src.get(p + name + ".weight"), src.get(p + name + ".bias")
            rm, rv = src.get(p + name + ".running_mean"), src.get(p + name + ".running_var")
            sc = g / torch.sqrt(rv + 1e-3)
            lin.set_affine(sc, b - rm * sc)

        self.conv1 = None
        if self.cnn_num == 2:
            w1 = src.get(p + "conv1d1.weight", torch.bfloat16)  # [2d, d, k] -> [2d, d*k] (col = c*k + j)
            self.conv1 = PackedLinear(w1.reshape(2 * d, d * k), src.get(p + "conv1d1.bias"))
            bn_affine(self.conv1, "bn1")
        cin = d if self.cnn_num == 1 else 2 * d
        w = src.get(p + "conv1d2.weight", torch.bfloat16)
        self.conv = PackedLinear(w.reshape(w.shape[0], cin * k), src.get(p + "conv1d2.bias"))
        self.ln = None
        if self.norm == "batch":
            bn_affine(self.conv, "bn2")
        else:
            self.ln = (src.get(p + "bn2.weight"), src.get(p + "bn2.bias"))
        self.project = PackedLinear(src.get(p + "project.weight", torch.bfloat16), src.get(p + "project.bias"))
        # cache[0]: inputs of the stride-2 conv; cache[1] (cnn_num 2): inputs of the stride-1 conv
        self.cache = torch.zeros(max_sessions, k - 1, cin, dtype=F32, device=self.device)
        self.cache1 = torch.zeros(max_sessions, k - 1, d, dtype=F32, device=self.device) if self.conv1 else None
        self.caches = [c for c in (self.cache, self.cache1) if c is not None]
        self.slots = SlotPool(max_sessions)

    @property
    def weight_bytes(self):
        return self.conv.nbytes + self.project.nbytes + (self.conv1.nbytes if self.conv1 else 0)

    def new_cache(self):
        return AdapterCache(self)

    def out_len(self, T):
        return (self.k - 1 + T - self.k) // 2 + 1

    def buffers(self, B, T):
        To, dev = self.out_len(T), self.device
        e = lambda *shape: torch.empty(*shape, dtype=F32, device=dev)  # noqa: E731
        bufs = {"cols": e(B * To, self.conv.Kp), "y": e(B * To, self.conv.N), "out": e(B * To, self.project.N),
                "slots": torch.empty(B, dtype=I32, device=dev)}
        if self.conv1 is not None:
            bufs["cols1"] = e(B * T, self.conv1.Kp)
            bufs["y1"] = e(B * T, self.conv1.N)
        return bufs

    def run(self, x, B, T, bufs):
        """Device part of __call__ with bufs['slots'] uploaded."""
        KC = self.k - 1
        slots = bufs["slots"]
        if self.conv1 is not None:  # models/adapter.py:123-134
            ops.im2col_conv1d(self.cache1, slots, x, B, KC, T, self.d, self.k, 1, bufs["cols1"])
            ops.conv_cache_update(self.cache1, slots, x, B, KC, T, self.d)
            x = self.conv1(bufs["cols1"], out=bufs["y1"], act="relu")
        cin = self.cache.shape[2]
        ops.im2col_conv1d(self.cache, slots, x, B, KC, T, cin, self.k, 2, bufs["cols"])
        ops.conv_cache_update(self.cache, slots, x, B, KC, T, cin)
        if self.ln is None:
            self.conv(bufs["cols"], out=bufs["y"], act=self.act)
        else:  # LayerNorm over the 2d channels of each frame (models/adapter.py:145-149)
            self.conv(bufs["cols"], out=bufs["y"])
            ops.layernorm(bufs["y"], *self.ln, eps=1e-3, out=bufs["y"], act=self.act)
        return self.project(bufs["y"], out=bufs["out"]), self.out_len(T)

    def __call__(self, x, T, caches):
        """x: device [B*T, d]; returns (out [B*To, L], To)."""
        B = len(caches)
        bufs = self.buffers(B, T)
        bufs["slots"].copy_(ops.h2d(np.asarray([c.slot for c in caches], np.int32), self.device))
        return self.run(x, B, T, bufs)
