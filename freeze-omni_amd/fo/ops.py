"""Thin torch-facing wrappers over the C-ABI kernels.

torch is used only for device memory and the current stream (plumbing); every computation
below is a hand-written gfx950 kernel in libfo_hip.so.
"""
import os
import threading

import numpy as np
import torch

from . import _lib

BF16 = torch.bfloat16
F32 = torch.float32

ACT = {"none": 0, "relu": 1, "silu": 2, "gelu": 3}


def ptr(t):
    return None if t is None else t.data_ptr()


def stream(device=None):
    return torch.cuda.current_stream(device).cuda_stream


_ENGINE_STREAMS = {}


# name prefixes of the streams created at the device's greatest priority: the AR decode's ("tts", "tts1": a second
# speech worker's).  The vocoder streams ("voc*") stay at the default priority: r03y A/B (bench, text steps queued
# ahead) tts + voc high 189.9 / 196.9x, tts only 197.4 / 197.8x (text stage 137-139 -> 134.5 ms, first PCM unchanged
# 58.7 ms), none 188.8 / 192.2x (first PCM 71 ms).  FO_HIGH_PRIO (comma-separated prefixes, "" none) overrides it.
HIGH_PRIORITY_STREAMS = tuple(p for p in os.environ.get("FO_HIGH_PRIO", "tts").split(",") if p)   # () matches none
# priority level of the side stream (the pipelined listen's encoder stage, the vocoder when no "voc" stream is
# given): 0 default, -1 the device's least (FO_SIDE_PRIORITY, A/B probes)
SIDE_STREAM_PRIORITY = int(os.environ.get("FO_SIDE_PRIORITY", "0"))
# and of the engine stream (the Qwen2 stages, the text decode): FO_MAIN_PRIORITY, 0 default, 1 greatest
MAIN_STREAM_PRIORITY = int(os.environ.get("FO_MAIN_PRIORITY", "0"))


# FO_ENC_CUS=k (probe): the side stream (the pipelined listen's encoder stage, fbank) runs on k CUs spread over the
# device's 32-CU blocks and the engine stream on the others, so no Qwen2 workgroup shares a CU with the encoder's
ENC_CUS = int(os.environ.get("FO_ENC_CUS", "0"))


def _enc_partition(idx):
    if ENC_CUS <= 0:
        return None
    n = torch.cuda.get_device_properties(idx).multi_processor_count
    blk = n // 8
    per = max(1, ENC_CUS // 8)
    enc = sorted({x * blk + j for x in range(8) for j in range(per)})
    return [c for c in range(n) if c not in set(enc)], enc, n


def engine_stream(device, side=False, name=None):
    """A blocking HIP stream per device (fo_stream_create) wrapped for torch: it orders against the
    legacy default stream implicitly, and graph capture (which needs a non-null stream) runs on it.
    side=True: a second such stream, for work that overlaps the main one (pipelined listen stages).
    name: further named streams ("tts", "voc": speech generation running beside the text decode; the AR decode's
    "tts*" streams are created at the device's greatest priority, HIGH_PRIORITY_STREAMS, so a sentence's codec
    tokens are not queued behind the text decode's weight streams)."""
    import ctypes
    d = torch.device(device)
    idx = d.index if d.index is not None else torch.cuda.current_device()
    key = (idx, name if name is not None else bool(side))
    if idx in getattr(_SERVE_TLS, "devices", ()):
        return _serve_stream(idx, key[1], name)
    if key not in _ENGINE_STREAMS:
        h = ctypes.c_void_p()
        with torch.cuda.device(idx):
            part = _enc_partition(idx) if name is None else None
            if part is not None:   # listen-stage CU partition: side stream on the encoder's CUs, engine on the rest
                cus = part[1] if side else part[0]
                words = (part[2] + 31) // 32
                m = (ctypes.c_uint * words)()
                for c in cus:
                    m[c // 32] |= 1 << (c % 32)
                with torch.cuda.device(idx):
                    _lib.call("fo_stream_create_cumask", ctypes.byref(h), m, words)
            elif name is not None and name.startswith(HIGH_PRIORITY_STREAMS):
                _lib.call("fo_stream_create_prio", ctypes.byref(h), 1)
            elif name is None and side and SIDE_STREAM_PRIORITY:
                _lib.call("fo_stream_create_prio", ctypes.byref(h), SIDE_STREAM_PRIORITY)
            elif name is None and not side and MAIN_STREAM_PRIORITY:
                _lib.call("fo_stream_create_prio", ctypes.byref(h), MAIN_STREAM_PRIORITY)
            else:
                _lib.call("fo_stream_create", ctypes.byref(h))
        _ENGINE_STREAMS[key] = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))
    return _ENGINE_STREAMS[key]


# The serving threads (fo.serve: one per replica for the listen / text work, one for speech) own their device's work:
# on such a thread engine_stream() hands out a private family of NON-blocking streams instead of the blocking ones
# above.  A caller thread of the reference's threading model (bin/dialog_state_pred.py:802-804) may then run work on
# the legacy default stream (a .cpu() of a PCM segment, a gater's fbank) while the serving thread captures a graph:
# a blocking stream would sync implicitly with that legacy work and invalidate the capture.  The serving thread
# orders its inputs (caller events) and outputs (synchronised before a call returns) itself.
_SERVE_TLS = threading.local()
_SERVE_STREAMS = {}


def serve_streams(idx):
    """Make engine_stream() on the calling thread return the serving stream family of device idx."""
    _SERVE_TLS.devices = tuple(getattr(_SERVE_TLS, "devices", ())) + (idx,)


def _serve_stream(idx, part, name):
    key = (idx, "serve", part)
    if key not in _SERVE_STREAMS:
        hi = name is not None and name.startswith(HIGH_PRIORITY_STREAMS)
        # torch's own streams are created hipStreamNonBlocking; priority -1 is the device's greatest
        _SERVE_STREAMS[key] = torch.cuda.Stream(device=torch.device("cuda", idx), priority=-1 if hi else 0)
    return _SERVE_STREAMS[key]


class Runtime:
    """Scratch (split-K slabs, counters) of the kernels issued on one stream of one device.  Keyed by
    (device, current stream): work on two streams may overlap (the pipelined listen stages), so each
    stream owns its scratch, and a graph's scratch is that of the stream it was captured on."""

    _inst = {}

    def __init__(self, device, ws_floats=1 << 25):
        self.device = torch.device(device)
        self.ws = torch.empty(ws_floats, dtype=F32, device=self.device)
        self.counters = torch.zeros(1 << 20, dtype=torch.int32, device=self.device)

    @classmethod
    def get(cls, device):
        d = torch.device(device)
        idx = d.index if d.index is not None else torch.cuda.current_device()
        key = (d.type, idx, torch.cuda.current_stream(idx).cuda_stream)
        if key not in cls._inst:
            cls._inst[key] = Runtime(torch.device("cuda", idx))
        return cls._inst[key]


def _check_dev(t):
    if not t.is_cuda:
        raise RuntimeError("Freeze-Omni MI355X kernels take device tensors only (no CPU fallback)")


class PackedLinear:
    """A linear layer's weight packed into MFMA fragment order (fo_pack_weight).

    w: [N, K] (f32 or bf16, any device tensor); bias: [N] or None.
    swiglu_up: optional second [N, K] weight; the pair is interleaved so one fo_gemm
    computes silu(x W^T) * (x U^T).
    """

    def __init__(self, w, bias=None, swiglu_up=None, rope_hd=None):
        """rope_hd: w is a fused q|k|v projection with this head dim; tiles are packed in (i, i + hd/2)
        pairs per head for the fused RoPE + KV-append epilogue (qkv_rope)."""
        _check_dev(w)
        w = w.contiguous()
        self.N, self.K = w.shape
        self.Kp = (self.K + 31) // 32 * 32
        self.swiglu = swiglu_up is not None
        nt = (self.N + 15) // 16
        ks = self.Kp // 32
        ntiles = nt * (2 if self.swiglu else 1)
        self.packed = torch.empty(ntiles * ks * 64 * 8, dtype=BF16, device=w.device)
        s = stream(w.device)
        src_bf16 = 1 if w.dtype == BF16 else 0
        if w.dtype not in (BF16, F32):
            w = w.float()
        self.rope_hd = rope_hd
        if rope_hd is not None:
            half = rope_hd // 2
            if rope_hd % 32 or self.N % rope_hd:
                raise ValueError(f"rope packing needs hd % 32 == 0 and N % hd == 0 (N={self.N}, hd={rope_hd})")
            es = w.element_size()
            for h in range(self.N // rope_hd):
                for p in (0, 1):
                    r0 = h * rope_hd + p * half
                    _lib.call("fo_pack_weight", w.data_ptr() + r0 * self.K * es, src_bf16, half, self.K, self.K,
                              self.packed.data_ptr(), h * (rope_hd // 16) + p, 2, s)
        elif self.swiglu:
            u = swiglu_up.contiguous().to(w.dtype)
            _lib.call("fo_pack_weight", w.data_ptr(), src_bf16, self.N, self.K, self.K, self.packed.data_ptr(), 0, 2, s)
            _lib.call("fo_pack_weight", u.data_ptr(), src_bf16, self.N, self.K, self.K, self.packed.data_ptr(), 1, 2, s)
        else:
            _lib.call("fo_pack_weight", w.data_ptr(), src_bf16, self.N, self.K, self.K, self.packed.data_ptr(), 0, 1, s)
        self.bias = None if bias is None else bias.detach().to(device=w.device, dtype=F32).contiguous()
        self.device = w.device

    @property
    def nbytes(self):
        return self.packed.numel() * 2

    def set_affine(self, scale, shift):
        """Per-column y*scale+shift after the bias (eval BatchNorm, models/adapter.py:103-104)."""
        self.scale = scale.detach().to(device=self.device, dtype=F32).contiguous()
        self.shift = shift.detach().to(device=self.device, dtype=F32).contiguous()

    scale = None
    shift = None

    def __call__(self, x, out=None, act="none", residual=False, out_dtype=F32, splitk=0, M=None, norm=None,
                 stats_out=None, xpack=None, ypack=None):
        """x: fp32 or bf16 [M, >=Kp] (row stride x.stride(0)); returns out [M, N].
        norm: (RowStats, eps): x is the producer's yg (= residual * gamma) and rows are scaled by the
        RMSNorm rstd from the producer's statistics; stats_out: RowStats this GEMM fills (see RowStats).
        xpack: XPack holding x (<= 64 rows) pre-split in fragment order (written by its producer), read instead of
        splitting x by the kernels that take packed X (include/fo_hip.h fo_gemm_set_xpack; the others read x);
        ypack: XPack this GEMM fills with stats_out's yg -- or, without stats_out, its output (<= 64 rows)."""
        if norm is not None or stats_out is not None:
            return self._call_norm(x, out, act, residual, out_dtype, splitk, M, norm, stats_out, xpack, ypack)
        _check_dev(x)
        if x.dtype not in (BF16, F32):
            raise TypeError("PackedLinear input must be fp32 or bf16")
        if x.stride(-1) != 1 or x.shape[-1] < self.Kp:
            raise ValueError(f"PackedLinear input needs unit stride and >= {self.Kp} columns, got {tuple(x.shape)}")
        M = x.shape[0] if M is None else M
        if out is None:
            out = torch.empty(M, self.N, dtype=out_dtype, device=x.device)
        rt = Runtime.get(x.device)
        with _packed(xpack, None):
            _lib.call("fo_gemm", x.data_ptr(), 1 if x.dtype == F32 else 0, x.stride(0), M, self.Kp,
                      self.packed.data_ptr(), self.N, 1 if self.swiglu else 0, ptr(self.bias), ptr(self.scale),
                      ptr(self.shift), out.data_ptr(), out.stride(0), 1 if out.dtype == BF16 else 0, ACT[act],
                      1 if residual else 0, rt.ws.data_ptr(), rt.ws.numel(), rt.counters.data_ptr(), splitk,
                      stream(x.device))
        return out


    def ln(self, x, lnw, lnb, stats, eps=1e-5, out=None, act="none", M=None, splitk=0, ypack=None, xpack32=None):
        """act(LayerNorm(x) W^T + b) with the norm applied as X is loaded (fo_gemm_ln; M <= 64); stats:
        the RowStats(with_sums=True) a rowstats() producer filled for x."""
        _check_dev(x)
        M = x.shape[0] if M is None else M
        if x.dtype != F32 or x.stride(-1) != 1 or x.shape[-1] < self.Kp or self.Kp != self.K:
            raise ValueError("fused LayerNorm GEMM needs fp32 unit-stride X with K % 32 == 0")
        if stats.groups <= 0 or stats.buf1 is None:
            raise RuntimeError("LayerNorm statistics consumed before a producer filled them")
        if out is None:
            out = torch.empty(M, self.N, dtype=F32, device=x.device)
        rt = Runtime.get(x.device)
        with _packed(None, ypack, xpack32):
            _lib.call("fo_gemm_ln", x.data_ptr(), x.stride(0), M, self.Kp, self.packed.data_ptr(), self.N,
                      ptr(self.bias), lnw.data_ptr(), lnb.data_ptr(), float(eps), stats.buf1.data_ptr(),
                      stats.buf.data_ptr(), stats.groups, out.data_ptr(), out.stride(0), ACT[act], rt.ws.data_ptr(),
                      rt.ws.numel(), splitk, stream(x.device))
        return out

    def rowstats(self, x, out, stats, residual=False, act="none", M=None, splitk=0, xpack=None, ypack32=None):
        """fp32 GEMM that also fills stats (per-row partial sums of out and out^2) for ln()."""
        import ctypes
        _check_dev(x)
        M = x.shape[0] if M is None else M
        if stats.buf1 is None:
            raise ValueError("rowstats needs RowStats(with_sums=True)")
        rt = Runtime.get(x.device)
        sg = ctypes.c_int(0)
        with _packed(xpack, None, None, ypack32):
            _lib.call("fo_gemm_rowstats", x.data_ptr(), 1 if x.dtype == F32 else 0, x.stride(0), M, self.Kp,
                      self.packed.data_ptr(), self.N, ptr(self.bias), out.data_ptr(), out.stride(0), ACT[act],
                      1 if residual else 0, rt.ws.data_ptr(), rt.ws.numel(), rt.counters.data_ptr(), splitk,
                      stats.buf1.data_ptr(), stats.buf.data_ptr(), ctypes.byref(sg), stream(x.device))
        if sg.value > stats.max_groups:
            raise RuntimeError(f"RowStats holds {stats.max_groups} groups per row, GEMM wrote {sg.value}")
        stats.groups = sg.value
        return out

    def qkv_rope(self, x, M, pos, slot, cos_t, sin_t, q_out, kc, vc, H, KVH, PS, norm=None, splitk=0, xpack=None):
        """Fused q|k|v projection + bias + RoPE + paged-KV append (weight packed with rope_hd):
        q_out [M, H*hd] gets the rotated queries, kc/vc (one layer's pages) the token's K/V rows at slot[m]."""
        _check_dev(x)
        if self.rope_hd is None:
            raise RuntimeError("qkv_rope needs a weight packed with rope_hd")
        if x.stride(-1) != 1 or x.shape[-1] < self.Kp or x.dtype not in (F32, BF16):
            raise ValueError("qkv_rope input needs unit stride, fp32/bf16 and >= Kp columns")
        rt = Runtime.get(x.device)
        rst, rg, eps = (None, 0, 0.0) if norm is None else (norm[0].buf.data_ptr(), norm[0].groups, float(norm[1]))
        if norm is not None and rg <= 0:
            raise RuntimeError("RowStats consumed before any GEMM produced them")
        with _packed(xpack, None):
            _lib.call("fo_gemm_qkv_rope", x.data_ptr(), 1 if x.dtype == F32 else 0, x.stride(0), M, self.Kp,
                      self.packed.data_ptr(), self.N, ptr(self.bias), rt.ws.data_ptr(), rt.ws.numel(),
                      rt.counters.data_ptr(), splitk, rst, rg, eps, pos.data_ptr(), slot.data_ptr(), cos_t.data_ptr(),
                      sin_t.data_ptr(), q_out.data_ptr(), kc.data_ptr(), vc.data_ptr(), H, KVH, self.rope_hd, PS,
                      stream(x.device))
        return q_out

    def _call_norm(self, x, out, act, residual, out_dtype, splitk, M, norm, stats_out, xpack=None, ypack=None):
        import ctypes
        _check_dev(x)
        if x.stride(-1) != 1 or x.shape[-1] < self.Kp or out_dtype != F32:
            raise ValueError("fused RMSNorm GEMM needs unit-stride X and fp32 output")
        M = x.shape[0] if M is None else M
        if out is None:
            out = torch.empty(M, self.N, dtype=F32, device=x.device)
        rt = Runtime.get(x.device)
        rst, rg, eps = (None, 0, 0.0) if norm is None else (norm[0].buf.data_ptr(), norm[0].groups, float(norm[1]))
        if norm is not None and rg <= 0:
            raise RuntimeError("RowStats consumed before any GEMM produced them")
        so = gn = yg = None
        if stats_out is not None:
            so, gn, yg = stats_out.buf.data_ptr(), stats_out.gamma.data_ptr(), stats_out.yg.data_ptr()
            if stats_out.yg.stride(0) != out.stride(0):
                raise ValueError("yg must share the output's row stride")
        sg = ctypes.c_int(0)
        if ypack is not None and stats_out is None:
            raise ValueError("ypack packs the stats_out yg: pass stats_out")
        with _packed(xpack, ypack):
            _lib.call("fo_gemm_rms", x.data_ptr(), 1 if x.dtype == F32 else 0, x.stride(0), M, self.Kp,
                      self.packed.data_ptr(), self.N, 1 if self.swiglu else 0, ptr(self.bias), out.data_ptr(),
                      out.stride(0), ACT[act], 1 if residual else 0, rt.ws.data_ptr(), rt.ws.numel(),
                      rt.counters.data_ptr(), splitk, rst, rg, eps, so, gn, yg, ctypes.byref(sg), stream(x.device))
        if stats_out is not None:
            if sg.value > stats_out.max_groups:
                raise RuntimeError(f"RowStats holds {stats_out.max_groups} groups per row, GEMM wrote {sg.value}")
            stats_out.groups = sg.value
        return out


# FO_XPACK=0 turns the packed <= 64-row activations off (A/B only)
XPACK = os.environ.get("FO_XPACK", "1") != "0"


class XPack:
    """An fp32 activation of <= 64 rows also held as bf16 hi + lo in MFMA A-fragment order ([K/32][row blocks][64][8]
    each; lane l = row l & 15 of the row block, columns 8 (l >> 4) .. + 8 of a 32-column k-step): its producer kernel writes it beside
    the fp32 rows, and the consuming one-row-tile GEMM reads one contiguous 1 KiB per wave and half instead of 16
    row segments per float4 (Qwen2 o 11.4 -> 9.2 us, q|k|v 13.7 -> 11.8 us at 16 rows, results bit-identical:
    scripts/gemm_xpack_probe.py)."""

    def __init__(self, K, device, rows=16):
        if K % 32 or not 1 <= rows <= 64:
            raise ValueError("XPack needs K % 32 == 0 and <= 64 rows")
        self.K, self.rows = K, rows
        self.rb = (rows + 15) // 16        # allocated row blocks (the extent the C-ABI setters pass along)
        n = K * 16 * self.rb               # [K/32][row blocks][64][8]
        self.hi = torch.empty(n, dtype=BF16, device=device)
        self.lo = torch.empty(n, dtype=BF16, device=device)


class XPack32:
    """The fp32 form of XPack's fragment order ([K/32][row blocks][64][8] floats): the speech encoder's residual
    stream for its LayerNorm-on-load GEMMs, which need the exact fp32 values (written by the out / FFN-down GEMMs
    beside the row-major rows)."""

    def __init__(self, K, device, rows):
        if K % 32 or not 1 <= rows <= 64:
            raise ValueError("XPack32 needs K % 32 == 0 and <= 64 rows")
        self.K, self.rows = K, rows
        self.rb = (rows + 15) // 16
        self.buf = torch.empty(K * 16 * self.rb, dtype=F32, device=device)


class _packed:
    """Arms fo_gemm's packed-X input / packed-yg output for the one launch inside the block (thread-local in the
    library, consumed by that launch -- also when the launch refuses its arguments, e.g. a pack whose extent does not
    fit); the disarm on an exception covers a failure between the setters and the launch."""

    def __init__(self, xpack, ypack, xpack32=None, ypack32=None):
        self.x, self.y, self.x32, self.y32 = xpack, ypack, xpack32, ypack32

    def __enter__(self):
        if self.x is not None:
            _lib.call("fo_gemm_set_xpack", self.x.hi.data_ptr(), self.x.lo.data_ptr(), self.x.K, self.x.rb)
        if self.y is not None:
            _lib.call("fo_gemm_set_ypack", self.y.hi.data_ptr(), self.y.lo.data_ptr(), self.y.K, self.y.rb)
        if self.x32 is not None:
            _lib.call("fo_gemm_set_xpack32", self.x32.buf.data_ptr(), self.x32.K, self.x32.rb)
        if self.y32 is not None:
            _lib.call("fo_gemm_set_ypack32", self.y32.buf.data_ptr(), self.y32.K, self.y32.rb)

    def __exit__(self, et, ev, tb):
        if et is not None:
            if self.x is not None:
                _lib.call("fo_gemm_set_xpack", None, None, 0, 0)
            if self.y is not None:
                _lib.call("fo_gemm_set_ypack", None, None, 0, 0)
            if self.x32 is not None:
                _lib.call("fo_gemm_set_xpack32", None, 0, 0)
            if self.y32 is not None:
                _lib.call("fo_gemm_set_ypack32", None, 0, 0)
        return False


class RowStats:
    """RMSNorm split across two GEMMs: the producer writes per-row partial sums of squares of its
    output (buf) and yg = output * gamma (the next norm's weight); the consumer GEMM reads yg as its
    input and scales rows by rsqrt(sum / K + eps).  set(gamma, yg) before each producer call."""

    def __init__(self, rows, device, max_groups=256, with_sums=False):
        self.max_groups = max_groups
        self.buf = torch.empty(rows * max_groups, dtype=F32, device=device)
        self.buf1 = torch.empty(rows * max_groups, dtype=F32, device=device) if with_sums else None  # LayerNorm
        self.groups = 0
        self.gamma = self.yg = None

    def set(self, gamma, yg):
        self.gamma, self.yg = gamma, yg
        return self


def h2d(a, device, dtype=None):
    """Host values -> a new device tensor WITHOUT a stream synchronisation (a plain `.to(device)` of pageable
    memory synchronises the stream, which on the eager paths -- duplex ticks, prefills -- stalls the host's launch
    queue behind the GPU): the values are staged in pinned memory from PyTorch's caching host allocator (which keeps
    the block until the copy recorded on the stream has run) and copied asynchronously on the current stream.
    Never used while a graph is being captured (a captured copy would keep reading a recycled staging block)."""
    t = a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    if torch.device(device).type != "cuda":   # host-only bookkeeping tests (tests/test_host_cpu.py)
        return t.clone()
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("ops.h2d inside a graph capture")
    p = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    if t.dtype in (torch.float32, torch.int32, torch.int64, torch.float64) and t.is_contiguous():
        # numpy's single-threaded copy: torch's copy_ of >= 32K elements fans out over the OpenMP pool, whose
        # spinning threads, on a CPU-quota'd host, got the process throttled (~60 ms duplex ticks, r05z)
        p.numpy()[...] = t.numpy()
    else:
        p.copy_(t)
    return p.to(device, non_blocking=True)


# ---------------------------------------------------------------- launch counters (include/fo_hip.h FoLaunchKind)
LAUNCH_KINDS = ("gemm_xs", "gemm_xsk", "gemm_xp", "gemm_reduce", "gemm_ln", "gemm_xp32", "gemm_ypack", "gemm_ypack32",
                "gemm_mid", "gemm_rope4", "gemm_pipe", "gemm_other", "attn_mfma", "attn_decode", "attn_opack", "relpos",
                "subsample", "attn_o", "enc_block", "gemm_rows")


def launch_counts():
    """{kind: launches issued since the last reset} (host-side counters; a captured graph counts at capture)."""
    import ctypes
    lib = _lib.load()
    n = lib.fo_launch_counts(None, 0)
    buf = (ctypes.c_longlong * n)()
    lib.fo_launch_counts(buf, n)
    return {k: int(buf[i]) for i, k in enumerate(LAUNCH_KINDS)}


def launch_counts_reset():
    _lib.call("fo_launch_counts_reset")


# ---------------------------------------------------------------- kernel wrappers
I32 = torch.int32


def fill_hash(out, key, center, scale):
    _check_dev(out)
    _lib.call("fo_fill_hash", out.data_ptr(), 1 if out.dtype == BF16 else 0, out.numel(), key & 0xFFFFFFFFFFFFFFFF,
              float(center), float(scale), stream(out.device))
    return out


def rmsnorm(x, w, eps, out=None, round_fp16=False, M=None):
    M = x.shape[0] if M is None else M
    out = torch.empty_like(x) if out is None else out
    _lib.call("fo_rmsnorm", x.data_ptr(), x.stride(0), M, x.shape[1], w.data_ptr(), float(eps), out.data_ptr(),
              out.stride(0), 1 if round_fp16 else 0, stream(x.device))
    return out


def layernorm(x, w, b, eps=1e-5, out=None, relu=False, M=None, act=None):
    """Row LayerNorm; act ('relu' | 'gelu', or relu=True) applied after the affine."""
    M = x.shape[0] if M is None else M
    out = torch.empty_like(x) if out is None else out
    a = ACT[act] if act is not None else (ACT["relu"] if relu else 0)
    _lib.call("fo_layernorm", x.data_ptr(), x.stride(0), M, x.shape[1], w.data_ptr(), b.data_ptr(), float(eps),
              out.data_ptr(), out.stride(0), a, stream(x.device))
    return out


def gather_rows(table, idx, out=None, round_fp16=False, D=None, M=None, out_rows=None):
    """out[out_rows[m]] = table[idx[m]] (None: identity).  table f32 or bf16 2-D."""
    D = table.shape[1] if D is None else D
    M = (idx.numel() if idx is not None else table.shape[0]) if M is None else M
    if out is None:
        out = torch.empty(M, D, dtype=F32, device=table.device)
    _lib.call("fo_gather_rows", table.data_ptr(), 1 if table.dtype == BF16 else 0, table.stride(0), ptr(idx), M, D,
              out.data_ptr(), out.stride(0), ptr(out_rows), 1 if round_fp16 else 0, stream(table.device))
    return out


def im2col_3x3s2(x, B, C, H, W, strides, out, mean=None, istd=None):
    _lib.call("fo_im2col_3x3s2", x.data_ptr(), B, C, H, W, *strides, ptr(mean), ptr(istd), out.data_ptr(),
              out.stride(0), stream(x.device))
    return out


def subsample(feats, B, R, F, mean, istd, w1, b1, C, y1, w2p, b2, z):
    """Conv2dSubsampling4 (+ GlobalCMVN) up to its output Linear: feats [B, R, F] -> z [B * H2, C * W2]
    (fo_subsample; split-K scratch at the HEAD of the stream's Runtime workspace -- the same floats the GEMMs' split-K
    slabs use, which is safe because launches on one stream run in order)."""
    n = int(_lib.load().fo_subsample_ws_floats(B, R, F, C))
    rt = Runtime.get(feats.device)
    if n > rt.ws.numel():
        raise RuntimeError(f"subsample: {n} workspace floats > {rt.ws.numel()}")
    _lib.call("fo_subsample", feats.data_ptr(), B, R, F, mean.data_ptr(), istd.data_ptr(), w1.data_ptr(), b1.data_ptr(),
              C, y1.data_ptr(), w2p.data_ptr(), b2.data_ptr(), z.data_ptr(), rt.ws.data_ptr(), rt.ws.numel(),
              stream(feats.device))
    return z


def tcf_permute(x, B, T, F, C, out):
    _lib.call("fo_tcf_permute", x.data_ptr(), B, T, F, C, out.data_ptr(), stream(x.device))
    return out


def im2col_conv1d(cache, slots, x, B, KC, T, D, K, S, out):
    _lib.call("fo_im2col_conv1d", ptr(cache), ptr(slots), x.data_ptr(), B, KC, T, D, K, S, out.data_ptr(),
              out.stride(0), stream(x.device))
    return out


def conv_cache_update(cache, slots, x, B, KC, T, D):
    _lib.call("fo_conv_cache_update", cache.data_ptr(), ptr(slots), x.data_ptr(), B, KC, T, D, stream(x.device))


def state_head(h, rows, W, b, out):
    _lib.call("fo_state_head", h.data_ptr(), h.stride(0), rows.data_ptr(), rows.numel(), W.data_ptr(), b.data_ptr(),
              h.shape[1], out.data_ptr(), stream(h.device))
    return out


def record_ids(ids, B, dst_ptr, ld, row):
    """dst[row[0] * ld + b] = ids[b] for b < B (dst: device pointer, e.g. HostBuffer.dev)."""
    _lib.call("fo_record_ids", ids.data_ptr(), B, dst_ptr, ld, row.data_ptr(), stream(ids.device))


class HostBuffer:
    """int32 [rows, cols] in pinned, device-mapped host memory (fo_host_alloc): kernels write through
    .dev, the host reads .np after the writing work has completed."""

    def __init__(self, rows, cols):
        import ctypes
        import numpy as np
        self.rows, self.cols = rows, cols
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.call("fo_host_alloc", rows * cols * 4, ctypes.byref(h), ctypes.byref(d))
        self.host, self.dev = h.value, d.value
        buf = (ctypes.c_int32 * (rows * cols)).from_address(self.host)
        self.np = np.frombuffer(buf, dtype=np.int32).reshape(rows, cols)

    def free(self):
        if self.host:
            self.np = None
            _lib.call("fo_host_free", self.host)
            self.host = self.dev = None


def scale_(x, s):
    _lib.call("fo_scale", x.data_ptr(), x.numel(), float(s), stream(x.device))
    return x


# FO_ATTN_ROWS=32: the Qwen2 prefills cut into work items of up to 32 query rows (4 tokens x 7 heads sharing one K / V
# read, k_attn_mfma<128, 8, 2>) instead of 16 -- measured on the duplex line (r05j, two rounds of 30 s): p50 decision
# 7.96 / 7.85 ms against 7.91 / 7.71 with 16-row items (half the work items, each with twice the MFMA and softmax work
# per key, one workgroup per CU at 103 KB of LDS), so 16 stays the policy (A/B only)
ATTN_ROWS32 = os.environ.get("FO_ATTN_ROWS") == "32"


def attn_max_rows(hd):
    """Query rows (tokens x query heads per kv head) one fo_attention work item may carry (the kernels' limit)."""
    return _lib.load().fo_attn_max_rows(int(hd))


def attn_item_rows(hd):
    """Query rows per work item the stacks cut their batches into (the policy, <= attn_max_rows)."""
    return attn_max_rows(hd) if ATTN_ROWS32 else 16


def attn_nsplit(max_keys, n_items, KVH):
    return _lib.load().fo_attn_nsplit(int(max_keys), int(n_items), int(KVH))


def rope_kv_write(qkv, T, H, KVH, hd, pos, slot, cos_t, sin_t, q_out, kc, vc, PS):
    _lib.call("fo_rope_kv_write", qkv.data_ptr(), qkv.stride(0), T, H, KVH, hd, pos.data_ptr(), slot.data_ptr(),
              cos_t.data_ptr(), sin_t.data_ptr(), q_out.data_ptr(), kc.data_ptr(), vc.data_ptr(), PS,
              stream(qkv.device))


# keys per split of the multi-row attention: 0 (default) = attn_keys_per_split() per launch; FO_ATTN_KPS fixes it
# (round 4: 128 everywhere)
ATTN_KEYS_PER_SPLIT = int(os.environ.get("FO_ATTN_KPS", "0"))
_CUS = {}


def attn_keys_per_split(max_keys, n_items, KVH, hd, device=None):
    """Keys per split of a k_attn_mfma launch with the in-launch merge: the smallest multiple of 64, at least 128,
    that keeps its grid (items x kv heads x splits) within one workgroup per CU.  The head-dim-128 kernel holds 256
    VGPRs a lane, so one 8-wave workgroup fills a CU and a larger grid runs in rounds, each paying the staging,
    partial stores and merge again: a duplex tick's 19 items x 4 kv heads x 7 splits of 128 keys were 532
    workgroups in 3 rounds.  At 8 sessions x 1-2 tokens (32 items x kv heads) this stays 128 up to 1024 keys,
    where r03c's sweep put 128 first (scripts/attn_kps_sweep.py: 800 keys 21.7 us vs 24.2 at 256)."""
    if hd != 128:
        return 128
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    cus = _CUS.get(dev)
    if cus is None:
        cus = _CUS[dev] = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 256
    slots = max(1, cus // max(1, n_items * KVH))
    per = -(-int(max_keys) // slots)
    # at most one split's LDS page table (256 pages of 16 keys; the kernel also keeps its split count at least
    # ceil(keys / 4096), so a longer sequence never takes the poison branch)
    return min(ATTN_MAX_SPLIT_KEYS, max(128, -(-per // 64) * 64))


ATTN_MAX_SPLIT_KEYS = 4096


def attention(q, T, items, n_items, max_rows, tok_nvis, block_table, PS, kc, vc, H, KVH, hd, scale, nsplit,
              part_ml, part_o, out, tickets=None, keys_per_split=128, opack=None):
    """tickets: zeroed int32 [>= n_items * KVH] -> splits sized from each item's key count (at most
    nsplit) merged inside the launch; None -> nsplit static splits + a combine launch.
    items None: a uniform batch, T / n_items tokens per sequence in sequence order (item b = sequence b); a
    decode batch is the one-token case."""
    if items is None and T % n_items:
        raise ValueError("attention: items=None needs T / n_items tokens per sequence")
    if tickets is not None and tickets.numel() < n_items * KVH:
        raise ValueError("attention tickets buffer smaller than n_items * KVH")
    if opack is not None:
        _lib.call("fo_attention_set_opack", opack.hi.data_ptr(), opack.lo.data_ptr(), opack.K, opack.rb)
    try:
        _lib.call("fo_attention", q.data_ptr(), T, ptr(items), n_items, max_rows, tok_nvis.data_ptr(),
                  block_table.data_ptr(), block_table.shape[1], PS, kc.data_ptr(), vc.data_ptr(), H, KVH, hd,
                  float(scale), nsplit, ptr(part_ml), ptr(part_o), out.data_ptr(), ptr(tickets), int(keys_per_split),
                  stream(q.device))
    except Exception:
        if opack is not None:   # the launch did not consume it: never leave it for the next one
            _lib.call("fo_attention_set_opack", None, None, 0, 0)
        raise
    return out


def attention_o(q, T, items, tok_nvis, block_table, PS, kc, vc, H, hd, scale, wo, part, tickets, x, gnext, yg, stats):
    """Decode attention (one token per sequence, MHA) + the o projection (PackedLinear wo) + residual into x + the
    next RMSNorm's statistics (stats: RowStats filled with one group; yg = x * gnext) -- fo_attention_o."""
    if tickets.numel() < T or part.numel() < T * H * wo.N:
        raise ValueError("attention_o: tickets / partial buffers too small")
    _lib.call("fo_attention_o", q.data_ptr(), T, ptr(items), tok_nvis.data_ptr(), block_table.data_ptr(),
              block_table.shape[1], PS, kc.data_ptr(), vc.data_ptr(), H, hd, float(scale), wo.packed.data_ptr(), wo.N,
              part.data_ptr(), tickets.data_ptr(), x.data_ptr(), x.stride(0), gnext.data_ptr(), yg.data_ptr(),
              stats.buf.data_ptr(), stream(q.device))
    stats.groups = 1
    return x


def enc_attn_block(x, B, T, h, ln1, qkv, kr, vr, cap, meta, ptab, bu, bv, out, scale, part, tickets, stats,
                   eps=1e-5):
    """The attention half of a speech-encoder block in one launch (fo_enc_attn_block): x [B*T, d] += linear_out(
    relpos attention(q|k|v(LayerNorm1(x)))) in place; stats (RowStats with_sums) gets the updated rows' sums in one
    group for the FFN's LayerNorm-on-load GEMM.  qkv / out: PackedLinear; meta: int32 [4B]."""
    d = x.shape[1]
    if part.numel() < B * h * T * d or tickets.numel() < B or stats.buf1 is None:
        raise ValueError("enc_attn_block: partial / ticket / statistics buffers too small")
    _lib.call("fo_enc_attn_block", x.data_ptr(), B, T, d, h, ln1[0].data_ptr(), ln1[1].data_ptr(), float(eps),
              qkv.packed.data_ptr(), qkv.bias.data_ptr(), kr.data_ptr(), vr.data_ptr(), cap, meta.data_ptr(),
              ptab.data_ptr(), bu.data_ptr(), bv.data_ptr(), out.packed.data_ptr(), out.bias.data_ptr(), float(scale),
              part.data_ptr(), tickets.data_ptr(), stats.buf1.data_ptr(), stats.buf.data_ptr(), stream(x.device))
    stats.groups = 1
    return x


def enc_attn_out(qkv, x, B, T, h, kr, vr, cap, meta, ptab, bu, bv, out, scale, part, tickets, stats):
    """fo_enc_attn_out: the rel-pos attention of the chunk's q|k|v rows (qkv [B*T, >= 3d], bias applied) + linear_out
    (PackedLinear out) + the residual into x (in place); stats (RowStats with_sums) gets the updated rows' sums in one
    group."""
    d = x.shape[1]
    if part.numel() < B * h * T * d or tickets.numel() < B or stats.buf1 is None:
        raise ValueError("enc_attn_out: partial / ticket / statistics buffers too small")
    _lib.call("fo_enc_attn_out", qkv.data_ptr(), qkv.stride(0), x.data_ptr(), B, T, d, h, kr.data_ptr(), vr.data_ptr(),
              cap, meta.data_ptr(), ptab.data_ptr(), bu.data_ptr(), bv.data_ptr(), out.packed.data_ptr(),
              out.bias.data_ptr(), float(scale), part.data_ptr(), tickets.data_ptr(), stats.buf1.data_ptr(),
              stats.buf.data_ptr(), stream(x.device))
    stats.groups = 1
    return x


def enc_kv_write(k, v, B, T, d, start, length, ring, cap, kr, vr):
    _lib.call("fo_enc_kv_write", k.data_ptr(), v.data_ptr(), k.stride(0), B, T, d, start.data_ptr(),
              length.data_ptr(), ptr(ring), cap, kr.data_ptr(), vr.data_ptr(), stream(k.device))


def relpos_attention_fused(qkv, kr, vr, cap, start, length, ring, ptab, pstart, bu, bv, B, T, h, dk, scale, out,
                           opack=None):
    if opack is not None:
        _lib.call("fo_attention_set_opack", opack.hi.data_ptr(), opack.lo.data_ptr(), opack.K, opack.rb)
    try:
        _relpos_fused_call(qkv, kr, vr, cap, start, length, ring, ptab, pstart, bu, bv, B, T, h, dk, scale, out)
    except Exception:
        if opack is not None:   # the launch did not consume it: never leave it for the next one
            _lib.call("fo_attention_set_opack", None, None, 0, 0)
        raise


def _relpos_fused_call(qkv, kr, vr, cap, start, length, ring, ptab, pstart, bu, bv, B, T, h, dk, scale, out):
    _lib.call("fo_relpos_attention_fused", qkv.data_ptr(), qkv.stride(0), kr.data_ptr(), vr.data_ptr(), cap,
              start.data_ptr(), length.data_ptr(), ptr(ring), ptab.data_ptr(), pstart.data_ptr(), bu.data_ptr(),
              bv.data_ptr(), B, T, h, dk, float(scale), out.data_ptr(), out.stride(0), stream(qkv.device))


def relpos_attention_chunks(qkv, kr, vr, cap, meta, B, C, ptab, bu, bv, T, h, dk, scale, out):
    """C consecutive chunks of B users' rel-pos attention in one launch (fo_relpos_attention_chunks); meta [C * 4 B]."""
    if meta.numel() < 4 * B * C or qkv.shape[0] < B * C * T or out.shape[0] < B * C * T:
        raise ValueError("relpos_attention_chunks: meta / q|k|v / out smaller than C chunks of B users x T rows")
    _lib.call("fo_relpos_attention_chunks", qkv.data_ptr(), qkv.stride(0), kr.data_ptr(), vr.data_ptr(), cap,
              meta.data_ptr(), B, C, ptab.data_ptr(), bu.data_ptr(), bv.data_ptr(), T, h, dk, float(scale),
              out.data_ptr(), out.stride(0), stream(qkv.device))
    return out


def relpos_attention(q, kr, vr, cap, start, length, ring, ptab, pstart, bu, bv, B, T, h, dk, scale, out):
    _lib.call("fo_relpos_attention", q.data_ptr(), q.stride(0), kr.data_ptr(), vr.data_ptr(), cap, start.data_ptr(),
              length.data_ptr(), ptr(ring), ptab.data_ptr(), pstart.data_ptr(), bu.data_ptr(), bv.data_ptr(), B, T, h,
              dk, float(scale), out.data_ptr(), out.stride(0), stream(q.device))
    return out


def fbank(samples, B, n_samples, wl, ws, nfft, window, tw_cos, tw_sin, mel, out, row0, zero_rows=None):
    """samples [B][ld] -> out [B][R*nmel] rows row0.. (one per frame); frames < zero_rows[b] are zeroed."""
    _lib.call("fo_fbank", samples.data_ptr(), samples.stride(0), B, n_samples, wl, ws, nfft, window.data_ptr(),
              tw_cos.data_ptr(), tw_sin.data_ptr(), mel.data_ptr(), mel.shape[0], out.data_ptr(), out.stride(0),
              row0, ptr(zero_rows), stream(samples.device))


def rows_shift(feats, B, R, ov, D):
    _lib.call("fo_rows_shift", feats.data_ptr(), B, R, ov, D, stream(feats.device))


def conv1d(x, B, Cin, Tin, w, bias, Cout, K, dil, pad, out, pre_leaky=None, residual=False, post_tanh=False):
    _lib.call("fo_conv1d", x.data_ptr(), B, Cin, Tin, w.data_ptr(), ptr(bias), Cout, K, dil, pad,
              0 if pre_leaky is None else 1, 0.0 if pre_leaky is None else float(pre_leaky), out.data_ptr(),
              1 if residual else 0, 1 if post_tanh else 0, stream(x.device))
    return out


class PackedConv:
    """Conv1d weight packed into MFMA A-fragment order for fo_conv_cl (channel-last activations).
    w: conv [Cout][Cin][K]; or, for one polyphase component of a ConvTranspose1d with stride u,
    w: [Cin][Cout][Ktot] with transposed=(j0, u) -> taps j0, j0+u, ... reversed."""

    def __init__(self, w, bias, transposed=None):
        _check_dev(w)
        w = w.contiguous()
        src_bf16 = 1 if w.dtype == BF16 else 0
        if w.dtype not in (BF16, F32):
            w = w.float()
        if transposed is None:
            self.Cout, self.Cin, self.K = w.shape
            Ktot, j0, u = self.K, 0, 1
        else:
            j0, u = transposed
            self.Cin, self.Cout, Ktot = w.shape
            self.K = (Ktot - j0 + u - 1) // u
        n = _lib.load().fo_conv_pack_elems(self.Cout, self.Cin, self.K)
        self.packed = torch.empty(n, dtype=BF16, device=w.device)
        _lib.call("fo_pack_conv", w.data_ptr(), src_bf16, self.Cout, self.Cin, self.K, 0 if transposed is None else 1,
                  Ktot, j0, u, self.packed.data_ptr(), stream(w.device))
        self.bias = None if bias is None else bias.detach().to(device=w.device, dtype=F32).contiguous()


def conv_cl(x, B, Cin, Tin, pc, dil, pad, out, Tq=None, ostride=1, ooff=0, Tout_total=None, pre_leaky=None,
            res=None, res2=None, oscale=1.0, gadd=None):
    """out[b][q*ostride+ooff][:] = (conv(x)[b][q] + res + res2) * oscale + gadd[b] for q < Tq;
    x [B][Tin][Cin], out/res/res2 [B][Tout_total][Cout] (res/res2 may be out itself), gadd [B][Cout]."""
    Tq = Tin + 2 * pad - dil * (pc.K - 1) if Tq is None else Tq
    Tout_total = Tq if Tout_total is None else Tout_total
    _lib.call("fo_conv_cl", x.data_ptr(), B, Cin, Tin, pc.packed.data_ptr(), ptr(pc.bias), pc.Cout, pc.K, dil, pad,
              Tq, ostride, ooff, Tout_total, 0 if pre_leaky is None else 1,
              0.0 if pre_leaky is None else float(pre_leaky), out.data_ptr(), ptr(res), ptr(res2), float(oscale),
              ptr(gadd), stream(x.device))
    return out


def conv_desc(x, Tin, pc, dil, pad, out, Tq=None, ostride=1, ooff=0, Tout_total=None, pre_leaky=None, res=None,
              res2=None, oscale=1.0, gadd=None):
    """One member of a conv_cl_multi launch (arguments as conv_cl's); returns (descriptor, keep-alive refs)."""
    Tq = Tin + 2 * pad - dil * (pc.K - 1) if Tq is None else Tq
    Tout_total = Tq if Tout_total is None else Tout_total
    d = _lib.FoConvDesc(x.data_ptr(), pc.packed.data_ptr(), ptr(pc.bias), out.data_ptr(), Tin, pc.K, dil, pad, Tq,
                        ostride, ooff, Tout_total, 0 if pre_leaky is None else 1,
                        0.0 if pre_leaky is None else float(pre_leaky), ptr(res), ptr(res2), float(oscale), ptr(gadd))
    return d


def conv_cl_multi(descs, B, Cin, Cout, device, summed=False):
    """G = len(descs) convolutions in one launch (fo_conv_cl_multi): independent members (polyphase components,
    parallel resblock chains), or summed=True: one output = (sum of the members' conv + bias + res) * oscale +
    gadd of descs[0]."""
    arr = (_lib.FoConvDesc * len(descs))(*descs)
    _lib.call("fo_conv_cl_multi", arr, len(descs), B, Cin, Cout, 1 if summed else 0, stream(device))


# channel counts that take fo_conv_pair_multi by default: 16 and 32 (r03l: the 16-channel stage 247 -> 173 us a
# call, the 32-channel one 272 -> 233 us); at 64 channels the kernel needs 122 KB of LDS (one workgroup per CU)
# and is slower than two launches (3 x 111 vs 6 x 43 us), so that stage keeps k_conv_cl
PAIR_CHANNELS = (16, 32)


def conv_pair_multi(members, B, C, T, device, slope=0.1, summed=False, oscale=1.0, gadd=None):
    """ResBlock1 steps y = x + c2(leaky(c1(leaky(x)))) side by side in one launch (fo_conv_pair_multi); members:
    (x, pc1, pc2, K, dil, out) with PackedConv weights.  summed=True: members[0]'s out = (sum of the members' y) *
    oscale + gadd."""
    arr = (_lib.FoPairDesc * len(members))(*[
        _lib.FoPairDesc(x.data_ptr(), p1.packed.data_ptr(), ptr(p1.bias), p2.packed.data_ptr(), ptr(p2.bias),
                        out.data_ptr(), K, dil) for x, p1, p2, K, dil, out in members])
    _lib.call("fo_conv_pair_multi", arr, len(members), B, C, T, 1 if summed else 0, float(slope), float(oscale),
              ptr(gadd), stream(device))


def codec_embed_cl(table, E, n_codes, ids, B, T, out):
    _lib.call("fo_codec_embed_cl", table.data_ptr(), E, n_codes, ids.data_ptr(), B, T, out.data_ptr(),
              stream(out.device))
    return out


def scale_add_cl(y, B, T, C, sc, g=None):
    _lib.call("fo_scale_add_cl", y.data_ptr(), B, T, C, float(sc), ptr(g), stream(y.device))
    return y


def conv_post_cl(x, B, T, C, w, bias, K, pad, slope, out):
    _lib.call("fo_conv_post_cl", x.data_ptr(), B, T, C, w.data_ptr(), ptr(bias), K, pad, float(slope), out.data_ptr(),
              stream(x.device))
    return out


def conv_transpose1d(x, B, Cin, Tin, w, bias, Cout, K, stride_, pad, out, slope=1.0):
    _lib.call("fo_conv_transpose1d", x.data_ptr(), B, Cin, Tin, w.data_ptr(), ptr(bias), Cout, K, stride_, pad,
              float(slope), out.data_ptr(), stream(x.device))
    return out


def codec_embed(table, ids, B, T, out):
    _lib.call("fo_codec_embed", table.data_ptr(), table.shape[1], table.shape[0], ids.data_ptr(), B, T,
              out.data_ptr(), stream(table.device))
    return out


def axpy_(y, x):
    _lib.call("fo_axpy", y.data_ptr(), x.data_ptr(), y.numel(), stream(y.device))
    return y


def scale_add_channel_(y, B, C, T, s, g=None):
    _lib.call("fo_scale_add_channel", y.data_ptr(), B, C, T, float(s), ptr(g), stream(y.device))
    return y


def silence_cut(x, N, res):
    _lib.call("fo_silence_cut", x.data_ptr(), x.numel(), N, res.data_ptr(), stream(x.device))
    return res


def silence_cut_rows(x, N, res):
    """find_min_sum_index's window search for every row of x [rows, L] (row stride x.stride(0)) in one launch;
    res [rows, 2] fp32 (min window sum, cut index)."""
    _lib.call("fo_silence_cut_rows", x.data_ptr(), x.stride(0), x.shape[0], x.shape[1], N, res.data_ptr(),
              stream(x.device))
    return res


class SampleCheck:
    """Host-mapped error word of the samplers (the C-ABI's `err`): a kernel sets it when a logits row holds a
    NaN or +inf (or only -inf) -- the rows the reference's torch.multinomial refuses (models/decoder/
    decoder.py:355-359, models/audioLLM.py:476: "probability tensor contains either inf, nan or element < 0").
    check() is read on the host after the sampling work has completed (an event / stream sync) and raises
    RuntimeError, as the reference does; the drawn ids themselves always stay inside the vocabulary."""

    def __init__(self):
        self.buf = HostBuffer(1, 1)
        self.buf.np[0, 0] = 0

    @property
    def dev(self):
        return self.buf.dev

    def check(self, what="sampler"):
        if self.buf.np is not None and int(self.buf.np[0, 0]) != 0:
            self.buf.np[0, 0] = 0
            raise RuntimeError(f"{what}: a logits row holds NaN / inf (probability tensor contains either inf, nan or "
                               "element < 0 -- torch.multinomial raises on it in the reference)")

    def free(self):
        self.buf.free()

    def __del__(self):   # the pinned word goes with its owner (a thread's default check dies with the thread)
        try:
            self.free()
        except Exception:
            pass


_CHECKS = threading.local()


def sample_check(device):
    """The default SampleCheck of a device FOR THE CALLING THREAD (used when a sampler call passes none).  Held in
    thread-local storage: the eager text step, AudioLLM._post_decode, LLM2TTSCodecAR.infer and speak's eager loop may
    run on several host threads (speech workers, server sessions), and a NaN row drawn by one thread must raise in that
    thread's check, not in another's (check() clears the word on read); a thread's checks are released when it ends,
    so a later thread (even one reusing its id) starts from a fresh, cleared word."""
    d = torch.device(device)
    idx = d.index if d.index is not None else torch.cuda.current_device()
    per = getattr(_CHECKS, "by_device", None)
    if per is None:
        per = _CHECKS.by_device = {}
    if idx not in per:
        per[idx] = SampleCheck()
    return per[idx]


def sample(logits, V, out_ids, top_k=None, temperature=None, top_p=None, seed=0, step=None, out_max=None, B=None,
           ban_id=-1, key=None, err=None, argmax_ws=False):
    """key: optional per-row int32 stream ids (defaults to the row index).  err: SampleCheck (default: the
    device's; read it with .check() after the work has completed).  argmax_ws=True: every row is top_k == 1,
    so large-vocabulary rows take the split arg-max (scratch at the tail of the stream's Runtime workspace)."""
    B = logits.shape[0] if B is None else B
    err = err or sample_check(logits.device)
    ws, wsn = None, 0
    if argmax_ws:
        wsn = int(_lib.load().fo_sample_ws_floats(B, V))
        rt = Runtime.get(logits.device)
        ws = rt.ws[rt.ws.numel() - wsn:].data_ptr()
    _lib.call("fo_sample", logits.data_ptr(), logits.stride(0), B, V, ptr(top_k), ptr(temperature), ptr(top_p),
              int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(step), ptr(key), int(ban_id), out_ids.data_ptr(), ptr(out_max),
              err.dev, ws, wsn, stream(logits.device))
    return out_ids


def sample_probs(logits, V, out_ids, probs, top_k=None, temperature=None, top_p=None, seed=0, step=None, B=None,
                 ban_id=-1, key=None, err=None):
    """sample() that also writes each row's sampling distribution (the reference's pre-multinomial probs)
    into probs [B, >=V] fp32."""
    B = logits.shape[0] if B is None else B
    assert probs.dtype == F32 and probs.is_contiguous() and probs.shape[0] >= B and probs.shape[1] >= V
    err = err or sample_check(logits.device)
    _lib.call("fo_sample_probs", logits.data_ptr(), logits.stride(0), B, V, ptr(top_k), ptr(temperature), ptr(top_p),
              int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(step), ptr(key), int(ban_id), out_ids.data_ptr(), probs.data_ptr(),
              probs.stride(0), err.dev, stream(logits.device))
    return out_ids


def conv1d_ex(x, B, Cin, Tin, w, bias, Cout, K, stride, dil, pad, pre_leaky, out, residual=False):
    """Channel-first conv [B][Cin][Tin] -> out [B][Cout][Tout] (fp32 weights [Cout][Cin][K])."""
    _lib.call("fo_conv1d_ex", x.data_ptr(), B, Cin, Tin, w.data_ptr(), ptr(bias), Cout, K, stride, dil, pad,
              0 if pre_leaky is None else 1, 0.0 if pre_leaky is None else float(pre_leaky), out.data_ptr(),
              1 if residual else 0, stream(x.device))
    return out


def group_norm(x, B, C, T, G, w, b, eps, scale, out):
    _lib.call("fo_group_norm", x.data_ptr(), B, C, T, G, w.data_ptr(), b.data_ptr(), float(eps), float(scale),
              out.data_ptr(), stream(x.device))
    return out


def gte_head(x, B, C, T, lw, lb, rm, rv, bw, bb, eps, out):
    _lib.call("fo_gte_head", x.data_ptr(), B, C, T, lw.data_ptr(), lb.data_ptr(), rm.data_ptr(), rv.data_ptr(),
              bw.data_ptr(), bb.data_ptr(), float(eps), out.data_ptr(), stream(x.device))
    return out


def vq_nearest(x, B, Ctot, T, ch0, D, codebook, ids, ids_ld, ids_col, residual=False):
    _lib.call("fo_vq_nearest", x.data_ptr(), B, Ctot, T, ch0, D, codebook.data_ptr(), codebook.shape[0],
              ids.data_ptr(), ids_ld, ids_col, 1 if residual else 0, stream(x.device))
    return ids


def penalty(logits, V, ids, win, step, penalty, B=None):
    """Repetition penalty (models/decoder/decoder.py:348-351) in place on logits [B, >=V]: stores this
    step's input ids into the ring win [B, W] at step % W, then divides each windowed id's logit."""
    B = logits.shape[0] if B is None else B
    assert logits.dtype == F32 and logits.stride(-1) == 1 and logits.shape[0] >= B and logits.shape[1] >= V
    assert win.dtype == I32 and win.is_contiguous() and win.dim() == 2 and win.shape[0] >= B
    assert ids.dtype == I32 and ids.is_contiguous() and ids.numel() >= B
    assert step.dtype == I32 and step.is_contiguous() and step.numel() >= B
    _lib.call("fo_penalty", logits.data_ptr(), logits.stride(0), B, V, ids.data_ptr(), win.data_ptr(), win.shape[1],
              step.data_ptr(), float(penalty), stream(logits.device))
    return logits


def sample_embed(logits, V, out_ids, emb, x, gamma, eps, h, top_k=None, temperature=None, top_p=None, seed=0,
                 step=None, B=None, ban_id=-1, key=None, hist_ptr=None, hist_row=None, hist_ld=0, meta=None, maxb=0,
                 PS=0, err=None):
    """sample(), then the next decode step's input from the drawn ids: x[b] = emb[id_b] (fp32), h[b] =
    RMSNorm(x[b]) * gamma, and (hist_ptr) hist[hist_row[0] * hist_ld + b] = id_b -- one launch.  meta: the
    captured step's metadata block (step / key are its rows): it advances to the next step in the same launch."""
    B = logits.shape[0] if B is None else B
    err = err or sample_check(logits.device)
    _lib.call("fo_sample_embed", logits.data_ptr(), logits.stride(0), B, V, ptr(top_k), ptr(temperature), ptr(top_p),
              int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(step), ptr(key), int(ban_id), out_ids.data_ptr(), hist_ptr,
              ptr(hist_row), hist_ld, emb.data_ptr(), emb.stride(0), emb.shape[1], x.data_ptr(), x.stride(0),
              gamma.data_ptr(), float(eps), h.data_ptr(), h.stride(0), ptr(meta), int(maxb), int(PS), err.dev,
              stream(logits.device))
    return out_ids

