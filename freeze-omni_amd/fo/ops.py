"""Thin torch-facing wrappers over the C-ABI kernels.

torch is used only for device memory and the current stream (plumbing); every computation
below is a hand-written gfx950 kernel in libfo_hip.so.
"""
import torch

from . import _lib

BF16 = torch.bfloat16
F32 = torch.float32

ACT = {"none": 0, "relu": 1, "silu": 2, "gelu": 3}


def ptr(t):
    return None if t is None else t.data_ptr()


def stream(device=None):
    return torch.cuda.current_stream(device).cuda_stream


class Runtime:
    """Per-device scratch shared by all kernels of one replica (single stream discipline)."""

    _inst = {}

    def __init__(self, device, ws_floats=1 << 25):
        self.device = torch.device(device)
        self.ws = torch.empty(ws_floats, dtype=F32, device=self.device)
        self.counters = torch.zeros(1 << 20, dtype=torch.int32, device=self.device)

    @classmethod
    def get(cls, device):
        d = torch.device(device)
        key = (d.type, d.index if d.index is not None else torch.cuda.current_device())
        if key not in cls._inst:
            cls._inst[key] = Runtime(torch.device("cuda", key[1]))
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

    def __init__(self, w, bias=None, swiglu_up=None):
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
        if self.swiglu:
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

    def __call__(self, x, out=None, act="none", residual=False, out_dtype=F32, splitk=0, M=None):
        """x: bf16 [M, >=Kp] (row stride x.stride(0)); returns out [M, N]."""
        _check_dev(x)
        if x.dtype != BF16:
            raise TypeError("PackedLinear input must be bf16")
        M = x.shape[0] if M is None else M
        if out is None:
            out = torch.empty(M, self.N, dtype=out_dtype, device=x.device)
        rt = Runtime.get(x.device)
        _lib.call("fo_gemm", x.data_ptr(), x.stride(0), M, self.Kp, self.packed.data_ptr(), self.N,
                  1 if self.swiglu else 0, ptr(self.bias), out.data_ptr(), out.stride(0),
                  1 if out.dtype == BF16 else 0, ACT[act], 1 if residual else 0, rt.ws.data_ptr(), rt.ws.numel(),
                  rt.counters.data_ptr(), splitk, stream(x.device))
        return out
