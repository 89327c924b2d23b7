"""The packed-activation C-ABI carries each buffer's extent (include/fo_hip.h fo_gemm_set_xpack & co.): a launch armed
with a pack built for another K / N or for fewer row blocks returns -2 before anything is enqueued, and the arming is
consumed by that refusal (nothing stays armed for the next launch).  Host-side argument checks only: these run without
a GPU (every refusal below happens before the library touches the device)."""
import ctypes
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("FO_LIB_PATH") or os.path.join(ROOT, "freeze-omni_amd", "fo", "libfo_hip.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libfo_hip.so not built (run __graft_entry__.build())")

FAKE = 1 << 20   # dummy device addresses: never dereferenced by a refused call


def _lib():
    from fo import _lib
    return _lib.load(), _lib.last_error


def _gemm(lib, M, K, N):
    """fo_gemm on dummy pointers (M x K fp32 X, N outputs)."""
    return lib.fo_gemm(FAKE, 1, K, M, K, FAKE, N, 0, None, None, None, FAKE, N, 0, 0, 0, FAKE, 1 << 20, None, 0, None)


def test_setters_validate_the_extent():
    lib, err = _lib()
    assert lib.fo_gemm_set_xpack(FAKE, None, 512, 1) == -2 and "both halves" in err()
    assert lib.fo_gemm_set_xpack(FAKE, FAKE, 500, 1) == -2 and "multiple of 32" in err()
    assert lib.fo_gemm_set_ypack(FAKE, FAKE, 512, 5) == -2 and "row blocks" in err()
    assert lib.fo_gemm_set_xpack32(FAKE, 512, 0) == -2
    assert lib.fo_attention_set_opack(FAKE, FAKE, 3584, 9) == -2
    for f in (lib.fo_gemm_set_xpack, lib.fo_gemm_set_ypack, lib.fo_attention_set_opack):   # NULL disarms
        assert f(None, None, 0, 0) == 0
    assert lib.fo_gemm_set_xpack32(None, 0, 0) == 0 and lib.fo_gemm_set_ypack32(None, 0, 0) == 0


@pytest.mark.parametrize("setter,two,cols,rb,M,K,N,what", [
    ("fo_gemm_set_xpack", True, 1024, 1, 16, 512, 256, "packed X"),        # built for another K
    ("fo_gemm_set_xpack", True, 512, 1, 17, 512, 256, "packed X"),         # one row block for 17 rows
    ("fo_gemm_set_xpack", True, 512, 2, 40, 512, 256, "packed X"),         # two row blocks for 40 rows
    ("fo_gemm_set_ypack", True, 512, 4, 16, 512, 256, "packed output"),    # built for another N
    ("fo_gemm_set_ypack", True, 256, 3, 64, 512, 256, "packed output"),    # three row blocks for 64 rows
    ("fo_gemm_set_xpack32", False, 256, 4, 32, 512, 256, "fp32 packed X"),
    ("fo_gemm_set_ypack32", False, 256, 1, 32, 512, 256, "fp32 packed output"),
])
def test_gemm_refuses_a_pack_that_does_not_fit(setter, two, cols, rb, M, K, N, what):
    lib, err = _lib()
    args = (FAKE, FAKE) if two else (FAKE,)
    assert getattr(lib, setter)(*args, cols, rb) == 0
    assert _gemm(lib, M, K, N) == -2
    assert what in err() and f"{cols} columns x {rb} row blocks" in err(), err()
    # the refusal consumed the arming: the next launch fails on its own (bad K) check, not on the pack
    assert _gemm(lib, M, 100, N) == -2
    assert "multiple of 32" in err(), err()


def test_attention_refuses_a_pack_that_does_not_fit():
    lib, err = _lib()
    H, KVH, hd = 28, 4, 128

    def attn(T):
        return lib.fo_attention(FAKE, T, None, T // 2, 14, FAKE, FAKE, 16, 16, FAKE, FAKE, H, KVH, hd,
                                ctypes.c_float(0.088), 1, None, None, FAKE, FAKE, 128, None)
    assert lib.fo_attention_set_opack(FAKE, FAKE, 3584, 1) == 0   # built for the 3584-wide o input, 1 row block
    assert attn(32) == -2 and "packed output" in err(), err()
    assert lib.fo_attention_set_opack(FAKE, FAKE, 1024, 4) == 0   # another width
    assert attn(16) == -2 and "1024 columns x 4 row blocks" in err(), err()
    # consumed: a bad head size now fails on its own check
    assert lib.fo_attention(FAKE, 16, None, 8, 14, FAKE, FAKE, 16, 16, FAKE, FAKE, H, KVH, 96, ctypes.c_float(0.1), 1,
                            None, None, FAKE, FAKE, 128, None) == -2
    assert "head_dim 96" in err(), err()
    assert lib.fo_attention_set_opack(FAKE, FAKE, 512, 1) == 0    # relpos: h * dk = 16 * 64 = 1024 != 512
    assert lib.fo_relpos_attention_fused(FAKE, 3072, FAKE, FAKE, 72, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, 2, 4,
                                         16, 64, ctypes.c_float(0.125), FAKE, 1024, None) == -2
    assert "fo_relpos_attention_fused: packed output" in err(), err()


def test_launch_counters_exist_and_reset():
    lib, _ = _lib()
    n = lib.fo_launch_counts(None, 0)
    assert n >= 16
    assert lib.fo_launch_counts_reset() == 0
    buf = (ctypes.c_longlong * n)()
    assert lib.fo_launch_counts(buf, n) == n
    assert list(buf) == [0] * n
