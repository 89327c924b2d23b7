"""ctypes binding of libfo_hip.so (the C-ABI declared in include/fo_hip.h).

torch is imported first on purpose: torch ships its own libamdhip64.so (soname
libamdhip64.so.7); loading it first makes the dynamic linker resolve our library's HIP
runtime to the same copy, so streams and device pointers are shared.

There is no fallback: if the library is missing or the device is not gfx950 the hot path
raises, it never silently reroutes to a CPU implementation.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FO_LIB_PATH") or os.path.join(_HERE, "libfo_hip.so")   # override: A/B sweeps only

c_int = ctypes.c_int
c_ll = ctypes.c_longlong
c_float = ctypes.c_float
c_vp = ctypes.c_void_p

class FoConvDesc(ctypes.Structure):
    """include/fo_hip.h FoConvDesc (fo_conv_cl_multi)."""
    _fields_ = [("x", c_vp), ("wp", c_vp), ("bias", c_vp), ("out", c_vp), ("Tin", c_int), ("K", c_int),
                ("dil", c_int), ("pad", c_int), ("Tq", c_int), ("ostride", c_int), ("ooff", c_int),
                ("Tout_total", c_int), ("pre_leaky", c_int), ("slope", c_float), ("res", c_vp), ("res2", c_vp),
                ("oscale", c_float), ("gadd", c_vp)]


class FoPairDesc(ctypes.Structure):
    """include/fo_hip.h FoPairDesc (fo_conv_pair_multi)."""
    _fields_ = [("x", c_vp), ("w1", c_vp), ("b1", c_vp), ("w2", c_vp), ("b2", c_vp), ("out", c_vp), ("K", c_int),
                ("dil", c_int)]


# name -> (restype, argtypes)
_SIGS = {
    "fo_version": (c_int, []),
    "fo_last_error": (c_int, [ctypes.c_char_p, c_int]),
    "fo_device_info": (c_int, [c_int, ctypes.c_char_p, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_ll)]),
    "fo_graph_begin": (c_int, [c_vp]),
    "fo_graph_end": (c_int, [c_vp, ctypes.POINTER(c_vp)]),
    "fo_graph_launch": (c_int, [c_vp, c_vp]),
    "fo_graph_destroy": (c_int, [c_vp]),
    "fo_stream_create": (c_int, [ctypes.POINTER(c_vp)]),
    "fo_stream_create_prio": (c_int, [ctypes.POINTER(c_vp), c_int]),
    "fo_stream_priority_range": (c_int, [ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "fo_stream_create_cumask": (c_int, [ctypes.POINTER(c_vp), ctypes.POINTER(ctypes.c_uint), c_int]),
    "fo_stream_destroy": (c_int, [c_vp]),
    "fo_stream_wait_event": (c_int, [c_vp, c_vp]),
    "fo_host_alloc": (c_int, [c_ll, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp)]),
    "fo_host_free": (c_int, [c_vp]),
    "fo_event_sync": (c_int, [c_vp]),
    "fo_event_query": (c_int, [c_vp]),
    "fo_event_create": (c_int, [ctypes.POINTER(c_vp)]),
    "fo_event_record": (c_int, [c_vp, c_vp]),
    "fo_event_elapsed_ms": (c_int, [c_vp, c_vp, ctypes.POINTER(c_float)]),
    "fo_event_destroy": (c_int, [c_vp]),
    "fo_gemm_tune": (c_int, [c_int, c_int]),
    "fo_gemm_set_u": (c_int, [c_int]),
    "fo_gemm_set_xs": (c_int, [c_int]),
    "fo_gemm_set_xs_variant": (c_int, [c_int]),
    "fo_gemm_set_merge": (c_int, [c_int]),
    "fo_gemm_set_trace": (c_int, [c_vp]),
    "fo_gemm_set_xpack": (c_int, [c_vp, c_vp, c_int, c_int]),
    "fo_gemm_set_ypack": (c_int, [c_vp, c_vp, c_int, c_int]),
    "fo_gemm_set_ypack32": (c_int, [c_vp, c_int, c_int]),
    "fo_gemm_set_xpack32": (c_int, [c_vp, c_int, c_int]),
    "fo_attention_set_opack": (c_int, [c_vp, c_vp, c_int, c_int]),
    "fo_launch_counts": (c_int, [ctypes.POINTER(c_ll), c_int]),
    "fo_launch_counts_reset": (c_int, []),
    "fo_subsample_ws_floats": (c_ll, [c_int, c_int, c_int, c_int]),
    "fo_attention_o": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_int, c_float, c_vp,
                               c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "fo_enc_attn_block": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_float, c_vp, c_vp, c_vp, c_vp,
                                  c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_float, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fo_enc_attn_out": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp,
                                c_vp, c_vp, c_vp, c_float, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fo_probe_seam": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_float, c_vp,
                              c_vp, c_vp, c_int, c_vp]),
    "fo_attn_max_rows": (c_int, [c_int]),
    "fo_gemm_set_xsk_min_mb": (c_int, [c_int]),
    "fo_gemm_set_rows": (c_int, [c_int]),
    "fo_set_kv_bf16": (c_int, [c_int]),
    "fo_conv_set_trace": (c_int, [c_vp]),
    "fo_attention_set_trace": (c_int, [c_vp]),
    "fo_subsample": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_ll, c_vp]),
    "fo_pack_weight_elems": (c_ll, [c_int, c_int]),
    "fo_pack_weight": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp]),
    "fo_gemm_pick_split": (c_int, [c_int, c_int, c_int]),
    "fo_gemm_workspace_floats": (c_ll, [c_int, c_int, c_int, c_int]),
    "fo_gemm": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int,
                        c_int, c_int, c_vp, c_ll, c_vp, c_int, c_vp]),
    "fo_gemm_rms": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int,
                            c_vp, c_ll, c_vp, c_int, c_vp, c_int, c_float, c_vp, c_vp, c_vp, ctypes.POINTER(c_int),
                            c_vp]),
    "fo_gemm_ln": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_float, c_vp, c_vp, c_int, c_vp,
                           c_int, c_int, c_vp, c_ll, c_int, c_vp]),
    "fo_gemm_rowstats": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp,
                                 c_ll, c_vp, c_int, c_vp, c_vp, ctypes.POINTER(c_int), c_vp]),
    "fo_gemm_qkv_rope": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_ll, c_vp, c_int, c_vp,
                                 c_int, c_float, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                 c_vp]),
    "fo_fill_hash": (c_int, [c_vp, c_int, c_ll, ctypes.c_ulonglong, c_float, c_float, c_vp]),
    "fo_rmsnorm": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_float, c_vp, c_int, c_int, c_vp]),
    "fo_layernorm": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_float, c_vp, c_int, c_int, c_vp]),
    "fo_gather_rows": (c_int, [c_vp, c_int, c_ll, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp]),
    "fo_im2col_3x3s2": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_ll, c_ll, c_ll, c_ll, c_vp, c_vp, c_vp, c_int,
                                c_vp]),
    "fo_tcf_permute": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "fo_im2col_conv1d": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp]),
    "fo_conv_cache_update": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    "fo_state_head": (c_int, [c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp]),
    "fo_record_ids": (c_int, [c_vp, c_int, c_vp, c_int, c_vp, c_vp]),
    "fo_scale": (c_int, [c_vp, c_ll, c_float, c_vp]),
    "fo_attn_nsplit": (c_int, [c_int, c_int, c_int]),
    "fo_rope_kv_write": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_int, c_vp]),
    "fo_attention": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_int,
                             c_int, c_float, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp]),
    "fo_enc_kv_write": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp]),
    "fo_relpos_attention_fused": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                          c_int, c_int, c_int, c_int, c_float, c_vp, c_int, c_vp]),
    "fo_relpos_attention_chunks": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int,
                                           c_int, c_int, c_float, c_vp, c_int, c_vp]),
    "fo_relpos_attention": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                    c_int, c_int, c_int, c_float, c_vp, c_int, c_vp]),
    "fo_fbank": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int,
                         c_int, c_vp, c_vp]),
    "fo_rows_shift": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp]),
    "fo_conv1d": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_float, c_vp,
                          c_int, c_int, c_vp]),
    "fo_conv_transpose1d": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_float, c_vp,
                                    c_vp]),
    "fo_codec_embed": (c_int, [c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp]),
    "fo_axpy": (c_int, [c_vp, c_vp, c_ll, c_vp]),
    "fo_scale_add_channel": (c_int, [c_vp, c_int, c_int, c_int, c_float, c_vp, c_vp]),
    "fo_conv_pack_elems": (c_ll, [c_int, c_int, c_int]),
    "fo_pack_conv": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "fo_conv_cl_multi": (c_int, [ctypes.POINTER(FoConvDesc), c_int, c_int, c_int, c_int, c_int, c_vp]),
    "fo_conv_pair_multi": (c_int, [ctypes.POINTER(FoPairDesc), c_int, c_int, c_int, c_int, c_int, c_float, c_float,
                                   c_vp, c_vp]),
    "fo_conv_cl": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                           c_int, c_int, c_float, c_vp, c_vp, c_vp, c_float, c_vp, c_vp]),
    "fo_codec_embed_cl": (c_int, [c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp]),
    "fo_scale_add_cl": (c_int, [c_vp, c_int, c_int, c_int, c_float, c_vp, c_vp]),
    "fo_conv_post_cl": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_float, c_vp, c_vp]),
    "fo_silence_cut": (c_int, [c_vp, c_int, c_int, c_vp, c_vp]),
    "fo_silence_cut_rows": (c_int, [c_vp, c_ll, c_int, c_int, c_int, c_vp, c_vp]),
    "fo_sample_ws_floats": (c_ll, [c_int, c_int]),
    "fo_sample": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, ctypes.c_ulonglong, c_vp, c_vp, c_int, c_vp,
                          c_vp, c_vp, c_vp, c_ll, c_vp]),
    "fo_sample_probs": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, ctypes.c_ulonglong, c_vp, c_vp, c_int,
                                c_vp, c_vp, c_int, c_vp, c_vp]),
    "fo_sample_embed": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, ctypes.c_ulonglong, c_vp, c_vp, c_int,
                                c_vp, c_vp, c_vp, c_int, c_vp, c_ll, c_int, c_vp, c_int, c_vp, c_float, c_vp, c_int,
                                c_vp, c_int, c_int, c_vp, c_vp]),
    "fo_gemm_set_pipe": (c_int, [c_int]),
    "fo_conv1d_ex": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                             c_vp, c_int, c_vp]),
    "fo_group_norm": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_float, c_float, c_vp, c_vp]),
    "fo_gte_head": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_float, c_vp, c_vp]),
    "fo_vq_nearest": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_int, c_int, c_vp]),
    "fo_penalty": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_float, c_vp]),
}

_lib = None


def declared_symbols():
    """Every symbol include/fo_hip.h declares (kept in sync by tests/test_capi_symbols.py)."""
    return list(_SIGS.keys())


def register(name, restype, argtypes):
    _SIGS[name] = (restype, argtypes)
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.restype = restype
        fn.argtypes = argtypes


def load(path=None):
    """Load the shared library (no device calls are made here)."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            f"libfo_hip.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the Freeze-Omni MI355X path has no CPU fallback)")
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    override = p != os.path.join(_HERE, "libfo_hip.so")
    for name, (rt, at) in _SIGS.items():
        if override and not hasattr(lib, name):
            continue   # an older build under A/B (FO_LIB_PATH): entries it predates stay unbound
        fn = getattr(lib, name)
        fn.restype = rt
        fn.argtypes = at
    _lib = lib
    return lib


def last_error():
    buf = ctypes.create_string_buffer(1024)
    load().fo_last_error(buf, 1024)
    return buf.value.decode(errors="replace")


def check(rc, what=""):
    if rc != 0:
        raise RuntimeError(f"{what or 'libfo_hip'} failed ({rc}): {last_error()}")
    return rc


def call(name, *args):
    """Call a C-ABI entry and raise RuntimeError with fo_last_error() on failure."""
    return check(getattr(load(), name)(*args), name)
