"""Shared event timer for the GPU sweep scripts."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "freeze-omni_amd"))
from fo import _lib, ops  # noqa: E402


def timeit(fn, reps=30):
    lib = _lib.load()
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.fo_event_create(ctypes.byref(e0))
    lib.fo_event_create(ctypes.byref(e1))
    for _ in range(3):
        fn()
    s = ops.stream()
    lib.fo_event_record(e0, s)
    for _ in range(reps):
        fn()
    lib.fo_event_record(e1, s)
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value / reps * 1e3
