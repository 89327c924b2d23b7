"""graph_time(fn, reps): per-launch device time of `reps` calls of fn captured as one hipGraph on the engine
stream and replayed (no host launch overhead in the number)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "freeze-omni_amd"))
from fo import _lib, ops  # noqa: E402

_ev = None


def graph_time(fn, reps):
    global _ev
    lib = _lib.load()
    dev = torch.device("cuda", torch.cuda.current_device())
    es = ops.engine_stream(dev)
    if _ev is None:
        _ev = (ctypes.c_void_p(), ctypes.c_void_p())
        lib.fo_event_create(ctypes.byref(_ev[0]))
        lib.fo_event_create(ctypes.byref(_ev[1]))
    e0, e1 = _ev
    s = es.cuda_stream
    with torch.cuda.stream(es):
        fn()  # allocate / warm outside the capture
        _lib.call("fo_graph_begin", s)
        try:
            for _ in range(reps):
                fn()
        finally:
            ex = ctypes.c_void_p()
            _lib.call("fo_graph_end", s, ctypes.byref(ex))
        _lib.call("fo_graph_launch", ex, s)
        lib.fo_event_record(e0, s)
        _lib.call("fo_graph_launch", ex, s)
        lib.fo_event_record(e1, s)
        torch.cuda.synchronize()
        _lib.call("fo_graph_destroy", ex)
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value / reps * 1e3
