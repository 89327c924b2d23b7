"""Device time of one listen chunk's LLM stage (28 Qwen2 layers + final norm + state head, 8 users x 2 rows)
and ENCODER stage at real geometry, each replayed alone from its captured ListenGraph, and both replayed
concurrently (encoder stage on the side stream, as ListenPipe overlaps them) -- the contention between
the two stages of a pipelined chunk.  python scripts/llm_stage_time.py (GPU only)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
from fo import _lib, ops  # noqa: E402
from fo.engine import FreezeOmniEngine  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
eng = FreezeOmniEngine(os.path.join(ROOT, "configs", "real"), device=dev, max_sessions=16)
B = 8
base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
kvs = [base.fork() for _ in range(B)]
fb = eng.fbank("A")
rng = np.random.default_rng(0)
wins = (rng.standard_normal((B, fb.n_samples)) * 3000).astype(np.float32)
feats = fb(wins, [True] * B)
items = [dict(identity="user", status="ipu_sl", feats=feats[b], kv=kvs[b], enc_cache=None, ada_cache=None, pe_index=0)
         for b in range(B)]
res = eng.listen(items)
for _ in range(3):   # steady-state chunks (graph path)
    items = [dict(identity="user", status="ipu_cl", feats=feats[b], kv=kvs[b], enc_cache=r["enc_cache"],
                  ada_cache=r["ada_cache"], pe_index=r["pe_index"]) for b, r in enumerate(res)]
    res = eng.listen(items)
g = eng._listen_graph_for(items, slots=2, extra=128)
pe = g.submit_encoder(items, 0)
g.submit_llm(items, pe, 0)
torch.cuda.synchronize()
main, side = g.main.cuda_stream, g.side.cuda_stream
e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
lib.fo_event_create(ctypes.byref(e0))
lib.fo_event_create(ctypes.byref(e1))


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    lib.fo_event_record(e0, main)
    for _ in range(reps):
        fn()
    lib.fo_event_record(e1, main)
    torch.cuda.synchronize()
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value / reps * 1e3


ev_side = ctypes.c_void_p()
lib.fo_event_create(ctypes.byref(ev_side))


def llm_only():
    _lib.call("fo_graph_launch", g.llm_exec[0], main)


def enc_only():
    _lib.call("fo_graph_launch", g.enc_exec[1], main)


def both():   # encoder stage of the next chunk on the side stream beside this chunk's LLM stage
    _lib.call("fo_graph_launch", g.enc_exec[1], side)
    _lib.call("fo_event_record", ev_side, side)
    _lib.call("fo_graph_launch", g.llm_exec[0], main)
    _lib.call("fo_stream_wait_event", main, ev_side)


t_llm = timed(llm_only)
t_enc = timed(enc_only)
t_both = timed(both)
wb = eng.llm.stack.weight_bytes
print(f"LLM stage alone     {t_llm:8.1f} us  ({wb / t_llm / 1e6:.2f} TB/s over {wb / 1e9:.2f} GB of layer weights)")
print(f"encoder stage alone {t_enc:8.1f} us")
print(f"both, overlapped    {t_both:8.1f} us  (max of the two {max(t_llm, t_enc):.1f}, sum {t_llm + t_enc:.1f})",
      flush=True)

# dispatch contention probe: beside the LLM stage, a side-stream graph of N tiny kernels (256-element axpy,
# ~no memory or CU time) -- if the LLM stage slows by ~N x the per-dispatch cost, the two streams' kernel
# dispatches, not HBM or CUs, are what the encoder stage contends for
from fo import ops as _ops  # noqa: E402
ta = torch.zeros(256, device=dev)
tb = torch.ones(256, device=dev)
side_s = g.side
for nk in (150, 300, 600):
    with torch.cuda.stream(side_s):
        _lib.call("fo_graph_begin", side)
        for _ in range(nk):
            _ops.axpy_(ta, tb)
        gx = ctypes.c_void_p()
        _lib.call("fo_graph_end", side, ctypes.byref(gx))

    def tiny_only(gx=gx):
        _lib.call("fo_graph_launch", gx, side)
        _lib.call("fo_event_record", ev_side, side)
        _lib.call("fo_stream_wait_event", main, ev_side)

    def both_tiny(gx=gx):
        _lib.call("fo_graph_launch", gx, side)
        _lib.call("fo_event_record", ev_side, side)
        _lib.call("fo_graph_launch", g.llm_exec[0], main)
        _lib.call("fo_stream_wait_event", main, ev_side)
    print(f"{nk:4d} tiny side-stream kernels: alone {timed(tiny_only):8.1f} us, beside the LLM stage "
          f"{timed(both_tiny):8.1f} us", flush=True)
