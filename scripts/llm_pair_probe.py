"""Ceiling of a two-chunk wavefront for the listen stage (DESIGN 8b's next lever): the captured LLM stage of a listen
chunk (28 Qwen2 layers, 8 users x 2 rows) replayed alone, twice back to back, and two instances replayed at once on
two streams (slots 0 and 1 of one ListenGraph; they write the same sessions' K / V rows, which only a timing probe may
do).  If two concurrent stages take much less than two sequential ones, overlapping consecutive chunks' stages one
layer apart would pay.  python scripts/llm_pair_probe.py (GPU only)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
from fo import _lib  # noqa: E402
from fo.engine import FreezeOmniEngine  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
eng = FreezeOmniEngine(os.path.join(ROOT, "configs", "real"), device=dev, max_sessions=16)
B = 8
base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
kvs = [base.fork() for _ in range(B)]
fb = eng.fbank("A")
rng = np.random.default_rng(0)
feats = fb((rng.standard_normal((B, fb.n_samples)) * 3000).astype(np.float32), [True] * B)
items = [dict(identity="user", status="ipu_sl", feats=feats[b], kv=kvs[b], enc_cache=None, ada_cache=None, pe_index=0)
         for b in range(B)]
res = eng.listen(items)
for _ in range(3):
    items = [dict(identity="user", status="ipu_cl", feats=feats[b], kv=kvs[b], enc_cache=r["enc_cache"],
                  ada_cache=r["ada_cache"], pe_index=r["pe_index"]) for b, r in enumerate(res)]
    res = eng.listen(items)
g = eng._listen_graph_for(items, slots=2, extra=128)
for k in (0, 1):
    pe = g.submit_encoder(items, k)
    g.submit_llm(items, pe, k)
torch.cuda.synchronize()
main, side = g.main.cuda_stream, g.side.cuda_stream
e0, e1, ev = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
for e in (e0, e1, ev):
    lib.fo_event_create(ctypes.byref(e))


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


def one():
    _lib.call("fo_graph_launch", g.llm_exec[0], main)


def seq2():
    _lib.call("fo_graph_launch", g.llm_exec[0], main)
    _lib.call("fo_graph_launch", g.llm_exec[1], main)


def par2():
    _lib.call("fo_event_record", ev, main)
    _lib.call("fo_stream_wait_event", side, ev)
    _lib.call("fo_graph_launch", g.llm_exec[1], side)
    _lib.call("fo_event_record", ev, side)
    _lib.call("fo_graph_launch", g.llm_exec[0], main)
    _lib.call("fo_stream_wait_event", main, ev)


for rep in range(2):
    t1, ts, tp = timed(one), timed(seq2), timed(par2)
    print(f"LLM stage alone {t1:8.1f} us | two back to back {ts:8.1f} us | two at once on two streams {tp:8.1f} us "
          f"({tp / ts:.3f} of sequential)", flush=True)
