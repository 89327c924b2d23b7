"""Device time of the listen's Qwen2 stage per chunk when C consecutive chunks of 8 users share one stage
(fo.engine.ListenGroupGraph, C x 16 rows) against one chunk per stage (ListenGraph, 16 rows), real geometry; each
stage graph-replayed alone, then with its C encoder stages beside it on the side stream (the pipe's overlap).
python scripts/group_stage_time.py [C ...] (GPU only)."""
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
Cs = [int(c) for c in sys.argv[1:]] or [1, 2, 3, 4]
base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
fb = eng.fbank("A")
rng = np.random.default_rng(0)
wins = (rng.standard_normal((B, fb.n_samples)) * 3000).astype(np.float32)
feats = fb(wins, [True] * B)
e0, e1, es = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
for e in (e0, e1, es):
    lib.fo_event_create(ctypes.byref(e))


def timed(fn, main, reps=20):
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


wb = eng.llm.stack.weight_bytes
for C in Cs:
    kvs = [base.fork() for _ in range(B)]
    items = [dict(identity="user", status="ipu_sl", feats=feats[b], kv=kvs[b], enc_cache=None, ada_cache=None,
                  pe_index=0) for b in range(B)]
    res = eng.listen(items)
    items = [dict(identity="user", status="ipu_cl", feats=feats[b], kv=kvs[b], enc_cache=r["enc_cache"],
                  ada_cache=r["ada_cache"], pe_index=r["pe_index"]) for b, r in enumerate(res)]
    if C == 1:
        g = eng._listen_graph_for(items, slots=2, extra=128)
        pe = g.submit_encoder(items, 0)
        g.submit_llm(items, pe, 0)
        llm_ex, enc_ex = g.llm_exec[0], [g.enc_exec[1]]
    else:
        g = eng._listen_graph_for(items, extra=128 * C, chunks=C)
        pes = [g.submit_encoder(items, 0, j) for j in range(C)]
        g.submit_llm([items] * C, pes, 0)
        g.collect_llm(0)
        for j in range(C):
            g.submit_encoder(items, 1, j)
        llm_ex, enc_ex = g.llm_exec[0][C], [g.enc_exec[1][C]]
    torch.cuda.synchronize()
    main, side = g.main.cuda_stream, g.side.cuda_stream

    def llm_only():
        _lib.call("fo_graph_launch", llm_ex, main)

    def both():
        for ex in enc_ex:
            _lib.call("fo_graph_launch", ex, side)
        _lib.call("fo_event_record", es, side)
        _lib.call("fo_graph_launch", llm_ex, main)
        _lib.call("fo_stream_wait_event", main, es)

    t = timed(llm_only, main)
    tb = timed(both, main)
    te = timed(lambda: [_lib.call("fo_graph_launch", ex, main) for ex in enc_ex], main)
    print(f"C={C}: encoder stage {te:8.1f} us for {C} chunk(s) = {te / C:7.1f} us/chunk", flush=True)
    print(f"C={C}: Qwen2 stage {t:8.1f} us for {C} chunk(s) = {t / C:7.1f} us/chunk "
          f"({wb / t / 1e6:.2f} TB/s over the layer weights); with the encoder stages beside it {tb:8.1f} us = "
          f"{tb / C:7.1f} us/chunk", flush=True)
    for kv in kvs:
        kv.free()
