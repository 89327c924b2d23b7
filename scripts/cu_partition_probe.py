"""Listen-stage CU partition probe: the encoder stage of chunk c+1 and the Qwen2 stage of chunk c replayed
concurrently from their captured graphs, each on a CU-masked stream (fo_stream_create_cumask), the encoder on a
few CUs and the Qwen2 stage on the complement -- so no Qwen2 workgroup shares a CU with the encoder's (the
round-2 probe masked only the encoder, and the overlapped time did not move).  Prints each stage alone and both
together per partition.  python scripts/cu_partition_probe.py (GPU only)."""
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
wins = (rng.standard_normal((B, fb.n_samples)) * 3000).astype(np.float32)
feats = fb(wins, [True] * B)
items = [dict(identity="user", status="ipu_sl", feats=feats[b], kv=kvs[b], enc_cache=None, ada_cache=None, pe_index=0)
         for b in range(B)]
res = eng.listen(items)
for _ in range(3):
    items = [dict(identity="user", status="ipu_cl", feats=feats[b], kv=kvs[b], enc_cache=r["enc_cache"],
                  ada_cache=r["ada_cache"], pe_index=r["pe_index"]) for b, r in enumerate(res)]
    res = eng.listen(items)
g = eng._listen_graph_for(items, slots=2, extra=256)
pe = g.submit_encoder(items, 0)
g.submit_llm(items, pe, 0)
torch.cuda.synchronize()
n_cu = ctypes.c_int()
name = ctypes.create_string_buffer(64)
hbm = ctypes.c_longlong()
_lib.call("fo_device_info", 0, name, 64, ctypes.byref(n_cu), ctypes.byref(hbm))
NCU = n_cu.value
print(f"{name.value.decode()} CUs {NCU}", flush=True)
e0, e1, ev = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
for e in (e0, e1, ev):
    lib.fo_event_create(ctypes.byref(e))


def stream_for(cus):
    words = (NCU + 31) // 32
    m = (ctypes.c_uint * words)()
    for c in cus:
        m[c // 32] |= 1 << (c % 32)
    h = ctypes.c_void_p()
    _lib.call("fo_stream_create_cumask", ctypes.byref(h), m, words)
    return h.value


def timed(fn, first, reps=20):
    fn()
    torch.cuda.synchronize()
    lib.fo_event_record(e0, first)
    for _ in range(reps):
        fn()
    lib.fo_event_record(e1, first)
    torch.cuda.synchronize()
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value / reps * 1e3


def run(label, llm_s, enc_s):
    t_llm = timed(lambda: _lib.call("fo_graph_launch", g.llm_exec[0], llm_s), llm_s)
    t_enc = timed(lambda: _lib.call("fo_graph_launch", g.enc_exec[1], enc_s), enc_s)

    def both():
        _lib.call("fo_graph_launch", g.enc_exec[1], enc_s)
        _lib.call("fo_event_record", ev, enc_s)
        _lib.call("fo_graph_launch", g.llm_exec[0], llm_s)
        _lib.call("fo_stream_wait_event", llm_s, ev)
    t_both = timed(both, llm_s)
    print(f"{label:44s} LLM {t_llm:7.1f}  enc {t_enc:7.1f}  both {t_both:7.1f} us", flush=True)


run("unmasked (engine / side streams)", g.main.cuda_stream, g.side.cuda_stream)
parts = []
for k, stride in ((8, 32), (16, 16), (16, 1), (32, 8), (32, 1), (24, 0)):
    if stride == 0:   # 3 per XCD under an XCD-major numbering: bits x * 32 + {0, 1, 2}
        enc = [x * (NCU // 8) + j for x in range(8) for j in range(3)]
        label = f"enc on {k} CUs (3 per 32-CU block)"
    else:
        enc = list(range(0, k * stride, stride))
        label = f"enc on {k} CUs (stride {stride})"
    llm = [c for c in range(NCU) if c not in set(enc)]
    run(label, stream_for(llm), stream_for(enc))
