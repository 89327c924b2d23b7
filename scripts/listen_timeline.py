"""Un-profiled timeline of the pipelined listen (rocprofv3's kernel trace serialises the two streams, so
it cannot show their overlap): HIP events around every encoder stage (side stream) and LLM stage
(engine stream) of one 8-user turn, all relative to one base event.
python scripts/listen_timeline.py (GPU only)."""
import ctypes
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from fo import _lib, ops  # noqa: E402
from fo.engine import FreezeOmniEngine, ListenGraph  # noqa: E402

dev = torch.device("cuda:0")
eng = FreezeOmniEngine(os.path.join(ROOT, "configs", "real"), device=dev, max_sessions=8)
lib = _lib.load()
marks = []   # (label, chunk, event)


def ev(stream):
    e = ctypes.c_void_p()
    lib.fo_event_create(ctypes.byref(e))
    lib.fo_event_record(e, stream.cuda_stream)
    return e


orig_enc, orig_llm = ListenGraph.submit_encoder, ListenGraph.submit_llm
counter = {"enc": 0, "llm": 0}


def enc_wrap(self, items, k=0):
    c = counter["enc"]
    counter["enc"] += 1
    marks.append(("enc0", c, ev(self.side)))
    r = orig_enc(self, items, k)
    marks.append(("enc1", c, ev(self.side)))
    return r


def llm_wrap(self, items, new_pe, k=0, wait=True):
    c = counter["llm"]
    counter["llm"] += 1
    marks.append(("llm0", c, ev(self.main)))
    r = orig_llm(self, items, new_pe, k, wait)
    marks.append(("llm1", c, ev(self.main)))
    return r


ListenGraph.submit_encoder, ListenGraph.submit_llm = enc_wrap, llm_wrap


class A:
    pipeline = True
    text_tokens = 8
    codec_tokens = 40
    top_k = 1


base_kv = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
pcms = [bench.synth_pcm(160000, 1234 + u) for u in range(8)]
bench.run_turn(eng, base_kv, pcms, A, torch.cuda.synchronize)   # warm: graphs captured
marks.clear()
counter.update(enc=0, llm=0)
base = ev(ops.engine_stream(dev))
bench.run_turn(eng, base_kv, pcms, A, torch.cuda.synchronize)
torch.cuda.synchronize()


def t(e):
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(base, e, ctypes.byref(ms))
    return ms.value


T = {}
for lab, c, e in marks:
    T[(lab, c)] = t(e)
n = counter["llm"]
llm = [T[("llm1", c)] - T[("llm0", c)] for c in range(n)]
enc = [T[("enc1", c)] - T[("enc0", c)] for c in range(counter["enc"])]
gap = [T[("llm0", c)] - T[("llm1", c - 1)] for c in range(1, n)]
print(f"chunks {n}: LLM stage {np.median(llm):.3f} ms median (sum {sum(llm):.1f}), encoder stage "
      f"{np.median(enc):.3f} ms median (sum {sum(enc):.1f}); engine-stream gap between LLM stages "
      f"{np.median(gap):.3f} ms median (sum {sum(gap):.1f}); listen wall {T[('llm1', n - 1)] - T[('llm0', 0)]:.1f} ms")
for c in range(1, min(n, 6)):
    print(f"  chunk {c}: enc {T[('enc0', c)]:.2f}-{T[('enc1', c)]:.2f}  llm {T[('llm0', c)]:.2f}-{T[('llm1', c)]:.2f}")
