"""Which tensors differ between a fully built engine and a receive-only engine after fo.replica's broadcast:
walks EVERY tensor reachable from both engines (skip lists ignored) with its attribute path and prints the
paths whose bytes differ -- the weight-derived state the broadcast does not reach.
python scripts/replica_diff.py (GPU only)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from fo.engine import FreezeOmniEngine  # noqa: E402
from fo.replica import broadcast_frozen  # noqa: E402
from test_replica_gpu import _Play, _Record  # noqa: E402


def walk(o, path, out, seen):
    if isinstance(o, torch.Tensor):
        out.setdefault(path, o)
        return
    if o is None or isinstance(o, (int, float, str, bool, bytes, torch.device, torch.dtype)) or id(o) in seen:
        return
    seen.add(id(o))
    if isinstance(o, dict):
        for k in sorted(o, key=str):
            walk(o[k], f"{path}[{k!r}]", out, seen)
    elif isinstance(o, (list, tuple)):
        for i, v in enumerate(o):
            walk(v, f"{path}[{i}]", out, seen)
    elif hasattr(o, "__dict__") and type(o).__module__.split(".")[0] not in ("torch", "numpy", "ctypes", "builtins"):
        for k in sorted(vars(o)):
            walk(vars(o)[k], f"{path}.{k}", out, seen)
    elif hasattr(o, "__slots__"):
        for k in o.__slots__:
            if hasattr(o, k):
                walk(getattr(o, k), f"{path}.{k}", out, seen)


dev = torch.device("cuda:0")
tiny = os.path.join(ROOT, "configs", "tiny")
a = FreezeOmniEngine(tiny, device=dev, max_sessions=4)
b = FreezeOmniEngine(tiny, device=dev, max_sessions=4, receive_weights=True)
rec = _Record()
broadcast_frozen(a, rec)
broadcast_frozen(b, _Play(rec.flats))
ta, tb = {}, {}
walk(a, "eng", ta, set())
walk(b, "eng", tb, set())
print(f"{len(ta)} / {len(tb)} tensors reachable", flush=True)
nd = 0
for p in sorted(ta):
    x, y = ta[p], tb.get(p)
    if y is None or x.shape != y.shape or x.dtype != y.dtype:
        print("shape/presence differs:", p, tuple(x.shape), None if y is None else tuple(y.shape))
        continue
    if x.is_floating_point():
        same = torch.equal(torch.nan_to_num(x.float(), 7.0), torch.nan_to_num(y.float(), 7.0))
    else:
        same = torch.equal(x, y)
    if not same:
        nd += 1
        print("differs:", p, tuple(x.shape), x.dtype, x.is_contiguous(), x.untyped_storage().nbytes(), flush=True)
print(f"{nd} differing tensors", flush=True)
