"""Wall and device time of one text-decode step (TextGraph: 28 Qwen2 layers + lm_head + sampler) for B
sessions at real geometry after a ~150-token context, as the bench's speak stage runs it.
python scripts/text_step_time.py [B] [steps] (GPU only; run under rocprofv3 --kernel-trace --stats for
the per-kernel split)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
from fo.engine import FreezeOmniEngine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dev = torch.device("cuda:0")
eng = FreezeOmniEngine(os.path.join(ROOT, "configs", "real"), device=dev, max_sessions=max(8, B))
base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
kvs = [base.fork() for _ in range(B)]
ctx = list(range(100, 230))
eng.text_step([(kv, ctx) for kv in kvs])          # ~150-token context per session
ids, _ = eng.text_step([(kv, [1]) for kv in kvs])
for _ in range(5):
    ids, _ = eng.text_step([(kv, [i]) for kv, i in zip(kvs, ids)])
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(N):
    ids, _ = eng.text_step([(kv, [i]) for kv, i in zip(kvs, ids)])
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / N
gb = (eng.llm.stack.weight_bytes + eng.llm.lm_head.nbytes) / 1e9
print(f"text step B={B}: {dt * 1e3:.3f} ms wall/step, {gb:.2f} GB weights -> {gb / dt / 1e3:.2f} TB/s "
      f"(roofline {gb / 8.0:.3f} ms at 8 TB/s)", flush=True)
