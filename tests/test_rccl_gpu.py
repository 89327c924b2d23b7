"""The multi-GPU replica path on RCCL, executed (bin/pool.py:61-91): a fresh child process -- started
before anything in it touches the GPU -- joins an `nccl` (RCCL) process group of world size 1 with a file store and
device_id cuda:0, builds a tiny engine, broadcasts its frozen weights with fo.replica.broadcast_frozen (the bucketed
per-dtype broadcast bench.py runs from rank 0 at N > 1), all_gathers fo.replica.frozen_checksum, passes a barrier and
destroys the group.  The child prints RCCL's version and the rank count; the test echoes them."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
sys.path[:0] = [{root!r}, {pkg!r}]
import torch
import torch.distributed as dist
dist.init_process_group("nccl", init_method="file://" + {store!r}, rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
torch.cuda.set_device(0)
from fo.engine import FreezeOmniEngine
from fo.replica import broadcast_frozen, frozen_checksum, frozen_storages
eng = FreezeOmniEngine(os.path.join({root!r}, "configs", "tiny"), device="cuda:0", max_sessions=2)
torch.cuda.synchronize()
before = frozen_checksum(eng)
t0 = time.perf_counter()
n, nbytes = broadcast_frozen(eng, dist)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
ck = torch.tensor([frozen_checksum(eng)], dtype=torch.int64, device="cuda:0")
cks = [torch.zeros_like(ck) for _ in range(dist.get_world_size())]
dist.all_gather(cks, ck)
dist.barrier()
out = {{"backend": dist.get_backend(), "world_size": dist.get_world_size(), "rank": dist.get_rank(),
        "rccl_version": ".".join(str(x) for x in torch.cuda.nccl.version()), "storages": n, "bytes": nbytes,
        "broadcast_s": round(dt, 4), "checksums": [int(c.item()) for c in cks], "checksum_before": before}}
dist.destroy_process_group()
print("RCCL_RESULT " + json.dumps(out), flush=True)
"""


def test_rccl_world1_broadcast_and_checksum(tmp_path, capsys):
    store = str(tmp_path / "store")
    code = CHILD.format(root=ROOT, pkg=os.path.join(ROOT, "freeze-omni_amd"), store=store)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("RCCL_RESULT ")]
    assert line, r.stdout[-2000:]
    res = json.loads(line[-1][len("RCCL_RESULT "):])
    with capsys.disabled():
        print(f"\n[rccl] backend {res['backend']} RCCL {res['rccl_version']} ranks {res['world_size']} "
              f"broadcast {res['bytes']} B in {res['storages']} storages, {res['broadcast_s']} s")
    assert res["backend"] == "nccl" and res["world_size"] == 1 and res["rank"] == 0
    assert res["storages"] > 0 and res["bytes"] > 0
    assert res["checksums"] == [res["checksum_before"]]   # the broadcast left rank 0's weights bit for bit
