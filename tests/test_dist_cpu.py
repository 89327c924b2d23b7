"""world_size-2 gloo tests of the N>1 path (bench aggregation + frozen-weight broadcast), on CPU."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Lin:
    def __init__(self, g, scale):
        self.packed = (torch.randn(1000, generator=g) * scale).to(torch.bfloat16)
        self.bias = torch.randn(17, generator=g) * scale


class _Slot:
    __slots__ = ("w", "b")   # like fo.stack.Layer: the weights live only in slots

    def __init__(self, g):
        self.w = torch.randn(64, generator=g)
        self.b = torch.randn(8, generator=g)


class _Model:
    def __init__(self, rank):
        g = torch.Generator().manual_seed(7 if rank == 0 else 100 + rank)
        self.layers = [_Lin(g, 1.0) for _ in range(5)]
        self.table = torch.randn(300, 4, generator=g)
        self.row = self.table[10:20]                 # a view at an offset: covered by the table's storage
        self.slotted = _Slot(g)
        self.alias = self.layers[0].packed          # shared storage is sent once
        self.pool = type("KVPool", (), {})()         # per-session state: never broadcast
        self.pool.k = torch.full((8,), float(rank))


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from fo.replica import broadcast_frozen, frozen_tensors
        vals = [float(rank * 10 + i) for i in range(rank + 1)]    # ragged per-rank lists
        got = bench.gather_list(dist, vals, world, torch.device("cpu"))
        m = _Model(rank)
        n, nbytes = broadcast_frozen(m, dist, bucket_bytes=3000)   # small buckets: exercise splitting
        ref = _Model(0)
        same = all(torch.equal(a, b) for a, b in zip(frozen_tensors(m), frozen_tensors(ref)))
        from fo.replica import frozen_checksum
        same = same and frozen_checksum(m) == frozen_checksum(ref) != frozen_checksum(_Model(1))
        q.put((rank, got, n, nbytes, same, float(m.pool.k[0]), m.alias.data_ptr() == m.layers[0].packed.data_ptr()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gather_and_weight_broadcast():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got, n, nbytes, same, kv0, alias in res:
        assert got == [0.0, 10.0, 11.0]
        assert n == 13 and nbytes == 5 * (1000 * 2 + 17 * 4) + 300 * 4 * 4 + (64 + 8) * 4
        assert same and alias
        assert kv0 == float(rank)


def _receive_worker(rank, world, port, q, empty_dir):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import types
        from oracle import configs
        from fo.engine import make_source
        from fo.params import all_shapes
        from fo.replica import broadcast_frozen, frozen_tensors
        from fo.weights import CheckpointSource, ReceiveSource
        cfg = configs.get("tiny")
        shapes = all_shapes(cfg)
        if rank == 0:
            g = torch.Generator().manual_seed(11)
            src = CheckpointSource({k: torch.randn(*v, generator=g) for k, v in shapes.items()}, "cpu")
        else:   # a model directory without any weight file: nothing may be read
            try:
                make_source(cfg, None, "cpu", model_path=empty_dir, llm_path=empty_dir)
                reads = "no error"
            except (FileNotFoundError, OSError):
                reads = "raised"
            src = make_source(cfg, None, "cpu", model_path=empty_dir, llm_path=empty_dir, receive=True)
            assert isinstance(src, ReceiveSource) and reads == "raised", reads

        def build(src):   # engine-shaped object: raw parameters, a bf16 "packed" copy and a derived tensor
            m = types.SimpleNamespace(p={k: src.get(k) for k in sorted(shapes)})
            m.packed = {k: src.get(k, torch.bfloat16) for k in sorted(shapes) if len(shapes[k]) == 2}
            m.affine = m.p["adpter_user.bn2.weight"] / torch.sqrt(m.p["adpter_user.bn2.running_var"].abs() + 1e-3)
            return m

        m = build(src)
        n, nbytes = broadcast_frozen(m, dist)
        digest = [float(t.double().sum()) for t in frozen_tensors(m)]
        q.put((rank, n, nbytes, digest))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_receive_only_replica(tmp_path):
    """Rank 1 builds from a model directory with no weight files (fo.weights.ReceiveSource: shapes only,
    nothing read or generated) and ends bit-identical to rank 0 after broadcast_frozen, derived tensors
    included (bench.py's N > 1 start-up)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_receive_worker, args=(r, 2, port, q, str(tmp_path))) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, n0, b0, d0), (r1, n1, b1, d1) = res
    assert n0 == n1 and b0 == b1 and n0 > 100
    assert d0 == d1
