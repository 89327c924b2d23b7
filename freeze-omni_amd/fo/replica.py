"""Data-parallel replicas: frozen-weight broadcast.

Sessions never cross replicas, so the only collective on the path is one broadcast of the frozen
weights from rank 0 at start-up (RCCL over xGMI on the GPU box; gloo in the CPU tests).  The
weights are coalesced into flat per-dtype buckets so the broadcast is a few large messages (xGMI is
point-to-point: large messages keep every ring link busy) instead of hundreds of small ones.
"""
import torch

# per-session / scratch state that must not be broadcast (it is replica-local by design)
_SKIP_CLASSES = {"KVPool", "KVSeq", "Runtime", "SlotPool", "EncoderCache", "AdapterCache", "Framer"}
_FOREIGN = {"torch", "numpy", "builtins", "ctypes", "transformers", "tokenizers", "threading", "logging"}
_SKIP_ATTRS = {"ws", "counters", "part_ml", "part_o", "scratch", "src"}


def frozen_tensors(root):
    """Every distinct tensor reachable from `root`'s attributes, in deterministic order
    (attribute-name order of a depth-first walk), excluding per-session state and scratch."""
    out, seen_obj, seen_ptr = [], set(), set()

    def walk(o):
        if isinstance(o, torch.Tensor):
            if o.numel() and o.data_ptr() not in seen_ptr:
                seen_ptr.add(o.data_ptr())
                out.append(o)
            return
        if o is None or isinstance(o, (int, float, str, bool, bytes, torch.device, torch.dtype)):
            return
        if id(o) in seen_obj or type(o).__name__ in _SKIP_CLASSES:
            return
        seen_obj.add(id(o))
        if isinstance(o, dict):
            for k in sorted(o, key=str):
                walk(o[k])
        elif isinstance(o, (list, tuple)):
            for v in o:
                walk(v)
        elif hasattr(o, "__dict__") and type(o).__module__.split(".")[0] not in _FOREIGN:
            for k in sorted(vars(o)):
                if k not in _SKIP_ATTRS:
                    walk(vars(o)[k])

    walk(root)
    return out


def broadcast_frozen(root, dist, src=0, bucket_bytes=256 << 20):
    """Broadcast every frozen tensor of `root` from rank `src`.  Returns (n_tensors, n_bytes)."""
    tens = [t for t in frozen_tensors(root) if t.is_contiguous()]
    by_dtype = {}
    for t in tens:
        by_dtype.setdefault(t.dtype, []).append(t)
    total = 0
    for dtype, ts in by_dtype.items():
        bucket, size = [], 0
        esz = torch.empty((), dtype=dtype).element_size()
        for t in ts + [None]:
            if t is not None and size + t.numel() * esz <= bucket_bytes or (t is not None and not bucket):
                bucket.append(t)
                size += t.numel() * esz
                continue
            if bucket:
                flat = torch.cat([b.reshape(-1) for b in bucket]) if len(bucket) > 1 else bucket[0].reshape(-1)
                dist.broadcast(flat, src)
                if len(bucket) > 1:
                    off = 0
                    for b in bucket:
                        b.reshape(-1).copy_(flat[off:off + b.numel()])
                        off += b.numel()
                total += size
            bucket, size = ([t], t.numel() * esz) if t is not None else ([], 0)
    return len(tens), total


def frozen_checksum(root):
    """Order-independent integer checksum of every frozen tensor's bytes (int64 sum of the raw 32-bit words of
    each tensor, mixed with its index): equal on every rank iff the broadcast delivered rank 0's weights."""
    acc = 0
    for i, t in enumerate(t for t in frozen_tensors(root) if t.is_contiguous()):
        b = t.reshape(-1).view(torch.uint8)
        n4 = b.numel() // 4 * 4
        w = b[:n4].view(torch.int32).to(torch.int64).sum().item() if n4 else 0
        tail = int(b[n4:].to(torch.int64).sum().item()) if b.numel() > n4 else 0
        acc = (acc * 1000003 + w + tail + i) & ((1 << 63) - 1)
    return acc
