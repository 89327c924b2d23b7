"""Data-parallel replicas: frozen-weight broadcast.

Sessions never cross replicas, so the only collective on the path is one broadcast of the frozen
weights from rank 0 at start-up (RCCL over xGMI on the GPU box; gloo in the CPU tests).  The
weights are coalesced into flat per-dtype buckets so the broadcast is a few large messages (xGMI is
point-to-point: large messages keep every ring link busy) instead of hundreds of small ones.
"""
import torch

# per-session / scratch state that must not be broadcast (it is replica-local by design), including the
# captured-graph caches a warm-up fills lazily (decode / text / listen graphs, vocoder buffers, fbank tables),
# so a replica that has run work before the broadcast walks the same storage list as one that has not
_SKIP_CLASSES = {"KVPool", "KVSeq", "Runtime", "SlotPool", "EncoderCache", "AdapterCache", "Framer", "DecodeGraph",
                 "TextGraph", "ListenGraph", "EncoderGraph", "ListenPipe", "FbankGPU", "HostBuffer", "SampleCheck", "_HostRing"}
_FOREIGN = {"torch", "numpy", "builtins", "ctypes", "transformers", "tokenizers", "threading", "logging"}
_SKIP_ATTRS = {"ws", "counters", "part_ml", "part_o", "scratch", "src", "_graphs", "_lgraphs", "_egraphs", "_tgraphs", "_fbank",
               "host", "meta_d", "hist", "err"}


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
        elif type(o).__module__.split(".")[0] not in _FOREIGN:
            # instance dict AND __slots__ (fo.stack.Layer is slotted: its weights live only in slots)
            names = set(vars(o)) if hasattr(o, "__dict__") else set()
            for c in type(o).__mro__:
                sl = getattr(c, "__slots__", ())
                names.update((sl,) if isinstance(sl, str) else sl)
            for k in sorted(names):
                if k not in _SKIP_ATTRS and k not in ("__dict__", "__weakref__") and hasattr(o, k):
                    walk(getattr(o, k))

    walk(root)
    return out


def frozen_storages(root):
    """A byte view over the WHOLE storage of every frozen tensor, one per storage, in walk order.  Broadcasting
    storages rather than tensors covers views at an offset, non-contiguous views and a smaller view that
    shares its first byte with a larger tensor (frozen_tensors keeps one tensor per data pointer)."""
    out, seen = [], set()
    for t in frozen_tensors(root):
        st = t.untyped_storage()
        if st.data_ptr() in seen or st.nbytes() == 0:
            continue
        seen.add(st.data_ptr())
        out.append(torch.empty(0, dtype=torch.uint8, device=t.device).set_(st))
    return out


def broadcast_frozen(root, dist, src=0, bucket_bytes=256 << 20):
    """Broadcast every frozen storage of `root` from rank `src`.  Returns (n_storages, n_bytes)."""
    tens = frozen_storages(root)
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
    """Integer checksum of every frozen storage's bytes (int64 sum of its raw 32-bit words, mixed in walk
    order): equal on every rank when the broadcast delivered rank 0's weights."""
    acc = 0
    for i, b in enumerate(frozen_storages(root)):
        n4 = b.numel() // 4 * 4
        w = b[:n4].view(torch.int32).to(torch.int64).sum().item() if n4 else 0
        tail = int(b[n4:].to(torch.int64).sum().item()) if b.numel() > n4 else 0
        acc = (acc * 1000003 + w + tail + i) & ((1 << 63) - 1)
    return acc


def copy_frozen(src_root, dst_root):
    """Fill a receive-only replica in the SAME process (fo.weights.ReceiveSource layouts, e.g. on another GPU
    of the node) from a loaded one: every frozen storage copied device to device (a peer copy over xGMI
    between GPUs), in the walk order broadcast_frozen uses, then checked by frozen_checksum.  The in-process
    form of the start-up broadcast (bin/pool.py's `devices` replicas), so one design serves both.
    Returns the bytes copied."""
    src, dst = frozen_storages(src_root), frozen_storages(dst_root)
    if len(src) != len(dst) or any(a.numel() != b.numel() for a, b in zip(src, dst)):
        raise RuntimeError(f"copy_frozen: the replicas' frozen layouts differ ({len(src)} vs {len(dst)} storages)")
    total = 0
    for a, b in zip(src, dst):
        b.copy_(a)
        total += a.numel()
    for r in {t.device for t in src} | {t.device for t in dst}:
        torch.cuda.synchronize(r)
    if frozen_checksum(src_root) != frozen_checksum(dst_root):
        raise RuntimeError("copy_frozen: replica weights differ from the source after the copy")
    return total
