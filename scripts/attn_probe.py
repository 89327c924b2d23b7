"""Event-timed fo_attention at bench-like shapes (run on the GPU box)."""
import ctypes
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))
import torch  # noqa: E402

from fo import _lib, ops  # noqa: E402
from fo.kv import BatchMeta, KVPool, KVSeq  # noqa: E402


def timeit(fn, reps=50):
    lib = _lib.load()
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.fo_event_create(ctypes.byref(e0))
    lib.fo_event_create(ctypes.byref(e1))
    for _ in range(3):
        fn()
    s = ops.stream()
    lib.fo_event_record(e0, s)
    for _ in range(reps):
        fn()
    lib.fo_event_record(e1, s)
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    return ms.value / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    for (H, KVH, hd, n_pages) in [(28, 4, 128, 8192), (14, 14, 64, 8192)]:
        pool = KVPool(1, KVH, hd, n_pages, 16, dev)
        pool.k.normal_()
        pool.v.normal_()
        for L in (150, 500, 2000):
            for ntok in (1, 2):
                seqs = [KVSeq(pool) for _ in range(8)]
                BatchMeta([(s, L, 0, True) for s in seqs], dev)
                meta = BatchMeta([(s, ntok, s.length, True) for s in seqs], dev, gqa=H // KVH)
                T = meta.T
                q = torch.randn(T, H * hd, device=dev)
                out = torch.empty_like(q)
                for ns in sorted({1, 2, 4, 16, ops.attn_nsplit(meta.max_keys, meta.n_items, KVH)}):
                    pm = torch.empty(T * H * ns * 2, device=dev)
                    po = torch.empty(T * H * ns * hd, device=dev)
                    us = timeit(lambda: ops.attention(q, T, meta.items, meta.n_items, meta.max_rows, meta.tok_nvis,
                                                      meta.block_table, 16, pool.k[0], pool.v[0], H, KVH, hd,
                                                      1 / math.sqrt(hd), ns, pm, po, out))
                    kv_bytes = 8 * (L + ntok) * KVH * hd * 4 * 2
                    print(f"H={H} KVH={KVH} hd={hd} L={L} ntok={ntok} nsplit={ns}: {us:7.2f} us  "
                          f"{kv_bytes / us / 1e3:7.1f} GB/s", flush=True)
                tk = torch.zeros(meta.n_items * KVH, dtype=torch.int32, device=dev)
                pm = torch.empty(T * H * 16 * 2, device=dev)
                po = torch.empty(T * H * 16 * hd, device=dev)
                for kps in (64, 128, 256, 512):
                    us = timeit(lambda: ops.attention(q, T, meta.items, meta.n_items, meta.max_rows, meta.tok_nvis,
                                                      meta.block_table, 16, pool.k[0], pool.v[0], H, KVH, hd,
                                                      1 / math.sqrt(hd), 16, pm, po, out, tickets=tk,
                                                      keys_per_split=kps))
                    print(f"H={H} KVH={KVH} hd={hd} L={L} ntok={ntok} merged in-launch, keys/split {kps}: "
                          f"{us:7.2f} us", flush=True)
                for s in seqs:
                    s.free()


if __name__ == "__main__":
    main()
