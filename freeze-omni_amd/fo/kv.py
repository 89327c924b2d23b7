"""Paged KV cache for the decoder stacks (Qwen2 in AudioLLM, Llama layers of the AR speech decoder).

The reference keeps one transformers DynamicCache per session and grows it with torch.cat on every
chunk (models/audioLLM.py:416-419, models/decoder/decoder.py:321); sessions deep-copy the system
prompt cache (bin/dialog_state_pred.py:110,218).  Here every layer's K/V live in one device pool of
fixed-size pages ([layer][page][kv_head][slot][hd], fp32).  A sequence is a block list; `fork()`
shares full pages copy-on-write (refcounts), so N sessions forked from one system prompt store it
once, and appending never moves existing keys.
"""
import threading

import numpy as np
import torch

from . import ops


class KVPool:
    def __init__(self, n_layers, n_kv, hd, n_pages, page_size, device):
        self.n_layers, self.n_kv, self.hd, self.PS = n_layers, n_kv, hd, page_size
        self.n_pages = n_pages
        self.k = torch.empty(n_layers, n_pages, n_kv, page_size, hd, dtype=torch.float32, device=device)
        self.v = torch.empty_like(self.k)
        self.ref = np.zeros(n_pages, dtype=np.int32)
        self.free = list(range(n_pages - 1, -1, -1))
        self.device = torch.device(device)
        # sequences of one pool may grow, fork and free from several host threads (speech workers, server sessions):
        # every refcount change goes through a method below, under this lock (numpy element updates are not atomic)
        self.lock = threading.RLock()

    @property
    def bytes_per_token(self):
        return self.n_layers * self.n_kv * self.hd * 4 * 2

    def alloc(self):
        with self.lock:
            if not self.free:
                raise RuntimeError(f"KV pool exhausted ({self.n_pages} pages of {self.PS} tokens)")
            p = self.free.pop()
            self.ref[p] = 1
            return p

    def release(self, p):
        with self.lock:
            self.ref[p] -= 1
            if self.ref[p] == 0:
                self.free.append(p)

    def share(self, pages):
        """One more holder of each page (fork / adopt)."""
        with self.lock:
            for p in pages:
                if self.ref[p] <= 0:
                    raise RuntimeError(f"KV page {p} shared after it was freed")
                self.ref[p] += 1

    def release_all(self, pages):
        with self.lock:
            for p in pages:
                self.release(p)

    def make_private(self, pg, keep):
        """Copy-on-write of one page a sequence is about to write: if another sequence holds it too, returns a fresh
        page (with the keys copied when keep) and drops this holder's reference; else returns pg.  The refcount check
        and the alloc / release it decides happen under one lock hold, so a concurrent release cannot slip between."""
        with self.lock:
            if self.ref[pg] <= 1:
                return pg
            fresh = self.alloc()
            if keep:
                self.copy_page(pg, fresh)
            self.release(pg)
            return fresh

    def copy_page(self, src, dst):
        self.k[:, dst].copy_(self.k[:, src])
        self.v[:, dst].copy_(self.v[:, src])

    def pages_in_use(self):
        return self.n_pages - len(self.free)


class KVSeq:
    """One sequence's view of a KVPool (block list + length).  `version` changes whenever the block list
    does (pages added, a shared page copied on write, truncation), so a device-side copy of the block table
    can tell whether it is still current."""

    def __init__(self, pool):
        self.pool = pool
        self.pages = []
        self.length = 0
        self.version = 0

    def reserve(self, new_len):
        """Make room for new_len tokens.  Every page that will be written and is shared with another
        sequence is made private first (copy on write): the partial tail page and any page past the
        current length (pages reserved ahead are never shared by fork(), this is the safety net)."""
        PS = self.pool.PS
        if new_len > self.length:
            first = self.length // PS   # first page the new tokens touch (the partial tail if length % PS)
            last_pg = min(len(self.pages), (new_len + PS - 1) // PS)
            for li in range(first, last_pg):
                pg = self.pages[li]
                fresh = self.pool.make_private(pg, keep=li * PS < self.length)   # live keys on it: kept
                if fresh != pg:
                    self.pages[li] = fresh
                    self.version += 1
        while len(self.pages) * PS < new_len:
            self.pages.append(self.pool.alloc())
            self.version += 1

    def slot(self, pos):
        PS = self.pool.PS
        return self.pages[pos // PS] * PS + pos % PS

    def fork(self):
        """A sequence sharing this one's keys copy-on-write: only the pages that hold keys (< length) are
        shared; pages reserved ahead stay this sequence's own."""
        n = KVSeq(self.pool)
        used = (self.length + self.pool.PS - 1) // self.pool.PS
        n.pages = list(self.pages[:used])
        n.length = self.length
        self.pool.share(n.pages)
        n.origin = (tuple(n.pages), n.length)
        return n

    origin = None   # (pages, length) at fork time: the content it was forked with

    def pristine(self):
        """Still exactly the content it was forked with (nothing appended, no page changed)?"""
        return self.origin is not None and self.length == self.origin[1] and tuple(self.pages) == self.origin[0]

    def content_key(self):
        """Identity of a pristine fork's content: the shared pages (held by every holder of the key, so they
        cannot be reused for other keys meanwhile) and the length."""
        return self.origin

    def adopt(self, other):
        """Become a copy-on-write fork of `other` (this sequence's own pages are released)."""
        self.free()
        used = (other.length + self.pool.PS - 1) // self.pool.PS
        pages = list(other.pages[:used])
        self.pool.share(pages)
        self.pages = pages
        self.length = other.length
        self.version += 1
        self.origin = None

    def truncate(self, new_len):
        PS = self.pool.PS
        keep = (new_len + PS - 1) // PS
        self.pool.release_all(self.pages[keep:])
        if keep < len(self.pages):
            self.version += 1
        self.pages = self.pages[:keep]
        self.length = new_len

    def free(self):
        self.pool.release_all(self.pages)
        self.pages = []
        self.length = 0
        self.version += 1

    def __del__(self):
        try:
            if self.pages:
                self.free()
        except Exception:
            pass


class BatchMeta:
    """Device-side metadata of one ragged forward over several sequences.

    entries: list of (KVSeq, n_new, rope_pos_start, causal).  Reserves KV for the new tokens and
    advances each sequence's length.  gqa = query heads per kv head of the stack that consumes it:
    attention work items hold up to rows // gqa tokens of one sequence (rows: query rows per item, at most
    ops.attn_max_rows(head_dim) -- 32 on the Qwen2 kernel, 16 otherwise; the stacks use ops.attn_item_rows).
    """

    def __init__(self, entries, device, gqa=1, rows=16):
        T = sum(n for _, n, _, _ in entries)
        tok_seq = np.empty(T, np.int32)
        tok_pos = np.empty(T, np.int32)
        tok_slot = np.empty(T, np.int32)
        tok_nvis = np.empty(T, np.int32)
        maxb = 1
        t = 0
        last_rows = []
        max_keys = 0
        PS = entries[0][0].pool.PS if entries else 1
        for s, (seq, n, p0, causal) in enumerate(entries):
            old = seq.length
            seq.reserve(old + n)
            if n > 8:   # vectorised (a sentence's speech prefill: ~64 rows a session)
                pos = np.arange(old, old + n, dtype=np.int64)
                tok_seq[t:t + n] = s
                tok_pos[t:t + n] = p0 + np.arange(n)
                tok_slot[t:t + n] = np.asarray(seq.pages, np.int64)[pos // PS] * PS + pos % PS
                tok_nvis[t:t + n] = pos + 1 if causal else old + n
                t += n
            else:
                for i in range(n):
                    tok_seq[t] = s
                    tok_pos[t] = p0 + i
                    tok_slot[t] = seq.slot(old + i)
                    tok_nvis[t] = old + i + 1 if causal else old + n
                    t += 1
            seq.length = old + n
            maxb = max(maxb, len(seq.pages))
            last_rows.append(t - 1)
            max_keys = max(max_keys, seq.length)
        bt = np.zeros((len(entries), maxb), np.int32)
        for s, (seq, _, _, _) in enumerate(entries):
            bt[s, :len(seq.pages)] = seq.pages
        tpi = max(1, rows // gqa)
        items = []
        t = 0
        for s, (seq, n, _, _) in enumerate(entries):
            for b in range(0, n, tpi):
                items += [s, t + b, min(tpi, n - b)]
            t += n
        self.n_items = len(items) // 3
        self.max_rows = max(items[2::3]) * gqa
        # every sequence adds the same count of tokens, one work item each (item b = sequence b): fo_attention
        # then takes no item table
        self.uniform = self.n_items == len(entries) and len({n for _, n, _, _ in entries}) == 1
        host = np.concatenate([tok_seq, tok_pos, tok_slot, tok_nvis, np.asarray(last_rows, np.int32), bt.ravel(),
                               np.asarray(items, np.int32)])
        dev = ops.h2d(host, device)   # pinned staging, no stream synchronisation
        S = len(entries)
        self.T, self.S, self.maxb, self.max_keys = T, S, maxb, max_keys
        self.tok_seq = dev[0:T]
        self.tok_pos = dev[T:2 * T]
        self.tok_slot = dev[2 * T:3 * T]
        self.tok_nvis = dev[3 * T:4 * T]
        self.last_rows = dev[4 * T:4 * T + S]
        self.block_table = dev[4 * T + S:4 * T + S + S * maxb].view(S, maxb)
        self.items = dev[4 * T + S + S * maxb:]
        self.last_rows_host = last_rows
        self._host = host  # keep the staging buffer alive until the copy is consumed
