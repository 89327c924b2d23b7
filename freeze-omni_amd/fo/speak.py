"""Batched speech generation: AR codec-token decode + 40/10 codec chunking + silence-cut emission.

Restates llm2TTS.run (models/decoder/llm2tts.py:114-160) for many sessions at once: every decode step
advances all live sessions with one launch sequence, and sessions that reach a codec chunk in the
same step share one vocoder launch.  Emission follows find_min_sum_index
(models/decoder/llm2tts.py:70-112) using the fo_silence_cut kernel for the window search.
"""
import collections
import os
import time

import torch

from . import _lib, ops
from .ops import F32, I32
from .tts import penalty_ring


class SpeakState:
    def __init__(self, seq, top_k, max_tokens, min_tokens):
        self.seq = seq
        self.top_k = top_k
        self.max_tokens = max_tokens
        self.min_tokens = min_tokens
        self.tokens = []          # tokens waiting for the vocoder (incl. left context)
        self.left = 0
        self.buffer = None        # held PCM (device 1-D)
        self.done = False
        self.n_generated = 0
        self.emitted = []         # device PCM segments
        self.all_ids = []
        self.t_first_pcm = None   # host time the first vocoder chunk's PCM was known (before the silence gate)


def silence_cut(buffer, syn, N, threshold, res, r=None):
    """find_min_sum_index(buffer, syn): returns (new_buffer, emitted or None); device tensors 1-D.
    r: the kernel's (min_sum, cut) already read back (batched by the caller), else launched and read here."""
    if r is None:
        ops.silence_cut(syn, N, res)
        r = res.cpu()
    min_sum, cut = float(r[0]), int(r[1])
    if min_sum / N < threshold:
        out = syn[:cut] if buffer is None or buffer.numel() == 0 else torch.cat([buffer, syn[:cut]])
        return syn[cut:].clone(), out
    nb = syn.clone() if buffer is None or buffer.numel() == 0 else torch.cat([buffer, syn])
    return nb, None


def speak(engine, items, top_k=1, codec_chunk_size=40, codec_padding_size=10, N=2401, seg_threshold=0.01,
          max_tokens=1000, min_tokens=0, states_out=None, seed=0, graph=True, window=32, penalty_window_size=-1,
          penalty=1.1, stream=None, voc_stream=None):
    """items: list of (hidden [T1, D] device, prefix [T2, D] device or None).
    min_tokens > 0 masks EOS until that many tokens (benchmark policy).
    Yields (session index, pcm segment device 1-D) as segments become available; the per-session
    SpeakState objects are appended to states_out.
    graph=True replays a captured decode step (fo.tts.DecodeGraph) and reads sampled ids back lazily,
    up to `window` steps behind the GPU; graph=False is the step-by-step eager loop.  Both produce the
    same ids (same kernels, same RNG stream).
    penalty_window_size > 0 applies the reference's repetition penalty (decoder.py:348-351, fo_penalty).
    stream / voc_stream: the streams of the AR decode and of the vocoder (default: the engine's main and side
    streams); the bench's concurrent speech generation runs on its own pair beside the text decode."""
    pen = (int(penalty_window_size), float(penalty)) if penalty_window_size and penalty_window_size > 0 else None
    es = stream if stream is not None else ops.engine_stream(engine.device)
    vs = voc_stream if voc_stream is not None else ops.engine_stream(engine.device, side=True)
    with torch.cuda.stream(es):
        seqs = engine.tts.start(items)
    states = [SpeakState(sq, top_k, max_tokens, min_tokens) for sq in seqs]
    if states_out is not None:
        states_out.extend(states)
    run = _speak_graph if graph else _speak_eager
    gen = run(engine, states, top_k, codec_chunk_size, codec_padding_size, N, seg_threshold, max_tokens, min_tokens,
              seed, window, pen, voc=vs)
    try:
        while True:
            with torch.cuda.stream(es):  # the engine stream is current only while engine code runs
                out = next(gen, None)
            if out is None:
                break
            yield from out
    finally:
        engine.tts.free(seqs)


def _after_token(states, i, t, eos, chunk_due, finished, codec_chunk_size, codec_padding_size):
    """llm2tts.py:122-129 bookkeeping for one sampled id of session i."""
    s = states[i]
    if t == eos or s.n_generated >= s.max_tokens:
        s.done = True
        finished.append(i)
        return
    s.tokens.append(t)
    s.all_ids.append(t)
    s.n_generated += 1
    if len(s.tokens) == s.left + codec_chunk_size + codec_padding_size:
        chunk_due.append(i)
    if s.n_generated >= s.max_tokens:
        s.done = True
        finished.append(i)


def _emit(engine, states, chunk_due, finished, up, pad, N, thr, res, voc):
    segs = []
    if chunk_due:
        segs += list(_vocode(engine, states, chunk_due, up, pad, N, thr, res, voc, final=False))
    if finished:
        segs += list(_vocode(engine, states, [i for i in finished if states[i].tokens], up, pad, N, thr, res, voc,
                             final=True))
    return segs


def _speak_eager(engine, states, top_k, codec_chunk_size, codec_padding_size, N, seg_threshold, max_tokens,
                 min_tokens, seed, window, pen=None, voc=None):
    tts = engine.tts
    dev = engine.device
    up = engine.codec.upsample
    res = torch.empty(2, dtype=F32, device=dev)
    cur = torch.full((len(states),), tts.sos, dtype=I32, device=dev)
    topk_d = torch.tensor([top_k] * len(states), dtype=I32).to(dev)
    out_ids = torch.empty(len(states), dtype=I32, device=dev)
    live = list(range(len(states)))
    step = 0
    while live:
        lg = tts.step([states[i].seq for i in live], cur[:len(live)])
        # benchmark policy: while EOS is masked, draw only real codec ids (random weights would otherwise
        # also emit the BOS/SOS/PAD specials that a trained decoder never produces)
        forced = bool(min_tokens and step < min_tokens)
        st = torch.tensor([step] * len(live) + live, dtype=I32).to(dev)  # RNG (step, session) per row
        if pen:
            win = torch.tensor([penalty_ring([tts.sos] + states[i].all_ids, pen[0]) for i in live], dtype=I32).to(dev)
            ops.penalty(lg, tts.vocab + 4, cur, win, st, pen[1], B=len(live))
        chk = ops.sample_check(dev)
        ops.sample(lg, tts.vocab if forced else tts.vocab + 4, out_ids, topk_d, None, None, seed=seed,
                   step=st[:len(live)], B=len(live), key=st[len(live):], err=chk)
        ids = out_ids[:len(live)].cpu().tolist()
        chk.check("speech decode")
        step += 1
        finished, chunk_due = [], []
        for j, i in enumerate(live):
            _after_token(states, i, ids[j], tts.eos, chunk_due, finished, codec_chunk_size, codec_padding_size)
        segs = _emit(engine, states, chunk_due, finished, up, codec_padding_size, N, seg_threshold, res, voc)
        live = [i for i in live if not states[i].done]
        if live:
            cur = torch.tensor([states[i].all_ids[-1] for i in live], dtype=I32).to(dev)
        if segs:
            yield segs


def _speak_graph(engine, states, top_k, codec_chunk_size, codec_padding_size, N, seg_threshold, max_tokens,
                 min_tokens, seed, window, pen=None, capture=True, voc=None):
    tts = engine.tts
    dev = engine.device
    up = engine.codec.upsample
    res = torch.empty(2, dtype=F32, device=dev)
    live = list(range(len(states)))
    max_keys = max(s.seq.kv.length for s in states) + max_tokens + 1
    pending = collections.deque()   # (step, live list, graph, event) launched but not yet read
    step = 0                        # decode steps launched (RNG step and history row)
    g = None
    while live or pending:
        # launch ahead while the window has room
        while live and len(pending) < window and step < max_tokens:
            forced = bool(min_tokens and step < min_tokens)
            ng = tts.decode_graph(len(live), tts.vocab if forced else tts.vocab + 4, top_k, seed, max_keys,
                                  max_tokens + 1, pen, capture)
            if ng is not g:
                if g is None or ng.B != g.B:
                    ng.ids.fill_(tts.sos) if step == 0 else ng.ids.copy_(torch.tensor(
                        [states[i].all_ids[-1] for i in live], dtype=I32).to(dev))
                    ng.set_window([[tts.sos] + states[i].all_ids for i in live])
                    ng.prime()
                else:
                    ng.adopt(g)  # same batch, other sampler bound: ids and input rows stay on the device
                g = ng
            ev = g.launch([states[i].seq for i in live], live, step, step)
            pending.append((step, list(live), g, ev))
            step += 1
        if not pending:
            break
        st, batch, pg, ev = pending.popleft()
        _lib.call("fo_event_sync", ev)
        pg.check()
        row = pg.hist.np[st].tolist()
        finished, chunk_due = [], []
        for j, i in enumerate(batch):
            if not states[i].done:
                _after_token(states, i, row[j], tts.eos, chunk_due, finished, codec_chunk_size, codec_padding_size)
        segs = _emit(engine, states, chunk_due, finished, up, codec_padding_size, N, seg_threshold, res, voc)
        if finished:
            # the batch shrinks: drain what was launched with the old batch (finished rows are ignored),
            # then continue with a graph for the survivors, seeded with their last ids
            while pending:
                st, batch, pg, ev = pending.popleft()
                _lib.call("fo_event_sync", ev)
                pg.check()
                row = pg.hist.np[st].tolist()
                fin2, due2 = [], []
                for j, i in enumerate(batch):
                    if not states[i].done:
                        _after_token(states, i, row[j], tts.eos, due2, fin2, codec_chunk_size, codec_padding_size)
                segs += _emit(engine, states, due2, fin2, up, codec_padding_size, N, seg_threshold, res, voc)
            live = [i for i in live if not states[i].done]
            g = None
        if step >= max_tokens and not pending:
            # every launched token is read; sessions still open ran into max_tokens
            rest = [i for i in live if not states[i].done]
            for i in rest:
                states[i].done = True
            segs += _emit(engine, states, [], [i for i in rest if states[i].tokens], up, codec_padding_size, N,
                          seg_threshold, res, voc)
            live = []
        if segs:
            yield segs


def _vocode(engine, states, idx, up, pad, N, thr, res, voc, final):
    """One batched vocoder call for sessions idx (equal token counts share a launch), on the vocoder stream
    (the engine's side stream by default): the MFMA-bound vocoder overlaps the launch-bound AR decode steps
    already queued on the decode stream instead of stalling them (the stream is blocking w.r.t. the legacy
    default stream, so callers reading the yielded PCM there are ordered after it)."""
    with torch.cuda.stream(voc if voc is not None else ops.engine_stream(engine.device, side=True)):
        yield from _vocode_on_stream(engine, states, idx, up, pad, N, thr, res, final)


def _vocode_on_stream(engine, states, idx, up, pad, N, thr, res, final):
    groups = {}
    for i in idx:
        groups.setdefault(len(states[i].tokens), []).append(i)
    for T, members in groups.items():
        ids = torch.tensor([states[i].tokens for i in members], dtype=I32).to(engine.device)
        pcm = engine.codec(ids)
        cuts = None
        if not final:   # every member's window search in one launch, one read-back for the call
            resb = torch.empty(len(members), 2, dtype=F32, device=engine.device)
            lefts = {states[i].left for i in members}
            if len(lefts) == 1:   # (equal token counts: always one left context)
                left = lefts.pop()
                ops.silence_cut_rows(pcm[:len(members), left * up: pcm.shape[1] - pad * up], N, resb)
            else:
                for j, i in enumerate(members):
                    s = states[i]
                    ops.silence_cut(pcm[j][s.left * up: pcm.shape[1] - pad * up], N, resb[j])
            cuts = resb.cpu()
        for j, i in enumerate(members):
            s = states[i]
            syn = pcm[j]
            if final:
                if s.t_first_pcm is None:
                    torch.cuda.current_stream(engine.device).synchronize()   # this call's PCM (not the other streams)
                    s.t_first_pcm = time.perf_counter()
                syn = syn[s.left * up:]
                seg = syn if s.buffer is None or s.buffer.numel() == 0 else torch.cat([s.buffer, syn])
                s.tokens = []
                s.emitted.append(seg)
                yield i, seg
                continue
            syn = syn[s.left * up: syn.numel() - pad * up]
            s.left = pad
            s.tokens = s.tokens[-(s.left + pad):]
            s.buffer, seg = silence_cut(s.buffer, syn, N, thr, res, cuts[j])   # PCM is final here (read back)
            if s.t_first_pcm is None:
                s.t_first_pcm = time.perf_counter()
            if seg is not None:
                s.emitted.append(seg)
                yield i, seg


class SpeechLane:
    """Continuous batching of the AR codec decode over groups of sessions that arrive over time (the sentences of
    a response, each started at its boundary as bin/inference.py:160-183 does; a server's new speakers).

    One captured decode step advances every live row of every group, so two sentences whose speech overlaps
    stream the decoder's weights once per step instead of once per sentence (the step is latency-bound: 8 or 16
    rows cost about the same).  A group's prefill (pre_nn, prefix KV, bidirectional prefill: TTSEngine.start)
    runs on its own stream beside the lane's decode steps; once it is done the group joins between two steps
    without a host round trip: the rows already decoding carry their next-step ids and input rows over from
    the old graph's buffers to the larger one's on the device, in stream order, and the new rows start from
    SOS.  While a group is joining the lane launches only a few steps ahead, so the join is not queued behind a
    long launch window.  Rows leave when they finish (the lane drains what it launched for them, then
    continues with a graph for the survivors).  Each row keeps the RNG stream it has in speak() (key = its
    index in its group, step = its own token count; the rows' steps differ inside a launch), so a row's ids --
    and its PCM -- are those of its group decoded alone (tests/test_engines_gpu.py::test_speech_lane_*).

    EOS masking (min_tokens) must cover a row's whole life (min_tokens == max_tokens, the benchmark policy) or none
    of it (min_tokens == 0), and all groups of a lane agree: one launch draws every row from one bound."""

    JOIN_WINDOW = int(os.environ.get("FO_LANE_JOIN_WINDOW", "4"))   # steps launched ahead while a group joins

    def __init__(self, engine, top_k=1, codec_chunk_size=40, codec_padding_size=10, N=2401, seg_threshold=0.01,
                 seed=0, window=32, stream=None, voc_stream=None, prefill_stream=None):
        self.engine, self.top_k, self.seed, self.window = engine, top_k, seed, window
        self.chunk, self.pad, self.N, self.thr = codec_chunk_size, codec_padding_size, N, seg_threshold
        self.es = stream if stream is not None else ops.engine_stream(engine.device)
        self.vs = voc_stream if voc_stream is not None else ops.engine_stream(engine.device, side=True)
        self.ps = prefill_stream if prefill_stream is not None else self.es
        self.states = []            # every row ever added; index = lane row id
        self.groups = {}            # tag -> [row ids]
        self.live = []              # rows decoding, in the current graph's batch order
        self.joining = []           # (row ids, prefill-done event) of groups not decoding yet
        self.pending = collections.deque()   # (batch rows, their steps, graph, event) launched, not yet read
        self.slot = 0               # launches so far (host-buffer / event ring slot)
        self.g = None               # decode graph of the current batch (None: rebuild before the next launch)
        self.forced = None
        self.res = torch.empty(2, dtype=F32, device=engine.device)
        self.done_groups = []       # tags whose rows are all finished and vocoded (drained by the caller)

    @property
    def idle(self):
        return not self.live and not self.pending and not self.joining

    def add(self, items, max_tokens, min_tokens=0, tag=None):
        """Prefill a group of sessions (items as speak()) on the prefill stream; the group joins the decode once
        that is done.  Returns the group's SpeakState objects (row order = items order)."""
        if min_tokens not in (0, max_tokens):
            raise ValueError("SpeechLane: EOS masking covers a row's whole life (min_tokens 0 or max_tokens)")
        forced = bool(min_tokens)
        if self.forced is not None and forced != self.forced and not self.idle:
            raise ValueError("SpeechLane: every live group must mask EOS the same way")
        self.forced = forced
        with torch.cuda.stream(self.ps):
            seqs = self.engine.tts.start(items)
            ev = torch.cuda.Event()
            ev.record()
        rows = []
        for j, sq in enumerate(seqs):
            st = SpeakState(sq, self.top_k, max_tokens, min_tokens)
            st.key, st.tag, st.launched = j, tag, 0
            rows.append(len(self.states))
            self.states.append(st)
        self.groups[tag] = rows
        self.joining.append((rows, ev))
        return [self.states[i] for i in rows]

    def pump(self):
        """Join the groups whose prefill is done, launch ahead while the window has room, then read the oldest
        launched step back.  Returns the PCM segments that became available: [(row id, pcm device 1-D)]."""
        segs = []
        with torch.cuda.stream(self.es):
            if self.joining:
                ready = [j for j in self.joining if j[1].query()]
                if not ready and not self.live and not self.pending:
                    ready = self.joining[:1]   # nothing else to do: wait for the first group's prefill on the device
                if ready:
                    # segments a join drains are returned by this pump, before _close_groups() below can report
                    # their group done (they were held for the next pump)
                    segs += self._join(ready)
            window = self.JOIN_WINDOW if self.joining else self.window
            while self.live and len(self.pending) < window:
                if any(self.states[i].launched >= self.states[i].max_tokens for i in self.live):
                    segs += self._shrink()   # launched-out rows leave; the rest go on without a host round trip
                    if not self.live:
                        break
                if self.g is None:
                    segs += self._rebuild()
                    if not self.live:
                        break
                self._launch()
            if self.pending:
                finished = self._read(self.pending.popleft(), segs)
                if any(i in self.live for i in finished):   # an EOS inside the batch: drain, rebuild from the host
                    segs += self._drain()
                    self.g = None
            elif self.live and self.g is not None:   # nothing launchable: the launched-out rows are done
                rest = [i for i in self.live if not self.states[i].done]
                for i in rest:
                    self.states[i].done = True
                segs += self._finish(rest)
                self.g = None
        self._close_groups()
        return segs

    def free(self):
        for s in self.states:
            if s.seq is not None:
                self.engine.tts.free([s.seq])
                s.seq = None

    # ---- internals
    def _busy(self, B):
        """A cached graph of batch size B still has launched steps unread (reusing it would overwrite their id
        history, regrowing it would destroy it)."""
        return any(e[2].B == B for e in self.pending)

    def _graph(self, rows):
        """The decode graph for batch `rows` (graphs are cached by batch size; callers make sure it is not busy)."""
        if self._busy(len(rows)):
            raise RuntimeError("SpeechLane: decode graph reused with steps still in flight")
        tts, st = self.engine.tts, self.states
        max_keys = max(st[i].seq.kv.length + st[i].max_tokens - st[i].launched for i in rows) + 1
        hist = max(st[i].max_tokens for i in rows) + 1
        V = tts.vocab if self.forced else tts.vocab + 4
        return tts.decode_graph(len(rows), V, self.top_k, self.seed, max_keys, hist, None, True)

    def _join(self, ready):
        """The ready groups join the batch between two steps (on the lane stream, after their prefill).  Returns the
        segments of the steps it had to drain."""
        tts = self.engine.tts
        new = []
        for rows, ev in ready:
            torch.cuda.current_stream().wait_event(ev)
            new += rows
        self.joining = [j for j in self.joining if all(j is not r for r in ready)]
        if self.g is None or not self.live or self._busy(len(self.live) + len(new)):
            # no device state to carry over (or the larger graph still has steps in flight): read everything
            # launched, then the next launch rebuilds from the host ids
            segs = self._drain()
            self.live += new
            self.g = None
            return segs
        old, B0 = self.g, len(self.live)
        rows = self.live + new
        g = self._graph(rows)
        # the old rows' next-step ids and input rows, written by the last launched step's sampler
        g.ids[:B0].copy_(old.ids[:B0])
        g.x[:B0].copy_(old.x[:B0])
        g.ws["h"][:B0].copy_(old.ws["h"][:B0])
        # the new rows start from SOS (DecodeGraph.prime's gather + norm on their rows only)
        g.ids[B0:].fill_(tts.sos)
        ops.gather_rows(tts.embedding, g.ids[B0:], out=g.x[B0:], M=len(new))
        ops.rmsnorm(g.x[B0:], tts.main.layers[0].ln1, tts.eps, out=g.ws["h"][B0:], M=len(new))
        g._uploaded = None
        self.g, self.live = g, rows
        return []

    def _launch(self):
        g, rows = self.g, self.live
        steps = [self.states[i].launched for i in rows]
        ev = g.launch([self.states[i].seq for i in rows], [self.states[i].key for i in rows], steps, self.slot)
        for i in rows:
            self.states[i].launched += 1
        self.pending.append((list(rows), steps, g, ev))
        self.slot += 1

    def _read(self, entry, segs):
        rows, steps, g, ev = entry
        _lib.call("fo_event_sync", ev)
        g.check()
        h = g.hist.np
        finished, due = [], []
        eos = self.engine.tts.eos
        for j, i in enumerate(rows):
            if not self.states[i].done:
                _after_token(self.states, i, int(h[steps[j], j]), eos, due, finished, self.chunk, self.pad)
        segs += _emit(self.engine, self.states, due, finished, self.engine.codec.upsample, self.pad, self.N,
                      self.thr, self.res, self.vs)
        return finished

    def _drain(self):
        """Read everything launched; rows that finished leave the batch."""
        segs = []
        while self.pending:
            self._read(self.pending.popleft(), segs)
        self.live = [i for i in self.live if not self.states[i].done]
        return segs

    def _shrink(self):
        """Rows that have launched their max_tokens leave the batch (their last steps are still being read); the
        others continue in a graph for the smaller batch with their next-step ids and input rows carried over on
        the device, as a join does."""
        st, old = self.states, self.g
        keep = [j for j, i in enumerate(self.live) if st[i].launched < st[i].max_tokens]
        rows = [self.live[j] for j in keep]
        if not rows:
            # every row launched out: the next pumps read their last steps one at a time, so a group that arrives
            # meanwhile is taken in (its prefill starts) at once -- its join drains what is left (r03zi: draining
            # here held the lane thread ~12.5 ms, a window of steps, while the next sentence waited in the queue;
            # r03zj)
            self.live, self.g = [], None
            return []
        if old is None or self._busy(len(rows)):
            # nothing to carry over, or the smaller graph still has steps in flight: drain (the launched-out rows
            # finish there) and rebuild from the host ids at the next launch
            self.live = rows
            segs = self._drain()
            self.g = None
            return segs
        self.live = rows
        g = self._graph(rows)
        if g is old:   # (unreachable: a smaller batch is another cache entry)
            raise RuntimeError("SpeechLane: shrink reused the running graph")
        idx = torch.tensor(keep, dtype=torch.long, device=self.engine.device)
        n = len(rows)
        g.ids[:n].copy_(old.ids.index_select(0, idx))
        g.x[:n].copy_(old.x.index_select(0, idx))
        g.ws["h"][:n].copy_(old.ws["h"][:old.B].index_select(0, idx))
        g._uploaded = None
        self.g = g
        return []

    def _finish(self, rows):
        segs = _emit(self.engine, self.states, [], [i for i in rows if self.states[i].tokens],
                     self.engine.codec.upsample, self.pad, self.N, self.thr, self.res, self.vs)
        self.live = [i for i in self.live if not self.states[i].done]
        return segs

    def _rebuild(self):
        """A graph for the live rows from the host-side ids (after a drain: the batch shrank, or rows joined an
        empty lane)."""
        segs = self._drain()
        if not self.live:
            return segs
        tts, st, rows = self.engine.tts, self.states, self.live
        g = self._graph(rows)
        g.ids.copy_(torch.tensor([st[i].all_ids[-1] if st[i].all_ids else tts.sos for i in rows], dtype=I32)
                    .to(self.engine.device))
        g.prime()
        self.g = g
        return segs

    def _close_groups(self):
        for tag, rows in list(self.groups.items()):
            if all(self.states[i].done for i in rows):
                self.engine.tts.free([self.states[i].seq for i in rows])
                for i in rows:
                    self.states[i].seq = None
                del self.groups[tag]
                self.done_groups.append(tag)
