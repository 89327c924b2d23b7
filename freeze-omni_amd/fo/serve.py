"""Serving threads: the reference's threading model made safe and batched (SURVEY §8(b) Threading).

The reference serves every session from threads of its own that call ONE pipeline object with no lock
(bin/dialog_state_pred.py:777-844, the shared call at :802-804; "Model as a Server", README.md:42) and one
llm2TTS object per speaking session (bin/pool.py:17-50).  On this engine that pattern would interleave two
callers' launch sequences on one stream: one caller's split-K reduce could sum the other's slabs, and both would
share the captured graphs' static buffers and the prefix-KV cache -- a silent wrong result.

Here each replica (one GPU) has
  * ReplicaScheduler: ONE thread that owns the device's listen / text work.  speech_dialogue, generate_step,
    set_system_role and _post_decode become requests it runs; concurrent speech_dialogue calls of different
    sessions are coalesced into one recognize_batch (one encoder / adapter / Qwen2 launch sequence) per round, and
    concurrent one-token generate_step calls into one text step.  Each caller blocks on its request, so the
    calls stay synchronous, with the reference's arguments, results and exceptions.
  * SpeechScheduler: ONE thread that owns the device's speech generation.  llm2TTS.run callers submit their
    sentence and read segments from a queue; every concurrent sentence decodes in one continuously batched AR
    decode (fo.speak.SpeechLane: a row's ids and PCM are those of its sentence decoded alone).

Both threads run their device work on a private family of non-blocking streams (fo.ops.serve_streams), so a
caller's own legacy-stream work never syncs with (or invalidates a graph capture on) the serving streams; inputs
a caller produced on the device are ordered by an event recorded on the caller's stream, and every result is
complete on the device before the call returns (or, for PCM, before the segment is yielded).

Ordering: requests of one session (the same KV sequence) run in submission order; requests of different sessions
may be coalesced.  A request that is not coalescable (a "call") runs alone, after everything submitted before it.
"""
import collections
import os
import queue
import threading
from concurrent.futures import Future

import torch

from . import ops

# FO_SERVE_WINDOW_US: how long the replica thread waits, once a request is queued, for more to coalesce with it
# (0: it takes what is queued when it gets round to it -- under load the requests that arrived while the previous
# batch ran)
WINDOW_US = float(os.environ.get("FO_SERVE_WINDOW_US", "0"))


def _dev_key(device):
    """torch.device of one GPU (the current one when no index is given); 'cpu' only for the host-logic tests."""
    d = torch.device(device)
    if d.type == "cpu":
        return d
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())


def _on_device(dev):
    """(stream context of the serving thread's main stream, that stream or None) for dev."""
    import contextlib
    if dev.type == "cpu":
        return contextlib.nullcontext(), None
    torch.cuda.set_device(dev)
    ops.serve_streams(dev.index)
    main = ops.engine_stream(dev)
    return torch.cuda.stream(main), main


def _caller_event(tensors):
    """An event on the caller's current stream if any input lives on the device (the serving stream waits on it)."""
    if any(torch.is_tensor(t) and t.is_cuda for t in tensors):
        ev = torch.cuda.Event()
        ev.record()
        return ev
    return None


class _Request:
    __slots__ = ("kind", "key", "payload", "seqs", "fut", "ev", "tag")

    def __init__(self, kind, key, payload, seqs, ev=None, tag=None):
        self.kind, self.key, self.payload, self.seqs, self.ev, self.tag = kind, key, payload, seqs, ev, tag
        self.fut = Future()


class ReplicaScheduler:
    """The one thread that issues a replica's listen / text work (module docstring)."""

    _inst = {}
    _inst_lock = threading.Lock()

    @classmethod
    def for_device(cls, device):
        dev = _dev_key(device)
        with cls._inst_lock:
            s = cls._inst.get(dev)
            if s is None or not s.thread.is_alive():
                s = cls._inst[dev] = cls(dev)
            return s

    def __init__(self, device, window_us=None):
        self.device = _dev_key(device)
        self.window = (WINDOW_US if window_us is None else window_us) * 1e-6
        self.cv = threading.Condition()
        self.q = collections.deque()
        self.stats = collections.Counter()
        self.batch_log = None   # set to a list: the tags of every coalesced group run, in order (tests)
        self.thread = threading.Thread(target=self._loop, name=f"fo-replica-{self.device}", daemon=True)
        self.thread.start()

    def on_thread(self):
        return threading.current_thread() is self.thread

    # ---------------------------------------------------------------- caller side
    def _submit(self, r):
        with self.cv:
            self.q.append(r)
            self.cv.notify()
        return r.fut.result()

    def call(self, fn, *args, **kw):
        """Run fn(*args, **kw) on the replica thread, after everything queued before it; returns its result."""
        if self.on_thread():
            return fn(*args, **kw)
        return self._submit(_Request("call", None, (fn, args, kw), None,
                                     _caller_event(list(args) + list(kw.values()))))

    def listen(self, model, requests, tag=None):
        """AudioLLM.recognize_batch(requests) run on the replica thread, coalesced with other sessions' concurrent
        listen requests of the same model and feature rows.  requests: [(speech, extra_inputs)], already checked."""
        if self.on_thread():
            return model._recognize_now(requests)
        rows = tuple(sorted({int(torch.as_tensor(s).shape[-2]) for s, _ in requests}))
        seqs = frozenset(id(ex["past_key_values"].seq) for _, ex in requests)
        if len(seqs) != len(requests):
            raise ValueError("recognize_batch: one KV context given twice in a batch")
        return self._submit(_Request("listen", ("listen", id(model), rows), (model, list(requests)), seqs,
                                     _caller_event([s for s, _ in requests]), tag))

    def text(self, model, past_key_values, input_ids, top_k, top_p, temperature, tag=None):
        """AudioLLM.generate_step on the replica thread; concurrent steps of other sessions with the same sampler
        settings share one text step (one-token steps replay the captured TextGraph for the batch)."""
        if self.on_thread():
            return model._generate_now(past_key_values, input_ids, top_k, top_p, temperature)
        key = ("text", id(model), int(top_k), float(top_p), float(temperature), len(input_ids) == 1)
        return self._submit(_Request("text", key, (model, past_key_values, list(input_ids)),
                                     frozenset([id(past_key_values.seq)]), None, tag))

    # ---------------------------------------------------------------- replica thread
    def _loop(self):
        ctx, main = _on_device(self.device)
        with ctx:
            while True:
                with self.cv:
                    while not self.q:
                        self.cv.wait()
                    if self.window > 0:
                        self.cv.wait(self.window)
                    batch = list(self.q)
                    self.q.clear()
                self._run(batch, main)

    def _run(self, batch, main):
        pending = batch
        while pending:
            head = pending[0]
            if head.kind == "call":
                self._exec([head], main)
                pending = pending[1:]
                continue
            # coalesce: every later request with the same key whose sessions are not in the group and not in a request
            # skipped before it (per-session order); nothing is taken past a call (it is a barrier)
            group, rest, taken, skipped, barrier = [head], [], set(head.seqs), set(), False
            for r in pending[1:]:
                if not barrier and r.kind != "call" and r.key == head.key and not (r.seqs & taken) \
                        and not (r.seqs & skipped):
                    group.append(r)
                    taken |= r.seqs
                else:
                    barrier = barrier or r.kind == "call"
                    if r.seqs:
                        skipped |= r.seqs
                    rest.append(r)
            self._exec(group, main)
            pending = rest

    def _exec(self, group, main):
        for r in group:
            if r.ev is not None and main is not None:
                main.wait_event(r.ev)
        kind = group[0].kind
        try:
            if kind == "call":
                fn, args, kw = group[0].payload
                out = [fn(*args, **kw)]
            elif kind == "listen":
                model = group[0].payload[0]
                flat = [rq for r in group for rq in r.payload[1]]
                res = model._recognize_now(flat)
                out, k = [], 0
                for r in group:
                    n = len(r.payload[1])
                    out.append(res[k:k + n])
                    k += n
                self.stats["listen_requests"] += len(group)
                self.stats["listen_batches"] += 1
            else:   # text
                model = group[0].payload[0]
                _, _, top_k, top_p, temperature, _ = group[0].key
                ids, hid = model.engine.text_step([(r.payload[1].seq, r.payload[2]) for r in group], top_k=top_k,
                                                  top_p=top_p, temperature=temperature)
                out = [(ids[b], hid[b:b + 1].reshape(1, 1, -1)) for b in range(len(group))]
                self.stats["text_requests"] += len(group)
                self.stats["text_batches"] += 1
            if main is not None:
                main.synchronize()   # every result complete on the device before its caller goes on
        except BaseException as e:   # noqa: BLE001 (handed to every caller of the group)
            for r in group:
                r.fut.set_exception(e)
            return
        if self.batch_log is not None and kind != "call":
            self.batch_log.append([r.tag for r in group])
        for r, o in zip(group, out):
            r.fut.set_result(o)


class _SpeechJob:
    def __init__(self, engine, hidden, prefix, ev, params):
        self.engine, self.hidden, self.prefix, self.ev, self.params = engine, hidden, prefix, ev, params
        self.out = queue.Queue()
        self.cancelled = False

    def segments(self):
        """The job's PCM segments as they become available (each complete on the device when yielded)."""
        try:
            while True:
                item = self.out.get()
                if item is None:
                    return
                if isinstance(item, BaseException):
                    raise item
                seg, ev = item
                ev.synchronize()
                yield seg
        finally:
            self.cancelled = True


class SpeechScheduler:
    """The one thread that runs a device's speech generation (module docstring).  One SpeechLane per (engine,
    sampler / chunking parameters); sentences with the repetition penalty on (which the lane does not batch) run
    through speak() on the same thread, one at a time."""

    _inst = {}
    _inst_lock = threading.Lock()

    @classmethod
    def for_device(cls, device):
        dev = _dev_key(device)
        with cls._inst_lock:
            s = cls._inst.get(dev)
            if s is None or not s.thread.is_alive():
                s = cls._inst[dev] = cls(dev)
            return s

    def __init__(self, device):
        self.device = _dev_key(device)
        self.cv = threading.Condition()
        self.new = collections.deque()
        self.lanes = {}     # key -> SpeechLane
        self.jobs = {}      # (lane key, tag) -> job
        self.n = 0
        self.stats = collections.Counter()
        self.thread = threading.Thread(target=self._loop, name=f"fo-speech-{self.device}", daemon=True)
        self.thread.start()

    def submit(self, engine, hidden, prefix, top_k, codec_chunk_size, codec_padding_size, N, seg_threshold,
               max_tokens=1000, penalty_window_size=-1, penalty=1.1):
        """Queue one sentence (hidden [T1, D], prefix [T2, D] or None, device fp32); returns its job, whose
        segments() yields the PCM segments llm2TTS.run yields."""
        params = (int(top_k), int(codec_chunk_size), int(codec_padding_size), int(N), float(seg_threshold),
                  int(max_tokens), int(penalty_window_size), float(penalty))
        job = _SpeechJob(engine, hidden, prefix, _caller_event([hidden, prefix]), params)
        with self.cv:
            self.new.append(job)
            self.cv.notify()
        return job

    def _loop(self):
        torch.cuda.set_device(self.device)
        ops.serve_streams(self.device.index)
        self.ts = ops.engine_stream(self.device, name="tts")
        self.vs = ops.engine_stream(self.device, name="voc")
        while True:
            with self.cv:
                while not self.new and all(l.idle for l in self.lanes.values()):
                    self.cv.wait()
                new = list(self.new)
                self.new.clear()
            for job in new:
                self._admit(job)
            for key, lane in list(self.lanes.items()):
                if lane.idle:
                    continue
                try:
                    segs = lane.pump()
                except BaseException as e:   # noqa: BLE001 (every sentence of the lane fails with it)
                    self._fail_lane(key, e)
                    continue
                self._deliver(key, lane, segs)

    def _admit(self, job):
        from .speak import SpeechLane, speak
        top_k, chunk, pad, N, thr, max_tokens, pen_w, pen = job.params
        if job.ev is not None:
            self.ts.wait_event(job.ev)
        if pen_w > 0:   # the lane does not batch the penalty: this sentence runs alone, to its end
            try:
                with torch.cuda.stream(self.ts):
                    for _, seg in speak(job.engine, [(job.hidden, job.prefix)], top_k=top_k, codec_chunk_size=chunk,
                                        codec_padding_size=pad, N=N, seg_threshold=thr, max_tokens=max_tokens,
                                        penalty_window_size=pen_w, penalty=pen, stream=self.ts, voc_stream=self.vs):
                        self._put(job, seg)
                job.out.put(None)
            except BaseException as e:   # noqa: BLE001
                job.out.put(e)
            self.stats["sentences_alone"] += 1
            return
        key = (id(job.engine), top_k, chunk, pad, N, thr)
        lane = self.lanes.get(key)
        if lane is None:
            lane = self.lanes[key] = SpeechLane(job.engine, top_k=top_k, codec_chunk_size=chunk,
                                                codec_padding_size=pad, N=N, seg_threshold=thr, stream=self.ts,
                                                voc_stream=self.vs, prefill_stream=self.ts)
        self.n += 1
        try:
            lane.add([(job.hidden, job.prefix)], max_tokens, 0, tag=self.n)
        except BaseException as e:   # noqa: BLE001
            job.out.put(e)
            return
        self.jobs[(key, self.n)] = job
        self.stats["sentences_lane"] += 1

    def _put(self, job, seg):
        if job.cancelled:
            return
        ev = torch.cuda.Event()
        ev.record(self.vs)   # the vocoder stream produced it (speak / SpeechLane: fo.speak._vocode)
        job.out.put((seg.view(1, 1, -1), ev))

    def _deliver(self, key, lane, segs):
        for i, seg in segs:
            job = self.jobs.get((key, lane.states[i].tag))
            if job is not None:
                self._put(job, seg)
        for tag in lane.done_groups:
            job = self.jobs.pop((key, tag), None)
            if job is not None:
                job.out.put(None)
        lane.done_groups.clear()

    def _fail_lane(self, key, e):
        lane = self.lanes.pop(key)
        for (k, tag) in [jk for jk in self.jobs if jk[0] == key]:
            self.jobs.pop((k, tag)).out.put(e)
        try:
            lane.free()
        except Exception:   # noqa: BLE001
            pass
