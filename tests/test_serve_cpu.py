"""Host logic of the serving layer on CPU (no GPU): the replica scheduler's coalescing and per-session ordering
(fo.serve.ReplicaScheduler, SURVEY §8(b) Threading), the pools' counters under threads (bin/pool.py:79-87, whose
reference form is unlocked), and a session surviving the loss of its replica (README.md:42)."""
import threading
import time

import numpy as np
import pytest
import torch


class _Seq:
    def __init__(self, sid):
        self.sid = sid
        self.n = 0


class _PKV:
    def __init__(self, sid):
        self.seq = _Seq(sid)


class _FakeModel:
    """recognize: each session's chunk k returns a value that depends on (session, k, the features) only, and the
    call checks that a session's chunks arrive in order; the batch sizes are recorded."""

    def __init__(self, delay=0.002, fail_on=None):
        self.batches = []
        self.delay = delay
        self.fail_on = fail_on
        self.engine = self
        self.lock = threading.Lock()

    def _recognize_now(self, requests):
        assert self.lock.acquire(blocking=False), "two groups at once"   # the scheduler runs one group at a time
        self.lock.release()
        self.batches.append(len(requests))
        time.sleep(self.delay)
        out = []
        for speech, ex in requests:
            seq = ex["past_key_values"].seq
            k = ex["k"]
            assert seq.n == k, (seq.sid, seq.n, k)   # per-session order
            if self.fail_on is not None and (seq.sid, k) == self.fail_on:
                raise RuntimeError("device fault")
            seq.n += 1
            out.append((float(np.asarray(speech).sum()) + 1000 * seq.sid + k, ex["past_key_values"], None, None, k + 1))
        return out

    def text_step(self, items, top_k=1, top_p=0.0, temperature=1.0):
        self.batches.append(("text", len(items)))
        time.sleep(self.delay)
        ids = [kv.sid * 100 + len(t) for kv, t in items]
        return ids, torch.zeros(len(items), 4)


def test_scheduler_coalesces_concurrent_sessions_and_keeps_their_order():
    from fo.serve import ReplicaScheduler
    sch = ReplicaScheduler("cpu")
    sch.batch_log = []
    model = _FakeModel()
    n_threads, n_chunks = 8, 20
    got, errs = {}, []

    def worker(t):
        try:
            pkv = _PKV(t)
            rng = np.random.default_rng(t)
            res = []
            for k in range(n_chunks):
                feats = torch.from_numpy(rng.standard_normal((1, 16, 4)).astype(np.float32))
                (r,) = sch.listen(model, [(feats, {"past_key_values": pkv, "k": k})], tag=(t, k))
                res.append((r[0], r[4], float(np.asarray(feats).sum())))
            got[t] = res
        except BaseException as e:   # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errs, errs
    for t in range(n_threads):
        for k, (val, pe, s) in enumerate(got[t]):
            assert pe == k + 1 and val == pytest.approx(s + 1000 * t + k)
    calls = n_threads * n_chunks
    assert sum(model.batches) == calls
    assert len(model.batches) < calls and max(model.batches) > 1      # concurrent calls were coalesced
    assert sch.stats["listen_requests"] == calls and sch.stats["listen_batches"] == len(model.batches)
    # the batch log names every request once, and each session's chunks appear in order
    flat = [tag for g in sch.batch_log for tag in g]
    assert sorted(flat) == sorted((t, k) for t in range(n_threads) for k in range(n_chunks))
    for t in range(n_threads):
        assert [k for (tt, k) in flat if tt == t] == list(range(n_chunks))
    assert all(len({tt for tt, _ in g}) == len(g) for g in sch.batch_log)   # one chunk per session per group


def test_scheduler_same_session_requests_stay_ordered_and_errors_reach_their_callers():
    from fo.serve import ReplicaScheduler
    sch = ReplicaScheduler(torch.device("cpu"), window_us=3000)   # a window so both requests are queued together
    model = _FakeModel(delay=0.0, fail_on=(7, 1))
    pkv = _PKV(7)
    out, errs = [None, None], []

    def call(k):
        try:
            out[k] = sch.listen(model, [(torch.ones(1, 2, 2), {"past_key_values": pkv, "k": k})])
        except RuntimeError as e:
            errs.append((k, str(e)))

    t0 = threading.Thread(target=call, args=(0,))
    t0.start()
    time.sleep(0.0005)
    t1 = threading.Thread(target=call, args=(1,))
    t1.start()
    t0.join(10)
    t1.join(10)
    # the session's second chunk was not coalesced with its first (same KV context): two groups, in order
    assert out[0][0][4] == 1
    assert errs == [(1, "device fault")]
    with pytest.raises(ValueError):   # one context twice in one batch
        sch.listen(model, [(torch.ones(1, 2, 2), {"past_key_values": pkv, "k": 1})] * 2)


def test_scheduler_calls_are_barriers_and_text_steps_coalesce():
    from fo.serve import ReplicaScheduler
    sch = ReplicaScheduler(torch.device("cpu"))
    model = _FakeModel(delay=0.003)
    order = []
    res = {}

    def text(t):
        res[t] = sch.text(model, _PKV(t), [5], 1, 0.0, 1.0)

    def call():
        order.append(sch.call(lambda: len(model.batches)))

    ts = [threading.Thread(target=text, args=(t,)) for t in range(6)] + [threading.Thread(target=call)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert sorted(res) == list(range(6))
    assert all(res[t][0] == t * 100 + 1 for t in range(6))
    assert sum(b[1] for b in model.batches if isinstance(b, tuple)) == 6
    assert sch.call(lambda: 42) == 42
    with pytest.raises(ZeroDivisionError):
        sch.call(lambda: 1 / 0)


# ------------------------------------------------------------------ bin/pool.py


class _StubPipeline:
    """speech_dialogue fork form over a host 'context': probs depend on everything the session fed, so a re-pinned
    session that re-prefilled its history gives the same probs as one that never moved."""
    n = 0

    def __init__(self, configs, weights_from=None):
        _StubPipeline.n += 1
        self.id = f"stub{_StubPipeline.n}"
        self.fail = False
        self.calls = 0

    def speech_dialogue(self, audio, identity=None, status=None, role=None, past_key_values=None, adapter_cache=None,
                        encoder_cache=None, pe_index=0):
        self.calls += 1
        if self.fail:
            raise RuntimeError("hipErrorLaunchFailure (stub)")
        if status == "pre":
            return None, [len(role or "")], None, None, None
        if identity not in ("user", "system"):
            raise ValueError(identity)
        ctx = past_key_values + [float(np.asarray(audio).sum())]
        pr = {"state_1": (sum(ctx) % 1.0), "state_2": 0.0} if identity == "user" else None
        return pr, ctx, None, None, (pe_index or 0) + 1


def test_pool_counters_under_threads():
    from bin.pool import TTSObjectPool, pipelineObjectPool
    pool = pipelineObjectPool(4, {"model_path": "x"}, factory=_StubPipeline)
    barrier = threading.Barrier(16)

    def worker():
        barrier.wait()
        for _ in range(2000):
            o = pool.acquire()
            pool.release(o)

    ts = [threading.Thread(target=worker) for _ in range(16)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert [o.user_count for o in pool.pool] == [0, 0, 0, 0]
    held = [pool.acquire() for _ in range(10)]          # least-loaded: 10 sessions over 4 replicas
    assert sorted(o.user_count for o in pool.pool) == [2, 2, 3, 3]
    for o in held:
        pool.release(o)

    class _Obj:
        def __init__(self, model_path, device, weights_from=None):
            self.in_use = False

    tp = TTSObjectPool(8, "x", factory=_Obj)
    owners, errs = {}, []
    barrier = threading.Barrier(8)

    def tts_worker(w):
        barrier.wait()
        for _ in range(500):
            o = tp.acquire()
            if id(o) in owners:
                errs.append("object handed out twice")
            owners[id(o)] = w
            del owners[id(o)]
            tp.release(o)

    ts = [threading.Thread(target=tts_worker, args=(w,)) for w in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errs and all(not o.in_use for o in tp.pool)
    for _ in range(8):
        tp.acquire()
    with pytest.raises(Exception, match="No available objects"):
        tp.acquire()


def test_session_survives_replica_loss():
    from bin.pool import PooledSession, pipelineObjectPool
    pool = pipelineObjectPool(3, {"model_path": "x"}, factory=_StubPipeline)
    rng = np.random.default_rng(5)
    chunks = [(rng.standard_normal((1, 8, 4)).astype(np.float32), "user" if k % 3 else "system",
               "ipu_sl" if k == 0 else "ipu_cl") for k in range(12)]
    ref = PooledSession(pool, role="you are a helper")
    want = [ref.speech_dialogue(a, i, s) for a, i, s in chunks]
    ref.release()
    s = PooledSession(pool, role="you are a helper")
    first = s.obj
    got = []
    for k, (a, i, st) in enumerate(chunks):
        if k == 7:
            first.pipeline_proc.fail = True    # the GPU under this session is lost
        got.append(s.speech_dialogue(a, i, st))
    assert got == want
    assert s.repins == 1 and s.obj is not first and not first.healthy
    assert first.user_count == 0 and s.obj.user_count == 1
    others = [pool.acquire() for _ in range(4)]
    assert all(o is not first for o in others)            # a failed replica admits no new session
    with pytest.raises(ValueError):                       # protocol errors are the caller's, no re-pin
        s.speech_dialogue(chunks[0][0], "robot", "ipu_cl")
    assert s.repins == 1
    for o in pool.pool:
        o.pipeline_proc.fail = True
    with pytest.raises(Exception, match="No healthy"):
        s.speech_dialogue(chunks[0][0], "user", "ipu_cl")
