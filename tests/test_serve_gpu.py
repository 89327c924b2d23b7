"""The reference's serving pattern on the device: many session threads calling ONE pipeline object
(bin/dialog_state_pred.py:777-844, the shared call at :802-804; README.md:42 "Model as a Server") and one llm2TTS per
speaking session called from its own thread (bin/pool.py:17-50).  fo.serve runs every call on the replica's
serving thread and coalesces concurrent sessions into one launch sequence (SURVEY §8(b) Threading).

Bit-exactness is checked against the serial execution of the same coalesced groups (the scheduler's batch log
replayed from one thread): the threaded run must not be perturbed by the interleaving at all.  Against each
session run on its own (batch of one) the GEMMs take other tilings (the row count picks the kernel), so the state
probabilities agree to 1e-4 -- the bound tests/test_duplex_gpu.py uses for the batched duplex tick -- and every
integer (pe_index, KV length, the decision away from 0.5) exactly."""
import copy
import os
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "configs", "tiny")
G = os.path.join(os.path.dirname(__file__), "golden")
N_THREADS, N_CHUNKS, N_TEXT = 8, 20, 4


@pytest.fixture(scope="module")
def pipe(dev):
    from models.pipeline import inferencePipeline
    return inferencePipeline({"model_path": TINY, "llm_path": os.path.join(TINY, "llm"), "device": "cuda:0",
                              "top_k": 1})


def _script(t):
    """Thread t's chunks: framing A rows (16 + 3 carried) on even threads, framing B (28 + 4) on odd ones; threads
    2, 3, 6, 7 alternate the user and system identities; a new IPU ('ipu_sl') starts again mid-stream at chunk 10."""
    R = 19 if t % 2 == 0 else 32
    rng = np.random.default_rng(1000 + t)
    out = []
    for k in range(N_CHUNKS):
        ident = "user" if (t % 4 < 2 or k % 3 != 2) else "system"
        status = "ipu_sl" if k in (0, 10) else ("ipu_el" if k in (9, 19) else "ipu_cl")
        feats = torch.from_numpy((rng.standard_normal((1, R, 80)) * 2.0).astype(np.float32))
        out.append((feats, ident, status))
    return out


def _kv_content(pipe, pkv):
    pool = pipe.model.engine.llm.pool
    seq = pkv.seq
    idx = torch.tensor(seq.pages, dtype=torch.long, device=pool.k.device)
    k = pool.k.index_select(1, idx)   # [L, n, KVH, PS, hd]
    v = pool.v.index_select(1, idx)
    L, n, H, PS, hd = k.shape
    k = k.permute(0, 2, 1, 3, 4).reshape(L, H, n * PS, hd)[:, :, :seq.length]
    v = v.permute(0, 2, 1, 3, 4).reshape(L, H, n * PS, hd)[:, :, :seq.length]
    return k.cpu(), v.cpu()


class _Session:
    def __init__(self, pipe, base, t):
        self.t = t
        self.pkv = copy.deepcopy(base)
        self.caches = {i: {"adapter_cache": None, "encoder_cache": None, "pe_index": 0} for i in ("user", "system")}
        self.out = []
        self.last_id = None

    def request(self, feats, ident, status):
        return dict(audio=feats, identity=ident, status=status, past_key_values=self.pkv, **self.caches[ident])

    def apply(self, ident, res):
        probs, pkv, ac, ec, pe = res
        self.pkv = pkv
        self.caches[ident] = {"adapter_cache": ac, "encoder_cache": ec, "pe_index": pe}
        self.out.append((ident, probs, pe, pkv.get_seq_length(), ec.start, ec.len))

    def text_ids(self, pipe, j):
        return pipe.model.prefix_ids("system") if j == 0 else [self.last_id]

    def apply_text(self, tok, hid):
        self.last_id = tok
        self.out.append(("text", tok, hid.detach().cpu().numpy().copy()))


def _threaded(pipe, base, sch):
    sess = [_Session(pipe, base, t) for t in range(N_THREADS)]
    errs = []
    barrier = threading.Barrier(N_THREADS)

    def worker(s):
        try:
            barrier.wait()
            for k, (feats, ident, status) in enumerate(_script(s.t)):
                r = s.request(feats, ident, status)
                # the fork form through the shared pipeline, tagged so the scheduler's batch log names it
                res = pipe.model._scheduler().listen(pipe.model, [(r.pop("audio"), r)], tag=("listen", s.t, k))[0]
                s.apply(ident, res)
            for j in range(N_TEXT):
                tok, hid = pipe.model._scheduler().text(pipe.model, s.pkv, s.text_ids(pipe, j), 1, 0.0, 1.0,
                                                        tag=("text", s.t, j))
                s.apply_text(tok, hid)
        except BaseException as e:   # noqa: BLE001 (re-raised by the test)
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(s,)) for s in sess]
    for th in ts:
        th.start()
    for th in ts:
        th.join(300)
    assert not errs, errs
    return sess


def _replay(pipe, base, log):
    """The logged groups, serially from this thread: each group as ONE request of its members."""
    sess = [_Session(pipe, base, t) for t in range(N_THREADS)]
    scripts = [_script(t) for t in range(N_THREADS)]
    eng = pipe.model.engine
    for group in log:
        kind = group[0][0]
        if kind == "listen":
            reqs, who = [], []
            for _, t, k in group:
                feats, ident, status = scripts[t][k]
                reqs.append(sess[t].request(feats, ident, status))
                who.append((t, ident))
            for (t, ident), res in zip(who, pipe.speech_dialogue_batch(reqs)):
                sess[t].apply(ident, res)
        else:
            items = [(sess[t].pkv.seq, sess[t].text_ids(pipe, j)) for _, t, j in group]
            ids, hid = pipe.model._run(eng.text_step, items, top_k=1, top_p=0.0, temperature=1.0)
            for b, (_, t, _) in enumerate(group):
                sess[t].apply_text(ids[b], hid[b:b + 1].reshape(1, 1, -1))
    return sess


def test_concurrent_speech_dialogue_threads_equal_their_serial_runs(pipe):
    from fo.serve import ReplicaScheduler
    sch = ReplicaScheduler.for_device(pipe.device)
    assert pipe.model._scheduler() is sch
    base = pipe.speech_dialogue(None, identity="", status="pre", role="You are a helpful assistant.")[1]
    eng = pipe.model.engine
    sch.batch_log = []
    n0 = dict(sch.stats)
    thr = _threaded(pipe, base, sch)
    log, sch.batch_log = sch.batch_log, None
    calls = N_THREADS * N_CHUNKS
    n_listen = sch.stats["listen_batches"] - n0.get("listen_batches", 0)
    n_text = sch.stats["text_batches"] - n0.get("text_batches", 0)
    # coalesced: fewer encoder / Qwen2 launch sequences than calls
    assert sch.stats["listen_requests"] - n0.get("listen_requests", 0) == calls
    assert n_listen < calls and max(len(g) for g in log if g[0][0] == "listen") > 1, n_listen
    assert n_text < N_THREADS * N_TEXT
    # every session's calls in its own order
    flat = [tag for g in log for tag in g]
    for t in range(N_THREADS):
        assert [k for kind, tt, k in flat if tt == t and kind == "listen"] == list(range(N_CHUNKS))
    rep = _replay(pipe, base, log)
    for a, b in zip(thr, rep):
        assert len(a.out) == len(b.out) == N_CHUNKS + N_TEXT
        for x, y in zip(a.out, b.out):
            if x[0] == "text":
                assert x[1] == y[1] and np.array_equal(x[2], y[2])
            else:
                assert x == y, (a.t, x, y)   # probs bit for bit, pe_index, KV length, encoder ring start / length
        ka, va = _kv_content(pipe, a.pkv)
        kb, vb = _kv_content(pipe, b.pkv)
        assert torch.equal(ka, kb) and torch.equal(va, vb)
    # each session alone (batch of one) through the same pipeline: same integers, probs within 1e-4
    for t in range(N_THREADS):
        s = _Session(pipe, base, t)
        for feats, ident, status in _script(t):
            s.apply(ident, pipe.speech_dialogue(**s.request(feats, ident, status)))
        for x, y in zip(s.out, thr[t].out):
            assert x[0] == y[0] and x[2:] == y[2:]
            if x[1] is None:
                assert y[1] is None
            else:
                for key in ("state_1", "state_2"):
                    assert abs(x[1][key] - y[1][key]) < 1e-4
    assert sum(1 for s in thr for x in s.out if x[0] == "system") > 0
    assert n_listen == len([g for g in log if g[0][0] == "listen"]) and n_text == len(log) - n_listen
    del eng


def test_upstream_form_and_protocol_errors_from_threads(pipe):
    """bin/inference.py's upstream form from two threads at once, and the reference's exceptions raised in the
    calling thread (not lost on the serving thread)."""
    g = np.load(os.path.join(G, "audiollm_tiny.npz"))
    feats = torch.from_numpy(g["feats"][0]).unsqueeze(0)
    res, errs = {}, []

    def run(t):
        try:
            out = pipe.speech_dialogue(None, stat="pre", role="hi")
            for k in range(3):
                out = pipe.speech_dialogue(feats, **dict(out, stat="dialog_sl" if k == 0 else "dialog_cl"))
            out = pipe.speech_dialogue(None, **dict(out, stat="dialog_ss"))
            res[t] = (out["last_id"], out["pe_index"], out["past_key_values"].get_seq_length())
        except BaseException as e:   # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=run, args=(t,)) for t in range(2)]
    for th in ts:
        th.start()
    for th in ts:
        th.join(120)
    assert not errs, errs
    assert res[0] == res[1]
    pkv = pipe.speech_dialogue(None, identity="", status="pre", role="hi")[1]
    errs = []

    def bad(kind):
        try:
            if kind == "identity":
                pipe.speech_dialogue(feats, identity="robot", status="ipu_cl", past_key_values=pkv)
            else:
                pipe.speech_dialogue(feats, identity="user", status="ipu_cl", past_key_values=None)
        except (ValueError, AssertionError) as e:
            errs.append(type(e).__name__)

    ts = [threading.Thread(target=bad, args=(k,)) for k in ("identity", "role")]
    for th in ts:
        th.start()
    for th in ts:
        th.join(60)
    assert sorted(errs) == ["AssertionError", "ValueError"]


def test_llm2tts_run_from_threads_matches_alone(dev):
    """Four llm2TTS objects' run() from four threads at once (the reference's one TTS object per speaking
    session): each yields exactly the PCM segments of its sentence decoded alone on the caller's thread."""
    from models.decoder.llm2tts import llm2TTS
    t = np.load(os.path.join(G, "tts_tiny.npz"))
    objs = [llm2TTS(TINY)]
    objs += [llm2TTS(TINY, weights_from=objs[0]) for _ in range(3)]
    rng = np.random.default_rng(3)
    jobs = []
    for j in range(4):
        h = t["hidden"] + (0.0 if j == 0 else 0.05 * rng.standard_normal(t["hidden"].shape).astype(np.float32))
        n = t["hidden"].shape[0] - 2 * j
        jobs.append((torch.from_numpy(h[:n]).unsqueeze(0), torch.from_numpy(t["prefix"]).unsqueeze(0)))

    def alone(o, h, p):
        o.SERVE = False
        try:
            return [s.cpu().numpy() for s in o.run(h.to(dev), 1, p.to(dev))]
        finally:
            del o.SERVE

    ref = [alone(objs[j], *jobs[j]) for j in range(4)]
    got, errs = [None] * 4, []

    def worker(j):
        try:
            got[j] = [s.cpu().numpy() for s in objs[j].run(jobs[j][0].to(dev), 1, jobs[j][1].to(dev))]
        except BaseException as e:   # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(j,)) for j in range(4)]
    for th in ts:
        th.start()
    for th in ts:
        th.join(300)
    assert not errs, errs
    for a, b in zip(got, ref):
        assert len(a) == len(b) and len(a) > 0
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    from fo.serve import SpeechScheduler
    assert SpeechScheduler.for_device(dev).stats["sentences_lane"] >= 4
