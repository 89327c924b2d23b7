"""Duplex session host logic (fo.duplex; reference bin/dialog_state_pred.py:330-844) with a stub
pipeline and feature gater: VAD labelling, IPU bookkeeping, user-priority serialisation / barge-in,
decision rule, and batched scheduling == per-session processing.  The device path is
tests/test_duplex_gpu.py."""
import copy

import numpy as np
import pytest

CH = 3584  # framing B chunk (224 ms at 16 kHz)


class _KV:
    def __init__(self, n=5):
        self.n = n
        self.freed = False

    def __deepcopy__(self, memo):
        return _KV(self.n)

    def get_seq_length(self):
        return self.n

    def free(self):
        self.freed = True


class _Pipe:
    """speech_dialogue stub: state_1 = the chunk's mean sample + 0.5 (so loud chunks answer)."""
    device = "cpu"

    def __init__(self):
        self.calls = []

    def speech_dialogue(self, audio, identity=None, status=None, role=None, past_key_values=None,
                        adapter_cache=None, encoder_cache=None, pe_index=0):
        if status == "pre":
            return None, _KV(), None, None, None
        self.calls.append((identity, status))
        past_key_values.n += 2 + (5 if status == "ipu_sl" else 0)
        probs = None
        if identity == "user":
            s1 = float(np.mean(audio)) + 0.5
            probs = {"state_1": s1, "state_2": 0.0}
        return probs, past_key_values, (adapter_cache or 0) + 1, (encoder_cache or 0) + 1, pe_index + 4

    def speech_dialogue_batch(self, reqs):
        return [self.speech_dialogue(**r) for r in reqs]


class _Gate:
    expected_frames_per_audio_chunk = CH

    def reset(self):
        pass

    def process_and_gate(self, ann):
        return {"feature": np.asarray(ann["audio"], np.float32), "status": ann["status"], "feature_last_chunk": []}


def _session(pipe, user_iv, sys_iv):
    from fo.duplex import DuplexSession, ScriptedVAD
    vad = {"user": ScriptedVAD(CH, user_iv), "system": ScriptedVAD(CH, sys_iv)}
    return DuplexSession(pipe, vad=vad, feature_gater={"user": _Gate(), "system": _Gate()})


def _feed(s, seconds, level, seed):
    rng = np.random.default_rng(seed)
    n = int(seconds * 16000 / CH)
    for k in range(n):
        for ident in ("user", "system"):
            x = np.clip(rng.normal(level[ident], 0.01, CH), -0.99, 0.99)
            s.enqueue_audio_data(ident, {"audio": (x * 32767).astype(np.int16).tobytes(), "sr": 16000,
                                         "enc": "s16le", "time_stamp": k * CH / 16000})


def test_scripted_vad_labels_and_preroll():
    from fo.duplex import ScriptedVAD
    v = ScriptedVAD(CH, [(0.5, 1.2)], cache_history_size=2)
    st = []
    for k in range(8):
        r = v.predict({"audio": np.full(CH, k, np.float32), "time_stamp": k})
        st.append(r["status"])
        if r["status"] == "ipu_sl":
            assert [int(c[0]) for c in r["cached_audio"]] == [k - 2, k - 1]
    # chunk centres 0.112, 0.336, 0.56, 0.784, 1.008, 1.232, ...
    assert st == [None, None, "ipu_sl", "ipu_cl", "ipu_cl", "ipu_el", None, None]


def test_barge_in_serialisation_and_decisions():
    pipe = _Pipe()
    # user speaks 0.5-2.0 s and again from 3.0 s (barge-in); the system answers 2.2-4.0 s
    s = _session(pipe, [(0.5, 2.0), (3.0, 4.5)], [(2.2, 4.0)])
    got = []
    s.set_dialog_callback(lambda sess, d: got.append(d["time_stamp"]))
    _feed(s, 5.0, {"user": 0.2, "system": -0.3}, 1)
    s.pump()
    seq = []
    while True:
        d = s.next_feature()
        if d is None:
            break
        seq.append((d["identity"], d["status"], s.llm_prefill(d)))
    idents = [x[0] for x in seq]
    # system chunks before the barge-in are sent (the first relabelled ipu_sl for the chat prefix), those
    # while the user is inside the new IPU are dropped
    first_sys = idents.index("system")
    assert seq[first_sys][1] == "ipu_sl"
    barge = [i for i, x in enumerate(seq) if x[0] == "user" and x[1] == "ipu_sl"][1]
    assert all(x[0] == "user" for x in seq[barge:])
    # decision rule: state_1 = 0.7 > 0.5 on every user chunk -> dialog_ss, callback fired each time
    assert all(x[2] == "dialog_ss" for x in seq if x[0] == "user")
    assert all(x[2] is None for x in seq if x[0] == "system")
    assert len(got) == sum(1 for x in seq if x[0] == "user")
    ipus = s.all_ipus["user"]
    assert sorted(ipus) == [1, 2] and ipus[1].end_timestamp is not None and ipus[1].response_state == "dialog_ss"
    # reset_context forks a fresh context from the system role and frees the old one
    old = s.past_key_values
    s.reset_context()
    assert old.freed and s.past_key_values.n == 5 and s.caches["user"]["pe_index"] == 0


def test_enqueue_validation():
    s = _session(_Pipe(), [], [])
    with pytest.raises(ValueError):
        s.enqueue_audio_data("user", {"audio": b"\0\0", "sr": 8000, "enc": "s16le", "time_stamp": 0})
    with pytest.raises(ValueError):
        s.enqueue_audio_data("user", {"audio": b"\0\0", "sr": 16000, "enc": "f32le", "time_stamp": 0})
    with pytest.raises(ValueError):
        s.enqueue_audio_data("robot", {"audio": b"\0\0", "sr": 16000, "enc": "s16le", "time_stamp": 0})


def test_scheduler_batches_one_feature_per_session_and_matches_sequential():
    from fo.duplex import DuplexScheduler
    plans = [([(0.3, 1.5), (2.5, 3.5)], [(1.7, 3.0)]), ([(0.0, 3.0)], []), ([(1.0, 1.6)], [(0.2, 0.9), (2.0, 3.4)])]
    levels = [{"user": 0.1, "system": 0.0}, {"user": -0.2, "system": 0.1}, {"user": 0.05, "system": -0.1}]

    def run(batched):
        pipe = _Pipe()
        sess = [_session(pipe, u, sy) for u, sy in plans]
        for i, s in enumerate(sess):
            _feed(s, 4.0, levels[i], 10 + i)
        if batched:
            sch = DuplexScheduler(pipe)
            for s in sess:
                sch.add(s)
            ticks = sch.drain()
            assert ticks == max(len(s.states) for s in sess)
        else:
            for s in sess:
                s.pump()
                while (d := s.next_feature()) is not None:
                    s.llm_prefill(d)
        return [(copy.deepcopy(s.states), s.past_key_values.n, dict(s.caches["user"])) for s in sess]

    a, b = run(True), run(False)
    for (sa, na, ca), (sb, nb, cb) in zip(a, b):
        assert [x[:3] for x in sa] == [x[:3] for x in sb] and na == nb and ca == cb


def test_deferred_gating_one_fbank_launch_per_framing_group():
    """DuplexScheduler.tick's batched gating (fo.duplex.deliver_deferred): the queued chunks of every session are
    computed by one fbank call per (framing, device) group of their gaters, user rows before system rows inside a
    group (one identity's rows adjacent), and finished / delivered in queue order with their own rows."""
    import torch

    from fo.duplex import deliver_deferred

    class _Fbank:
        def __init__(self):
            self.calls = []

        def __call__(self, windows, firsts):   # row i of the batch = the window's first sample, as a [R, 80] block
            self.calls.append([float(w[0]) for w in windows])
            return torch.tensor([[[float(w[0])] * 80] * 2 for w in windows])

    class _Gater:
        def __init__(self, kind, fb):
            self.kind, self.device, self.fbank = kind, torch.device("cpu"), fb
            self.got = []

        def finish(self, ann, feat):
            self.got.append((ann["n"], float(feat[0, 0, 0])))
            return {"feature": feat, "status": ann["status"], "feature_last_chunk": []}

    class _Sess:
        def __init__(self, gaters):
            self.feature_gater = gaters
            self.delivered = []

        def _deliver(self, ident, ann, gated):
            self.delivered.append((ident, ann["n"], float(gated["feature"][0, 0, 0])))

    fa, fb_ = _Fbank(), _Fbank()
    s0 = _Sess({"user": _Gater("B", fa), "system": _Gater("B", fa)})
    s1 = _Sess({"user": _Gater("B", fa), "system": _Gater("A", fb_)})
    defer = []
    n = 0
    for s in (s0, s1):
        for ident in ("user", "system"):
            for _ in range(2):
                n += 1
                defer.append((s, ident, {"n": n, "status": "ipu_cl"}, (np.full(4, float(n), np.float32), False)))
    deliver_deferred(defer)
    # framing B: s0 user 1 2, s1 user 5 6 first, then s0 system 3 4; framing A: s1 system 7 8 on its own call
    assert fa.calls == [[1.0, 2.0, 5.0, 6.0, 3.0, 4.0]]
    assert fb_.calls == [[7.0, 8.0]]
    # every chunk delivered in queue order with its own rows
    assert s0.delivered == [("user", 1, 1.0), ("user", 2, 2.0), ("system", 3, 3.0), ("system", 4, 4.0)]
    assert s1.delivered == [("user", 5, 5.0), ("user", 6, 6.0), ("system", 7, 7.0), ("system", 8, 8.0)]
    deliver_deferred([])   # nothing queued: nothing to launch
