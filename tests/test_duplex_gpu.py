"""Duplex sessions on the device path (fo.duplex over models.pipeline, tiny config): the batched
scheduler (one speech_dialogue_batch per tick for every session) gives each session the results of
its own sequential llm_prefill loop (bin/dialog_state_pred.py:719-844), with user barge-in over
system speech."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "configs", "tiny")


@pytest.fixture(scope="module")
def pipe(dev):
    from models.pipeline import inferencePipeline
    return inferencePipeline({"model_path": TINY, "llm_path": os.path.join(TINY, "llm"), "device": "cuda:0",
                              "top_k": 1})


def _pcm(n, seed):
    rng = np.random.default_rng(seed)
    w = np.convolve(rng.standard_normal(n + 64), np.hanning(33), mode="same")[:n]
    t = np.arange(n) / 16000.0
    return 0.1 * w / (np.abs(w).max() + 1e-9) * 0.5 * (1 + np.sin(2 * np.pi * 4 * t))


PLANS = [([(0.3, 1.6), (2.6, 3.8)], [(1.8, 3.2)]),   # barge-in at 2.6 s into the system's answer
         ([(0.0, 2.5)], [(2.7, 3.9)]),
         ([(1.0, 1.7), (2.2, 3.0)], [(0.1, 0.9)])]


def _run(pipe, batched, seconds=4.0):
    from fo.duplex import DuplexScheduler, DuplexSession, ScriptedVAD
    sess = []
    for i, (u, s) in enumerate(PLANS):
        ch = 3584
        vad = {"user": ScriptedVAD(ch, u), "system": ScriptedVAD(ch, s)}
        ds = DuplexSession(pipe, sid=i, vad=vad)
        n = int(seconds * 16000 / ch)
        pcm = {"user": _pcm(n * ch, 100 + i), "system": _pcm(n * ch, 200 + i)}
        for k in range(n):
            for ident in ("user", "system"):
                x = (np.clip(pcm[ident][k * ch:(k + 1) * ch], -1, 1) * 32767).astype(np.int16)
                ds.enqueue_audio_data(ident, {"audio": x.tobytes(), "sr": 16000, "enc": "s16le",
                                              "time_stamp": k * ch / 16000})
        sess.append(ds)
    if batched:
        sch = DuplexScheduler(pipe)
        for s in sess:
            sch.add(s)
        sch.drain()
    else:
        for s in sess:
            s.pump()
            while (d := s.next_feature()) is not None:
                s.llm_prefill(d)
    out = [(list(s.states), s.past_key_values.get_seq_length(), s.caches["user"]["pe_index"]) for s in sess]
    for s in sess:
        s.release()
    return out


def test_dialog_state_params_api(dev):
    """The reference class surface: DialogStateParams(sid, socketio, event_outlet, outlets) from the pool,
    enqueue_audio_data / start_all_threads / reset_context / release; two sessions share one replica's
    scheduler and pipeline."""
    import copy
    from bin.dialog_state_pred import DialogStateParams
    from fo.duplex import DEFAULT_CONFIG, ScriptedVAD
    cfg = copy.deepcopy(DEFAULT_CONFIG)
    cfg.update(model_path=TINY, llm_path=os.path.join(TINY, "llm"), device="cuda:0")
    DialogStateParams.DIALOG_STATE_PRED_CONFIGS = cfg
    DialogStateParams.PIPELINE_POOL = None
    events = []
    sess = [DialogStateParams(f"sid{i}", None, events.append, [],
                              vad={"user": ScriptedVAD(3584, [(0.2, 1.2)]), "system": ScriptedVAD(3584, [(1.3, 2.0)])})
            for i in range(2)]
    assert sess[0].pipeline_obj is sess[1].pipeline_obj and sess[0].pipeline_obj.user_count == 2
    for s in sess:
        s.start_all_threads()
        s.reset_context()
    assert sess[0].scheduler is sess[1].scheduler and len(sess[0].scheduler.sessions) == 2
    pcm = (_pcm(9 * 3584, 7) * 32767).astype(np.int16)
    for s in sess:
        for k in range(9):
            for ident in ("user", "system"):
                s.enqueue_audio_data(ident, {"audio": pcm[k * 3584:(k + 1) * 3584].tobytes(), "sr": 16000,
                                             "enc": "s16le", "time_stamp": k * 0.224})
    n = sess[0].run_scheduler()
    assert n > 0 and len(events) == 2                       # one user IPU opened per session
    for s in sess:
        idents = [x[0] for x in s.states]
        assert idents[0] == "user" and "system" in idents
        assert all(x[2] in ("dialog_ss", "dialog_cl") for x in s.states if x[0] == "user")
    obj = sess[0].pipeline_obj
    for s in sess:
        s.release()
    assert obj.user_count == 0
    DialogStateParams.PIPELINE_POOL = None


def test_duplex_scheduler_matches_per_session(pipe):
    bat, seq = _run(pipe, True), _run(pipe, False)
    n_sys = 0
    for (sb, nb, pb), (ss, ns, ps) in zip(bat, seq):
        assert nb == ns and pb == ps
        assert [x[:2] for x in sb] == [x[:2] for x in ss]
        n_sys += sum(1 for x in sb if x[0] == "system")
        for (i1, _, st1, p1), (_, _, st2, p2) in zip(sb, ss):
            if i1 == "user":
                assert abs(p1["state_1"] - p2["state_1"]) < 1e-4 and abs(p1["state_2"] - p2["state_2"]) < 1e-4
                if abs(p2["state_1"] - 0.5) > 1e-3:
                    assert st1 == st2
            else:
                assert p1 is None and st1 is None
    assert n_sys > 0   # system speech really went through the system encoder / prefill


def test_server_transport_on_device(dev, pipe):
    """bin/server.py with the production session factory (DialogStateParams on the replica pool, tiny
    config) over loopback TCP: the emitted VAD events follow the scripted schedule and the emitted
    dialog states equal a direct sequential llm_prefill run of the same audio."""
    import argparse
    import threading
    from bin.dialog_state_pred import DialogStateParams
    from bin.server import DialogClient, DialogServer, TransportServer, dialog_session_factory
    from fo.duplex import DuplexSession, ScriptedVAD

    u_iv, s_iv = [(0.2, 1.3)], [(1.5, 2.2)]
    ch, n = 3584, 11
    pcm = {"user": (np.clip(_pcm(n * ch, 31), -1, 1) * 32767).astype(np.int16),
           "system": (np.clip(_pcm(n * ch, 32), -1, 1) * 32767).astype(np.int16)}
    # direct run
    ds = DuplexSession(pipe, sid=0, vad={"user": ScriptedVAD(ch, u_iv), "system": ScriptedVAD(ch, s_iv)},
                       config=None)
    for k in range(n):
        for ident in ("user", "system"):
            ds.enqueue_audio_data(ident, {"audio": pcm[ident][k * ch:(k + 1) * ch].tobytes(), "sr": 16000,
                                          "enc": "s16le", "time_stamp": k * ch / 16000})
    ds.pump()
    while (d := ds.next_feature()) is not None:
        ds.llm_prefill(d)
    want = [(st, p["state_1"]) for ident, _, st, p in ds.states if ident == "user"]
    ds.release()

    DialogStateParams.PIPELINE_POOL = None
    args = argparse.Namespace(config=None, model_path=TINY, llm_path=os.path.join(TINY, "llm"), top_k=1, top_p=0.0,
                              temperature=1.0, llm_exec_nums=1)
    dialog = DialogServer(dialog_session_factory(args), max_users=2, timeout=60.0)
    srv = TransportServer(("127.0.0.1", 0), dialog)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    c = DialogClient(*srv.server_address, timeout=120.0)
    try:
        c.send("start", {"vad_intervals": u_iv, "system_vad_intervals": s_iv})
        c.wait("started")
        for k in range(n):
            for ident in ("user", "system"):
                c.send_audio(ident, pcm[ident][k * ch:(k + 1) * ch], k * ch / 16000)
        c.send("stop")
        c.wait("stopped")
    finally:
        c.close()
        srv.shutdown()
        srv.server_close()
        dialog.shutdown()
        DialogStateParams.PIPELINE_POOL = None
    vad_u = [m["data"]["event_type"] for m in c.events if m["event"] == "vad_event" and m["data"]["identity"] == "user"]
    assert vad_u == ["ipu_sl"] + ["ipu_cl"] * 4 + ["ipu_el"]
    got = [m["data"]["dialog_state"] for m in c.events if m["event"] == "dialog_state_update"]
    assert len(got) == len(want) > 0
    for g, (w, p1) in zip(got, want):
        if abs(p1 - 0.5) > 1e-3:
            assert g == w
    assert sum(m["event"] == "dialog_ss" for m in c.events) == got.count("dialog_ss")


def test_duplex_encoder_graph_and_two_streams_match_eager(pipe):
    """The duplex tick's steady-state encoder + adapter stage replays a captured EncoderGraph, the second identity's
    on its own stream ('enc2'); with graphs off the same tick runs the eager encoder / adapter launches.  Both must
    give the same state probabilities bit for bit and the same KV lengths / pe indices (same kernels, same order,
    each stream with its own scratch)."""
    eng = pipe.model.engine
    assert eng.use_graphs
    with_graphs = _run(pipe, True)
    eng.use_graphs = False
    try:
        eager = _run(pipe, True)
    finally:
        eng.use_graphs = True
    assert with_graphs == eager
    assert any(x[0] == "system" for s, _, _ in with_graphs for x in s)   # both parties took part


def test_batched_fbank_matches_single_chunk_gating(dev):
    """DuplexScheduler.tick frames every session's chunk first and computes all their fbank rows in one launch
    (AudioFeatureGating.prepare / fbank_batch / finish): each chunk's gated features, onset replay included, are
    bit-identical to the one-chunk process_and_gate of an identical gater."""
    import torch

    from fo.duplex import DEFAULT_CONFIG
    from models.AudioFeatureGating import AudioFeatureGating, fbank_batch
    g = DEFAULT_CONFIG["audio_feature_gating"]
    # (an onset replay of 6 chunks: the fork's config replays none)
    mk = lambda: AudioFeatureGating(16000, g["feature_gating_history_size"], 6, g["fbank"], device="cuda:0",  # noqa: E731
                                    as_tensor=True)
    single, batched = [mk() for _ in range(3)], [mk() for _ in range(3)]
    n = single[0].expected_frames_per_audio_chunk
    statuses = [None, None, "ipu_sl", "ipu_cl", "ipu_el"]
    for k, st in enumerate(statuses):
        anns = [{"audio": _pcm(n, 100 * k + i).astype(np.float32), "status": st} for i in range(3)]
        want = [gt.process_and_gate(a) for gt, a in zip(single, anns)]
        reqs = [gt.prepare(a) for gt, a in zip(batched, anns)]
        got = [gt.finish(a, f) for gt, a, f in zip(batched, anns, fbank_batch(batched, reqs))]
        for w, o in zip(want, got):
            if w is None:
                assert o is None
                continue
            assert w["status"] == o["status"]
            assert torch.equal(w["feature"], o["feature"])
            if st == "ipu_sl":
                assert torch.equal(w["feature_last_chunk"], o["feature_last_chunk"])
    for a, b in zip(single, batched):
        assert torch.equal(a.history, b.history)
