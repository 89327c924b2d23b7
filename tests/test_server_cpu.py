"""Server transport (bin/server.py, web/emit.py) over loopback TCP with a stub
pipeline and feature gater: the session's emits (bin/dialog_state_pred.py:565-590, 818-837) reach the
client in order, the task manager gets 'tm_audio_chunk' in the reference's payload form (:577-585),
max_users refuses a start with the pool-exhaustion message, idle sessions time out.  The device path is
the same DuplexSession driven by tests/test_duplex_gpu.py."""
import threading

import numpy as np
import pytest

from test_duplex_cpu import CH, _Gate, _Pipe


def _serve(max_users=2, timeout=30.0):
    from bin.server import DialogServer, TransportServer
    from fo.duplex import DuplexSession, ScriptedVAD

    pipe = _Pipe()

    def factory(sid, hub, data):
        vad = {"user": ScriptedVAD(CH, data.get("vad_intervals", [])),
               "system": ScriptedVAD(CH, data.get("system_vad_intervals", []))}
        return DuplexSession(pipe, sid=sid, vad=vad, feature_gater={"user": _Gate(), "system": _Gate()},
                             socketio=hub)

    dialog = DialogServer(factory, max_users=max_users, timeout=timeout, tick_sleep=0.001)
    srv = TransportServer(("127.0.0.1", 0), dialog)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    return srv, dialog, pipe


def _close(srv, dialog):
    srv.shutdown()
    srv.server_close()
    dialog.shutdown()


def _pcm(level, seed):
    rng = np.random.default_rng(seed)
    return (np.clip(rng.normal(level, 0.01, CH), -0.99, 0.99) * 32767).astype(np.int16)


def test_emit_payloads_follow_reference():
    from web import emit as ev

    a = np.array([0.0, 0.5, -1.0, 1.2, -1.5], np.float32)
    assert ev.np_float32_audio_to_np_int16_audio(a).tolist() == [0, 16384, -32767, 32767, -32768]
    p = ev.tm_audio_chunk_payload("user", "ipu_sl", a[:2], 1.5, [a[:1], a[1:2]])
    assert sorted(p) == ["audio_int_list", "cached_audio_int_list", "identity", "status", "time_stamp"]
    assert p["audio_int_list"] == [0, 16384] and p["cached_audio_int_list"] == [[0], [16384]]
    assert ev.tm_audio_chunk_payload("system", "ipu_cl", a[:1], 2.0)["cached_audio_int_list"] == []

    class Sock:
        def __init__(self):
            self.out = []

        def emit(self, event, data, to=None):
            self.out.append((event, data, to))

    s = Sock()
    ev.emit_dialog_state_update(s, 7, "dialog_ss")
    ev.emit_tm_audio_chunk(s, None, "user", "ipu_cl", a, 0.0)   # no task manager: nothing sent
    ev.emit_dialog_state_update(None, 7, "dialog_cl")           # no transport: nothing sent
    assert s.out == [("dialog_state_update", {"dialog_state": "dialog_ss"}, 7)]


def test_server_streams_session_events_and_tm_chunks():
    from bin.server import DialogClient

    srv, dialog, pipe = _serve()
    host, port = srv.server_address
    c = DialogClient(host, port)
    tm = DialogClient(host, port)
    try:
        # user speech from 0.3 s to 1.5 s (chunk centres 0.112, 0.336, ... step 0.224)
        c.send("start", {"vad_intervals": [[0.3, 1.5]]})
        st = c.wait("started")
        assert st["sid"] == c.sid
        # a guessed sid without the session's token is refused, and so is a second registration
        tm.send("register_tm", {"sid": c.sid})
        assert "wrong token" in tm.wait("error")["message"]
        tm.send("register_tm", {"sid": c.sid, "token": st["token"]})
        assert tm.wait("registered")["sid"] == c.sid
        spy = DialogClient(host, port)
        spy.send("register_tm", {"sid": c.sid, "token": st["token"]})
        assert "already registered" in spy.wait("error")["message"]
        spy.close()
        n = 9
        for k in range(n):
            c.send_audio("user", _pcm(0.2, k), k * CH / 16000)
        c.send("stop")
        c.wait("stopped")
        ev = [m for m in c.events if m["event"] in ("vad_event", "dialog_state_update", "dialog_ss")]
        vad = [m["data"]["event_type"] for m in ev if m["event"] == "vad_event"]
        # centres 0.336..1.456 are speech (6 chunks), 1.68 closes the IPU
        assert vad == ["ipu_sl"] + ["ipu_cl"] * 5 + ["ipu_el"]
        states = [m["data"]["dialog_state"] for m in ev if m["event"] == "dialog_state_update"]
        # stub state_1 = mean + 0.5 = 0.7 on every prefilled user chunk -> dialog_ss each time
        assert states and all(s == "dialog_ss" for s in states)
        assert sum(m["event"] == "dialog_ss" for m in ev) == len(states)
        assert len(states) == sum(1 for ident, _ in pipe.calls if ident == "user")
        # every emitted state follows the VAD event of its chunk
        first_state = next(i for i, m in enumerate(ev) if m["event"] == "dialog_state_update")
        assert ev[first_state - 1]["event"] in ("vad_event", "dialog_ss") or first_state > 0
        # the task manager saw every IPU chunk, in the reference's payload form
        tm_chunks = []
        while len(tm_chunks) < 7:
            m = tm.recv()
            assert m is not None
            if m["event"] == "tm_audio_chunk":
                tm_chunks.append(m["data"])
        assert [d["status"] for d in tm_chunks] == ["ipu_sl"] + ["ipu_cl"] * 5 + ["ipu_el"]
        assert all(len(d["audio_int_list"]) == CH and d["identity"] == "user" for d in tm_chunks)
        assert len(tm_chunks[0]["cached_audio_int_list"]) == 1   # one silent pre-roll chunk before the onset
        ref = _pcm(0.2, 1).astype(np.float32) / 32767.0
        back = np.rint(ref * 32767).astype(np.int16)
        assert tm_chunks[0]["audio_int_list"] == back.tolist()
    finally:
        c.close()
        tm.close()
        _close(srv, dialog)


def test_task_manager_reregisters_after_its_connection_drops():
    import time

    from bin.server import DialogClient

    srv, dialog, _ = _serve()
    host, port = srv.server_address
    c = DialogClient(host, port)
    try:
        c.send("start", {})
        st = c.wait("started")
        tm = DialogClient(host, port)
        tm.send("register_tm", {"sid": c.sid, "token": st["token"]})
        assert tm.wait("registered")["sid"] == c.sid
        tm.close()   # the task manager's connection drops: its registration goes with it
        deadline = time.monotonic() + 10
        while getattr(dialog.sessions[c.sid], "tm_sid", None) is not None and time.monotonic() < deadline:
            time.sleep(0.01)
        assert dialog.sessions[c.sid].tm_sid is None
        tm2 = DialogClient(host, port)
        tm2.send("register_tm", {"sid": c.sid, "token": st["token"]})
        assert tm2.wait("registered")["sid"] == c.sid
        tm2.close()
    finally:
        c.close()
        _close(srv, dialog)


def test_server_max_users_errors_and_timeout():
    from bin.server import DialogClient

    srv, dialog, _ = _serve(max_users=1, timeout=1.5)
    host, port = srv.server_address
    a, b = DialogClient(host, port), DialogClient(host, port)
    try:
        a.send("start")
        a.wait("started")
        b.send("start")
        assert b.wait("error")["message"] == "Failed to get pipeline object from pool"
        # protocol errors are reported and the connection stays usable
        b.send("audio", {"identity": "user", "audio": ""})
        assert "start" in b.wait("error")["message"]
        a.send("audio", {"identity": "robot", "audio": "", "sr": 16000, "enc": "s16le", "time_stamp": 0.0})
        assert "Unknown identity" in a.wait("error")["message"]
        a.send("audio", {"identity": "user", "audio": "", "sr": 8000, "enc": "s16le", "time_stamp": 0.0})
        assert "sampling rate" in a.wait("error")["message"]
        # a idles past the timeout: released, told, disconnected; its slot frees up for b
        assert a.wait("timeout")["sid"] == a.sid
        with pytest.raises(ConnectionError):
            a.wait("anything")
        b.send("start")
        assert b.wait("started")["sid"] == b.sid
    finally:
        a.close()
        b.close()
        _close(srv, dialog)


def test_server_cli_matches_launch_script():
    """scripts/run_demo_server.sh:20-30 flags parse unchanged."""
    from bin.server import get_parser

    a = get_parser().parse_args(["--ip", "127.0.0.1", "--port", "8081", "--max_users", "3", "--llm_exec_nums", "1",
                                 "--timeout", "180", "--model_path", "./checkpoints", "--llm_path",
                                 "./Qwen2-7B-Instruct", "--top_p", "0.8", "--top_k", "20", "--temperature", "0.8"])
    assert (a.max_users, a.llm_exec_nums, a.top_k, a.top_p, a.temperature) == (3, 1, 20, 0.8, 0.8)
