"""Server transport for the duplex dialog-state sessions.

Upstream `bin/server.py` is absent from the snapshot; what is pinned is its launch contract
(scripts/run_demo_server.sh:20-30: --ip --port --max_users --llm_exec_nums --timeout --model_path
--llm_path --top_p --top_k --temperature) and the emits of the session it drives
(bin/dialog_state_pred.py:565-590, 818-837; web/emit.py).  flask-socketio is not installed, so the
socket.io event model is kept over a plain TCP stream of JSON lines, one event per line:

    {"event": <name>, "data": <payload>}

client -> server
    start        {"prompt": str?, "vad_intervals": [[s, e], ...]?}  open this connection's session
    audio        {"identity": "user"|"system", "audio": base64 s16le, "sr": 16000, "enc": "s16le",
                  "time_stamp": float}                               enqueue_audio_data (:330-400)
    prompt       {"text": str}                                       set_prompt (:290-300)
    reset        {}                                                  reset_context (:170-238)
    register_tm  {"sid": int, "token": str}  this connection receives that session's 'tm_audio_chunk' stream;
                 the token is the one 'started' returned to the session's own connection (a guessed sid
                 alone is refused), and a session's stream, once registered, is not taken over
    stop         {}                                                  release the session
server -> client
    connected {"sid"}, started {"sid", "token"}, registered {"sid"}, error {"message"}, timeout {"sid"},
    stopped {"sid"}, and the
    session's emits: vad_state_update, vad_event, dialog_ss, dialog_state_update, tm_audio_chunk.

Sessions are not threads here: one worker thread ticks every replica's DuplexScheduler, which batches
all of that GPU's sessions into one prefill per tick (fo/duplex.py), and the emits are written to the
sockets from that thread.  --max_users caps concurrent sessions (a refused start gets an 'error'
event, the reference pool's exhaustion message); sessions idle longer than --timeout seconds are
released and their connection closed.
"""
import argparse
import base64
import itertools
import json
import os
import secrets
import socket
import socketserver
import sys
import threading
import time

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fo.duplex import DuplexScheduler, EnergyVAD, ScriptedVAD  # noqa: E402

TICK_SLEEP = 0.005   # DialogStateParams.SLEEP_INTERVAL: the reference threads poll every 5 ms


class Connection:
    def __init__(self, sock):
        self.sock = sock
        self.wlock = threading.Lock()
        self.alive = True

    def send(self, event, data):
        line = (json.dumps({"event": event, "data": data}, separators=(",", ":")) + "\n").encode()
        with self.wlock:
            if not self.alive:
                return
            try:
                self.sock.sendall(line)
            except OSError:
                self.alive = False

    def close(self):
        with self.wlock:
            if self.alive:
                self.alive = False
                try:
                    self.sock.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass


class Hub:
    """The socketio object the sessions emit through: emit(event, data, to=sid)."""

    def __init__(self):
        self.conns = {}
        self.lock = threading.Lock()

    def register(self, sid, conn):
        with self.lock:
            self.conns[sid] = conn

    def unregister(self, sid):
        with self.lock:
            self.conns.pop(sid, None)

    def emit(self, event, data, to=None):
        with self.lock:
            conn = self.conns.get(to)
        if conn is not None:
            conn.send(event, data)


class DialogServer:
    """Session table + the worker that ticks the replicas' schedulers.

    session_factory(sid, hub, start_data) -> a DuplexSession (DialogStateParams in production); it must
    expose .pipeline, enqueue_audio_data, set_prompt, reset_context, release and a tm_sid attribute."""

    def __init__(self, session_factory, max_users=3, timeout=180.0, tick_sleep=TICK_SLEEP):
        self.factory, self.max_users, self.timeout, self.tick_sleep = session_factory, max_users, timeout, tick_sleep
        self.hub = Hub()
        self.sessions, self.last_active = {}, {}
        self.tokens = {}     # sid -> the secret 'started' returned (register_tm must present it)
        self.schedulers = {}
        self.lock = threading.RLock()
        self._sids = itertools.count(1)
        self._stop = threading.Event()
        self.worker = threading.Thread(target=self._run, name="fo-dialog-server", daemon=True)
        self.worker.start()

    def new_connection(self, conn):
        sid = next(self._sids)
        self.hub.register(sid, conn)
        conn.send("connected", {"sid": sid})
        return sid

    # ---------------------------------------------------------------- session lifecycle
    def start(self, sid, data):
        with self.lock:
            if sid in self.sessions:
                raise ValueError(f"session {sid} already started")
            if len(self.sessions) >= self.max_users:
                raise Exception("Failed to get pipeline object from pool")   # bin/pool.py:46 / :55-56
            s = self.factory(sid, self.hub, data or {})
            key = id(s.pipeline)
            if key not in self.schedulers:
                self.schedulers[key] = DuplexScheduler(s.pipeline)
            self.schedulers[key].add(s)
            self.sessions[sid] = s
            self.last_active[sid] = time.monotonic()
            self.tokens[sid] = token = secrets.token_hex(16)
        self.hub.emit("started", {"sid": sid, "token": token}, to=sid)

    def stop(self, sid, event="stopped", drain=False):
        """Release a session; drain=True first prefills everything it has received (a client 'stop')."""
        with self.lock:
            s = self.sessions.get(sid)
            if s is None:
                return
            sch = next((c for c in self.schedulers.values() if s in c.sessions), None)
            if drain and sch is not None:
                for _ in range(1 << 16):
                    s.pump()
                    if not s.context_serializer.feature_queue:
                        break
                    sch.tick()
            self.sessions.pop(sid, None)
            self.last_active.pop(sid, None)
            self.tokens.pop(sid, None)
            if sch is not None:
                sch.sessions.remove(s)
            s.release()
        self.hub.emit(event, {"sid": sid}, to=sid)

    def disconnect(self, sid):
        self.stop(sid)
        with self.lock:   # a dropped task-manager connection frees the streams it registered for re-registration
            for s in self.sessions.values():
                if getattr(s, "tm_sid", None) == sid:
                    s.tm_sid = None
        self.hub.unregister(sid)

    # ---------------------------------------------------------------- events
    def handle(self, sid, event, data):
        data = data or {}
        if event == "start":
            self.start(sid, data)
            return
        if event == "register_tm":
            with self.lock:
                tsid = int(data["sid"])
                target = self.sessions.get(tsid)
                token = str(data.get("token", ""))
                if target is None or not secrets.compare_digest(token, self.tokens.get(tsid, "")):
                    raise ValueError("register_tm: unknown session or wrong token")   # no hint which
                if getattr(target, "tm_sid", None) not in (None, sid):
                    raise ValueError(f"register_tm: session {tsid}'s stream is already registered")
                target.tm_sid = sid
            self.hub.emit("registered", {"sid": tsid}, to=sid)
            return
        with self.lock:
            s = self.sessions.get(sid)
            if s is None:
                raise ValueError("no session: send 'start' first")
            self.last_active[sid] = time.monotonic()
            if event == "audio":
                s.enqueue_audio_data(data["identity"], {
                    "audio": base64.b64decode(data["audio"]), "sr": data.get("sr", 16000),
                    "enc": data.get("enc", "s16le"), "time_stamp": data.get("time_stamp", time.time())})
            elif event == "prompt":
                s.set_prompt(data["text"])
            elif event == "reset":
                s.reset_context()
            elif event == "stop":
                pass
            else:
                raise ValueError(f"unknown event {event!r}")
        if event == "stop":
            self.stop(sid, drain=True)

    # ---------------------------------------------------------------- worker
    def tick(self):
        """One batched prefill per replica; the sessions emit their results.  Returns the work count.  A
        replica whose prefill fails reports it to the sessions of that batch only (the others go on)."""
        n = 0
        with self.lock:
            for sch in list(self.schedulers.values()):
                if not sch.sessions:
                    continue
                try:
                    n += len(sch.tick())
                except Exception as e:
                    members = [sid for sid, s in self.sessions.items() if s in sch.sessions]
                    for sid in members:
                        self.hub.emit("error", {"message": f"prefill failed: {e}"}, to=sid)
        return n

    def _reap(self):
        now = time.monotonic()
        with self.lock:
            idle = [sid for sid, t in self.last_active.items() if now - t > self.timeout]
        for sid in idle:
            self.stop(sid, event="timeout")
            with self.hub.lock:
                conn = self.hub.conns.get(sid)
            if conn is not None:
                conn.close()

    def _run(self):
        while not self._stop.is_set():
            n = self.tick()   # a failing prefill is reported to its batch's sessions, never kills the transport
            self._reap()
            if n == 0:
                time.sleep(self.tick_sleep)

    def shutdown(self):
        self._stop.set()
        self.worker.join(timeout=5)
        with self.lock:
            sids = list(self.sessions)
        for sid in sids:
            self.stop(sid)


class _Handler(socketserver.StreamRequestHandler):
    def handle(self):
        srv = self.server.dialog
        conn = Connection(self.request)
        sid = srv.new_connection(conn)
        try:
            for raw in self.rfile:
                if not raw.strip():
                    continue
                try:
                    msg = json.loads(raw)
                    srv.handle(sid, msg.get("event"), msg.get("data"))
                except Exception as e:   # protocol / ValueError / pool exhaustion: reported, connection kept
                    conn.send("error", {"message": str(e)})
                if not conn.alive:
                    break
        except OSError:   # peer reset / closed by the timeout reaper
            pass
        finally:
            srv.disconnect(sid)
            conn.close()


class TransportServer(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, addr, dialog):
        self.dialog = dialog
        super().__init__(addr, _Handler)


class DialogClient:
    """Minimal client of the transport (demo GUI / task manager side, and the tests)."""

    def __init__(self, host, port, timeout=30.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.rfile = self.sock.makefile("rb")
        self.events = []
        self.sid = self.wait("connected")["sid"]

    def send(self, event, data=None):
        self.sock.sendall((json.dumps({"event": event, "data": data or {}}) + "\n").encode())

    def send_audio(self, identity, pcm_int16, time_stamp, sr=16000):
        self.send("audio", {"identity": identity, "audio": base64.b64encode(pcm_int16.astype("<i2").tobytes()).decode(),
                            "sr": sr, "enc": "s16le", "time_stamp": time_stamp})

    def recv(self):
        line = self.rfile.readline()
        if not line:
            return None
        m = json.loads(line)
        self.events.append(m)
        return m

    def wait(self, event, limit=10000):
        for _ in range(limit):
            m = self.recv()
            if m is None:
                raise ConnectionError(f"closed while waiting for {event!r}")
            if m["event"] == event:
                return m["data"]
            if m["event"] == "error" and event != "error":
                raise RuntimeError(m["data"]["message"])
        raise TimeoutError(event)

    def close(self):
        try:   # shutdown first: a makefile() reader keeps the descriptor open past close(), the peer would see no EOF
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        try:
            self.sock.close()
        except OSError:
            pass


def dialog_session_factory(args):
    """Production factory: one DialogStateParams per started connection, on the replica pool."""
    from bin.dialog_state_pred import DialogStateParams, get_args

    cfg = get_args(args.config)
    cfg["model_path"] = args.model_path or cfg["model_path"]
    if args.llm_path:
        cfg["llm_path"] = args.llm_path
    ic = cfg.setdefault("inference_control", {})
    ic.update(top_k=args.top_k, top_p=args.top_p, temperature=args.temperature)
    DialogStateParams.DIALOG_STATE_PRED_CONFIGS = cfg
    DialogStateParams.MAX_PIPELINE_NUN = args.llm_exec_nums

    def make(sid, hub, data):
        chunk = int(round(cfg["audio_feature_gating"]["fbank"]["expected_audio_chunk_duration_in_sec"] *
                          cfg["audio"]["expected_sampling_rate"]))
        hist = cfg["vad"]["vad_history_cache_chunk_cnt"]
        sr = cfg["audio"]["expected_sampling_rate"]
        if data.get("vad_intervals") is not None:
            vad = {"user": ScriptedVAD(chunk, data["vad_intervals"], sr, hist),
                   "system": ScriptedVAD(chunk, data.get("system_vad_intervals", []), sr, hist)}
        else:
            vad = {i: EnergyVAD(chunk, sr, hist, min_silent_duration_second=cfg["vad"]["min_silent_duration_second"])
                   for i in ("user", "system")}
        s = DialogStateParams(sid, socketio=hub, vad=vad)
        if data.get("prompt"):
            s.set_prompt(data["prompt"])
        return s

    return make


def get_parser():
    p = argparse.ArgumentParser(description="Freeze-Omni duplex dialog-state server (MI355X build)")
    p.add_argument("--ip", default="127.0.0.1")
    p.add_argument("--port", type=int, default=8081)
    p.add_argument("--max_users", type=int, default=3)
    p.add_argument("--llm_exec_nums", type=int, default=1)
    p.add_argument("--timeout", type=float, default=180.0)
    p.add_argument("--model_path", default=None)
    p.add_argument("--llm_path", default=None)
    p.add_argument("--top_p", type=float, default=0.8)
    p.add_argument("--top_k", type=int, default=20)
    p.add_argument("--temperature", type=float, default=0.8)
    p.add_argument("--config", default=None, help="duplex YAML (configs/dialog_state_pred_config.yaml form)")
    return p


def main(argv=None):
    args = get_parser().parse_args(argv)
    dialog = DialogServer(dialog_session_factory(args), max_users=args.max_users, timeout=args.timeout)
    with TransportServer((args.ip, args.port), dialog) as srv:
        print(f"serving on {args.ip}:{srv.server_address[1]}", flush=True)
        try:
            srv.serve_forever()
        finally:
            dialog.shutdown()


if __name__ == "__main__":
    main()
