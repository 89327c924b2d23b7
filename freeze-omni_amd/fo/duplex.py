"""Full-duplex dialogue sessions: the bin/dialog_state_pred.py path.

Reference (bin/dialog_state_pred.py:65-844): per session, five polling threads share one pipeline
without locks:
    receive_raw_audio_chunk (:348-400)  s16le bytes -> float32 / 32767
    vad_annotation          (:405-598)  PureVAD -> ipu_sl / ipu_cl / ipu_el / None, IPU handles
    feature_gating          (:600-684)  AudioFeatureGating.process_and_gate (+ onset replay)
    serialize_context       (:686-717)  ContextSerializer: timestamp order, user priority
    predict_dialog_state    (:719-775)  -> llm_prefill (:777-844) -> speech_dialogue; state_1 > 0.5 -> dialog_ss

Here a DuplexSession keeps exactly those per-session stages and their state, run synchronously by
pump() (no polling threads, no 5 ms sleeps), and a DuplexScheduler owns every session of one replica:
each tick it takes at most one serialized feature per session (a session's context is sequential) and
runs ALL of them through one batched speech_dialogue_batch call -- one encoder / adapter / Qwen2 launch
sequence for every session's chunk instead of one un-batched call per session thread.

ScriptedVAD stands in for periphrals.PureVAD (absent from the reference tree; silero-vad 5.1.2 is not
installed): it labels chunks from a speech-interval schedule with the same output contract.
"""
import collections
import copy
import os

import numpy as np
import torch

from web import emit as ev

RESPONSE_THRESHOLD = 0.5   # configs/dialog_state_pred_config.yaml:40-41

DEFAULT_CONFIG = {         # configs/dialog_state_pred_config.yaml (the fork's duplex settings)
    "audio": {"expected_sampling_rate": 16000},
    "vad": {"use_standalone_vad": True, "vad_threshold": 0.5, "min_silent_duration_second": 0.5,
            "speech_pad_second": 0.03, "vad_history_cache_chunk_cnt": 2},
    "audio_feature_gating": {"feature_gating_history_size": 10, "onset_input_chunk_cache_size": 0,
                             "fbank": {"expected_audio_chunk_duration_in_sec": 0.224, "feat_dim": 80,
                                       "audio_to_proc_per_step_in_sec": 0.016, "step_size_in_sec": 0.008,
                                       "context_duration_in_sec": 0.032}},
    "inference_control": {"top_k": 5, "top_p": 0.8, "temperature": 0.7,
                          "default_prompt": "Start new response if the user provided new information or gave "
                                            "new instructions."},
    "dialog_state_decision": {"resp_threshold": RESPONSE_THRESHOLD},
}


class ScriptedVAD:
    """PureVAD stand-in with its predict() contract (bin/dialog_state_pred.py:476-483): returns
    {'audio', 'status' in ipu_sl / ipu_cl / ipu_el / None, 'cached_audio', 'time_stamp'} per chunk of
    get_chunk_size() samples.  A chunk is speech when its centre falls inside one of the scheduled
    [start, end) intervals (seconds of this stream); the first speech chunk after silence opens an IPU
    (ipu_sl, carrying the last `cache_history_size` silent chunks as pre-roll), the first silent
    chunk after speech closes it (ipu_el)."""

    def __init__(self, chunk_size, intervals, sample_rate=16000, cache_history_size=2):
        self.chunk_size = chunk_size
        self.sr = sample_rate
        self.intervals = sorted((float(a), float(b)) for a, b in intervals)
        self.cache_history_size = cache_history_size
        self.reset()

    def get_chunk_size(self):
        return self.chunk_size

    def reset(self):
        self.n = 0
        self.in_speech = False
        self.history = collections.deque(maxlen=max(self.cache_history_size, 1))

    def is_speech(self, k):
        t = (k + 0.5) * self.chunk_size / self.sr
        return any(a <= t < b for a, b in self.intervals)

    def predict(self, audio_dict):
        audio = audio_dict["audio"]
        speech = self.is_speech(self.n)
        self.n += 1
        cached = None
        if speech and not self.in_speech:
            status = "ipu_sl"
            cached = list(self.history)[-self.cache_history_size:] if self.cache_history_size > 0 else []
        elif speech:
            status = "ipu_cl"
        elif self.in_speech:
            status = "ipu_el"
        else:
            status = None
        self.in_speech = speech
        self.history.append(audio)
        return {"audio": audio, "status": status, "cached_audio": cached, "time_stamp": audio_dict.get("time_stamp")}


class EnergyVAD(ScriptedVAD):
    """Live-audio PureVAD stand-in for the server transport (silero-vad is not installed): a chunk is
    speech when its RMS is above `threshold_dbfs`; an IPU closes only after `min_silent_duration_second`
    of consecutive silence (the YAML's hangover, configs/dialog_state_pred_config.yaml vad block), so
    short pauses stay inside one IPU.  Same predict() contract and pre-roll as ScriptedVAD."""

    def __init__(self, chunk_size, sample_rate=16000, cache_history_size=2, threshold_dbfs=-40.0,
                 min_silent_duration_second=0.5):
        self.threshold = 10.0 ** (threshold_dbfs / 20.0)
        self.hang = max(1, int(round(min_silent_duration_second * sample_rate / chunk_size)))
        super().__init__(chunk_size, [], sample_rate, cache_history_size)

    def reset(self):
        super().reset()
        self.silent = 0

    def is_speech(self, k):
        a = self._audio
        loud = a.size > 0 and float(np.sqrt(np.mean(np.square(a, dtype=np.float64)))) > self.threshold
        self.silent = 0 if loud else self.silent + 1
        return loud or (self.in_speech and self.silent < self.hang)

    def predict(self, audio_dict):
        self._audio = np.asarray(audio_dict["audio"], dtype=np.float32)
        return super().predict(audio_dict)


class IPURecord:
    """One inter-pausal unit of a speaker (stands in for AudioLLMInterface.IPUHandle, absent from the
    reference tree): the response state the predictor last registered for it."""

    def __init__(self, ipu_id, identity, start_timestamp):
        self.id, self.identity = ipu_id, identity
        self.start_timestamp, self.end_timestamp = start_timestamp, None
        self.n_chunks = 1
        self.response_state, self.prediction_cnt = None, 0

    def add_chunk(self, _audio=None):
        self.n_chunks += 1

    def set_end_timestamp(self, ts):
        self.end_timestamp = ts

    def register_response_state(self, state, cnt):
        self.response_state, self.prediction_cnt = state, cnt


class DuplexSession:
    """Per-session state of DialogStateParams (bin/dialog_state_pred.py:79-238) with the thread bodies
    as synchronous stages.  pipeline: a models.pipeline.inferencePipeline (fork API)."""

    def __init__(self, pipeline, sid=0, config=None, vad=None, event_outlet=None, user_ipu_outlet_list=(),
                 dialog_state_callback=None, feature_gater=None, socketio=None):
        cfg = copy.deepcopy(DEFAULT_CONFIG if config is None else config)
        self.cfg, self.sid, self.pipeline = cfg, sid, pipeline
        # transport (bin/server.py): emit(event, data, to=sid) or None; tm_sid receives 'tm_audio_chunk'
        self.socketio = socketio
        self.tm_sid = getattr(self, "tm_sid", None)
        self.sr = cfg["audio"]["expected_sampling_rate"]
        self.threshold = cfg["dialog_state_decision"]["resp_threshold"]
        g = cfg["audio_feature_gating"]
        if feature_gater is None:
            from models.AudioFeatureGating import AudioFeatureGating
            feature_gater = {ident: AudioFeatureGating(self.sr, g["feature_gating_history_size"],
                                                       g["onset_input_chunk_cache_size"], g["fbank"],
                                                       device=pipeline.device, as_tensor=True)
                             for ident in ("user", "system")}
        self.feature_gater = feature_gater
        chunk = self.feature_gater["user"].expected_frames_per_audio_chunk
        self.vad = vad if vad is not None else {
            ident: ScriptedVAD(chunk, [], self.sr, cfg["vad"]["vad_history_cache_chunk_cnt"])
            for ident in ("user", "system")}
        self.event_outlet = event_outlet
        self.user_ipu_outlet_list = list(user_ipu_outlet_list)
        self.dialog_state_callback = dialog_state_callback
        _, kv, _, _, _ = pipeline.speech_dialogue(None, identity="", status="pre",
                                                  role=cfg["inference_control"]["default_prompt"])
        self.system_role = kv                       # :108-110
        self.past_key_values = None
        self.prediction_cnt = 0
        self.states = []                            # (identity, status, predicted state, probs) per prefill
        self.reset_context()

    # ------------------------------------------------------------------ :170-238
    def reset_context(self):
        from models.ContextSerializer import ContextSerializer
        self.raw = {"user": collections.deque(), "system": collections.deque()}
        self.pending = {"user": np.zeros(0, np.float32), "system": np.zeros(0, np.float32)}
        self.pending_ts = {"user": None, "system": None}
        self.all_ipus = {"user": {}, "system": {}}
        self.current_ipu = {"user": None, "system": None}
        self.total_ipus = {"user": 0, "system": 0}
        for ident in ("user", "system"):
            self.feature_gater[ident].reset()
            self.vad[ident].reset()
        if not hasattr(self, "context_serializer"):
            self.context_serializer = ContextSerializer()
        self.context_serializer.reset()
        if self.past_key_values is not None:
            self.past_key_values.free()
        self.past_key_values = copy.deepcopy(self.system_role)    # :218 (copy-on-write fork)
        self.caches = {ident: {"encoder_cache": None, "adapter_cache": None, "pe_index": 0}
                       for ident in ("user", "system")}

    def set_prompt(self, prompt):
        # the reference stores the whole 5-tuple here (:296-300, SURVEY §8(c) ii); the KV is what it means
        old = self.system_role
        _, self.system_role, _, _, _ = self.pipeline.speech_dialogue(None, identity=None, status="pre", role=prompt)
        old.free()

    def set_dialog_callback(self, callback):
        self.dialog_state_callback = callback

    def release(self):
        if self.past_key_values is not None:
            self.past_key_values.free()
            self.past_key_values = None
        if self.system_role is not None:
            self.system_role.free()
            self.system_role = None

    # ------------------------------------------------------------------ :330-400
    def enqueue_audio_data(self, identity, audio_data_dict):
        if identity not in ("user", "system"):
            raise ValueError(f"Unknown identity: {identity}. Must be 'user' or 'system'.")
        if audio_data_dict["sr"] != self.sr:
            raise ValueError(f"Expected audio sampling rate {self.sr}, but got {audio_data_dict['sr']}")
        if audio_data_dict["enc"] != "s16le":
            raise ValueError(f"Expected audio encoding 's16le', but got {audio_data_dict['enc']}")
        audio = np.frombuffer(audio_data_dict["audio"], dtype=np.int16).astype(np.float32) / 32767.0
        self.raw[identity].append((audio, audio_data_dict["time_stamp"]))

    # ------------------------------------------------------------------ :405-684 as one synchronous pass
    def pump(self, defer=None):
        """Run VAD annotation and feature gating over every complete VAD chunk received so far; gated
        features go to the context serializer.  defer (a list): the gating of each chunk is queued there as
        (session, identity, annotation, fbank request) instead, for DuplexScheduler.tick to compute every
        session's fbank rows in one launch and deliver them in order (deliver_deferred)."""
        for ident in ("user", "system"):
            vad, n = self.vad[ident], self.vad[ident].get_chunk_size()
            while self.raw[ident]:
                audio, ts = self.raw[ident].popleft()
                buf = np.concatenate([self.pending[ident], audio])
                self.pending_ts[ident] = ts
                while buf.shape[0] >= n:
                    self._annotate(ident, vad.predict({"audio": buf[:n], "time_stamp": ts}), defer)
                    buf = buf[n:]
                self.pending[ident] = buf

    def _annotate(self, ident, ann, defer=None):
        status = ann["status"]
        if status == "ipu_sl":                                     # :484-526
            if self.current_ipu[ident] is not None:
                raise ValueError(f"We currently have IPU {self.current_ipu[ident].id}, but a new IPU start is detected.")
            self.total_ipus[ident] += 1
            ipu = IPURecord(self.total_ipus[ident], ident, ann["time_stamp"])
            self.current_ipu[ident] = ipu
            self.all_ipus[ident][ipu.id] = ipu
            if ident == "user":
                for outlet in self.user_ipu_outlet_list:
                    outlet(ipu)
                if self.event_outlet is not None:
                    self.event_outlet(ipu)
        elif status in ("ipu_cl", "ipu_el"):                       # :528-558
            ipu = self.current_ipu[ident]
            if ipu is None:
                return
            ipu.add_chunk(ann["audio"])
            if status == "ipu_el":
                ipu.set_end_timestamp(ann["time_stamp"])
                self.current_ipu[ident] = None
        else:
            return  # outside any IPU: the VAD thread forwards nothing to feature gating (:565-571)
        ann["ipu_id"] = self.current_ipu[ident].id if self.current_ipu[ident] is not None else ipu.id
        if self.socketio is not None:                              # :565-590
            ev.emit_vad_state_update(self.socketio, self.sid, status != "ipu_el", ident)
            ev.emit_vad_event(self.socketio, self.sid, status, ident)
            ev.emit_tm_audio_chunk(self.socketio, self.tm_sid, ident, status, ann["audio"], ann["time_stamp"],
                                   ann.get("cached_audio"))
        gater = self.feature_gater[ident]
        if defer is not None and hasattr(gater, "prepare"):
            defer.append((self, ident, ann, gater.prepare(ann)))
            return
        self._deliver(ident, ann, gater.process_and_gate(ann))

    def _deliver(self, ident, ann, gated):
        """Feature gating's output to the context serializer (:639-670)."""
        if not gated:
            return
        ser = self.context_serializer
        base = {"identity": ident, "time_stamp": ann["time_stamp"], "ipu_id": ann["ipu_id"]}
        if gated["status"] == "ipu_sl":                            # :639-670 onset replay
            last = gated["feature_last_chunk"]
            for i in range(len(last)):
                ser.add_feature_chunk(dict(base, feature=last[i], status="ipu_sl" if i == 0 else "ipu_cl"))
            ser.add_feature_chunk(dict(base, feature=gated["feature"],
                                       status="ipu_cl" if len(last) > 0 else "ipu_sl"))
        else:
            ser.add_feature_chunk(dict(base, feature=gated["feature"], status=gated["status"]))

    def next_feature(self):
        """The next serialized feature (serialize_context, :686-717), or None."""
        while self.context_serializer.feature_queue:
            f = self.context_serializer.get_next_feature()
            if f is not None:
                return f
        return None

    def request(self, data):
        """speech_dialogue keyword arguments of llm_prefill's call (:793-805)."""
        return dict(audio=data["feature"], identity=data["identity"], status=data["status"],
                    past_key_values=self.past_key_values, **self.caches[data["identity"]])

    def apply(self, data, result):
        """llm_prefill steps 3-4 (:808-844) + the IPU bookkeeping of predict_dialog_state (:758-770)."""
        probs, pkv, ada_cache, enc_cache, pe_index = result
        ident = data["identity"]
        self.past_key_values = pkv
        self.caches[ident] = {"encoder_cache": enc_cache, "adapter_cache": ada_cache, "pe_index": pe_index}
        state = None
        if ident == "user" and probs is not None:
            state = "dialog_ss" if probs["state_1"] > self.threshold else "dialog_cl"
            if state == "dialog_ss":
                ev.emit_dialog_ss_callback(self.socketio, self.sid)       # :826
                if self.dialog_state_callback is not None:
                    self.dialog_state_callback(self, data)
            ev.emit_dialog_state_update(self.socketio, self.sid, state)  # :833-837
        self.prediction_cnt += 1
        if ident == "user":
            ipu = self.all_ipus["user"].get(data["ipu_id"])
            if ipu is not None:
                ipu.register_response_state(state, self.prediction_cnt)
        self.states.append((ident, data["status"], state, probs))
        return state

    def llm_prefill(self, data):
        """One chunk through the pipeline on its own (the reference's per-session call)."""
        return self.apply(data, self.pipeline.speech_dialogue(**self.request(data)))


# every session's fbank rows of a tick in one launch (FO_DUPLEX_BATCH_FBANK=0: one launch per chunk, A/B only)
BATCH_FBANK = os.environ.get("FO_DUPLEX_BATCH_FBANK", "1") != "0"


def deliver_deferred(defer):
    """Gate the chunks DuplexSession.pump(defer) queued: every session's fbank rows in one launch (sessions whose
    gaters share a framing and device; models.AudioFeatureGating.fbank_batch), then each chunk finished and
    delivered in queue order, which is chunk order within every session and identity."""
    if not defer:
        return
    from models.AudioFeatureGating import fbank_batch
    gaters = [s.feature_gater[i] for s, i, _, _ in defer]
    # one launch per (framing, device) among the tick's gaters (one in practice); the batch's rows grouped by
    # identity (user rows, then system rows, each in queue order), so that one identity's features of the tick are
    # adjacent rows of one tensor and its encoder stage takes them with one copy
    groups = {}
    for q in sorted(range(len(defer)), key=lambda q: defer[q][1] != "user"):
        groups.setdefault((gaters[q].kind, str(gaters[q].device)), []).append(q)
    feats = [None] * len(defer)
    for order in groups.values():
        for q, f in zip(order, fbank_batch([gaters[q] for q in order], [defer[q][3] for q in order])):
            feats[q] = f
    for (s, ident, ann, _), f in zip(defer, feats):
        s._deliver(ident, ann, s.feature_gater[ident].finish(ann, f))


class DuplexScheduler:
    """Every duplex session of one replica (one GPU).  tick(): pump each session, take at most one
    serialized feature per session, and prefill all of them with ONE speech_dialogue_batch call."""

    def __init__(self, pipeline):
        self.pipeline = pipeline
        self.sessions = []

    def add(self, session):
        self.sessions.append(session)
        return session

    def tick(self):
        defer = [] if BATCH_FBANK else None
        for s in self.sessions:
            s.pump(defer)
        deliver_deferred(defer)
        work = []
        for s in self.sessions:
            d = s.next_feature()
            if d is not None:
                work.append((s, d))
        if not work:
            return []
        with torch.no_grad():
            results = self.pipeline.speech_dialogue_batch([s.request(d) for s, d in work])
        return [(s, d, s.apply(d, r)) for (s, d), r in zip(work, results)]

    def drain(self, max_ticks=1 << 30):
        n = 0
        while n < max_ticks:
            done = self.tick()
            if not done:
                break
            n += 1
        return n
