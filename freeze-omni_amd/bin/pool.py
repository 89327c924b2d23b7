"""Model-as-a-Server object pools (reference: bin/pool.py:17-91), replica-aware, thread-safe.

TTSObjectPool: first free object, raises when exhausted.  pipelineObjectPool: least-loaded replica.
configs may carry 'devices' (e.g. ['cuda:0', ..., 'cuda:7']): replica i is placed on
devices[i % len(devices)], so one pool spans the GPUs of a node as data-parallel replicas (sessions
stay pinned to the replica that admitted them, their KV lives there).  As in the one-process-per-GPU
launch (bench.py, fo.replica.broadcast_frozen), only the first replica reads or generates the frozen
weights; every other replica allocates the packed layouts receive-only and is filled from it device to
device (fo.replica.copy_frozen, xGMI peer copies between GPUs), checksum-verified.

The reference's acquire / release mutate the counters from many session threads without a lock (bin/pool.py:
79-87); here every counter change happens under the pool's lock.

Replica loss (README.md:42: "any model ... could respond to any chunk of any user", because every cache lives with
the user): a replica whose device call fails with a RuntimeError is marked unhealthy and admits no new session.
PooledSession is the caller-side handle that survives it: it keeps the session's history (system role and every
chunk it fed, on the host), and when its replica fails it re-pins to the least-loaded healthy one and re-prefills
that history there before serving the chunk again.
"""
import threading

import numpy as np

from models.decoder.llm2tts import llm2TTS
from models.pipeline import inferencePipeline


class PooledCodecTTSObject:
    def __init__(self, model_path, device="cuda:0", weights_from=None):
        self.in_use = False
        self.tts_proc = llm2TTS(model_path, device=device,
                                weights_from=None if weights_from is None else weights_from.tts_proc)


class TTSObjectPool:
    def __init__(self, size=10, model_path="", devices=None, factory=None):
        """factory(model_path, device, weights_from) -> pooled object (default PooledCodecTTSObject; tests)."""
        devices = devices or ["cuda:0"]
        factory = factory or PooledCodecTTSObject
        self.lock = threading.Lock()
        self.pool = []
        for i in range(size):
            self.pool.append(factory(model_path, devices[i % len(devices)], self.pool[0] if self.pool else None))

    def acquire(self):
        with self.lock:
            for obj in self.pool:
                if not obj.in_use:
                    obj.in_use = True
                    return obj
        raise Exception("No available objects in the pool")

    def release(self, obj):
        with self.lock:
            obj.in_use = False

    def print_info(self):
        with self.lock:
            for i, obj in enumerate(self.pool):
                print(f"TTS Object {i} is in use: {obj.in_use}")


class inferencePipelineObject:
    def __init__(self, configs, weights_from=None, factory=None):
        self.user_count = 0
        self.healthy = True
        self.pipeline_proc = (factory or inferencePipeline)(
            configs, weights_from=None if weights_from is None else weights_from.pipeline_proc)
        self.id = self.pipeline_proc.id


class pipelineObjectPool:
    def __init__(self, size, configs, factory=None):
        """factory(configs, weights_from=...) -> pipeline (default models.pipeline.inferencePipeline; tests)."""
        devices = configs.get("devices") if isinstance(configs, dict) else None
        self.lock = threading.Lock()
        self.pool = []
        for i in range(size):
            c = dict(configs) if isinstance(configs, dict) else configs
            if devices:
                c["device"] = devices[i % len(devices)]
            self.pool.append(inferencePipelineObject(c, weights_from=self.pool[0] if self.pool else None,
                                                     factory=factory))

    def acquire(self):
        """The least-loaded healthy replica (bin/pool.py:79-83), its count taken under the lock."""
        with self.lock:
            live = [o for o in self.pool if o.healthy]
            if not live:
                raise Exception("No healthy pipeline object in the pool")
            obj = min(live, key=lambda o: o.user_count)
            obj.user_count += 1
            return obj

    def release(self, obj):
        with self.lock:
            if obj.user_count > 0:
                obj.user_count -= 1

    def mark_failed(self, obj):
        """A replica whose device failed: it admits no new session (its sessions re-pin, PooledSession)."""
        with self.lock:
            obj.healthy = False

    def print_info(self):
        with self.lock:
            for i, obj in enumerate(self.pool):
                print(f"Pipeline Object {i} user count: {obj.user_count}" + ("" if obj.healthy else " (failed)"))


class PooledSession:
    """One user session pinned to a replica of a pipelineObjectPool, in the fork form of speech_dialogue
    (bin/dialog_state_pred.py:777-844), that survives the loss of its replica.

    The session's device state (KV pages, encoder / adapter caches) lives on its replica; its history -- the role
    and every (features, identity, status) chunk it fed -- is kept on the host by this handle.  When a call fails
    with a RuntimeError (a device fault, a lost GPU), the replica is marked failed, the session is re-pinned to the
    least-loaded healthy replica, the history is re-prefilled there (the same chunks in the same order: the same
    context), and the chunk is served again.  Protocol errors (AssertionError, ValueError) are the caller's and
    propagate unchanged."""

    def __init__(self, pool, role=None):
        self.pool, self.role = pool, role
        self.history = []
        self.repins = 0
        self.obj = pool.acquire()
        try:
            self._open()
        except BaseException:
            pool.release(self.obj)
            raise

    def _open(self):
        p = self.obj.pipeline_proc
        _, self.past_key_values, _, _, _ = p.speech_dialogue(None, identity="", status="pre", role=self.role)
        self.caches = {i: {"adapter_cache": None, "encoder_cache": None, "pe_index": 0} for i in ("user", "system")}

    def _feed(self, audio, identity, status):
        probs, pkv, ac, ec, pe = self.obj.pipeline_proc.speech_dialogue(
            audio, identity=identity, status=status, past_key_values=self.past_key_values,
            **self.caches.get(identity, {}))
        self.past_key_values = pkv
        self.caches[identity] = {"adapter_cache": ac, "encoder_cache": ec, "pe_index": pe}
        return probs

    def speech_dialogue(self, audio, identity, status):
        """One chunk; returns the prediction probs (or None) as the fork form does."""
        host = np.array(audio.detach().cpu() if hasattr(audio, "detach") else audio, dtype=np.float32, copy=True)
        src = audio
        while True:
            try:
                probs = self._feed(src, identity, status)
                break
            except RuntimeError:
                self._repin()   # raises once no healthy replica is left
                src = host
        self.history.append((host, identity, status))
        return probs

    def _repin(self):
        """Move to the least-loaded healthy replica and re-prefill the history there; a replica that fails meanwhile
        is marked too and the next one tried, until none is left (pool.acquire raises)."""
        while True:
            old = self.obj
            self.pool.mark_failed(old)
            self.pool.release(old)
            self.obj = None
            self.obj = self.pool.acquire()
            self.repins += 1
            try:
                self._open()
                for audio, identity, status in self.history:
                    self._feed(audio, identity, status)
                return
            except RuntimeError:
                continue

    def release(self):
        if self.obj is not None:
            self.pool.release(self.obj)
            self.obj = None
