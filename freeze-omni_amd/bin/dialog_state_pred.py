"""DialogStateParams (reference: bin/dialog_state_pred.py:65-844) on the MI355X engine.

Same class name, constructor arguments, public methods and decision rule as the reference's duplex
session; the five polling threads become synchronous stages (fo.duplex.DuplexSession.pump) and every
session of a replica is prefilled in one batched launch sequence per tick by the replica's
fo.duplex.DuplexScheduler (start_all_threads registers the session with it; run_scheduler() or
tick() drives it).  Transport: `socketio` is any object with
emit(event, data, to=sid) -- bin/server.py's hub -- and receives the reference's emits (VAD state and
events, dialog_ss, dialog state updates, and 'tm_audio_chunk' to the task manager's sid; web/emit.py).
"""
import os

import yaml

from bin.pool import pipelineObjectPool
from fo.duplex import DEFAULT_CONFIG, DuplexScheduler, DuplexSession

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def get_args(path=None):
    """The duplex YAML (reference get_args, :40-49): configs/dialog_state_pred_config.yaml keys;
    `path` or $FO_DIALOG_CONFIG, else the fork's defaults with the bundled synthetic model."""
    path = path or os.environ.get("FO_DIALOG_CONFIG")
    if path:
        with open(path) as f:
            return yaml.safe_load(f)
    cfg = dict(DEFAULT_CONFIG)
    cfg.update(model_path=os.path.join(ROOT, "configs", "real"), llm_path=None, device="cuda:0",
               thread_sleep_interval=0.005, debug_time=False)
    return cfg


class DialogStateParams(DuplexSession):
    DIALOG_STATE_PRED_CONFIGS = None
    MAX_PIPELINE_NUN = 1
    PIPELINE_POOL = None
    SCHEDULERS = {}   # pipeline id -> DuplexScheduler (one per replica)

    @classmethod
    def _pool(cls):
        if cls.PIPELINE_POOL is None:
            if cls.DIALOG_STATE_PRED_CONFIGS is None:
                cls.DIALOG_STATE_PRED_CONFIGS = get_args()
            c = cls.DIALOG_STATE_PRED_CONFIGS
            ic = c.get("inference_control", {})
            cls.PIPELINE_POOL = pipelineObjectPool(size=cls.MAX_PIPELINE_NUN, configs={
                "model_path": c["model_path"], "llm_path": c.get("llm_path"), "device": c.get("device", "cuda:0"),
                "top_k": ic.get("top_k", 1), "top_p": ic.get("top_p", 0.0), "temperature": ic.get("temperature", 1.0)})
        return cls.PIPELINE_POOL

    def __init__(self, sid, socketio=None, event_outlet=None, user_ipu_outlet_list=(), parent_logger=None, vad=None):
        self.pipeline_pool = self._pool()
        self.pipeline_obj = self.pipeline_pool.acquire()
        if self.pipeline_obj is None:
            raise Exception("Failed to get pipeline object from pool")
        self.tm_sid = None
        try:
            super().__init__(self.pipeline_obj.pipeline_proc, sid, self.DIALOG_STATE_PRED_CONFIGS, vad=vad,
                             event_outlet=event_outlet, user_ipu_outlet_list=user_ipu_outlet_list,
                             socketio=socketio)
        except Exception:
            self.pipeline_pool.release(self.pipeline_obj)
            raise

    def set_tm_sid(self, tm_sid):
        self.tm_sid = tm_sid

    @property
    def scheduler(self):
        key = self.pipeline_obj.id
        if key not in self.SCHEDULERS:
            self.SCHEDULERS[key] = DuplexScheduler(self.pipeline_obj.pipeline_proc)
        return self.SCHEDULERS[key]

    def start_all_threads(self):
        """The reference starts five polling threads per session (:240-288); here the session joins its
        replica's scheduler, which batches it with every other session on that GPU."""
        if self not in self.scheduler.sessions:
            self.scheduler.add(self)

    def tick(self):
        """One scheduler step of this session's replica (all of its sessions)."""
        return self.scheduler.tick()

    def run_scheduler(self):
        return self.scheduler.drain()

    def release(self):
        sch = self.SCHEDULERS.get(self.pipeline_obj.id) if self.pipeline_obj is not None else None
        if sch is not None and self in sch.sessions:
            sch.sessions.remove(self)
        super().release()
        if self.pipeline_obj is not None:
            self.pipeline_pool.release(self.pipeline_obj)
            self.pipeline_obj = None
