"""Model-as-a-Server object pools (reference: bin/pool.py:17-91), replica-aware.

TTSObjectPool: first free object, raises when exhausted.  pipelineObjectPool: least-loaded replica.
configs may carry 'devices' (e.g. ['cuda:0', ..., 'cuda:7']): replica i is placed on
devices[i % len(devices)], so one pool spans the GPUs of a node as data-parallel replicas (sessions
stay pinned to the replica that admitted them, their KV lives there).  As in the one-process-per-GPU
launch (bench.py, fo.replica.broadcast_frozen), only the first replica reads or generates the frozen
weights; every other replica allocates the packed layouts receive-only and is filled from it device to
device (fo.replica.copy_frozen, xGMI peer copies between GPUs), checksum-verified.
"""
from models.decoder.llm2tts import llm2TTS
from models.pipeline import inferencePipeline


class PooledCodecTTSObject:
    def __init__(self, model_path, device="cuda:0", weights_from=None):
        self.in_use = False
        self.tts_proc = llm2TTS(model_path, device=device,
                                weights_from=None if weights_from is None else weights_from.tts_proc)


class TTSObjectPool:
    def __init__(self, size=10, model_path="", devices=None):
        devices = devices or ["cuda:0"]
        self.pool = []
        for i in range(size):
            self.pool.append(PooledCodecTTSObject(model_path, devices[i % len(devices)],
                                                  weights_from=self.pool[0] if self.pool else None))

    def acquire(self):
        for obj in self.pool:
            if not obj.in_use:
                obj.in_use = True
                return obj
        raise Exception("No available objects in the pool")

    def release(self, obj):
        obj.in_use = False

    def print_info(self):
        for i, obj in enumerate(self.pool):
            print(f"TTS Object {i} is in use: {obj.in_use}")


class inferencePipelineObject:
    def __init__(self, configs, weights_from=None):
        self.user_count = 0
        self.pipeline_proc = inferencePipeline(configs, weights_from=None if weights_from is None
                                               else weights_from.pipeline_proc)
        self.id = self.pipeline_proc.id


class pipelineObjectPool:
    def __init__(self, size, configs):
        devices = configs.get("devices") if isinstance(configs, dict) else None
        self.pool = []
        for i in range(size):
            c = dict(configs) if isinstance(configs, dict) else configs
            if devices:
                c["device"] = devices[i % len(devices)]
            self.pool.append(inferencePipelineObject(c, weights_from=self.pool[0] if self.pool else None))

    def acquire(self):
        obj = min(self.pool, key=lambda o: o.user_count)
        obj.user_count += 1
        return obj

    def release(self, obj):
        if obj.user_count > 0:
            obj.user_count -= 1

    def print_info(self):
        for i, obj in enumerate(self.pool):
            print(f"Pipeline Object {i} user count: {obj.user_count}")
