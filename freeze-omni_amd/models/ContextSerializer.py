"""Timestamp-ordered serialisation of user/system audio features for one shared LLM context
(reference behaviour: models/ContextSerializer.py:30-121).

Rules: features are released earliest-timestamp first; user features are always forwarded and track
whether the user is inside an IPU (ipu_sl/ipu_cl -> inside, ipu_el -> outside); system features are
dropped while the user is inside an IPU, and the first system feature of each run is re-labelled
'ipu_sl' so the chat prefix is inserted.
"""
import heapq


class ContextSerializer:
    def __init__(self):
        self.reset()

    def reset(self):
        self.user_in_actual_ipu = False
        self.system_in_pseudo_ipu = False
        self.feature_queue = []
        self._seq = 0

    def add_feature_chunk(self, feature_chunk):
        # heap key (timestamp, identity, status) as the reference's tuple; an arrival counter breaks the
        # remaining ties so feature payloads (device tensors here) are never compared
        entry = (feature_chunk.get("time_stamp"), feature_chunk.get("identity"), feature_chunk.get("status"),
                 self._seq, feature_chunk.get("feature"), feature_chunk.get("ipu_id"))
        self._seq += 1
        heapq.heappush(self.feature_queue, entry)

    def gate_feature(self, identity, status):
        if identity == "user":
            if status in ("ipu_sl", "ipu_cl"):
                self.user_in_actual_ipu = True
            elif status == "ipu_el":
                self.user_in_actual_ipu = False
            self.system_in_pseudo_ipu = False
            return True, False
        if identity == "system" and not self.user_in_actual_ipu:
            first = not self.system_in_pseudo_ipu
            self.system_in_pseudo_ipu = True
            return True, first
        return False, False

    def get_next_feature(self):
        if not self.feature_queue:
            return None
        ts, identity, status, _, feature, ipu_id = heapq.heappop(self.feature_queue)
        send, force_sl = self.gate_feature(identity, status)
        if not send:
            return None
        return {"time_stamp": ts, "identity": identity, "status": "ipu_sl" if force_sl else status,
                "feature": feature, "ipu_id": ipu_id}
