"""Event emission of the duplex session (server transport).

The reference's session (bin/dialog_state_pred.py) emits through helpers of the absent
FloorState.floor_state_emission module (`from FloorState.floor_state_emission import *`, :34) and
socketio.emit:
  * emit_vad_state_update / emit_vad_event  per VAD-labelled chunk inside an IPU   (:565-568)
  * 'tm_audio_chunk' to the task manager's sid                                    (:573-590)
  * emit_dialog_ss_callback                 when state_1 > threshold              (:818-826)
  * emit_dialog_state_update                after every user prediction           (:832-837)
The helpers keep the reference's names and keyword arguments; their event names and payload keys
are this build's (the module that defined them is not in the snapshot).  The 'tm_audio_chunk' payload
follows :577-585 exactly.  `socketio` is anything with emit(event, data, to=sid): the transport of
bin/server.py, or None (then nothing is sent).
"""
import numpy as np

EV_VAD_STATE = "vad_state_update"
EV_VAD_EVENT = "vad_event"
EV_DIALOG_SS = "dialog_ss"
EV_DIALOG_STATE = "dialog_state_update"
EV_TM_AUDIO = "tm_audio_chunk"


def np_float32_audio_to_np_int16_audio(audio):
    """float32 samples in [-1, 1] -> int16 (utils.audio_helpers, absent upstream; the inverse of the
    receive path's int16 / 32767, bin/dialog_state_pred.py:384).  Out-of-range samples saturate."""
    a = np.asarray(audio, dtype=np.float32)
    return np.clip(np.rint(a * 32767.0), -32768, 32767).astype(np.int16)


def _emit(socketio, event, data, sid):
    if socketio is not None:
        socketio.emit(event, data, to=sid)


def emit_vad_state_update(socketio, sid, vad_state, identity):
    _emit(socketio, EV_VAD_STATE, {"vad_state": bool(vad_state), "identity": identity}, sid)


def emit_vad_event(socketio, sid, event_type, identity):
    _emit(socketio, EV_VAD_EVENT, {"event_type": event_type, "identity": identity}, sid)


def emit_dialog_ss_callback(socketio, sid):
    _emit(socketio, EV_DIALOG_SS, {"sid": sid}, sid)


def emit_dialog_state_update(socketio, sid, dialog_state):
    _emit(socketio, EV_DIALOG_STATE, {"dialog_state": dialog_state}, sid)


def tm_audio_chunk_payload(identity, status, audio, time_stamp, cached_audio=None):
    """The JSON-serialisable chunk the task manager receives (bin/dialog_state_pred.py:577-585)."""
    return {
        "identity": identity,
        "status": status,
        "audio_int_list": np_float32_audio_to_np_int16_audio(audio).tolist(),
        "time_stamp": time_stamp,
        "cached_audio_int_list": [np_float32_audio_to_np_int16_audio(c).tolist() for c in cached_audio]
        if cached_audio is not None else [],
    }


def emit_tm_audio_chunk(socketio, tm_sid, identity, status, audio, time_stamp, cached_audio=None):
    if tm_sid is not None:
        _emit(socketio, EV_TM_AUDIO, tm_audio_chunk_payload(identity, status, audio, time_stamp, cached_audio), tm_sid)
