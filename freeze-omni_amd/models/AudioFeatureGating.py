"""Stateful fbank extraction + VAD gating for the duplex path (reference: models/AudioFeatureGating.py).

Same constructor, process_and_gate(dict) contract and output format as the reference (features as
nested lists unless as_tensor=True); the kaldi fbank runs on the GPU (fo_fbank) and the carried frames
are recomputed from the retained samples instead of being kept on the host.
"""
import numpy as np
import torch

from fo.speech import FRAMINGS, FbankGPU, Framer

_DEFAULT = {"feat_dim": 80, "expected_audio_chunk_duration_in_sec": 0.16, "audio_to_proc_per_step_in_sec": 0.025,
            "step_size_in_sec": 0.01, "context_duration_in_sec": 0.03}


def _framing_for(cfg, sr):
    wl = int(cfg["audio_to_proc_per_step_in_sec"] * sr)
    ws = int(cfg["step_size_in_sec"] * sr)
    for k, (nf, ov, w, s, nfft, scale) in FRAMINGS.items():
        if w == wl and s == ws:
            return k
    raise ValueError(f"no fbank framing for window {wl} / shift {ws} samples")


class AudioFeatureGating:
    def __init__(self, sample_rate, cache_history_size=10, onset_input_chunk_cache_size=6, fbank_config=None,
                 device="cuda:0", as_tensor=False):
        cfg = dict(fbank_config or _DEFAULT)
        self.sample_rate = sample_rate
        self.cache_history_size = cache_history_size
        self.onset_input_chunk_cache_size = onset_input_chunk_cache_size
        self.feat_dim = cfg["feat_dim"]
        self.step_size_in_frames = int(cfg["step_size_in_sec"] * sample_rate)
        self.step_cnt_per_chunk = int(cfg["expected_audio_chunk_duration_in_sec"] / cfg["step_size_in_sec"])
        self.context_step_cnt = int(cfg["context_duration_in_sec"] / cfg["step_size_in_sec"])
        self.expected_frames_per_audio_chunk = self.step_size_in_frames * self.step_cnt_per_chunk
        self.kind = _framing_for(cfg, sample_rate)
        nf, ov = FRAMINGS[self.kind][:2]
        if (nf, ov) != (self.step_cnt_per_chunk, self.context_step_cnt):
            raise ValueError(f"fbank config does not match framing {self.kind}")
        self.device = torch.device(device)
        self.as_tensor = as_tensor
        self.framer = Framer(self.kind)
        self.fbank = FbankGPU(self.kind, self.device)
        self.reset()

    def reset(self):
        self.framer.reset()
        self.history = torch.zeros(self.cache_history_size, self.step_cnt_per_chunk + self.context_step_cnt,
                                   self.feat_dim, device=self.device)

    def _extract_fbank(self, audio_chunk):
        # the reference scales by 32767 here (models/AudioFeatureGating.py:58); FRAMINGS['B'] does the same
        w, first = self.framer.push(np.asarray(audio_chunk, dtype=np.float32))
        return self.fbank(w[None], [first])  # [1, R, 80] device

    def process_and_gate(self, annotated_audio):
        return self.finish(annotated_audio, self.fbank(*self._one(self.prepare(annotated_audio))))

    @staticmethod
    def _one(req):
        w, first = req
        return w[None], [first]

    # process_and_gate in two halves, so that a scheduler holding many gaters (fo.duplex.DuplexScheduler) frames
    # every session's chunk first and computes all their fbank rows in one launch (fbank_batch)
    def prepare(self, annotated_audio):
        """Host half: push the chunk through the framer (the carried samples advance here).  Returns the fbank
        request (window [n_samples] float32, first chunk?) that finish() consumes, in chunk order."""
        return self.framer.push(np.asarray(annotated_audio["audio"], dtype=np.float32))

    def finish(self, annotated_audio, feat):
        """Device half: feat = this chunk's fbank rows [1, R, 80] (device) -> the gated output, or None outside
        an IPU (the chunk then only enters the onset history)."""
        status = annotated_audio["status"]
        if status is None:
            if self.cache_history_size > 0:
                self.history = torch.cat([self.history[1:], feat])
            return None
        out = {"feature": feat if self.as_tensor else feat.cpu().numpy().tolist(), "status": status,
               "feature_last_chunk": []}
        if status == "ipu_sl" and self.onset_input_chunk_cache_size > 0:
            last = self.history[-self.onset_input_chunk_cache_size:].unsqueeze(1)
            out["feature_last_chunk"] = last if self.as_tensor else last.cpu().numpy().tolist()
        return out


def fbank_batch(gaters, requests):
    """One fbank launch for chunks prepared by several gaters of the same framing and device (one row per
    request; k_fbank computes every (row, frame) on its own, so each row equals its single-chunk launch).
    Returns each request's [1, R, 80] device rows."""
    g0 = gaters[0]
    for g in gaters:
        if g.kind != g0.kind or g.device != g0.device:
            raise ValueError("fbank_batch: gaters of different framings or devices")
    feats = g0.fbank(np.stack([w for w, _ in requests]), [f for _, f in requests])
    return [feats[i:i + 1] for i in range(len(requests))]
