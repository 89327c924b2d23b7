"""llm2TTS on the MI355X engine (reference: models/decoder/llm2tts.py).

llm2TTS(model_path).run(hidden, top_k, prefix, codec_chunk_size=40, codec_padding_size=10,
penalty_window_size=-1, penalty=1.1, N=2401, seg_threshold=0.01) is a generator of [1, 1, S] device
PCM tensors (24 kHz) with the reference's chunking and emission rules; run_batch() serves many
sessions with one launch sequence per decode step.
"""
import os

import torch

from fo.codec import CodecEngine
from fo.engine import load_model_dir, make_source
from fo.speak import silence_cut, speak
from fo.tts import TTSEngine


class _SpeechEngine:
    def __init__(self, model_path, device, receive=False):
        self.device = torch.device(device)
        self.cfg, synth, _ = load_model_dir(model_path)
        src = make_source(self.cfg, synth, self.device, model_path, receive=receive)
        self.tts = TTSEngine(src, self.cfg["decoder_json"], self.device)
        self.codec = CodecEngine(src, self.cfg["codec_json"], self.device)


class llm2TTS:
    def __init__(self, model_path, device="cuda:0", weights_from=None):
        """weights_from: another llm2TTS whose frozen weights this one copies (fo.replica.copy_frozen)."""
        self.engine = _SpeechEngine(model_path, device, receive=weights_from is not None)
        if weights_from is not None:
            from fo.replica import copy_frozen
            copy_frozen(weights_from.engine, self.engine)
        self.model = self.engine.tts          # .vocab_size mirrors LLM2TTSCodecAR.vocab_size
        self.model.vocab_size = self.engine.tts.vocab
        self.codec_model = self.engine.codec

    def find_min_sum_index(self, buffer, syn, N, threshold):
        """Reference signature (models/decoder/llm2tts.py:70-112); tensors [1, 1, L] on the device."""
        res = torch.empty(2, dtype=torch.float32, device=syn.device)
        b = None if buffer is None or buffer.numel() == 0 else buffer.reshape(-1)
        nb, out = silence_cut(b, syn.reshape(-1).contiguous(), N, threshold, res)
        return nb.view(1, 1, -1), (None if out is None else out.view(1, 1, -1))

    # run() goes through the device's speech thread (fo.serve.SpeechScheduler): the reference gives every speaking
    # session an llm2TTS object of its own and calls run() from that session's thread (bin/pool.py:17-50); here the
    # concurrent sentences of every such object on one GPU decode together in one continuously batched AR decode,
    # each with the ids and PCM it gets alone.  FO_SERVE=0: run() decodes on the caller's thread (one caller only).
    SERVE = os.environ.get("FO_SERVE", "1") != "0"

    def run(self, hidden, top_k, prefix, codec_chunk_size=40, codec_padding_size=10, penalty_window_size=-1,
            penalty=1.1, N=2401, seg_threshold=0.01):
        if not self.SERVE:
            for _, seg in self.run_batch([(hidden, prefix)], top_k, codec_chunk_size, codec_padding_size,
                                         penalty_window_size, penalty, N, seg_threshold):
                yield seg.view(1, 1, -1)
            return
        from fo.serve import SpeechScheduler
        (h, p), = self._prepare([(hidden, prefix)])
        job = SpeechScheduler.for_device(self.engine.device).submit(
            self.engine, h, p, top_k, codec_chunk_size, codec_padding_size, N, seg_threshold,
            penalty_window_size=penalty_window_size if penalty_window_size is not None else -1, penalty=penalty)
        yield from job.segments()

    def _prepare(self, items):
        prepared = []
        for hidden, prefix in items:
            h = torch.as_tensor(hidden).reshape(-1, torch.as_tensor(hidden).shape[-1])
            p = None if prefix is None else torch.as_tensor(prefix).reshape(-1, h.shape[-1])
            prepared.append((h.to(self.engine.device, torch.float32).contiguous(),
                             None if p is None else p.to(self.engine.device, torch.float32).contiguous()))
        return prepared

    def run_batch(self, items, top_k, codec_chunk_size=40, codec_padding_size=10, penalty_window_size=-1,
                  penalty=1.1, N=2401, seg_threshold=0.01, max_tokens=1000, min_tokens=0):
        """Many sentences with one launch sequence per decode step, on the caller's thread (the single-caller batch
        form the benchmark uses; concurrent callers use run())."""
        prepared = self._prepare(items)
        yield from speak(self.engine, prepared, top_k=top_k, codec_chunk_size=codec_chunk_size,
                         codec_padding_size=codec_padding_size, N=N, seg_threshold=seg_threshold,
                         max_tokens=max_tokens, min_tokens=min_tokens, penalty_window_size=penalty_window_size,
                         penalty=penalty)
