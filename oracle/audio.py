"""Oracle (TEST INFRASTRUCTURE): CPU restatement of the audio front end, numpy only.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker; the
product path never imports this package.

Parity pinning: torchaudio 2.2.0 (pinned at requirements.txt:9) is absent from the container, so
kaldi_fbank below restates its published algorithm (torchaudio/compliance/kaldi.py: fbank ->
_get_window -> get_mel_banks) and is pinned against tests/golden/fbank.npz, which the reference's
own framing code (bin/inference.py:43-80, models/AudioFeatureGating.py:54-75) produced with
transformers.audio_utils' documented kaldi restatement standing in for torchaudio.
"""
import numpy as np

EPS_F32 = np.float32(np.finfo(np.float32).eps)


def mel_scale(f):
    return 1127.0 * np.log(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def mel_banks(num_bins, nfft, sample_freq=16000.0, low_freq=20.0, high_freq=0.0):
    """torchaudio.compliance.kaldi.get_mel_banks (no VTLN) -> [num_bins, nfft//2 + 1] (last column 0)."""
    num_fft_bins = nfft // 2
    nyquist = 0.5 * sample_freq
    if high_freq <= 0.0:
        high_freq += nyquist
    fft_bin_width = sample_freq / nfft
    mel_low, mel_high = mel_scale(low_freq), mel_scale(high_freq)
    delta = (mel_high - mel_low) / (num_bins + 1)
    b = np.arange(num_bins, dtype=np.float64)[:, None]
    left = mel_low + b * delta
    center = mel_low + (b + 1.0) * delta
    right = mel_low + (b + 2.0) * delta
    mel = mel_scale(fft_bin_width * np.arange(num_fft_bins, dtype=np.float64))[None, :]
    up = (mel - left) / (center - left)
    down = (right - mel) / (right - center)
    banks = np.maximum(0.0, np.minimum(up, down))
    return np.concatenate([banks, np.zeros((num_bins, 1))], axis=1)


def povey_window(wl):
    n = np.arange(wl, dtype=np.float64)
    hann = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / (wl - 1))  # torch.hann_window(periodic=False)
    return hann ** 0.85


def kaldi_fbank(wave, frame_length_ms=25.0, frame_shift_ms=10.0, num_mel_bins=80, sample_freq=16000.0):
    """kaldi fbank with the reference's arguments (dither=0, snip_edges, povey, preemph 0.97,
    remove DC, power spectrum, log(max(x, f32 eps))).  wave: 1-D samples already x32768/x32767."""
    x = np.asarray(wave, dtype=np.float64)
    wl = int(sample_freq * frame_length_ms * 0.001)
    ws = int(sample_freq * frame_shift_ms * 0.001)
    nfft = 1 << (wl - 1).bit_length()
    n_frames = 1 + (len(x) - wl) // ws
    if n_frames <= 0:
        return np.zeros((0, num_mel_bins), np.float32)
    idx = np.arange(wl)[None, :] + ws * np.arange(n_frames)[:, None]
    fr = x[idx]
    fr = fr - fr.mean(axis=1, keepdims=True)
    prev = np.concatenate([fr[:, :1], fr[:, :-1]], axis=1)
    fr = (fr - 0.97 * prev) * povey_window(wl)[None, :]
    spec = np.abs(np.fft.rfft(fr, n=nfft, axis=1)) ** 2
    mel = spec @ mel_banks(num_mel_bins, nfft, sample_freq).T
    return np.log(np.maximum(mel, float(EPS_F32))).astype(np.float32)


class EncoderFraming:
    """bin/inference.py:43-80 audioEncoderProcessor (framing A: 16 frames + 3 carried)."""

    def __init__(self, chunk_size=16, chunk_overlap=3, frame_size=400, frame_shift=160, scale=32768.0,
                 frame_length_ms=25.0, frame_shift_ms=10.0):
        self.chunk_size, self.chunk_overlap = chunk_size, chunk_overlap
        self.frame_overlap = frame_size - frame_shift
        self.CHUNK = frame_shift * chunk_size
        self.scale = scale
        self.fl, self.fs = frame_length_ms, frame_shift_ms
        self.reset()

    def reset(self):
        self.input_chunk = np.zeros((self.chunk_size + self.chunk_overlap, 80), np.float32)
        self.input_sample = np.zeros(self.CHUNK + self.frame_overlap, np.float32)

    def process(self, audio):
        s = np.asarray(audio, dtype=np.float32).reshape(-1) * np.float32(self.scale)
        self.input_sample[:self.frame_overlap] = self.input_sample[-self.frame_overlap:].copy()
        self.input_sample[self.frame_overlap:] = s
        xs = kaldi_fbank(self.input_sample, self.fl, self.fs)
        self.input_chunk[:self.chunk_overlap] = self.input_chunk[-self.chunk_overlap:].copy()
        self.input_chunk[self.chunk_overlap:] = xs
        return self.input_chunk[None].copy()


def framing_b():
    """models/AudioFeatureGating.py:33-45 with configs/dialog_state_pred_config.yaml:24-29."""
    sr = 16000
    fl, fs, chunk_s, ctx_s = 0.016, 0.008, 0.224, 0.032
    frames_per_step = int(fl * sr)
    step = int(fs * sr)
    steps = int(chunk_s / fs)
    ctx = int(ctx_s / fs)
    f = EncoderFraming(chunk_size=steps, chunk_overlap=ctx, frame_size=frames_per_step, frame_shift=step,
                       scale=32767.0, frame_length_ms=fl * 1000, frame_shift_ms=fs * 1000)
    return f
