"""Host-precomputed constant tables (computed once, uploaded, read by kernels).

* kaldi fbank window / FFT twiddles / mel banks (torchaudio.compliance.kaldi get_mel_banks &
  povey window, as used at bin/inference.py:77 and models/AudioFeatureGating.py:65)
* RoPE cos/sin per position (transformers rotary: inv_freq in fp32, angle pos*inv_freq in fp32,
  cast to the embeds dtype: fp16 for Qwen2 fed .half() embeds, models/audioLLM.py:338,410)
* rel-pos sinusoid rows (models/encoder/attention.py:105-121, fp32 like the reference)
"""
import math

import numpy as np
import torch


def kaldi_tables(wl, nfft, num_bins=80, sample_freq=16000.0, low_freq=20.0):
    n = np.arange(wl, dtype=np.float64)
    window = (0.5 - 0.5 * np.cos(2.0 * np.pi * n / (wl - 1))) ** 0.85
    k = np.arange(nfft // 2, dtype=np.float64)
    tw_cos = np.cos(2.0 * np.pi * k / nfft)
    tw_sin = np.sin(2.0 * np.pi * k / nfft)

    def mel(f):
        return 1127.0 * np.log(1.0 + f / 700.0)

    nyq = 0.5 * sample_freq
    width = sample_freq / nfft
    ml, mh = mel(low_freq), mel(nyq)
    delta = (mh - ml) / (num_bins + 1)
    b = np.arange(num_bins, dtype=np.float64)[:, None]
    left, center, right = ml + b * delta, ml + (b + 1) * delta, ml + (b + 2) * delta
    m = mel(width * np.arange(nfft // 2, dtype=np.float64))[None, :]
    banks = np.maximum(0.0, np.minimum((m - left) / (center - left), (right - m) / (right - center)))
    banks = np.concatenate([banks, np.zeros((num_bins, 1))], axis=1)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))  # noqa: E731
    return f32(window), f32(tw_cos), f32(tw_sin), f32(banks)


def rope_tables(theta, hd, max_pos, round_fp16):
    """cos/sin [max_pos][hd/2] for rotate_half RoPE."""
    inv = 1.0 / (torch.tensor(float(theta), dtype=torch.float32) **
                 (torch.arange(0, hd, 2, dtype=torch.int64).float() / hd))
    pos = torch.arange(max_pos, dtype=torch.float32)[:, None]
    ang = pos * inv[None, :]
    c, s = torch.cos(ang), torch.sin(ang)
    if round_fp16:
        c, s = c.half().float(), s.half().float()
    return c.contiguous(), s.contiguous()


def relpos_sinusoid(n_pos, d):
    """pe[p] = interleaved sin/cos(p * div_term) for p in [0, n_pos)."""
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pos = torch.arange(n_pos, dtype=torch.float32).unsqueeze(1)
    pe = torch.zeros(n_pos, d)
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe
