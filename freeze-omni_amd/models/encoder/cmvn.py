"""CMVN statistics loaders (reference: models/encoder/cmvn.py:37-107): json and kaldi-text formats
-> (mean, istd) numpy arrays.  The normalisation itself is fused into the encoder's first im2col."""
import json
import math

import numpy as np


def _finish(means, var_sums, count):
    mean = [m / count for m in means]
    istd = []
    for m, v in zip(mean, var_sums):
        var = v / count - m * m
        istd.append(1.0 / math.sqrt(max(var, 1.0e-20)))
    return np.array(mean), np.array(istd)


def load_json_cmvn(path):
    with open(path) as f:
        st = json.load(f)
    return _finish(st["mean_stat"], st["var_stat"], st["frame_num"])


def load_kaldi_cmvn(path):
    with open(path) as f:
        head = f.read(2)
        if head == "\0B":
            raise ValueError("kaldi binary cmvn is not supported; recompute with compute-cmvn-stats --binary=false")
        f.seek(0)
        arr = f.read().split()
    if arr[0] != "[" or arr[-2] != "0" or arr[-1] != "]":
        raise ValueError(f"{path}: not a kaldi text cmvn file")
    d = (len(arr) - 4) // 2
    means = [float(x) for x in arr[1:d + 1]]
    count = float(arr[d + 1])
    var = [float(x) for x in arr[d + 2:2 * d + 2]]
    return _finish(means, var, count)


def load_cmvn(cmvn_file, is_json):
    return load_json_cmvn(cmvn_file) if is_json else load_kaldi_cmvn(cmvn_file)


class GlobalCMVN:
    """GlobalCMVN(mean, istd, norm_var=True) (reference: models/encoder/cmvn.py:7-35): the statistics a
    speechEncoder folds into its first kernel ((x - mean) * istd; norm_var=False subtracts the mean only).
    It is a parameter holder here: the normalisation runs inside the encoder's im2col on the device."""

    def __init__(self, mean, istd, norm_var=True):
        import torch
        self.mean = torch.as_tensor(mean).float()
        self.istd = torch.as_tensor(istd).float() if norm_var else torch.ones_like(self.mean)
        self.norm_var = norm_var
