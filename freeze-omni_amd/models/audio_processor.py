"""Drop-in for bin/inference.py's audioEncoderProcessor (bin/inference.py:43-80): 2560-sample chunks
-> [1, 19, 80] kaldi fbank features, computed on the GPU (framing A)."""
import numpy as np

from fo.speech import FbankGPU, Framer


class audioEncoderProcessor:
    def __init__(self, chunk_size=16, device="cuda:0"):
        self.chunk_size = 16
        self.chunk_overlap = 3
        self.feat_dim = 80
        self.frame_size = 400
        self.frame_shift = 160
        self.frame_overlap = self.frame_size - self.frame_shift
        self.CHUNK = self.frame_shift * self.chunk_size
        self.framer = Framer("A")
        self.fbank = FbankGPU("A", device)

    def get_chunk_size(self):
        return self.CHUNK

    def reset(self):
        self.framer.reset()

    def process(self, audio):
        a = audio.numpy() if hasattr(audio, "numpy") else np.asarray(audio)
        w, first = self.framer.push(np.asarray(a, dtype=np.float32).reshape(-1))
        return self.fbank(w[None], [first])  # [1, 19, 80] on the device
