"""Host side of the offline driver (freeze-omni_amd/bin/inference.py; reference bin/inference.py):
command line, wav I/O and resampling. No GPU calls."""
import numpy as np


def _mod():
    import importlib
    return importlib.import_module("bin.inference")


def test_args_mirror_reference_cli():
    a = _mod().get_args(["--model_path", "m", "--llm_path", "l", "--input_wav", "i.wav", "--output_wav", "o.wav"])
    # bin/inference.py:29-41 defaults
    assert (a.top_k, a.top_p, a.temperature) == (5, 0.8, 0.7)
    assert a.model_path == "m" and a.llm_path == "l" and a.input_wav == "i.wav" and a.output_wav == "o.wav"
    assert a.max_text_tokens == 128


def test_wav_roundtrip_int16_exact(tmp_path):
    m = _mod()
    rng = np.random.default_rng(0)
    q = rng.integers(-32768, 32767, size=4000).astype(np.int16)
    p = str(tmp_path / "x.wav")
    m.write_wav(p, q.astype(np.float64) / 32768.0, 16000)
    x, fs = m.read_wav(p)
    assert fs == 16000 and x.dtype == np.float64
    np.testing.assert_array_equal(np.round(x * 32768.0).astype(np.int16), q)
    m.write_wav(p, np.array([2.0, -2.0]), 24000)         # clipped, not wrapped
    y, fs = m.read_wav(p)
    assert fs == 24000 and y[0] == 32767 / 32768.0 and y[1] == -1.0


def test_float_wav_and_resample(tmp_path):
    from scipy.io import wavfile
    m = _mod()
    t = np.arange(48000) / 48000.0
    x = (0.5 * np.sin(2 * np.pi * 440.0 * t)).astype(np.float32)
    p = str(tmp_path / "f.wav")
    wavfile.write(p, 48000, x)
    y, fs = m.read_wav(p)
    assert fs == 48000
    z = m.resample_to_16k(y, fs)
    assert z.shape[0] == 16000
    # a 440 Hz tone survives the 3:1 decimation: compare against the analytic tone away from the edges
    ref = 0.5 * np.sin(2 * np.pi * 440.0 * np.arange(16000) / 16000.0)
    assert np.max(np.abs(z[500:-500] - ref[500:-500])) < 1e-2
    assert m.resample_to_16k(y[:10], 16000) is not None
