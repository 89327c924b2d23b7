"""NaN / inf logits are an error, as in the reference: torch.multinomial raises on the NaN probabilities such a
row gives after the softmax (models/decoder/decoder.py:355-359, models/audioLLM.py:476).  The samplers flag the
row in a host-mapped error word (the drawn id stays a valid table index, so nothing downstream faults) and the
host raises RuntimeError.  Also: one NaN does not win the arg-max over the real maximum of the rest of the row
(block path and the split arg-max of the 152,064-wide text rows)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("V,fast", [(1028, False), (152064, False), (152064, True)])
def test_partial_nan_row_flags_and_keeps_true_argmax(dev, V, fast):
    from fo import ops
    g = torch.Generator(device=dev).manual_seed(3)
    lg = torch.randn(3, V, device=dev, generator=g)
    lg[0, 5] = float("nan")            # partial NaN: flagged, the pick is the max of the others
    lg[1, 7] = float("inf")            # +inf: flagged
    want = [int(torch.nan_to_num(lg[0], nan=-1e30).argmax()), 7, int(lg[2].argmax())]
    chk = ops.SampleCheck()
    try:
        out = torch.empty(3, dtype=torch.int32, device=dev)
        ops.sample(lg, V, out, torch.ones(3, dtype=torch.int32, device=dev), err=chk, argmax_ws=fast)
        got = out.cpu().tolist()
        assert got[0] == want[0] and got[2] == want[2], (got, want)
        assert 0 <= got[1] < V
        with pytest.raises(RuntimeError, match="NaN"):
            chk.check()
        chk.check()   # cleared once raised
        # a clean batch does not raise
        ops.sample(lg[2:], V, out, torch.ones(1, dtype=torch.int32, device=dev), err=chk, argmax_ws=fast)
        torch.cuda.synchronize()
        chk.check()
        # a row of -inf only and the general (top_k = 0 / top_p) path
        lg2 = torch.full((2, V), float("-inf"), device=dev)
        lg2[1] = torch.randn(V, device=dev, generator=g)
        lg2[1, 11] = float("nan")
        k = torch.tensor([1, 0], dtype=torch.int32, device=dev)
        ops.sample(lg2, V, out, k, torch.ones(2, device=dev), torch.full((2,), 0.8, device=dev), err=chk)
        assert all(0 <= i < V for i in out[:2].cpu().tolist())
        with pytest.raises(RuntimeError):
            chk.check()
    finally:
        chk.free()


def test_speech_decode_raises_on_nan_logits(dev):
    """An injected NaN in the AR decoder's output head (every logits row then holds a NaN): the captured decode
    step flags it and speak() raises instead of decoding plausible ids."""
    from fo.engine import FreezeOmniEngine
    from fo.speak import speak
    eng = FreezeOmniEngine(os.path.join(ROOT, "configs", "tiny"), device=dev, max_sessions=4)
    rng = np.random.default_rng(0)
    D = eng.cfg["decoder_json"][0]
    items = [(torch.from_numpy(rng.standard_normal((8, D)).astype(np.float32)).to(dev), None) for _ in range(2)]
    n = sum(seg.numel() for _, seg in speak(eng, items, top_k=1, min_tokens=20, max_tokens=20))
    assert n > 0
    b = eng.tts.out_fnn.bias
    keep = b[3].item()
    b[3] = float("nan")
    try:
        with pytest.raises(RuntimeError, match="NaN"):
            for _ in speak(eng, items, top_k=1, min_tokens=20, max_tokens=20):
                pass
    finally:
        b[3] = keep
    assert eng.tts.pool.pages_in_use() == 0


def test_default_check_is_per_thread_and_dies_with_it(dev):
    """ops.sample_check (the check a sampler call uses when it passes none) is thread-local: a NaN row drawn on one
    thread raises in that thread's check only, and a thread that ends takes its check (and pinned word) with it --
    a later thread starts from a fresh, cleared word."""
    import gc
    import threading
    import weakref

    from fo import ops
    V = 1028
    lg = torch.randn(1, V, device=dev)
    lg[0, 3] = float("nan")
    out = torch.empty(1, dtype=torch.int32, device=dev)
    seen = {}

    def worker():
        chk = ops.sample_check(dev)
        assert ops.sample_check(dev) is chk
        seen["ref"] = weakref.ref(chk)
        seen["id"] = id(chk)
        ops.sample(lg, V, out, torch.ones(1, dtype=torch.int32, device=dev))
        torch.cuda.synchronize()
        seen["flagged"] = int(chk.buf.np[0, 0]) != 0   # left unread: it must not leak into another thread

    t = threading.Thread(target=worker)
    t.start()
    t.join()
    gc.collect()
    assert seen["flagged"]
    assert seen["ref"]() is None, "a finished thread's default check is released"
    mine = ops.sample_check(dev)
    mine.check()   # this thread never drew the NaN row: no error
    t2 = threading.Thread(target=lambda: seen.update(fresh=ops.sample_check(dev).buf.np[0, 0] == 0))
    t2.start()
    t2.join()
    assert seen["fresh"]
