"""The duplex state head (k_state_head): softmax over the three predictor-head logits of selected rows, as the
reference's LLM computes for its listen / speak / interrupt decision (models/audioLLM.py:215 / :488 predictor_head, softmax over
the first three logits).  Compared with a torch fp32 restatement on the same rows, D below, at and above one 4096-wide
slab of the single-pass loop.  Tolerance 1e-5 absolute on probabilities (fp32 sums in a different order)."""
import pytest
import torch

from fo import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D", [64, 896, 3584, 5000])
def test_state_head_matches_fp32(D):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(D)
    h = torch.randn(11, D, device=dev, generator=g)
    W = torch.randn(3, D, device=dev, generator=g) / D ** 0.5
    b = torch.randn(3, device=dev, generator=g)
    rows = torch.tensor([10, 0, 3, 7, 7], dtype=torch.int32, device=dev)
    out = torch.empty(rows.numel(), 3, device=dev)
    ops.state_head(h, rows, W, b, out)
    ref = torch.softmax(h[rows.long()].double() @ W.double().t() + b.double(), dim=-1).float()
    torch.testing.assert_close(out, ref, rtol=0, atol=1e-5)
