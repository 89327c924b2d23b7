"""fo_subsample (the encoder's Conv2dSubsampling4 + GlobalCMVN up to its output Linear, models/encoder/
subsampling.py:67-73, cmvn.py:24-35) against a plain torch fp32 reference of the same op on the same bf16-valued
weights: framings A (19 frames) and B (32 frames), 1 and 8 sessions, 32 and 1024 channels (the tiny and real
geometries), the transposed Linear-input layout z[(b, t)][c * W2 + f].  Tolerance 2e-5 x max|ref| (fp32 arithmetic
with bf16 hi + lo activations against bf16 weights)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,R,C", [(1, 19, 32), (8, 19, 1024), (8, 32, 1024), (3, 32, 64), (2, 19, 96)])
def test_subsample_matches_torch_fp32(dev, B, R, C):
    from fo import ops
    g = torch.Generator().manual_seed(B * 100 + R + C)
    F = 80
    feats = (torch.randn(B, R, F, generator=g) * 3 + 8).float()
    mean = (8 + torch.randn(F, generator=g)).float()
    istd = (0.25 + 0.05 * torch.rand(F, generator=g)).float()
    w1 = (torch.randn(C, 1, 3, 3, generator=g) / 3).to(torch.bfloat16).float()
    b1 = (0.05 * torch.randn(C, generator=g)).float()
    w2 = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(torch.bfloat16).float()
    b2 = (0.05 * torch.randn(C, generator=g)).float()
    x = ((feats - mean) * istd).unsqueeze(1).double()
    y = torch.relu(torch.nn.functional.conv2d(x, w1.double(), b1.double(), stride=2))
    y = torch.relu(torch.nn.functional.conv2d(y, w2.double(), b2.double(), stride=2))   # [B, C, H2, W2]
    Bn, Cn, H2, W2 = y.shape
    ref = y.transpose(1, 2).reshape(B * H2, C * W2).float()
    H1, W1 = (R - 3) // 2 + 1, (F - 3) // 2 + 1
    w2p = ops.PackedLinear(w2.permute(0, 2, 3, 1).reshape(C, 9 * C).to(torch.bfloat16).to(dev))
    y1 = torch.empty(B * H1 * W1, C, device=dev)
    z = torch.full((B * H2, C * W2), float("nan"), device=dev)
    ops.launch_counts_reset()
    ops.subsample(feats.to(dev), B, R, F, mean.to(dev), istd.to(dev), w1.reshape(C, 9).contiguous().to(dev),
                  b1.to(dev), C, y1, w2p.packed, b2.to(dev), z)
    torch.cuda.synchronize()
    assert ops.launch_counts()["subsample"] == 1
    got = z.cpu()
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item()
    assert err <= 2e-5 * ref.abs().max().item(), (err, ref.abs().max().item())
