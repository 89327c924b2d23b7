"""VQVAE.encode on the GPU (fo_codec_enc.hip through the C-ABI) vs the reference's own outputs
(tests/golden/codec_encoder_tiny.*, counter-hash weights regenerated on the device): encoder output
within fp32 tolerance, local (2-layer residual VQ) and global token ids exact."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def test_codec_encoder_matches_reference_golden(dev):
    from fo.codec import CodecEncoderEngine
    from fo.weights import SynthSource
    from models.decoder.ticodec.vqvae import VQVAE
    meta = json.load(open(os.path.join(G, "codec_encoder_tiny.json")))
    g = np.load(os.path.join(G, "codec_encoder_tiny.npz"))
    eng = CodecEncoderEngine(SynthSource(meta["seed"], meta["shapes"], dev), meta["codec_json"], dev)
    wav = torch.from_numpy(g["wav"]).to(dev)
    c, gfeat, L = eng.encoder(wav)
    np.testing.assert_allclose(c.cpu().numpy(), g["enc_out"], atol=2e-5, rtol=1e-4)
    np.testing.assert_allclose(gfeat.cpu().numpy(), g["global_features"], atol=2e-5, rtol=1e-4)
    local, gst = VQVAE(None, eng).encode(wav.unsqueeze(-1))
    np.testing.assert_array_equal(local.cpu().numpy(), g["local_tokens"])
    np.testing.assert_array_equal(gst.cpu().numpy(), g["global_tokens"])
