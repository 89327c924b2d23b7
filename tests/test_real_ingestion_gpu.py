"""Real-geometry checkpoint ingestion: an engine built from the REFERENCE'S FILE FORMATS at
configs/real geometry (reduced depth: 2 Qwen2 layers with the real 152,064-row embedding and lm_head, 2 encoder
blocks, the full 4-layer AR decoder, the 512-channel codec; tests/refdir.py make_reference_dir_real) reproduces
the reference-run T2 goldens:
  * Qwen2 from three bf16 safetensors shards + index (models/audioLLM.py:70-74, from_pretrained): the
    real_qwen2_t2 prefill / chunks / text steps (hidden 2e-3, state probs 5e-4, logits 1e-3, ids exact);
  * the speech encoder + adapter from audiollm/final.pt under the UPSTREAM names 'encoder.*' / 'adpter.*'
    (models/utils.py:11-28; fo.checkpoint fans them out to both identities): real_encoder_t2 on both identities;
  * the AR decoder from decoder/final.pt (models/decoder/llm2tts.py:32-68): real_tts_t2's 48 greedy ids;
  * the vocoder from codec/final.pt's weight-normed generator (models/decoder/ticodec/vqvae.py:21-35, weight norm
    folded at load): real_codec_t2's 36,146 samples.
Tolerances as in the synthetic-weight tests of the same goldens (test_real_qwen2_gpu.py, test_parity_r02_gpu.py)."""
import os

import numpy as np
import pytest
import torch

from refdir import make_reference_dir_real
from test_real_qwen2_gpu import check_llm_against_golden

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _close(a, b, rtol, atol):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


@pytest.fixture(scope="module")
def eng(dev, tmp_path_factory):
    from fo.engine import FreezeOmniEngine
    d = str(tmp_path_factory.mktemp("real_t2") / "model")
    make_reference_dir_real(d, dev)
    assert not os.path.exists(os.path.join(d, "synthetic.json"))   # the checkpoint path, not the hash fill
    e = FreezeOmniEngine(d, device=dev, max_sessions=8)
    assert (e.llm.D, e.llm.V, e.llm.stack.n) == (3584, 152064, 2)
    yield e


def test_qwen2_from_sharded_safetensors_matches_reference(dev, eng):
    check_llm_against_golden(eng.llm, dev, np.load(os.path.join(G, "real_qwen2_t2.npz")))


@pytest.mark.parametrize("ident", ["user", "system"])
def test_encoder_adapter_from_upstream_names_match_reference(dev, eng, ident):
    g = np.load(os.path.join(G, "real_encoder_t2.npz"))
    enc, ada = eng.enc[ident], eng.ada[ident]
    for kind in ("A", "B"):
        ec, ac, pe = enc.new_cache(), ada.new_cache(), int(g[f"{kind}_pe0"])
        for i in range(g[f"{kind}_feats"].shape[0]):
            out, T, pes = enc.infer(torch.from_numpy(g[f"{kind}_feats"][i][None]).to(dev), [ec], [pe])
            pe = pes[0]
            assert pe == int(g[f"{kind}_pe"][i])
            ref = g[f"{kind}_enc"][i]
            _close(out, ref, 2e-3, 2e-3 * float(np.abs(ref).max()))
            emb, To = ada(out, T, [ac])
            ref = g[f"{kind}_ada"][i]
            _close(emb, ref, 2e-3, 2e-3 * float(np.abs(ref).max()))


def test_tts_and_vocoder_from_reference_files_match_reference(dev, eng):
    from fo import ops
    g = np.load(os.path.join(G, "real_tts_t2.npz"))
    tts = eng.tts
    seqs = tts.start([(torch.from_numpy(g["hidden"]).to(dev), torch.from_numpy(g["prefix"]).to(dev))])
    cur = torch.full((1,), tts.sos, dtype=torch.int32, device=dev)
    ids = []
    for i in range(len(g["ids"])):
        lg = tts.step(seqs, cur)
        if i < 4:
            ref = g["logits"][i]
            _close(lg[0, :ref.size], ref, 1e-3, 1e-3)
        cur = ops.sample(lg, tts.vocab + 4, torch.empty(1, dtype=torch.int32, device=dev))
        ids.append(int(cur.item()))
    tts.free(seqs)
    assert ids == g["ids"].tolist()
    c = np.load(os.path.join(G, "real_codec_t2.npz"))
    pcm = eng.codec(torch.from_numpy(c["ids"][None]).to(dev, torch.int32))[0]
    assert pcm.numel() == c["pcm"].size
    _close(pcm, c["pcm"], 1e-3, 1e-4)
