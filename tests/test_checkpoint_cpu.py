"""fo.checkpoint: the reference's checkpoint files -> engine parameter names (CPU).

The model directory is written in the reference's formats (tests/refdir.py) with the tiny
configuration's counter-hash weights, so every ingested tensor can be compared with its source."""
import json
import os

import numpy as np
import pytest
import torch

from refdir import make_reference_dir


def _state(tmp_path, **kw):
    from fo.checkpoint import load_reference_checkpoints
    from fo.engine import load_model_dir
    d = str(tmp_path / "model")
    cfg_o, W, cmvn = make_reference_dir(d, **kw)
    cfg, synth, llm_path = load_model_dir(d)
    assert synth is None
    return load_reference_checkpoints(cfg, d, llm_path, "cpu"), W, cmvn, d


def test_fork_names_roundtrip(tmp_path):
    src, W, cmvn, _ = _state(tmp_path)
    for k in W.keys():
        if k.startswith("task_embeddings."):
            continue
        got = src.get(k).numpy()
        want = W[k]
        if ".weight" in k and k.startswith("codec.generator.") and W[k].ndim > 1:
            np.testing.assert_allclose(got, want, rtol=2e-6, atol=1e-7, err_msg=k)  # folded weight norm
        else:
            np.testing.assert_array_equal(got, want, err_msg=k)


def test_upstream_names_fill_both_identities(tmp_path):
    src, W, _, _ = _state(tmp_path, upstream_names=True)
    for k in W.keys():
        if k.startswith(("encoder_system.", "adpter_system.")):
            user = k.replace("_system.", "_user.", 1)
            np.testing.assert_array_equal(src.get(k).numpy(), W[user], err_msg=k)


def test_cmvn_file_then_checkpoint_override(tmp_path):
    src, W, (mean, istd), _ = _state(tmp_path, cmvn_in_ckpt=False)
    np.testing.assert_allclose(src.get("encoder_user.global_cmvn.mean").numpy(), mean, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(src.get("encoder_system.global_cmvn.istd").numpy(), istd, rtol=1e-6)
    src2, W2, _, _ = _state(tmp_path / "b", cmvn_in_ckpt=True)
    np.testing.assert_array_equal(src2.get("encoder_user.global_cmvn.mean").numpy(), W2["encoder_user.global_cmvn.mean"])


def test_kaldi_cmvn_text(tmp_path):
    from fo.checkpoint import load_cmvn
    p = tmp_path / "global_cmvn"
    means, var, n = [2.0, -4.0, 6.0], [8.0, 20.0, 40.0], 2.0
    p.write_text("[ " + " ".join(map(str, means + [n])) + "\n " + " ".join(map(str, var + [0])) + " ]\n")
    m, istd = load_cmvn(str(p), is_json=False)
    np.testing.assert_allclose(m.numpy(), [1.0, -2.0, 3.0])
    np.testing.assert_allclose(istd.numpy(), 1 / np.sqrt([4 - 1, 10 - 4, 20 - 9]), rtol=1e-6)


def test_llm_decoder_entries_override_safetensors(tmp_path):
    src, W, _, d = _state(tmp_path, llm_in_final=True)
    sd = torch.load(os.path.join(d, "audiollm", "final.pt"), weights_only=True)
    sd["llm_decoder.model.norm.weight"] = sd["llm_decoder.model.norm.weight"] * 0 + 3.0
    torch.save(sd, os.path.join(d, "audiollm", "final.pt"))
    from fo.checkpoint import load_reference_checkpoints
    from fo.engine import load_model_dir
    cfg, _, llm_path = load_model_dir(d)
    s2 = load_reference_checkpoints(cfg, d, llm_path, "cpu")
    assert float(s2.get("model.norm.weight")[0]) == 3.0


def test_missing_and_misshaped_tensors_raise(tmp_path):
    from fo.checkpoint import load_reference_checkpoints
    from fo.engine import load_model_dir
    _, _, _, d = _state(tmp_path)
    snap = torch.load(os.path.join(d, "decoder", "final.pt"), weights_only=True)
    del snap["model"]["norm.weight"]
    snap["model"]["out_fnn.bias"] = torch.zeros(3)
    torch.save(snap, os.path.join(d, "decoder", "final.pt"))
    cfg, _, llm_path = load_model_dir(d)
    with pytest.raises(RuntimeError) as e:
        load_reference_checkpoints(cfg, d, llm_path, "cpu")
    assert "tts.norm.weight" in str(e.value) and "tts.out_fnn.bias" in str(e.value)


def test_single_file_safetensors_and_bin(tmp_path):
    from safetensors.torch import load_file, save_file
    from fo.checkpoint import load_reference_checkpoints
    from fo.engine import load_model_dir
    _, W, _, d = _state(tmp_path)
    ld = os.path.join(d, "llm")
    idx = json.load(open(os.path.join(ld, "model.safetensors.index.json")))
    allt = {}
    for fn in sorted(set(idx["weight_map"].values())):
        allt.update(load_file(os.path.join(ld, fn)))
        os.remove(os.path.join(ld, fn))
    os.remove(os.path.join(ld, "model.safetensors.index.json"))
    save_file(allt, os.path.join(ld, "model.safetensors"))
    cfg, _, llm_path = load_model_dir(d)
    s = load_reference_checkpoints(cfg, d, llm_path, "cpu")
    np.testing.assert_array_equal(s.get("model.layers.1.mlp.down_proj.weight").numpy(),
                                  W["model.layers.1.mlp.down_proj.weight"])
    os.remove(os.path.join(ld, "model.safetensors"))
    torch.save(allt, os.path.join(ld, "pytorch_model.bin"))
    s = load_reference_checkpoints(cfg, d, llm_path, "cpu")
    np.testing.assert_array_equal(s.get("lm_head.weight").float().numpy(), W["lm_head.weight"])
