"""The reference-signature constructors on the GPU, each built the reference's way and loaded with the
reference module's own state-dict names, against the reference's goldens:
  * CNNSubsampling(enc_out_dim, llm_embed_dim, kernel_size, activation_func, norm) + load_state_dict
    (models/adapter.py:72-157) on every adapter_variants_tiny branch (5e-4 abs, as the engine-level test);
  * speechEncoder(input_dim, overview_conf, para_conf, GlobalCMVN(mean, istd)) + load_state_dict
    (models/encoder/encoder.py:45-155) at real geometry (2 blocks, d 1024) on real_encoder_t2's framing-A
    chunks (2e-3 of the output's scale, as the engine-level test);
  * init_encoder_llm(configs) with the train.yaml dict inferencePipeline builds (cmvn_file + llm_path
    injected, models/pipeline.py:21-24) -> AudioLLM whose fork-form recognize matches audiollm_tiny.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import configs
from oracle.weights import synth_param

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _state(m, seed, prefix):
    """The reference module's state dict with the goldens' counter-hash values (make_golden.init_module)."""
    return {k: torch.from_numpy(synth_param(seed, prefix + k, shp)) for k, shp in m.state_dict_shapes().items()}


def test_cnn_subsampling_reference_constructor_matches_golden(dev):
    from models.adapter import CNNSubsampling
    meta = json.load(open(os.path.join(G, "adapter_variants_tiny.json")))
    g = np.load(os.path.join(G, "adapter_variants_tiny.npz"))
    for vi, v in enumerate(meta["variants"]):
        m = CNNSubsampling(v["enc_out_dim"], v["llm_embed_dim"], v["kernel_size"], v["activation_func"], v["norm"],
                           seed=1)   # built with other weights, then loaded the reference way
        assert m.cnn_num == int(g[f"v{vi}_cnn_num"])
        r = m.load_state_dict(_state(m, meta["seed"], "adpter_user."))
        assert not r.missing_keys and not r.unexpected_keys
        cache = None
        for ci in range(6):
            x = torch.from_numpy(g[f"v{vi}_c{ci}_x"]).to(dev).unsqueeze(0)
            mask = torch.ones(1, 1, x.shape[1], dtype=torch.bool, device=dev)
            y, mo, cache = m(x, mask, cache=cache, return_cache=True)
            assert mo.shape[-1] == (x.shape[1] + 1) // 2
            np.testing.assert_allclose(y[0].cpu().numpy(), g[f"v{vi}_c{ci}_y"], atol=5e-4)
    with pytest.raises(RuntimeError, match="size mismatch"):
        m.load_state_dict({"project.weight": torch.zeros(3, 3)}, strict=False)


def test_speech_encoder_reference_constructor_matches_golden(dev):
    from models.encoder.cmvn import GlobalCMVN
    from models.encoder.encoder import speechEncoder
    cfg = configs.get("real")
    ec = cfg["train_yaml"]["encoder_conf"]
    ec["para_conf"]["transformer"]["transformer-num-blocks"] = 2
    enc = speechEncoder(80, ec["overview_conf"], ec["para_conf"], GlobalCMVN(torch.zeros(80), torch.ones(80)),
                        seed=3)
    assert enc.output_size() == 1024 and enc.enc[1].num_blocks == 2
    sd = _state(enc, cfg["seed"], "encoder_user.")   # the golden's global_cmvn buffers are hashed too (init_module)
    r = enc.load_state_dict(sd)
    assert not r.missing_keys and not r.unexpected_keys
    g = np.load(os.path.join(G, "real_encoder_t2.npz"))
    buf, pe = None, int(g["A_pe0"])
    for i in range(g["A_feats"].shape[0]):
        o, buf, _, _, pe = enc.infer(torch.from_numpy(g["A_feats"][i]).unsqueeze(0), buf, 0, None, pe)
        ref = g["A_enc"][i]   # the engine-level test's tolerance, relative to the output's scale
        np.testing.assert_allclose(o[0].cpu().numpy(), ref, rtol=2e-3, atol=2e-3 * float(np.abs(ref).max()),
                                   err_msg=f"chunk {i}")
        assert pe == int(g["A_pe"][i])


def test_init_encoder_llm_from_reference_configs(dev):
    import yaml
    from models.utils import init_encoder_llm
    tiny = os.path.join(ROOT, "configs", "tiny")
    with open(os.path.join(tiny, "audiollm", "train.yaml")) as f:
        ty = yaml.safe_load(f)
    ty["cmvn_file"] = os.path.join(tiny, "audiollm", "global_cmvn")   # models/pipeline.py:23 (absent here: synthetic)
    ty["model_conf"]["llm_path"] = os.path.join(tiny, "llm")         # models/pipeline.py:24
    model = init_encoder_llm(ty, device="cuda:0")
    assert model.encoder_user.enc[1].num_blocks == ty["encoder_conf"]["para_conf"]["transformer"][
        "transformer-num-blocks"]
    assert model.adpter_user.cnn_num in (1, 2)
    meta = json.load(open(os.path.join(G, "audiollm_tiny.json")))
    g = np.load(os.path.join(G, "audiollm_tiny.npz"))
    pkv = model.set_system_role({"role_prompt": "<|im_start|>system\nYou are a helpful assistant."})
    ex = {"identity": "user", "status": "ipu_sl", "past_key_values": pkv, "adapter_cache": None,
          "encoder_cache": None, "pe_index": 0}
    step = meta["steps"][0]
    probs, pkv, ac, ec, pe = model.recognize(torch.from_numpy(g["feats"][0]).unsqueeze(0), ex)
    assert pe == step["pe_index"] and pkv.get_seq_length() == step["kv_len"]
    assert abs(probs["state_1"] - step["probs"]["state_1"]) < 2e-4
    pkv.free()
