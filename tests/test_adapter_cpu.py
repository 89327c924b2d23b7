"""Adapter configuration checks that need no GPU: the engine rejects what the reference cannot stream
(models/audioLLM.py:159-165,386-387; models/adapter.py:100-107)."""
import pytest

from oracle import configs


@pytest.mark.parametrize("conf,msg", [({"adpter_type": "cnn"}, "adpter_type"), ({"adpter_type": "linear"}, "adpter_type"),
                                      ({"norm": "instance"}, "norm")])
def test_adapter_rejects_unstreamable_configs(conf, msg):
    from fo.speech import AdapterEngine
    c = configs.get("tiny")
    c["train_yaml"]["model_conf"].update(conf)
    with pytest.raises(ValueError, match=msg):
        AdapterEngine(None, c, "user", "cpu", 1)


def test_adapter_branch_inventory():
    """cnn_num follows 4*d < L (models/adapter.py:84); the layer-norm branch has no running stats."""
    from oracle.params import adapter_shapes
    c = configs.get("tiny")
    c["train_yaml"]["model_conf"].update(enc_out_dim=16, llm_embed_dim=128)
    s = adapter_shapes(c, "user")
    assert s["adpter_user.conv1d1.weight"] == [32, 16, 5] and s["adpter_user.conv1d2.weight"] == [64, 32, 5]
    assert s["adpter_user.project.weight"] == [128, 64]
    c = configs.get("tiny")
    c["train_yaml"]["model_conf"]["norm"] = "layer"
    s = adapter_shapes(c, "user")
    assert "adpter_user.bn2.running_mean" not in s and s["adpter_user.bn2.weight"] == [64]
