"""The Python surface keeps the reference's constructor signatures:
models.adapter.CNNSubsampling(enc_out_dim, llm_embed_dim, kernel_size, activation_func, norm)
(models/adapter.py:72-80), models.encoder.encoder.speechEncoder(input_dim, overview_conf, para_conf,
global_cmvn) (models/encoder/encoder.py:45-51), models.utils.init_encoder_llm(configs, device)
(models/utils.py:30), models.encoder.cmvn.GlobalCMVN(mean, istd, norm_var) (models/encoder/cmvn.py:7-22).
No GPU here: building one must fail loudly (no CPU fallback)."""
import inspect

import pytest
import torch

from oracle import configs


def _params(fn):
    return [(p.name, p.default) for p in inspect.signature(fn).parameters.values()
            if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD) and p.name != "self"]


def test_reference_signatures():
    from models.adapter import CNNSubsampling
    from models.encoder.cmvn import GlobalCMVN
    from models.encoder.encoder import speechEncoder
    from models.utils import init_encoder_llm, load_checkpoint
    assert _params(CNNSubsampling.__init__) == [("enc_out_dim", 512), ("llm_embed_dim", 4096), ("kernel_size", 5),
                                                ("activation_func", "relu"), ("norm", "batch")]
    assert _params(speechEncoder.__init__) == [("input_dim", inspect.Parameter.empty), ("overview_conf", None),
                                               ("para_conf", None), ("global_cmvn", None)]
    assert [n for n, _ in _params(init_encoder_llm)][:2] == ["configs", "device"]
    assert [n for n, _ in _params(load_checkpoint)] == ["model", "path"]
    assert [n for n, _ in _params(GlobalCMVN.__init__)] == ["mean", "istd", "norm_var"]
    c = GlobalCMVN(torch.zeros(4), torch.full((4,), 2.0), norm_var=False)
    assert torch.equal(c.istd, torch.ones(4))


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_constructors_need_the_gpu():
    from models.adapter import CNNSubsampling
    from models.encoder.encoder import speechEncoder
    from models.utils import init_encoder_llm
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        CNNSubsampling(1024, 3584, 5, "relu", "batch")
    ec = configs.get("tiny")["train_yaml"]["encoder_conf"]
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        speechEncoder(80, ec["overview_conf"], ec["para_conf"], None)
    ty = configs.get("tiny")["train_yaml"]
    with pytest.raises(ValueError, match="cmvn_file"):
        init_encoder_llm(dict(ty, cmvn_file=None))
