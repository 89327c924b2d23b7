"""Model factory / checkpoint entry points (reference: models/utils.py:11-49)."""
import os

from models.audioLLM import AudioLLM


def init_encoder_llm(configs, device="cuda:0", model_path=None, llm_path=None):
    """models/utils.py:30-49 with the reference's `configs`: the parsed train.yaml carrying the cmvn_file and
    model_conf.llm_path that inferencePipeline injects (models/pipeline.py:21-24).  The model directory is the
    one cmvn_file sits in (<model_path>/audiollm/global_cmvn) unless model_path is given; its decoder and codec
    configs and weights (or synthetic.json) load with it, the CMVN statistics come from cmvn_file when it
    exists, and the train.yaml settings are the dict's (not the file's)."""
    import copy
    configs = copy.deepcopy(configs)
    cmvn = configs.get("cmvn_file")
    mp = model_path or configs.get("model_path") or (os.path.dirname(os.path.dirname(cmvn)) if cmvn else None)
    if mp is None:
        raise ValueError("init_encoder_llm: configs carry no cmvn_file (models/pipeline.py:23 sets "
                         "<model_path>/audiollm/global_cmvn); pass model_path")
    lp = llm_path or configs.get("model_conf", {}).get("llm_path") or os.path.join(mp, "llm")
    return AudioLLM.from_model_dir(mp, lp, device=device, train_yaml=configs)


def load_checkpoint(model, path):
    """models/utils.py:11-28: load an audiollm final.pt into the model (strict=False: unknown keys are
    ignored; the fork's 'encoder_*' / 'adpter_*' names and the upstream 'encoder.' / 'adpter.' names
    both bind, see fo.checkpoint.audiollm_state) and return the configs of a sibling final.yaml, or {}.
    The encoders, adapters and state head (and the Qwen2 weights for 'llm_decoder.*' entries) are
    re-packed on the device from the file; a tensor of the wrong shape raises."""
    import re

    import yaml

    from fo.checkpoint import audiollm_state
    if not isinstance(model, AudioLLM):
        raise TypeError(f"load_checkpoint: expected models.audioLLM.AudioLLM, got {type(model).__name__}")
    print(f"Checkpoint: loading from checkpoint {path} for GPU")
    model.rebind(model.engine.rebind_audiollm(audiollm_state(path)))
    info_path = re.sub(r"\.pt$", ".yaml", path)
    if os.path.exists(info_path):
        with open(info_path) as f:
            return yaml.safe_load(f)
    return {}
