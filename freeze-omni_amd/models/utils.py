"""Model factory / checkpoint entry points (reference: models/utils.py:11-49)."""
import os

from models.audioLLM import AudioLLM


def init_encoder_llm(configs, device="cuda:0", model_path=None, llm_path=None):
    """Build the AudioLLM for a model directory.  `configs` is the parsed train.yaml as in the
    reference; the MI355X engine reads the same files itself, so model_path must be given (or
    configs['model_path'])."""
    mp = model_path or configs.get("model_path")
    if mp is None:
        raise ValueError("init_encoder_llm: pass model_path (directory holding audiollm/train.yaml)")
    lp = llm_path or configs.get("model_conf", {}).get("llm_path") or os.path.join(mp, "llm")
    return AudioLLM.from_model_dir(mp, lp, device=device)


def load_checkpoint(model, path):
    """Weights are bound when the engine is built from the model directory (synthetic.json or the
    reference checkpoint files); kept for API parity with models/utils.py:11-28."""
    return {}
