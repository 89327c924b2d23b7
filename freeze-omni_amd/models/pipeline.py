"""inferencePipeline: the reference's Python entry point (models/pipeline.py) on the MI355X engine.

Accepts both calling conventions found in the reference tree:
  * fork form (models/pipeline.py:36-88, bin/dialog_state_pred.py:777-844):
      speech_dialogue(audio, identity, status, role=None, past_key_values=None, adapter_cache=None,
                      encoder_cache=None, pe_index=0)
      -> (prediction_probs, past_key_values, adapter_cache, encoder_cache, pe_index)
      status 'pre' -> (None, past_key_values, None, None, None)
  * upstream form used by bin/inference.py:119-187: speech_dialogue(audio, stat=..., role=..., **outputs)
      -> dict(stat, past_key_values, adapter_cache, encoder_cache, pe_index, text, hidden_state,
              past_tokens, last_id); stats 'pre' | 'dialog_sl' | 'dialog_cl' | 'dialog_el' | 'dialog_ss'
      | 'dialog_cs'.  The speak states reconstruct the text decode the fork removed.
args may be a dict (reference) or an argparse.Namespace (bin/inference.py:191).
"""
import argparse
import re
import uuid

import torch

from models.audioLLM import AudioLLM

_UPSTREAM_TO_STATUS = {"dialog_sl": "ipu_sl", "dialog_cl": "ipu_cl", "dialog_el": "ipu_el"}


class inferencePipeline:
    def __init__(self, args, weights_from=None):
        """weights_from: another inferencePipeline (any device) whose frozen weights this replica copies
        instead of reading / generating its own (fo.replica.copy_frozen: the in-process form of the
        start-up broadcast, bin/pool.py's `devices` replicas)."""
        if isinstance(args, argparse.Namespace):
            args = vars(args)
        self.args = args
        self.device = args.get("device", "cuda:0")
        self.id = uuid.uuid4().hex[:22]
        print(f"Using device: {self.device} for inference pipeline of freeze-omni model.")
        top_k = args.get("top_k", 1)
        self.model = AudioLLM.from_model_dir(args["model_path"], args.get("llm_path"), device=self.device,
                                             top_k=top_k if top_k is not None else 1,
                                             top_p=args.get("top_p", 0.0) or 0.0,
                                             temperature=args.get("temperature", 1.0) or 1.0,
                                             receive_weights=weights_from is not None)
        if weights_from is not None:
            from fo.replica import copy_frozen
            copy_frozen(weights_from.model.engine, self.model.engine)
            self.model.rebind()
        self.model.init_template_compilation()
        self.logger = None

    @classmethod
    def from_engine(cls, engine, top_k=1, top_p=0.0, temperature=1.0):
        """A pipeline over an already loaded FreezeOmniEngine (replica-local serving, benchmarks)."""
        self = cls.__new__(cls)
        self.args = {"device": str(engine.device)}
        self.device = engine.device
        self.id = uuid.uuid4().hex[:22]
        self.model = AudioLLM(engine, top_k=top_k, top_p=top_p, temperature=temperature)
        self.logger = None
        return self

    # ------------------------------------------------------------------ speech_dialogue
    def speech_dialogue(self, audio, identity=None, status=None, role=None, past_key_values=None,
                        adapter_cache=None, encoder_cache=None, pe_index=0, stat=None, **upstream):
        if stat is not None:
            return self._upstream(audio, stat, role, past_key_values, adapter_cache, encoder_cache, pe_index,
                                  **upstream)
        with torch.no_grad():
            extra = {"identity": identity, "status": status, "past_key_values": past_key_values,
                     "adapter_cache": adapter_cache, "encoder_cache": encoder_cache, "pe_index": pe_index}
            if role is not None and past_key_values is None:
                extra["role_prompt"] = "<|im_start|>system\n" + role
            if status == "pre":
                return None, self.model.set_system_role(extra), None, None, None
            return self.model.recognize(audio, extra)

    def speech_dialogue_batch(self, requests):
        """Batched fork-form calls: requests = list of dicts with the keyword arguments of
        speech_dialogue; one device launch sequence serves all of them."""
        rq = []
        for r in requests:
            extra = {k: r.get(k) for k in ("identity", "status", "past_key_values", "adapter_cache",
                                           "encoder_cache")}
            extra["pe_index"] = r.get("pe_index", 0) or 0
            rq.append((r["audio"], extra))
        return self.model.recognize_batch(rq)

    def _upstream(self, audio, stat, role, pkv, adapter_cache, encoder_cache, pe_index, text="",
                  hidden_state=None, past_tokens=None, last_id=None, **_):
        out = {"stat": stat, "past_key_values": pkv, "adapter_cache": adapter_cache,
               "encoder_cache": encoder_cache, "pe_index": pe_index, "text": text or "",
               "hidden_state": hidden_state, "past_tokens": list(past_tokens or []), "last_id": last_id}
        m = self.model
        if stat == "pre":
            extra = {"past_key_values": None}
            if role is not None:
                extra["role_prompt"] = "<|im_start|>system\n" + role
            out.update(stat="dialog_sl", past_key_values=m.set_system_role(extra), adapter_cache=None,
                       encoder_cache=None, pe_index=0, text="", hidden_state=None, past_tokens=[], last_id=None)
            return out
        if stat in _UPSTREAM_TO_STATUS:
            if audio is None:
                return out
            extra = {"identity": "user", "status": _UPSTREAM_TO_STATUS[stat], "past_key_values": pkv,
                     "adapter_cache": adapter_cache, "encoder_cache": encoder_cache, "pe_index": pe_index}
            probs, pkv, ac, ec, pe = m.recognize(audio, extra)
            nstat = "dialog_cl"
            if probs is not None:
                if probs["state_1"] > 0.5:
                    nstat = "dialog_ss"
                elif probs["state_2"] > 0.5:
                    nstat = "dialog_el"
            out.update(stat=nstat, past_key_values=pkv, adapter_cache=ac, encoder_cache=ec, pe_index=pe,
                       prediction_probs=probs)
            return out
        if stat in ("dialog_ss", "dialog_cs"):
            ids = m.prefix_ids("system") if stat == "dialog_ss" else [out["last_id"]]
            tok, hid = m.generate_step(pkv, ids)
            toks = ([] if stat == "dialog_ss" else out["past_tokens"]) + [tok]
            eod = m.tokenizer.eod_id
            out.update(last_id=tok, past_tokens=toks, hidden_state=hid,
                       text=m.tokenizer.decode([t for t in toks if t != eod]),
                       stat="dialog_sl" if tok == eod else "dialog_cs")
            return out
        raise ValueError(f"unknown stat {stat!r}")

    # ------------------------------------------------------------------ models/pipeline.py:90-130
    def post_process(self, text):
        text = text.replace("、", "，")
        text = text.replace("(", ",")
        text = text.replace(")", ",")
        text = text.replace("（", "，")
        text = text.replace("）", "，")
        text = re.sub(r"[\n\r\t]", "", text)
        text = re.sub(r"[*_`~]", "", text)
        text = re.sub(r"(\.|\:)\s+", r"\1", text)
        if re.search("[\u4e00-\u9fa5]", text):
            text = re.sub("(\\d+)\\.\\s*([\u4e00-\u9fa5A-Za-z])", r"\1：\2", text)
        else:
            text = re.sub(r"(\d+)\.\s*([\w])", r"\1:\2", text)
        if text and text[-1] not in ["。", "？", "！", ".", "?", "!"]:
            if text[-1] in [",", "，", ";", "；", ":", "：", "、"]:
                text = text[:-1] + "。"
            else:
                text += "。"
        return text

    def setup_logger(self, parent_logger):
        if parent_logger is not None:
            self.logger = parent_logger.getChild("FOPipe")
        else:
            from logger.logger import setup_logger
            self.logger = setup_logger(f"FOPipe_{self.id}", file_log_level="DEBUG", terminal_log_level="INFO")
        self.model.setup_logger(self.logger)
