"""AudioLLM facade over the MI355X engine (reference: models/audioLLM.py).

Same entry points and argument meaning as the reference class: set_system_role(extra_inputs),
recognize(speech, extra_inputs), _post_decode(output, temperature, top_k, top_p), plus the
attributes callers touch (tokenizer, chat_template, llm_decoder.model.embed_tokens,
encoder_user.enc[1].num_blocks).  Per-user state stays caller-owned exactly as in the reference
(past_key_values, adapter_cache, encoder_cache, pe_index), but as opaque handles into device pools:
PastKeyValues (paged KV; copy.deepcopy forks it copy-on-write), fo.speech.EncoderCache /
AdapterCache (ring / carried-frame slots).
The text decode step that the fork removed is reconstructed from its caller
contract in bin/inference.py:133-187: generate_step(...).
"""
import copy
import os

import torch

from fo import ops
from fo.engine import FreezeOmniEngine
from fo.ops import F32, I32


class PastKeyValues:
    """Caller-owned LLM context (reference: transformers DynamicCache, models/audioLLM.py:416-419)."""

    def __init__(self, seq):
        self.seq = seq

    def get_seq_length(self, layer_idx=0):
        return self.seq.length

    def __len__(self):
        return self.seq.pool.n_layers

    def __deepcopy__(self, memo):
        # bin/dialog_state_pred.py:110,218 deep-copies the system-role cache per session: fork the
        # block list, sharing full pages copy-on-write.
        return PastKeyValues(self.seq.fork())

    def free(self):
        self.seq.free()


class _EmbedTokens:
    def __init__(self, engine):
        self.engine = engine

    def __call__(self, ids):
        ids = torch.as_tensor(ids).reshape(-1).to(device=self.engine.device, dtype=I32)
        return self.engine.llm.embed(ids)


class _LLMDecoder:
    """Exposes llm_decoder.model.embed_tokens / .transformer.wte like the reference (bin/inference.py:86)."""

    def __init__(self, engine):
        self.model = type("Qwen2Model", (), {})()
        self.model.embed_tokens = _EmbedTokens(engine)
        self.transformer = self.model
        self.transformer.wte = self.model.embed_tokens


class AudioLLM:
    def __init__(self, engine: FreezeOmniEngine, top_k=1, top_p=0.0, temperature=1.0):
        self.engine = engine
        self.device = engine.device
        self.tokenizer = engine.tokenizer
        self.chat_template = None if engine.chat_template is None else {
            k: torch.tensor([v]) for k, v in engine.chat_template.items()}
        self.llm_decoder = _LLMDecoder(engine)
        self._views()
        self.predictor_head = engine.llm.head_w
        self.top_k, self.top_p, self.temperature = top_k, top_p, temperature
        self.logger = None

    def rebind(self, loaded=None):
        """Refresh the views on the engine after models.utils.load_checkpoint re-packed weights."""
        eng = self.engine
        self._views()
        self.predictor_head = eng.llm.head_w
        self.llm_decoder = _LLMDecoder(eng)
        return loaded

    def _views(self):
        """encoder_user / encoder_system / adpter_user / adpter_system as the reference names them
        (models/audioLLM.py:67-68,159-166): speechEncoder / CNNSubsampling facades over the engine's own."""
        from models.adapter import CNNSubsampling
        from models.encoder.encoder import speechEncoder
        for i in ("user", "system"):
            setattr(self, f"encoder_{i}", speechEncoder(self.engine.enc[i]))
            setattr(self, f"adpter_{i}", CNNSubsampling(self.engine.ada[i]))

    @classmethod
    def from_model_dir(cls, model_path, llm_path=None, device="cuda:0", train_yaml=None, receive_weights=False, **kw):
        return cls(FreezeOmniEngine(model_path, llm_path, device=device, train_yaml=train_yaml,
                                    receive_weights=receive_weights), **kw)

    def setup_logger(self, parent_logger=None):
        if parent_logger is not None:
            self.logger = parent_logger.getChild("AudioLLM")

    def init_template_compilation(self):
        """Reference: precompute chat-prefix embeds + torch.compile.  The engine precomputes the
        prefix ids at load and its kernels are ahead-of-time compiled, so nothing is left to do."""
        return None

    # ------------------------------------------------------------------ models/audioLLM.py:312-348
    def set_system_role(self, extra_inputs=None):
        extra_inputs = extra_inputs or {}
        assert extra_inputs.get("past_key_values", None) is None, "past key values already exist!!!"
        return PastKeyValues(self._run(self.engine.system_role, extra_inputs.get("role_prompt", None)))

    # every entry below runs on the replica's serving thread (fo.serve.ReplicaScheduler): the reference calls one
    # pipeline from many session threads (bin/dialog_state_pred.py:802-804); FO_SERVE=0 runs on the caller's thread
    SERVE = os.environ.get("FO_SERVE", "1") != "0"

    def _scheduler(self):
        if not self.SERVE:
            return None
        from fo.serve import ReplicaScheduler
        return ReplicaScheduler.for_device(self.device)

    def _run(self, fn, *args, **kw):
        sch = self._scheduler()
        return fn(*args, **kw) if sch is None else sch.call(fn, *args, **kw)

    # ------------------------------------------------------------------ models/audioLLM.py:350-429
    def recognize(self, speech, extra_inputs=None):
        return self.recognize_batch([(speech, extra_inputs)])[0]

    def recognize_batch(self, requests):
        """Batched recognize: requests = [(speech [1,T,80], extra_inputs)] -> list of 5-tuples.
        All users' chunks run through one encoder/adapter/LLM launch sequence (on the serving thread, together with
        the concurrent calls of other sessions)."""
        for speech, ex in requests:   # the reference's protocol errors, raised in the caller's thread
            assert ex.get("past_key_values", None) is not None, "must set system role first!!!"
            ident = ex.get("identity")
            if ident not in ("user", "system"):
                raise ValueError(f"Unknown identity: {ident}. Must be 'user' or 'system'.")
        sch = self._scheduler()
        return self._recognize_now(requests) if sch is None else sch.listen(self, requests)

    def _recognize_now(self, requests):
        items = []
        for speech, ex in requests:
            ident = ex.get("identity")
            feats = torch.as_tensor(speech)
            feats = feats.reshape(feats.shape[-2], feats.shape[-1]).to(self.device, F32)
            items.append(dict(identity=ident, status=ex.get("status"), feats=feats,
                              kv=ex["past_key_values"].seq, enc_cache=ex.get("encoder_cache"),
                              ada_cache=ex.get("adapter_cache"), pe_index=ex.get("pe_index", 0) or 0))
        res = self.engine.listen(items)
        out = []
        for (speech, ex), r in zip(requests, res):
            out.append((r["probs"], ex["past_key_values"], r["ada_cache"], r["enc_cache"], r["pe_index"]))
            # (buffer, row) of the last request's final hidden row (a probe for single-caller tests: the buffer is the
            # engine's and is rewritten by the next listen)
            self._last_hidden = r["hidden_row"]
        return out

    # ------------------------------------------------------------------ models/audioLLM.py:431-477
    def _post_decode(self, output, temperature=1.0, top_k=0, top_p=0.0, seed=None):
        """Sample one token id from logits [1, 1, V] with the reference's rule (models/audioLLM.py:
        431-477): temperature, top_k > 0 keeps the k largest (0 = no top-k filtering: the whole
        vocabulary), top_p > 0 the nucleus, then one draw (fo_sample).  The draw comes from the
        kernel's counter stream: `seed` pins it, otherwise each call takes the next stream."""
        if seed is None:
            self._draws = getattr(self, "_draws", 0) + 1
            seed = self._draws
        return self._run(self._post_decode_now, output, temperature, top_k, top_p, seed)

    def _post_decode_now(self, output, temperature, top_k, top_p, seed):
        lg = torch.as_tensor(output).reshape(1, -1).to(self.device, F32).contiguous()
        V = lg.shape[1]
        out = torch.empty(1, dtype=I32, device=self.device)
        chk = ops.sample_check(self.device)
        ops.sample(lg, V, out, torch.tensor([int(top_k)], dtype=I32).to(self.device),
                   torch.tensor([temperature], dtype=F32).to(self.device),
                   torch.tensor([top_p], dtype=F32).to(self.device), seed=seed, err=chk)
        tok = out.view(1, 1).long().cpu()
        chk.check("_post_decode")   # NaN / inf logits: the reference's torch.multinomial raises
        return tok.to(self.device)

    # ------------------------------------------------------------------ A17: text decode step
    def generate_step(self, past_key_values, input_ids, top_k=None, top_p=None, temperature=None):
        """Forward `input_ids` on the session context and sample the next token from the last
        position.  Returns (token id, last hidden state [1, 1, D] device).  Concurrent one-token steps of other
        sessions with the same sampler settings share one text step on the serving thread."""
        top_k = self.top_k if top_k is None else top_k
        top_p = self.top_p if top_p is None else top_p
        temperature = self.temperature if temperature is None else temperature
        sch = self._scheduler()
        if sch is None:
            return self._generate_now(past_key_values, input_ids, top_k, top_p, temperature)
        return sch.text(self, past_key_values, input_ids, top_k, top_p, temperature)

    def _generate_now(self, past_key_values, input_ids, top_k, top_p, temperature):
        ids, hid = self.engine.text_step([(past_key_values.seq, list(input_ids))], top_k=top_k, top_p=top_p,
                                         temperature=temperature)
        return ids[0], hid.view(1, 1, -1)

    def prefix_ids(self, identity):
        return list(self.engine.prefix_ids[identity])

    def deepcopy_kv(self, pkv):
        return copy.deepcopy(pkv)
