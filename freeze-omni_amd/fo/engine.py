"""One Freeze-Omni replica on one MI355X: model loading plus the batched hot-path primitives that the
reference-API layer (freeze-omni_amd/models) and the benchmark drive.

Reference flow being replaced: inferencePipeline.__init__ (models/pipeline.py:12-34)
loads train.yaml + final.pt + Qwen2; speech_dialogue -> AudioLLM.set_system_role / recognize
(models/audioLLM.py:312-429); llm2TTS.run -> LLM2TTSCodecAR.infer + VQVAE (models/decoder/*).
Where the reference runs one user per call with ~hundreds of small launches, every primitive here
takes a list of sessions and issues one launch sequence for all of them.
"""
import contextlib
import ctypes
import json
import os
import time
from types import SimpleNamespace

import numpy as np
import torch

from . import _lib, ops
from .codec import CodecEngine
from .llm import LLMEngine
from .ops import F32, I32
from .params import all_shapes
from .speech import AdapterEngine, FbankGPU, SpeechEncoderEngine
from .tokenizer import load_tokenizer
from .tts import TTSEngine
from .weights import SynthSource


def load_model_dir(model_path, llm_path=None):
    """Parse the reference's config files: audiollm/train.yaml, decoder/model.json,
    codec/model.json and the Qwen2 config.json under llm_path (default <model_path>/llm)."""
    import yaml
    llm_path = llm_path or os.path.join(model_path, "llm")
    with open(os.path.join(model_path, "audiollm", "train.yaml")) as f:
        train = yaml.safe_load(f)
    with open(os.path.join(model_path, "decoder", "model.json")) as f:
        dec = json.load(f)
    with open(os.path.join(model_path, "codec", "model.json")) as f:
        codec = json.load(f)
    with open(os.path.join(llm_path, "config.json")) as f:
        llm = json.load(f)
    cfg = {"train_yaml": train, "llm": llm, "decoder_json": dec, "codec_json": codec}
    synth = None
    sp = os.path.join(model_path, "synthetic.json")
    if os.path.exists(sp):
        with open(sp) as f:
            synth = json.load(f)
    return cfg, synth, llm_path


def make_source(cfg, synth, device, model_path=None, llm_path=None, receive=False):
    """synthetic.json in the model dir -> counter-hash weights generated on the device; otherwise the
    reference's checkpoint files (fo.checkpoint: audiollm/final.pt, the Qwen2 safetensors,
    decoder/final.pt, codec/final.pt).  receive=True: a replica that gets its weights from rank 0's
    broadcast (fo.replica) -- shapes only, nothing is read or generated."""
    if receive:
        from .weights import ReceiveSource
        return ReceiveSource(all_shapes(cfg), device)
    if synth is not None:
        return SynthSource(synth["seed"], all_shapes(cfg), device, {k: tuple(v) for k, v in
                                                                   synth.get("overrides", {}).items()})
    from .checkpoint import load_reference_checkpoints
    return load_reference_checkpoints(cfg, model_path, llm_path, device)


class FreezeOmniEngine:
    def __init__(self, model_path, llm_path=None, device="cuda:0", max_sessions=64, llm_kv_tokens=None,
                 tts_kv_tokens=None, source=None, receive_weights=False, train_yaml=None):
        """receive_weights=True: allocate every packed layout without reading or generating weights; the
        caller fills them with fo.replica.broadcast_frozen(engine, dist) from rank 0 before any use.
        train_yaml: the parsed audiollm/train.yaml as a dict (models/utils.py:init_encoder_llm's configs) in
        place of the file; its cmvn_file, when present on disk, supplies the CMVN statistics
        (models/utils.py:31-38)."""
        if not torch.cuda.is_available():
            raise RuntimeError("FreezeOmniEngine needs an MI355X (gfx950) device: there is no CPU fallback")
        self.device = torch.device(device)
        torch.cuda.set_device(self.device)
        self.cfg, self.synth, self.llm_path = load_model_dir(model_path, llm_path)
        if train_yaml is not None:
            self.cfg["train_yaml"] = train_yaml
        src = source or make_source(self.cfg, self.synth, self.device, model_path, self.llm_path,
                                    receive=receive_weights)
        cmvn = (train_yaml or {}).get("cmvn_file")
        if cmvn and os.path.exists(cmvn) and not receive_weights:
            from .checkpoint import load_cmvn
            from .weights import CheckpointSource, OverlaySource
            mean, istd = load_cmvn(cmvn, bool(self.cfg["train_yaml"].get("is_json_cmvn", True)))
            st = {f"encoder_{i}.global_cmvn.{n}": torch.from_numpy(np.asarray(v, np.float32))
                  for i in ("user", "system") for n, v in (("mean", mean), ("istd", istd))}
            src = OverlaySource(CheckpointSource(st, self.device), src)
        self.src = src
        self.max_sessions = max_sessions
        ty = self.cfg["train_yaml"]
        self.enc = {i: SpeechEncoderEngine(src, self.cfg, i, self.device, max_sessions) for i in ("user", "system")}
        self.ada = {i: AdapterEngine(src, self.cfg, i, self.device, max_sessions) for i in ("user", "system")}
        V = self.cfg["llm"]["vocab_size"]
        self.llm = LLMEngine(src, self.cfg["llm"], self.device,
                             kv_tokens=llm_kv_tokens or min(max_sessions * 4096, 1 << 17))
        self.tts = TTSEngine(src, self.cfg["decoder_json"], self.device,
                             kv_tokens=tts_kv_tokens or min(max_sessions * 2048, 1 << 17))
        self.codec = CodecEngine(src, self.cfg["codec_json"], self.device)
        self.tokenizer = load_tokenizer(self.llm_path, V)
        if not hasattr(self.tokenizer, "eod_id"):
            self.tokenizer.eod_id = self.tokenizer.eos_token_id
        self._fbank = {}
        self._lgraphs = {}
        self._egraphs = {}   # (identity, B, R, stream) -> EncoderGraph (eager listen of steady-state sessions)
        self._tgraphs = {}
        self._prefix_kv = {}   # shared-context chat-prefix KV (listen: _apply_cached_prefixes)
        self.use_graphs = True
        self.predict_usr_state = ty["model_conf"].get("predict_usr_state", 0)
        self._chat_template(ty["model_conf"].get("chat_template"))

    # ------------------------------------------------------------------ models/utils.py:11-28
    def rebind_audiollm(self, state):
        """Load an audiollm/final.pt state (fo.checkpoint.audiollm_state) over this engine, as the
        reference's load_checkpoint does after the model is built: the speech encoders, adapters and
        state head are rebuilt from it; 'llm_decoder.*' entries rebuild the Qwen2 weights too (the KV
        pool with them, so no session may be open).  Unknown keys are ignored (strict=False, utils.py:20);
        a key the path reads with the wrong shape raises."""
        from .checkpoint import CheckpointSource
        from .weights import OverlaySource
        need = all_shapes(self.cfg)
        bad = [f"{k}: {tuple(v.shape)} != {tuple(need[k])}" for k, v in state.items()
               if k in need and tuple(v.shape) != tuple(need[k])]
        if bad:
            raise RuntimeError("load_checkpoint: shape mismatch: " + "; ".join(bad[:20]))
        state = {k: v for k, v in state.items() if k in need}
        src = OverlaySource(CheckpointSource(state, self.device), self.src)
        for g in list(self._lgraphs.values()) + list(self._tgraphs.values()):
            g.destroy()
        self._lgraphs, self._tgraphs = {}, {}
        self.enc = {i: SpeechEncoderEngine(src, self.cfg, i, self.device, self.max_sessions) for i in ("user", "system")}
        self.ada = {i: AdapterEngine(src, self.cfg, i, self.device, self.max_sessions) for i in ("user", "system")}
        if any(k.startswith(("model.", "lm_head.")) for k in state):
            if self.llm.pool.pages_in_use():
                raise RuntimeError("load_checkpoint: Qwen2 weights cannot be replaced while sessions hold KV pages")
            kv_tokens = self.llm.pool.n_pages * self.llm.pool.PS
            self.llm = None   # release the old weights and pool first (15 GB at Qwen2-7B size)
            torch.cuda.empty_cache()
            self.llm = LLMEngine(src, self.cfg["llm"], self.device, kv_tokens=kv_tokens)
        elif "predictor_head.weight" in src:
            self.llm.head_w, self.llm.head_b = src.get("predictor_head.weight"), src.get("predictor_head.bias")
        self.src = src
        return sorted(state)

    # ------------------------------------------------------------------ chat template (audioLLM.py:112-126)
    def _ids(self, text):
        r = self.tokenizer([text])["input_ids"]
        r = r[0]
        return [int(i) for i in (r.tolist() if torch.is_tensor(r) else r)]

    def _chat_template(self, tpl):
        self.chat_template = None
        if tpl is None:
            return
        tok = self.tokenizer
        self.tokenizer.eod_id = self._ids("<|im_end|>")[0]
        a, b = tpl.split("<audio>")
        pre = a.split("<|im_end|>")
        self.chat_template = {"role_prompt": self._ids(pre[0] + "<|im_end|>"),
                              "prefix_for_user_utterance": self._ids(pre[1]),
                              "prefix_for_system_utterance": self._ids(b)}
        self.prefix_ids = {"user": [tok.eod_id] + self.chat_template["prefix_for_user_utterance"],
                           "system": list(self.chat_template["prefix_for_system_utterance"])}

    def fbank(self, kind):
        if kind not in self._fbank:
            self._fbank[kind] = FbankGPU(kind, self.device)
        return self._fbank[kind]

    # ------------------------------------------------------------------ system role (audioLLM.py:312-348)
    def system_role(self, role_prompt=None):
        if role_prompt is not None:
            ids = self._ids(role_prompt)
        else:
            ids = self.chat_template["role_prompt"][:-1]
        x = self.llm.embed(ids, round_fp16=True)  # inputs_embeds.half()
        seq = self.llm.new_seq()
        self.llm.forward(x, [(seq, len(ids))])
        return seq

    # ------------------------------------------------------------------ listen step (audioLLM.py:350-429)
    def listen(self, items, graph=True):
        """items: list of dicts with keys identity ('user'|'system'), status, feats (device [R,80]),
        kv (KVSeq), enc_cache, ada_cache, pe_index (None caches -> fresh state).
        Returns a list of dicts {probs, enc_cache, ada_cache, pe_index, hidden_row} in order.
        Steady-state chunks (one identity, no chat prefix, caches already open) replay a captured
        ListenGraph; everything else runs the eager launch sequence.  hidden_row = (buffer, row):
        the buffer is reused by the next listen call."""
        with torch.cuda.stream(ops.engine_stream(self.device)):
            items = self._apply_cached_prefixes(items)
            if graph and self._graphable(items):
                return self._listen_graph(items)
            return self._listen_eager(items)

    def apply_chat_prefix(self, items):
        """The first chunk's chat-prefix rows applied ahead of its listen (the shared-context prefix cache below):
        afterwards the items are steady-state chunks with open caches, so a ListenPipe can take them too."""
        with torch.cuda.stream(ops.engine_stream(self.device)):
            return self._apply_cached_prefixes(items)

    PREFIX_CACHE = 8
    use_prefix_cache = True

    def _apply_cached_prefixes(self, items):
        """Shared-context prefix caching for the first chunk of a turn (status 'ipu_sl' with the chat
        template): when a session's KV is still exactly the context it was forked from (e.g. the system role
        every session starts from, bin/dialog_state_pred.py:110,218), the chat-prefix rows it is about to
        append (models/audioLLM.py:404-406) are the same tokens on the same keys for every such session, so
        they are computed once per (context, identity), kept as a cached KV extension, and each session
        becomes a copy-on-write fork of it; the chunk then carries only its adapter rows and runs as a
        steady-state (captured) step.  Causal attention makes this exact: the prefix rows never see the audio
        rows.  Sessions with history of their own take the ordinary path."""
        if not self.chat_template or not self.use_prefix_cache:
            return items
        out = []
        for it in items:
            kv = it.get("kv")
            if (it.get("status") == "ipu_sl" and not it.get("prefix_applied") and kv is not None and
                    it.get("identity") in ("user", "system") and kv.pristine()):
                key = (kv.content_key(), it["identity"])
                ext = self._prefix_kv.pop(key, None)
                if ext is None:
                    if len(self._prefix_kv) >= self.PREFIX_CACHE:   # least recently used goes
                        self._prefix_kv.pop(next(iter(self._prefix_kv))).free()
                    ids = self.prefix_ids[it["identity"]]
                    ext = kv.fork()
                    self.llm.forward(self.llm.embed(ids, round_fp16=True), [(ext, len(ids))])
                self._prefix_kv[key] = ext
                kv.adopt(ext)
                it = dict(it, prefix_applied=True)
                if it.get("enc_cache") is None:
                    it["enc_cache"] = self.enc[it["identity"]].new_cache()
                if it.get("ada_cache") is None:
                    it["ada_cache"] = self.ada[it["identity"]].new_cache()
            out.append(it)
        return out

    def _graphable(self, items):
        if not items or not self.use_graphs:
            return False
        ident = items[0]["identity"]
        R = items[0]["feats"].shape[0]
        for it in items:
            if it["identity"] != ident or it["kv"] is None or it["enc_cache"] is None or it["ada_cache"] is None:
                return False
            if it["feats"].shape[0] != R or (self.chat_template and it["status"] == "ipu_sl" and
                                              not it.get("prefix_applied")):
                return False
        if ident not in ("user", "system"):
            return False
        # the captured step gives each session one 16-row attention work item (framing B's 4 LLM
        # tokens x 7 query heads per kv head do not fit: those chunks run eagerly)
        To = self.ada[ident].out_len(self.enc[ident].dims(R)[2])
        return To * (self.llm.H // self.llm.KVH) <= 16

    def _listen_graph_for(self, items, slots=1, extra=64, chunks=1):
        ident = items[0]["identity"]
        B, R = len(items), items[0]["feats"].shape[0]
        need = max(it["kv"].length for it in items) + extra
        key = (ident, B, R, slots) if chunks == 1 else (ident, B, R, "group", chunks)
        g = self._lgraphs.get(key)
        if g is None or g.max_keys < need:
            if g is not None:
                g.destroy()
            if chunks == 1:
                g = ListenGraph(self, ident, B, R, max(need + 1024, 2048), slots=slots)
            else:
                g = ListenGroupGraph(self, ident, B, R, max(need + 1024, 2048), chunks)
            self._lgraphs[key] = g
        return g

    def _listen_graph(self, items):
        return self._listen_graph_for(items).run(items)

    def listen_pipe(self, chunks=1):
        """A ListenPipe over this engine (encoder stage of chunk c+1 overlapped with the LLM of chunk c); chunks > 1:
        that many consecutive chunks per Qwen2 stage (ListenGroupGraph)."""
        return ListenPipe(self, chunks)

    MAX_ENC_GRAPHS = 32

    def _enc_graph(self, ident, B, R):
        """The cached EncoderGraph for (identity, sessions, rows) on the current stream (captured on first use;
        least recently used first out)."""
        st = torch.cuda.current_stream(self.device)
        key = (ident, B, R, st.cuda_stream)
        g = self._egraphs.pop(key, None)
        if g is None:
            if len(self._egraphs) >= self.MAX_ENC_GRAPHS:
                okey = next(iter(self._egraphs))
                torch.cuda.ExternalStream(okey[3], device=self.device).synchronize()   # its last replay's stream only
                self._egraphs.pop(okey).destroy()
            g = EncoderGraph(self, ident, B, R, st)
        self._egraphs[key] = g
        return g

    # stage probe (bench.py --scenario duplex): a list to append (name, HIP event) marks to on the engine stream, or None
    stage_probe = None

    def _mark(self, name):
        if self.stage_probe is not None:
            ev = ctypes.c_void_p()
            _lib.call("fo_event_create", ctypes.byref(ev))
            _lib.call("fo_event_record", ev, ops.stream(self.device))
            self.stage_probe.append((name, ev, time.perf_counter()))

    def _listen_eager(self, items):
        self._mark("start")
        for it in items:
            if it["identity"] not in ("user", "system"):
                raise ValueError(f"Unknown identity: {it['identity']}. Must be 'user' or 'system'.")
            if it["kv"] is None:
                raise AssertionError("must set system role first!!!")
        results = [dict() for _ in items]
        rows = {}
        idents = [d for d in ("user", "system") if any(it["identity"] == d for it in items)]
        # both parties in one call (a duplex tick): the two identities' encoders + adapters are independent, so the
        # second runs on its own stream beside the first (latency-bound launch chains overlap) and the LLM input
        # gather waits for both
        main = torch.cuda.current_stream()
        s2 = ops.engine_stream(self.device, name="enc2") if len(idents) == 2 else None
        if s2 is not None:
            ev_in = torch.cuda.Event()
            ev_in.record(main)
        for k, ident in enumerate(idents):
            idx = [i for i, it in enumerate(items) if it["identity"] == ident]
            side = s2 is not None and k == 1
            with torch.cuda.stream(s2) if side else contextlib.nullcontext():
                if side:
                    s2.wait_event(ev_in)
                    for i in idx:
                        items[i]["feats"].record_stream(s2)
                enc, ada = self.enc[ident], self.ada[ident]
                R = items[idx[0]]["feats"].shape[-2]
                eg = None
                if (self.use_graphs and all(items[i]["enc_cache"] is not None and items[i]["ada_cache"] is not None
                                            and items[i]["feats"].shape[-2] == R for i in idx)):
                    eg = self._enc_graph(ident, len(idx), R)
                if eg is not None:   # steady state: the captured encoder + adapter stage (one launch)
                    ecs = [items[i]["enc_cache"] for i in idx]
                    acs = [items[i]["ada_cache"] for i in idx]
                    emb, To, pes = eg.run([items[i] for i in idx])
                else:
                    ecs = [items[i]["enc_cache"] or enc.new_cache() for i in idx]
                    acs = [items[i]["ada_cache"] or ada.new_cache() for i in idx]
                    feats = torch.stack([items[i]["feats"] for i in idx]) if len(idx) > 1 else items[idx[0]]["feats"][None]
                    out, T, pes = enc.infer(feats.contiguous(), ecs, [items[i]["pe_index"] or 0 for i in idx])
                    emb, To = ada(out, T, acs)
                if side:
                    emb.record_stream(main)
                    ev_out = torch.cuda.Event()
                    ev_out.record(s2)
            for j, i in enumerate(idx):
                results[i].update(enc_cache=ecs[j], ada_cache=acs[j], pe_index=pes[j])
                rows[i] = (emb, j * To, To)
            if s2 is None:
                self._mark("encoder_" + ident)
        if s2 is not None:
            main.wait_event(ev_out)
            self._mark("encoders_both")
        # assemble LLM input rows: [chat prefix (ipu_sl)] + adapter rows, all rounded to fp16 (.half())
        n_tok, pre_ids, pre_pos, ada_src, ada_pos = [], [], [], [], []
        r = 0
        for i, it in enumerate(items):
            emb, r0, To = rows[i]
            p = self.prefix_ids[it["identity"]] if (self.chat_template and it["status"] == "ipu_sl" and
                                                    not it.get("prefix_applied")) else []
            pre_ids += p
            pre_pos += list(range(r, r + len(p)))
            r += len(p)
            ada_pos += list(range(r, r + To))
            ada_src.append((emb, r0, To))
            r += To
            n_tok.append(len(p) + To)
        x = torch.empty(r, self.llm.D, dtype=F32, device=self.device)
        if pre_ids:
            meta = ops.h2d(np.asarray(pre_ids + pre_pos, np.int32), self.device)
            ops.gather_rows(self.llm.embed_tokens, meta[:len(pre_ids)], out=x, round_fp16=True,
                            out_rows=meta[len(pre_ids):])
        emb0 = ada_src[0][0]
        if all(e is emb0 for e, _, _ in ada_src):
            src_rows = [r0 + k for _, r0, To in ada_src for k in range(To)]
            meta = ops.h2d(np.asarray(src_rows + ada_pos, np.int32), self.device)
            ops.gather_rows(emb0, meta[:len(src_rows)], out=x, round_fp16=True, out_rows=meta[len(src_rows):])
        else:
            k = 0
            for (e, r0, To) in ada_src:
                meta = ops.h2d(np.asarray(list(range(r0, r0 + To)) + ada_pos[k:k + To], np.int32), self.device)
                ops.gather_rows(e, meta[:To], out=x, round_fp16=True, out_rows=meta[To:])
                k += To
        self._mark("gather")
        h, bm = self.llm.forward(x, [(it["kv"], n) for it, n in zip(items, n_tok)])
        self._mark("qwen2")
        pred = [i for i, it in enumerate(items) if it["identity"] == "user" and self.predict_usr_state]
        probs = None
        if pred:
            sp = self.llm.state_probs(h, [bm.last_rows_host[i] for i in pred])
            self._mark("state_head")
            probs = sp.cpu().numpy()
        for i in range(len(items)):
            results[i]["probs"] = None
            results[i]["hidden_row"] = (h, bm.last_rows_host[i])
        for j, i in enumerate(pred):
            results[i]["probs"] = {"state_1": float(probs[j, 1]), "state_2": float(probs[j, 2])}
        return results

    # ------------------------------------------------------------------ text decode (A17 reconstruction)
    def text_step(self, items, top_k=1, top_p=0.0, temperature=1.0, seed=0, graph=True):
        """items: list of (kv, input_ids list): forward those tokens, sample the next from the last
        position.  Returns (next ids list, last hidden rows [B, D] device).  One token per session
        (every step after the assistant prefix) replays a captured TextGraph; the result is the same
        launch sequence as the eager path."""
        if graph and self.use_graphs and items and all(len(t) == 1 for _, t in items):
            with torch.cuda.stream(ops.engine_stream(self.device)):
                return self._text_graph_for(items, top_k, top_p, temperature, seed).run(items)
        B = len(items)
        ids = [t for _, toks in items for t in toks]
        x = self.llm.embed(ids, round_fp16=True)
        h, bm = self.llm.forward(x, [(kv, len(toks)) for kv, toks in items])
        rows = torch.tensor(bm.last_rows_host, dtype=I32).to(self.device)
        hid = ops.gather_rows(h, rows)
        logits = self.llm.lm_head(hid)
        par = torch.tensor([top_k] * B, dtype=I32).to(self.device)
        tp = torch.tensor([temperature] * B + [top_p] * B, dtype=F32).to(self.device)
        step = torch.tensor([kv.length for kv, _ in items], dtype=I32).to(self.device)
        out = torch.empty(B, dtype=I32, device=self.device)
        chk = ops.sample_check(self.device)
        ops.sample(logits, self.llm.V, out, par, tp[:B], tp[B:], seed=seed, step=step, err=chk, argmax_ws=top_k == 1)
        ids = out.cpu().tolist()
        chk.check("text decode")
        return ids, hid


    def text_graph(self, kvs, n_tokens, top_k=1, top_p=0.0, temperature=1.0, seed=0):
        """The captured one-token text step for the sessions kvs, sized for n_tokens more tokens: launch() /
        read() queue a step before the previous one is read back (its ids stay on the device)."""
        with torch.cuda.stream(ops.engine_stream(self.device)):
            return self._text_graph_for([(kv, [0]) for kv in kvs], top_k, top_p, temperature, seed,
                                        extra=n_tokens + 64)

    def _text_graph_for(self, items, top_k, top_p, temperature, seed, extra=64):
        B = len(items)
        need = max(kv.length for kv, _ in items) + extra
        key = (B, top_k, float(top_p), float(temperature), seed)
        g = self._tgraphs.get(key)
        if g is None or g.max_keys < need:
            if g is not None:
                g.destroy()
            g = TextGraph(self, B, max(need + 1024, 2048), top_k, top_p, temperature, seed)
            self._tgraphs[key] = g
        return g


def _rows_of_one_tensor(items, n):
    """The items' feature tensors are consecutive [R, 80] rows of ONE storage (a batched fbank's output), so one
    strided copy takes them all.  Separate tensors that merely sit next to each other in the caching allocator's
    memory (each session's features uploaded on its own) do not qualify: a view over the first one's storage would
    run past its end."""
    f0 = items[0]["feats"]
    st = f0.untyped_storage()
    base, size = st.data_ptr(), st.nbytes()
    return (f0.data_ptr() - base + len(items) * n * 4 <= size and
            all(it["feats"].is_contiguous() and it["feats"].numel() == n and
                it["feats"].untyped_storage().data_ptr() == base and
                it["feats"].data_ptr() == f0.data_ptr() + b * n * 4 for b, it in enumerate(items)))


class _HostRing:
    """Pinned host staging buffers for one metadata block, reused once their upload has run."""

    def __init__(self, n, depth=4):
        self.bufs = [torch.empty(n, dtype=I32).pin_memory() for _ in range(depth)]
        self.events = []
        for _ in self.bufs:
            e = ctypes.c_void_p()
            _lib.call("fo_event_create", ctypes.byref(e))
            self.events.append(e)
        self.i = 0

    def next(self):
        k = self.i % len(self.bufs)
        if self.i >= len(self.bufs):
            _lib.call("fo_event_sync", self.events[k])  # that buffer's previous upload has run
        self.i += 1
        return k, self.bufs[k].numpy()

    def upload(self, k, dst, stream):
        with torch.cuda.stream(stream):
            dst.copy_(self.bufs[k], non_blocking=True)
        _lib.call("fo_event_record", self.events[k], stream.cuda_stream)

    def destroy(self):
        for e in self.events:
            _lib.call("fo_event_destroy", e)
        self.events = []


class EncoderGraph:
    """The encoder + adapter stage of B steady-state sessions of one identity (encoder and adapter caches open) as
    one captured hipGraph on the stream it replays on: features -> Conv2dSubsampling4 -> 24 transformer blocks ->
    CNNSubsampling -> the adapter's output rows [B*To, D] (a static buffer, read by the caller before the next run).
    The eager duplex tick (two parties, framing B, no ListenGraph: 4 LLM rows per session) launched these ~150
    kernels one by one and was host-bound there (its enqueue time equalled the stage's GPU span, r04f); the replay is
    one launch.  Same kernels in the same order as the eager path, so the same results."""

    def __init__(self, eng, ident, B, R, stream):
        dev = eng.device
        self.enc, self.ada, self.B, self.R = eng.enc[ident], eng.ada[ident], B, R
        self.feats = torch.empty(B, R, 80, dtype=F32, device=dev)
        self.eb = self.enc.buffers(B, R)
        self.T = self.enc.dims(R)[2]
        self.ab = self.ada.buffers(B, self.T)
        self.To = self.ada.out_len(self.T)
        self.meta_d = torch.zeros(5 * B, dtype=I32, device=dev)
        self.ring = _HostRing(5 * B)
        self.eb["meta"] = self.meta_d[0:4 * B]
        self.ab["slots"] = self.meta_d[4 * B:5 * B]
        self.stream = stream
        self.out = None
        self.exec = ListenGraph._capture(stream, self._body)

    def _body(self):
        xe, T = self.enc.run(self.feats, self.B, self.R, self.eb)
        self.out, _ = self.ada.run(xe, self.B, T, self.ab)

    def run(self, items):
        """items: this identity's items, in order (on self.stream).  Returns (out, To, new pe_indices)."""
        B = self.B
        caches = [it["enc_cache"] for it in items]
        emeta, new_pe = self.enc.host_meta(caches, [it["pe_index"] or 0 for it in items])
        j, h = self.ring.next()
        h[0:4 * B] = emeta
        h[4 * B:5 * B] = [it["ada_cache"].slot for it in items]
        st = self.stream
        with torch.cuda.stream(st):
            # the duplex tick's batched fbank puts one identity's rows next to each other (deliver_deferred): one copy
            f0, n = items[0]["feats"], self.R * 80
            if _rows_of_one_tensor(items, n):
                self.feats.copy_(f0.as_strided((B, self.R, 80), (n, 80, 1)))
            else:
                for b, it in enumerate(items):
                    self.feats[b].copy_(it["feats"].reshape(self.R, 80))
        self.ring.upload(j, self.meta_d, st)
        _lib.call("fo_graph_launch", self.exec, st.cuda_stream)
        self.enc.advance(caches, self.T)
        return self.out, self.To, new_pe

    def destroy(self):
        if self.exec is not None:
            _lib.call("fo_graph_destroy", self.exec)
            self.ring.destroy()
            self.exec = None


class ListenGraph:
    """Steady-state listen step for B sessions of one identity (status ipu_cl / ipu_el: no chat
    prefix) as two captured hipGraphs (models/audioLLM.py:350-429):
      encoder stage: features -> encoder -> adapter -> fp16-rounded LLM input rows (x slot)
      LLM stage:     x slot -> Qwen2 chunk prefill on paged KV -> final norm -> dialog-state head
    Per-call inputs go through static buffers: the features (device copy) and one metadata block per
    stage (encoder ring positions / adapter cache slots; LLM positions, cache slots, visible keys,
    block tables), each uploaded with a single async copy from pinned memory.

    run(items): both stages back to back on the engine stream.
    pipelined: with slots=2, the encoder stage of chunk c+1 runs on a side stream while the LLM stage
    of chunk c runs on the engine stream (ListenPipe); the two stages share nothing but the x slot,
    ordered by events.  The state decision of chunk c does not depend on chunk c+1, so the results are
    those of the sequential order."""

    def __init__(self, eng, ident, B, R, max_keys, slots=1):
        dev = eng.device
        self.eng, self.ident, self.B, self.R, self.max_keys = eng, ident, B, R, max_keys
        enc, ada, llm = eng.enc[ident], eng.ada[ident], eng.llm
        self.enc, self.ada, self.llm = enc, ada, llm
        self.feats = torch.empty(B, R, 80, dtype=F32, device=dev)
        self.eb = enc.buffers(B, R)
        self.T = enc.dims(R)[2]
        self.ab = ada.buffers(B, self.T)
        self.To = To = ada.out_len(self.T)
        n = B * To
        G = llm.H // llm.KVH
        assert To * G <= 16, "listen graph: one attention work item per session"
        PS = llm.pool.PS
        self.maxb = (max_keys + PS - 1) // PS
        # encoder metadata [enc 4B | ada slots B]; LLM metadata [tok_pos n | tok_slot n | tok_nvis n | block table]
        self.emeta_d = torch.zeros(5 * B, dtype=I32, device=dev)
        self.lmeta_d = torch.zeros(3 * n + B * self.maxb, dtype=I32, device=dev)
        self.ering, self.lring = _HostRing(5 * B), _HostRing(3 * n + B * self.maxb)
        self.eb["meta"] = self.emeta_d[0:4 * B]
        self.ab["slots"] = self.emeta_d[4 * B:5 * B]
        m = self.lmeta_d
        items = torch.tensor([[b, b * To, To] for b in range(B)], dtype=I32).reshape(-1).to(dev)
        self.rows = torch.tensor([b * To + To - 1 for b in range(B)], dtype=I32).to(dev)
        self.meta = SimpleNamespace(T=n, S=B, tok_pos=m[0:n], tok_slot=m[n:2 * n], tok_nvis=m[2 * n:3 * n],
                                    block_table=m[3 * n:].view(B, self.maxb), items=items, n_items=B,
                                    max_rows=To * G, max_keys=max_keys, uniform=True)
        self.slots = slots
        self.xs = [torch.empty(n, llm.D, dtype=F32, device=dev) for _ in range(slots)]
        self.x = self.xs[0]
        self.ws = llm.stack.workspace(n, ops.attn_nsplit(max_keys, B, llm.KVH), dev)
        self.predict = ident == "user" and bool(eng.predict_usr_state) and llm.head_w is not None
        self.probs = torch.empty(B, 3, dtype=F32, device=dev)
        self.probs_host = [torch.empty(B, 3, dtype=F32).pin_memory() for _ in range(slots)]
        self.inflight = [None] * slots
        self.main = ops.engine_stream(dev)
        self.side = ops.engine_stream(dev, side=True) if slots > 1 else self.main
        # the encoder stage is captured on the stream it replays on, so its split-K scratch (ops.Runtime)
        # is not the LLM stage's while the two overlap
        self.enc_exec = [self._capture(self.side, lambda k=k: self._enc_body(k), ENC_GEMM_TUNE) for k in range(slots)]
        self.llm_exec = [self._capture(self.main, lambda k=k: self._llm_body(k)) for k in range(slots)]
        self.ev_enc = [self._event() for _ in range(slots)]
        self.ev_llm = [self._event() for _ in range(slots)]
        self.llm_used = [False] * slots
        self.exec = True

    @staticmethod
    def _event():
        e = ctypes.c_void_p()
        _lib.call("fo_event_create", ctypes.byref(e))
        return e

    @staticmethod
    def _capture(stream, body, tune=None):
        """tune: (waves, tiles per workgroup) forced on the GEMMs captured in body (fo_gemm_tune; probes)."""
        s = stream.cuda_stream
        if tune:
            _lib.call("fo_gemm_tune", *tune)
        _lib.call("fo_graph_begin", s)
        try:
            with torch.cuda.stream(stream):
                body()
        finally:
            ex = ctypes.c_void_p()
            _lib.call("fo_graph_end", s, ctypes.byref(ex))
            if tune:
                _lib.call("fo_gemm_tune", 0, 0)
        return ex

    def _enc_body(self, k):
        B, R = self.B, self.R
        xe, T = self.enc.run(self.feats, B, R, self.eb)
        emb, To = self.ada.run(xe, B, T, self.ab)
        ops.gather_rows(emb, None, out=self.xs[k], round_fp16=True)   # inputs_embeds.half()

    def _llm_body(self, k):
        llm, x = self.llm, self.xs[k]
        llm.stack.forward(x, self.meta, self.ws)
        ops.rmsnorm(x, llm.norm, llm.eps, out=x)
        if self.predict:
            ops.state_head(x, self.rows, llm.head_w, llm.head_b, self.probs)

    # ---------------------------------------------------------------- stages
    def submit_encoder(self, items, k=0):
        """Encoder stage of one chunk into x slot k (side stream when pipelined).  Advances the
        encoder caches; returns the per-session pe_index after this chunk."""
        B = self.B
        caches = [it["enc_cache"] for it in items]
        emeta, new_pe = self.enc.host_meta(caches, [it["pe_index"] or 0 for it in items])
        j, h = self.ering.next()
        h[0:4 * B] = emeta
        h[4 * B:5 * B] = [it["ada_cache"].slot for it in items]
        st = self.side
        if self.slots > 1 and self.llm_used[k]:
            _lib.call("fo_stream_wait_event", st.cuda_stream, self.ev_llm[k])  # slot k's last reader is done
        with torch.cuda.stream(st):
            f0 = items[0]["feats"]
            if _rows_of_one_tensor(items, self.R * 80):
                self.feats.copy_(f0.as_strided((B, self.R, 80), (self.R * 80, 80, 1)))  # one batched tensor
            else:
                for b, it in enumerate(items):
                    self.feats[b].copy_(it["feats"])
        self.ering.upload(j, self.emeta_d, st)
        _lib.call("fo_graph_launch", self.enc_exec[k], st.cuda_stream)
        _lib.call("fo_event_record", self.ev_enc[k], st.cuda_stream)
        self.enc.advance(caches, self.T)
        return new_pe

    def submit_llm(self, items, new_pe, k=0, wait=True):
        """LLM stage of the chunk whose encoder stage filled x slot k (engine stream); appends To KV
        rows per session.  wait=True returns the per-session results (reads the state head back);
        wait=False only queues the stage and its state-head copy: collect_llm(k) reads them later."""
        B, To, maxb = self.B, self.To, self.maxb
        n = B * To
        j, h = self.lring.next()
        bt = h[3 * n:].reshape(B, maxb)
        for b, it in enumerate(items):
            kv = it["kv"]
            old = kv.length
            kv.reserve(old + To)
            if len(kv.pages) > maxb:
                raise RuntimeError("listen graph block table too small")
            for i in range(To):
                r = b * To + i
                h[r] = old + i
                h[n + r] = kv.slot(old + i)
                h[2 * n + r] = old + i + 1
            bt[b, :len(kv.pages)] = kv.pages
            kv.length = old + To
        st = self.main
        self.lring.upload(j, self.lmeta_d, st)
        if self.side is not self.main:
            _lib.call("fo_stream_wait_event", st.cuda_stream, self.ev_enc[k])
        _lib.call("fo_graph_launch", self.llm_exec[k], st.cuda_stream)
        if self.predict:
            with torch.cuda.stream(st):
                self.probs_host[k].copy_(self.probs, non_blocking=True)
        _lib.call("fo_event_record", self.ev_llm[k], st.cuda_stream)
        self.llm_used[k] = True
        self.inflight[k] = (items, new_pe)
        return self.collect_llm(k) if wait else None

    def collect_llm(self, k):
        """Results of the LLM stage queued in slot k (waits for it)."""
        items, new_pe = self.inflight[k]
        self.inflight[k] = None
        To = self.To
        _lib.call("fo_event_sync", self.ev_llm[k])
        probs = self.probs_host[k].numpy() if self.predict else None
        res = []
        for b, it in enumerate(items):
            r = {"enc_cache": it["enc_cache"], "ada_cache": it["ada_cache"], "pe_index": new_pe[b],
                 "hidden_row": (self.xs[k], b * To + To - 1), "probs": None}
            if probs is not None:
                r["probs"] = {"state_1": float(probs[b, 1]), "state_2": float(probs[b, 2])}
            res.append(r)
        return res

    def run(self, items):
        return self.submit_llm(items, self.submit_encoder(items, 0), 0)

    def destroy(self):
        if self.exec is not None:
            for ex in self.enc_exec + self.llm_exec:
                _lib.call("fo_graph_destroy", ex)
            for e in self.ev_enc + self.ev_llm:
                _lib.call("fo_event_destroy", e)
            self.ering.destroy()
            self.lring.destroy()
            self.exec = None


class ListenGroupGraph:
    """C consecutive steady-state chunks of B sessions in ONE Qwen2 stage (the listen of an offline input: the
    reference feeds a wav's chunks back to back, bin/inference.py:119-150).  Each chunk's encoder stage is its own
    captured replay (the encoder is chunk-recurrent), writing its rows into the group's x slot chunk-major
    ([chunk][session][token]); the LLM stage then prefills all C x B x To rows at once -- each session's C chunks are
    its next C*To positions, causal, so chunk j's rows see chunks < j of the same stage as the sequential order does
    -- and the dialog-state head reads every chunk's last row (one decision per chunk, models/audioLLM.py:420-429).
    Work items are (session, chunk): To tokens each, as in ListenGraph.  The Qwen2 weights stream once per C chunks
    instead of once per chunk; the GEMMs run at C x 16 rows (k_gemm_xsk / the 17..64-row paths), whose row-count
    dependent tilings give the sequential results to fp32 rounding, not bit for bit.  A group of m < C chunks (the
    end of the input) replays an LLM stage captured for m.  Two slots: the encoder stages of group g+1 run on the side
    stream while group g's LLM stage runs (ListenPipe)."""

    def __init__(self, eng, ident, B, R, max_keys, C):
        dev = eng.device
        self.eng, self.ident, self.B, self.R, self.max_keys, self.C = eng, ident, B, R, max_keys, C
        enc, ada, llm = eng.enc[ident], eng.ada[ident], eng.llm
        self.enc, self.ada, self.llm = enc, ada, llm
        # the group's features, chunk-major ([chunk][session] windows): each push copies its chunk's rows in
        self.feats = torch.empty(C * B, R, 80, dtype=F32, device=dev)
        self.eb = enc.buffers(C * B, R)
        self.T = enc.dims(R)[2]
        self.ab = ada.buffers(B, self.T)
        self.To = To = ada.out_len(self.T)
        G = llm.H // llm.KVH
        assert To * G <= 16, "listen group graph: one attention work item per (session, chunk)"
        self.n1 = n1 = B * To
        self.n = n = C * n1
        PS = llm.pool.PS
        self.maxb = (max_keys + PS - 1) // PS
        # encoder metadata [chunk j: enc 4B] x C | ada slots B -- filled chunk by chunk on the host, uploaded once
        self.emeta_d = torch.zeros(4 * B * C + B, dtype=I32, device=dev)
        self.hmeta = np.zeros(4 * B * C + B, np.int32)
        self.lmeta_d = torch.zeros(3 * n + B * self.maxb, dtype=I32, device=dev)
        self.ering, self.lring = _HostRing(4 * B * C + B), _HostRing(3 * n + B * self.maxb)
        self.eb["meta"] = self.emeta_d[0:4 * B * C]
        self.ab["slots"] = self.emeta_d[4 * B * C:]
        lm = self.lmeta_d
        self.items = torch.tensor([[b, j * n1 + b * To, To] for j in range(C) for b in range(B)],
                                  dtype=I32).reshape(-1).to(dev)
        self.rows = torch.tensor([j * n1 + b * To + To - 1 for j in range(C) for b in range(B)], dtype=I32).to(dev)
        bt = lm[3 * n:].view(B, self.maxb)
        self.metas = {m: SimpleNamespace(T=m * n1, S=B, tok_pos=lm[0:m * n1], tok_slot=lm[n:n + m * n1],
                                         tok_nvis=lm[2 * n:2 * n + m * n1], block_table=bt,
                                         items=self.items[:3 * m * B], n_items=m * B, max_rows=To * G,
                                         max_keys=max_keys, uniform=False)
                      for m in range(1, C + 1)}
        self.xs = [torch.empty(n, llm.D, dtype=F32, device=dev) for _ in range(2)]
        self.ws = llm.stack.workspace(n, ops.attn_nsplit(max_keys, C * B, llm.KVH), dev)
        self.predict = ident == "user" and bool(eng.predict_usr_state) and llm.head_w is not None
        self.probs = torch.empty(C * B, 3, dtype=F32, device=dev)
        self.probs_host = [torch.empty(C * B, 3, dtype=F32).pin_memory() for _ in range(2)]
        self.inflight = [None, None]
        self.main = ops.engine_stream(dev)
        self.side = ops.engine_stream(dev, side=True)
        self.enc_exec = [{}, {}]   # slot -> {chunks in the group: captured encoder stage}
        self.llm_exec = [{}, {}]   # slot -> {chunks in the group: captured LLM stage}
        self.enc_todo = [0, 0]     # chunks whose features are in the slot but whose encoder stage is not queued
        self.ev_enc = [ListenGraph._event() for _ in range(2)]
        self.ev_llm = [ListenGraph._event() for _ in range(2)]
        self.llm_used = [False, False]
        self.exec = True

    def _enc_body(self, k, m):
        """The encoder stage of m chunks: one encoder pass over all their rows (SpeechEncoderEngine.run(chunks=m)),
        then the adapter chunk by chunk (its causal conv cache carries from one to the next), each chunk's rows
        rounded to fp16 into its block of x slot k."""
        B, ne = self.B, self.B * self.T
        xe, T = self.enc.run(self.feats, B, self.R, self.eb, chunks=m)
        for j in range(m):
            emb, To = self.ada.run(xe[j * ne:(j + 1) * ne], B, T, self.ab)
            ops.gather_rows(emb, None, out=self.xs[k][j * self.n1:(j + 1) * self.n1], round_fp16=True)   # .half()

    def _llm_body(self, k, m):
        llm, x = self.llm, self.xs[k][:m * self.n1]
        llm.stack.forward(x, self.metas[m], self.ws)
        ops.rmsnorm(x, llm.norm, llm.eps, out=x)
        if self.predict:
            ops.state_head(x, self.rows[:m * self.B], llm.head_w, llm.head_b, self.probs)

    def submit_encoder(self, items, k, j):
        """Chunk j of the group in slot k: its ring / position metadata (the encoder caches advanced as the
        sequential order does) and its features into the slot's group buffers; the group's encoder stage (side
        stream) is queued with its last chunk (launch_encoder).  Returns the per-session pe_index after this chunk."""
        B = self.B
        caches = [it["enc_cache"] for it in items]
        emeta, new_pe = self.enc.host_meta(caches, [it["pe_index"] or 0 for it in items])
        self.hmeta[4 * B * j:4 * B * (j + 1)] = emeta
        if j == 0:
            self.hmeta[4 * B * self.C:] = [it["ada_cache"].slot for it in items]
        st = self.side
        if j == 0 and self.llm_used[k]:
            _lib.call("fo_stream_wait_event", st.cuda_stream, self.ev_llm[k])   # slot k's last reader is done
        with torch.cuda.stream(st):
            dst = self.feats[j * B:(j + 1) * B]
            if _rows_of_one_tensor(items, self.R * 80):
                dst.copy_(items[0]["feats"].as_strided((B, self.R, 80), (self.R * 80, 80, 1)))
            else:
                for b, it in enumerate(items):
                    dst[b].copy_(it["feats"])
        self.enc.advance(caches, self.T)
        self.enc_todo[k] = j + 1
        if j + 1 == self.C:
            self.launch_encoder(k)
        return new_pe

    def launch_encoder(self, k):
        """Queue slot k's encoder stage over the chunks submitted to it (C, or fewer at the end of the input)."""
        m = self.enc_todo[k]
        if m == 0:
            return
        ex = self.enc_exec[k].get(m)
        if ex is None:
            ex = self.enc_exec[k][m] = ListenGraph._capture(self.side, lambda: self._enc_body(k, m), ENC_GEMM_TUNE)
        q, h = self.ering.next()
        h[:] = self.hmeta
        st = self.side
        self.ering.upload(q, self.emeta_d, st)
        _lib.call("fo_graph_launch", ex, st.cuda_stream)
        _lib.call("fo_event_record", self.ev_enc[k], st.cuda_stream)
        self.enc_todo[k] = 0

    def submit_llm(self, groups, pes, k):
        """The LLM stage of the m = len(groups) chunks whose encoder stages filled slot k (engine stream); appends
        m * To KV rows per session.  collect_llm(k) reads its results."""
        B, To, n1, n, maxb = self.B, self.To, self.n1, self.n, self.maxb
        m = len(groups)
        if self.enc_todo[k]:   # a partial group (the end of the input): its encoder stage is queued now
            self.launch_encoder(k)
        ex = self.llm_exec[k].get(m)
        if ex is None:
            ex = self.llm_exec[k][m] = ListenGraph._capture(self.main, lambda: self._llm_body(k, m))
        q, h = self.lring.next()
        bt = h[3 * n:].reshape(B, maxb)
        for b, it in enumerate(groups[0]):
            kv = it["kv"]
            old = kv.length
            kv.reserve(old + m * To)
            if len(kv.pages) > maxb:
                raise RuntimeError("listen group graph block table too small")
            for j in range(m):
                for i in range(To):
                    r = j * n1 + b * To + i
                    pos = old + j * To + i
                    h[r] = pos
                    h[n + r] = kv.slot(pos)
                    h[2 * n + r] = pos + 1
            bt[b, :len(kv.pages)] = kv.pages
            kv.length = old + m * To
        st = self.main
        self.lring.upload(q, self.lmeta_d, st)
        _lib.call("fo_stream_wait_event", st.cuda_stream, self.ev_enc[k])
        _lib.call("fo_graph_launch", ex, st.cuda_stream)
        if self.predict:
            with torch.cuda.stream(st):
                self.probs_host[k][:m * B].copy_(self.probs[:m * B], non_blocking=True)
        _lib.call("fo_event_record", self.ev_llm[k], st.cuda_stream)
        self.llm_used[k] = True
        self.inflight[k] = (groups, pes)

    def collect_llm(self, k):
        """Results of the LLM stage queued in slot k (waits for it): one result list per chunk, in chunk order."""
        groups, pes = self.inflight[k]
        self.inflight[k] = None
        B, To, n1 = self.B, self.To, self.n1
        _lib.call("fo_event_sync", self.ev_llm[k])
        probs = self.probs_host[k].numpy() if self.predict else None
        out = []
        for j, (items, pe) in enumerate(zip(groups, pes)):
            res = []
            for b, it in enumerate(items):
                r = {"enc_cache": it["enc_cache"], "ada_cache": it["ada_cache"], "pe_index": pe[b],
                     "hidden_row": (self.xs[k], j * n1 + b * To + To - 1), "probs": None}
                if probs is not None:
                    r["probs"] = {"state_1": float(probs[j * B + b, 1]), "state_2": float(probs[j * B + b, 2])}
                res.append(r)
            out.append(res)
        return out

    def destroy(self):
        if self.exec is not None:
            for ex in [e for d in self.enc_exec + self.llm_exec for e in d.values()]:
                _lib.call("fo_graph_destroy", ex)
            for e in self.ev_enc + self.ev_llm:
                _lib.call("fo_event_destroy", e)
            self.ering.destroy()
            self.lring.destroy()
            self.exec = None


class TextGraph:
    """One text-decode step for B sessions (A17 reconstruction, the caller contract of
    bin/inference.py:152-179: one token per session in, the next token out) as one captured hipGraph:
    embedding rows rounded to fp16 (inputs_embeds.half(), models/audioLLM.py:338), the Qwen2 layers on
    paged KV, the final norm, lm_head and the sampler (models/audioLLM.py:431-477).  Per-call inputs
    (token ids, positions, cache slots, visible keys, sampler steps, block tables) go up in one pinned
    upload and the drawn ids come back in one pinned download."""

    def __init__(self, eng, B, max_keys, top_k, top_p, temperature, seed):
        dev = eng.device
        llm = eng.llm
        self.eng, self.B, self.max_keys, self.seed = eng, B, max_keys, seed
        PS = llm.pool.PS
        self.maxb = (max_keys + PS - 1) // PS
        # metadata [ids B | tok_pos B | tok_slot B | tok_nvis B | sampler step B | block table B x maxb]
        n_meta = 5 * B + B * self.maxb
        self.meta_d = torch.zeros(n_meta, dtype=I32, device=dev)
        self.ring = _HostRing(n_meta)
        m = self.meta_d
        self.ids, self.step = m[0:B], m[4 * B:5 * B]
        items = torch.tensor([[b, b, 1] for b in range(B)], dtype=I32).reshape(-1).to(dev)
        self.meta = SimpleNamespace(T=B, S=B, tok_pos=m[B:2 * B], tok_slot=m[2 * B:3 * B], tok_nvis=m[3 * B:4 * B],
                                    block_table=m[5 * B:].view(B, self.maxb), items=items, n_items=B,
                                    max_rows=llm.H // llm.KVH, max_keys=max_keys)
        self.x = torch.empty(B, llm.D, dtype=F32, device=dev)
        self.logits = torch.empty(B, llm.lm_head.N, dtype=F32, device=dev)
        self.ws = llm.stack.workspace(B, ops.attn_nsplit(max_keys, B, llm.KVH), dev)
        self.par = torch.tensor([top_k] * B, dtype=I32).to(dev)
        self.tp = torch.tensor([temperature] * B + [top_p] * B, dtype=F32).to(dev)
        self.out = torch.empty(B, dtype=I32, device=dev)
        # steps in flight (launch() / read()): each has its own pinned id read-back and event
        self.out_host = [torch.empty(B, dtype=I32).pin_memory() for _ in range(self.DEPTH)]
        self.evs = [ListenGraph._event() for _ in range(self.DEPTH)]
        self.n_launched = self.n_read = 0
        self.top_k = top_k
        self.err = ops.SampleCheck()
        self.main = ops.engine_stream(dev)
        self.exec = ListenGraph._capture(self.main, self._body)

    DEPTH = 4

    def _body(self):
        # the step's input ids are read from `out`: the previous step's draw (a step queued behind it, launch()
        # without ids), or the host's ids copied there first; the draw then overwrites them
        llm, B = self.eng.llm, self.B
        ops.gather_rows(llm.embed_tokens, self.out, out=self.x, round_fp16=True)
        llm.stack.forward(self.x, self.meta, self.ws)
        ops.rmsnorm(self.x, llm.norm, llm.eps, out=self.x)
        llm.lm_head(self.x, out=self.logits)
        ops.sample(self.logits, llm.V, self.out, self.par, self.tp[:B], self.tp[B:], seed=self.seed, step=self.step,
                   err=self.err, argmax_ws=self.top_k == 1)

    def run(self, items):
        """items: list of (kv, [token id]) in batch order; appends one KV position per session."""
        return self.read(self.launch([kv for kv, _ in items], [toks[0] for _, toks in items]))

    def launch(self, kvs, ids=None):
        """Queue one step for the sessions kvs (batch order) and return its handle for read().  ids: the input
        token per session from the host; None: the ids the previous launched step draws (still on the device),
        so the step can be queued before that one is read back.  Appends one KV position per session."""
        B, maxb = self.B, self.maxb
        if self.n_launched - self.n_read >= self.DEPTH:
            raise RuntimeError("text graph: more than DEPTH steps in flight")
        if ids is None and self.n_launched == 0:
            raise ValueError("text graph: the first step needs its input ids")
        j, h = self.ring.next()
        bt = h[5 * B:].reshape(B, maxb)
        for b, kv in enumerate(kvs):
            L = kv.length
            kv.reserve(L + 1)
            if len(kv.pages) > maxb:
                raise RuntimeError("text graph block table too small")
            if ids is not None:
                h[b] = ids[b]
            h[B + b] = L
            h[2 * B + b] = kv.slot(L)
            h[3 * B + b] = L + 1
            h[4 * B + b] = L + 1   # the eager path's sampler step: the sequence length after the forward
            bt[b, :len(kv.pages)] = kv.pages
            kv.length = L + 1
        st = self.main
        self.ring.upload(j, self.meta_d, st)
        k = self.n_launched % self.DEPTH
        with torch.cuda.stream(st):
            if ids is not None:
                self.out.copy_(self.ids)
            _lib.call("fo_graph_launch", self.exec, st.cuda_stream)
            self.out_host[k].copy_(self.out, non_blocking=True)
            hid = self.x.clone()
        _lib.call("fo_event_record", self.evs[k], st.cuda_stream)
        self.n_launched += 1
        return (k, hid)

    def read(self, handle):
        """Wait for a launched step; returns (drawn ids list, last hidden rows [B, D] device)."""
        k, hid = handle
        _lib.call("fo_event_sync", self.evs[k])
        self.n_read += 1
        self.err.check("text decode step")
        return self.out_host[k].tolist(), hid

    def destroy(self):
        if self.exec is not None:
            _lib.call("fo_graph_destroy", self.exec)
            for e in self.evs:
                _lib.call("fo_event_destroy", e)
            self.ring.destroy()
            self.err.free()
            self.exec = None


# probe knob: FO_ENC_TUNE="waves,tiles" forces the GEMM shape of the pipelined encoder stage's graph (the stage
# beside the Qwen2 stage, off the critical path: fewer, wider workgroups re-read its activations less often)
ENC_GEMM_TUNE = tuple(int(v) for v in os.environ["FO_ENC_TUNE"].split(",")) if os.environ.get("FO_ENC_TUNE") else None


class ListenPipe:
    """Pipelined steady-state listen for one batch of sessions (ListenGraph with two x slots).

        pipe = engine.listen_pipe()
        pe_next, prev = pipe.push(items_c, decide)   # chunk c's next pe_index per session; results of c-1
        ...; last = pipe.flush()

    push(items_c): queues chunk c's encoder stage (side stream) and, behind chunk c-1's, chunk c's LLM stage
    (engine stream), then waits for chunk c-1's LLM stage and reads its results (the state decision).  If
    decide(results of c-1) returns False -- the reference's "stop listening on dialog_ss" -- chunk c's LLM
    stage is rolled back (waited for, its KV rows truncated), so the context holds exactly the chunks before
    it, as if it had never been queued.  The encoder stage of chunk c overlaps the LLM stage of chunk c-1,
    the engine stream never idles on the host's read-back, and the caller prepares chunk c+1 (framing,
    fbank) while chunk c's LLM stage runs.  A refused chunk's encoder stage has run (its caches are reset
    on dialog_ss anyway, bin/inference.py:133-135).
    (encoder / adapter caches are advanced in place at submission, like listen().)

    Every push must be graphable (same identity and batch, no chat prefix, open caches); the results
    are identical to calling listen() chunk by chunk."""

    def __init__(self, eng, chunks=1):
        self.eng, self.g, self.pending, self.k = eng, None, None, 0
        self.stopped = False
        self.C = int(chunks)
        self.acc = []   # chunks > 1: (items, pe) of the group being assembled in slot k

    def push(self, items, decide=None):
        eng = self.eng
        if self.stopped:
            raise RuntimeError("ListenPipe: decide() stopped this pipe (flush and start a new one)")
        if self.C > 1:
            return self._push_group(items, decide)
        with torch.cuda.stream(ops.engine_stream(eng.device)):
            if not eng._graphable(items):
                raise ValueError("ListenPipe.push: items must be steady-state chunks (no chat prefix, open caches)")
            g = eng._listen_graph_for(items, slots=2, extra=64 * 2)
            if self.g is not None and g is not self.g:
                raise RuntimeError("ListenPipe: the batch changed (flush before changing sessions)")
            self.g = g
            k = self.k
            pe = g.submit_encoder(items, k)
            # chunk c's LLM stage is queued speculatively right behind chunk c-1's on the engine stream, so the
            # stream never idles while the host reads c-1's state head back; if the decision on c-1 stops the
            # listen (dialog_ss), chunk c is rolled back below and never reaches the context
            g.submit_llm(items, pe, k, wait=False)
            out = None
            if self.pending is not None:
                out = g.collect_llm(self.pending)
            self.pending = k
            self.k = 1 - k
            if decide is not None and out is not None and not decide(out):
                self._roll_back(k)
                self.stopped = True
            return pe, out

    def _roll_back(self, k):
        """Undo the speculative LLM stage in slot k: wait for it, drop the KV rows it appended."""
        g = self.g
        items, _ = g.inflight[k]
        _lib.call("fo_event_sync", g.ev_llm[k])
        g.inflight[k] = None
        for it in items:
            it["kv"].truncate(it["kv"].length - g.To)
        self.pending = None

    def flush(self):
        if self.C > 1:
            return self._flush_group()
        if self.pending is None:
            return None
        with torch.cuda.stream(ops.engine_stream(self.eng.device)):
            k, self.pending = self.pending, None
            return self.g.collect_llm(k)

    # ---- chunks > 1 (ListenGroupGraph): push returns (pe after this chunk, None or the per-chunk result lists of the
    # previous group, in chunk order); decide() is asked chunk by chunk, and a refusal rolls back every later chunk
    # already in a stage (the rest of its group and the speculative next group)
    def _push_group(self, items, decide):
        eng = self.eng
        with torch.cuda.stream(ops.engine_stream(eng.device)):
            if not eng._graphable(items):
                raise ValueError("ListenPipe.push: items must be steady-state chunks (no chat prefix, open caches)")
            g = eng._listen_graph_for(items, extra=64 * 2 * self.C, chunks=self.C)
            if self.g is not None and g is not self.g:
                raise RuntimeError("ListenPipe: the batch changed (flush before changing sessions)")
            self.g = g
            k = self.k
            pe = g.submit_encoder(items, k, len(self.acc))
            self.acc.append((items, pe))
            self.kvs = [it["kv"] for it in items]
            out = None
            if len(self.acc) == self.C:
                g.submit_llm([a for a, _ in self.acc], [p for _, p in self.acc], k)
                self.acc = []
                if self.pending is not None:
                    out = g.collect_llm(self.pending)
                self.pending = k
                self.k = 1 - k
                if decide is not None and out is not None:
                    self._decide_group(out, decide, newer=[k])
            return pe, out

    def _decide_group(self, out, decide, newer):
        """Ask decide() chunk by chunk; on a refusal drop the chunks after it from `out` and from every session's KV,
        together with every stage in `newer` (waited for first): the context holds exactly the chunks up to the
        refused one, as in the sequential order."""
        for j, res in enumerate(out):
            if decide(res):
                continue
            g = self.g
            drop = (len(out) - 1 - j) * g.To
            for k in newer:
                if g.inflight[k] is not None:
                    _lib.call("fo_event_sync", g.ev_llm[k])
                    drop += len(g.inflight[k][0]) * g.To
                    g.inflight[k] = None
            for kv in self.kvs:
                kv.truncate(kv.length - drop)
            del out[j + 1:]
            self.pending = None
            self.acc = []
            self.stopped = True
            return

    def _flush_group(self):
        g = self.g
        if g is None:
            return None
        with torch.cuda.stream(ops.engine_stream(self.eng.device)):
            out = []
            if self.pending is not None:
                out += g.collect_llm(self.pending)
                self.pending = None
            if self.acc:   # the end of the input: a partial group of m < C chunks
                k = self.k
                g.submit_llm([a for a, _ in self.acc], [p for _, p in self.acc], k)
                self.acc = []
                out += g.collect_llm(k)
                self.k = 1 - k
            return out or None
