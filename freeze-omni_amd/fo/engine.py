"""One Freeze-Omni replica on one MI355X: model loading plus the batched hot-path primitives that the
reference-API layer (freeze-omni_amd/models) and the benchmark drive.

Reference flow being replaced: inferencePipeline.__init__ (models/pipeline.py:12-34)
loads train.yaml + final.pt + Qwen2; speech_dialogue -> AudioLLM.set_system_role / recognize
(models/audioLLM.py:312-429); llm2TTS.run -> LLM2TTSCodecAR.infer + VQVAE (models/decoder/*).
Where the reference runs one user per call with ~hundreds of small launches, every primitive here
takes a list of sessions and issues one launch sequence for all of them.
"""
import ctypes
import json
import os
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


def make_source(cfg, synth, device, model_path=None, llm_path=None):
    """synthetic.json in the model dir -> counter-hash weights generated on the device; otherwise the
    reference's checkpoint files (fo.checkpoint: audiollm/final.pt, the Qwen2 safetensors,
    decoder/final.pt, codec/final.pt)."""
    if synth is not None:
        return SynthSource(synth["seed"], all_shapes(cfg), device, {k: tuple(v) for k, v in
                                                                   synth.get("overrides", {}).items()})
    from .checkpoint import load_reference_checkpoints
    return load_reference_checkpoints(cfg, model_path, llm_path, device)


class FreezeOmniEngine:
    def __init__(self, model_path, llm_path=None, device="cuda:0", max_sessions=64, llm_kv_tokens=None,
                 tts_kv_tokens=None, source=None):
        if not torch.cuda.is_available():
            raise RuntimeError("FreezeOmniEngine needs an MI355X (gfx950) device: there is no CPU fallback")
        self.device = torch.device(device)
        torch.cuda.set_device(self.device)
        self.cfg, self.synth, self.llm_path = load_model_dir(model_path, llm_path)
        src = source or make_source(self.cfg, self.synth, self.device, model_path, self.llm_path)
        self.src = src
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
        self.use_graphs = True
        self.predict_usr_state = ty["model_conf"].get("predict_usr_state", 0)
        self._chat_template(ty["model_conf"].get("chat_template"))

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
            if graph and self._graphable(items):
                return self._listen_graph(items)
            return self._listen_eager(items)

    def _graphable(self, items):
        if not items or not self.use_graphs:
            return False
        ident = items[0]["identity"]
        R = items[0]["feats"].shape[0]
        for it in items:
            if it["identity"] != ident or it["kv"] is None or it["enc_cache"] is None or it["ada_cache"] is None:
                return False
            if it["feats"].shape[0] != R or (self.chat_template and it["status"] == "ipu_sl"):
                return False
        return ident in ("user", "system")

    def _listen_graph(self, items):
        ident = items[0]["identity"]
        B, R = len(items), items[0]["feats"].shape[0]
        need = max(it["kv"].length for it in items) + 64
        key = (ident, B, R)
        g = self._lgraphs.get(key)
        if g is None or g.max_keys < need:
            if g is not None:
                g.destroy()
            g = ListenGraph(self, ident, B, R, max(need + 1024, 2048))
            self._lgraphs[key] = g
        return g.run(items)

    def _listen_eager(self, items):
        for it in items:
            if it["identity"] not in ("user", "system"):
                raise ValueError(f"Unknown identity: {it['identity']}. Must be 'user' or 'system'.")
            if it["kv"] is None:
                raise AssertionError("must set system role first!!!")
        results = [dict() for _ in items]
        rows = {}
        for ident in ("user", "system"):
            idx = [i for i, it in enumerate(items) if it["identity"] == ident]
            if not idx:
                continue
            enc, ada = self.enc[ident], self.ada[ident]
            ecs = [items[i]["enc_cache"] or enc.new_cache() for i in idx]
            acs = [items[i]["ada_cache"] or ada.new_cache() for i in idx]
            feats = torch.stack([items[i]["feats"] for i in idx]) if len(idx) > 1 else items[idx[0]]["feats"][None]
            out, T, pes = enc.infer(feats.contiguous(), ecs, [items[i]["pe_index"] or 0 for i in idx])
            emb, To = ada(out, T, acs)
            for j, i in enumerate(idx):
                results[i].update(enc_cache=ecs[j], ada_cache=acs[j], pe_index=pes[j])
                rows[i] = (emb, j * To, To)
        # assemble LLM input rows: [chat prefix (ipu_sl)] + adapter rows, all rounded to fp16 (.half())
        n_tok, pre_ids, pre_pos, ada_src, ada_pos = [], [], [], [], []
        r = 0
        for i, it in enumerate(items):
            emb, r0, To = rows[i]
            p = self.prefix_ids[it["identity"]] if (self.chat_template and it["status"] == "ipu_sl") else []
            pre_ids += p
            pre_pos += list(range(r, r + len(p)))
            r += len(p)
            ada_pos += list(range(r, r + To))
            ada_src.append((emb, r0, To))
            r += To
            n_tok.append(len(p) + To)
        x = torch.empty(r, self.llm.D, dtype=F32, device=self.device)
        if pre_ids:
            meta = torch.tensor(pre_ids + pre_pos, dtype=I32).to(self.device)
            ops.gather_rows(self.llm.embed_tokens, meta[:len(pre_ids)], out=x, round_fp16=True,
                            out_rows=meta[len(pre_ids):])
        emb0 = ada_src[0][0]
        if all(e is emb0 for e, _, _ in ada_src):
            src_rows = [r0 + k for _, r0, To in ada_src for k in range(To)]
            meta = torch.tensor(src_rows + ada_pos, dtype=I32).to(self.device)
            ops.gather_rows(emb0, meta[:len(src_rows)], out=x, round_fp16=True, out_rows=meta[len(src_rows):])
        else:
            k = 0
            for (e, r0, To) in ada_src:
                meta = torch.tensor(list(range(r0, r0 + To)) + ada_pos[k:k + To], dtype=I32).to(self.device)
                ops.gather_rows(e, meta[:To], out=x, round_fp16=True, out_rows=meta[To:])
                k += To
        h, bm = self.llm.forward(x, [(it["kv"], n) for it, n in zip(items, n_tok)])
        pred = [i for i, it in enumerate(items) if it["identity"] == "user" and self.predict_usr_state]
        probs = None
        if pred:
            probs = self.llm.state_probs(h, [bm.last_rows_host[i] for i in pred]).cpu().numpy()
        for i in range(len(items)):
            results[i]["probs"] = None
            results[i]["hidden_row"] = (h, bm.last_rows_host[i])
        for j, i in enumerate(pred):
            results[i]["probs"] = {"state_1": float(probs[j, 1]), "state_2": float(probs[j, 2])}
        return results

    # ------------------------------------------------------------------ text decode (A17 reconstruction)
    def text_step(self, items, top_k=1, top_p=0.0, temperature=1.0, seed=0):
        """items: list of (kv, input_ids list): forward those tokens, sample the next from the last
        position.  Returns (next ids list, last hidden rows [B, D] device)."""
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
        ops.sample(logits, self.llm.V, out, par, tp[:B], tp[B:], seed=seed, step=step)
        return out.cpu().tolist(), hid


class ListenGraph:
    """Steady-state listen step for B sessions of one identity (status ipu_cl / ipu_el: no chat
    prefix), captured once as a hipGraph: features -> encoder -> adapter -> fp16-rounded LLM rows ->
    Qwen2 chunk prefill on paged KV -> final norm -> dialog-state head (models/audioLLM.py:350-429).
    Per-call inputs go through static buffers: the features (device copy) and one metadata block
    (encoder ring positions, adapter cache slots, LLM positions / cache slots / visible keys / block
    tables) uploaded with a single async copy from pinned memory."""

    def __init__(self, eng, ident, B, R, max_keys):
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
        # metadata block: [enc 4B | ada slots B | tok_pos n | tok_slot n | tok_nvis n | block table B*maxb]
        self.n_meta = 5 * B + 3 * n + B * self.maxb
        self.meta_d = torch.zeros(self.n_meta, dtype=I32, device=dev)
        self.host = [torch.empty(self.n_meta, dtype=I32).pin_memory() for _ in range(4)]
        self.host_ev = []
        for _ in self.host:
            e = ctypes.c_void_p()
            _lib.call("fo_event_create", ctypes.byref(e))
            self.host_ev.append(e)
        self.hi = 0
        m = self.meta_d
        self.eb["meta"] = m[0:4 * B]
        self.ab["slots"] = m[4 * B:5 * B]
        o = 5 * B
        items = torch.tensor([[b, b * To, To] for b in range(B)], dtype=I32).reshape(-1).to(dev)
        self.rows = torch.tensor([b * To + To - 1 for b in range(B)], dtype=I32).to(dev)
        self.meta = SimpleNamespace(T=n, S=B, tok_pos=m[o:o + n], tok_slot=m[o + n:o + 2 * n],
                                    tok_nvis=m[o + 2 * n:o + 3 * n], block_table=m[o + 3 * n:].view(B, self.maxb),
                                    items=items, n_items=B, max_rows=To * G, max_keys=max_keys)
        self.x = torch.empty(n, llm.D, dtype=F32, device=dev)
        self.ws = llm.stack.workspace(n, ops.attn_nsplit(max_keys, B, llm.KVH), dev)
        self.predict = ident == "user" and bool(eng.predict_usr_state) and llm.head_w is not None
        self.probs = torch.empty(B, 3, dtype=F32, device=dev)
        self.probs_host = torch.empty(B, 3, dtype=F32).pin_memory()
        self.exec = None
        s = ops.stream(dev)
        _lib.call("fo_graph_begin", s)
        try:
            self._body()
        finally:
            ex = ctypes.c_void_p()
            _lib.call("fo_graph_end", s, ctypes.byref(ex))
        self.exec = ex

    def _body(self):
        B, R, llm = self.B, self.R, self.llm
        xe, T = self.enc.run(self.feats, B, R, self.eb)
        emb, To = self.ada.run(xe, B, T, self.ab)
        ops.gather_rows(emb, None, out=self.x, round_fp16=True)   # inputs_embeds.half()
        llm.stack.forward(self.x, self.meta, self.ws)
        ops.rmsnorm(self.x, llm.norm, llm.eps, out=self.x)
        if self.predict:
            ops.state_head(self.x, self.rows, llm.head_w, llm.head_b, self.probs)

    def run(self, items):
        B, To, maxb = self.B, self.To, self.maxb
        enc = self.enc
        caches = [it["enc_cache"] for it in items]
        emeta, new_pe = enc.host_meta(caches, [it["pe_index"] or 0 for it in items])
        slot = self.hi % len(self.host)
        self.hi += 1
        if self.hi > len(self.host):
            _lib.call("fo_event_sync", self.host_ev[slot])  # that slot's previous upload has run
        h = self.host[slot].numpy()
        h[0:4 * B] = emeta
        h[4 * B:5 * B] = [it["ada_cache"].slot for it in items]
        n = B * To
        o = 5 * B
        bt = h[o + 3 * n:].reshape(B, maxb)
        for b, it in enumerate(items):
            kv = it["kv"]
            old = kv.length
            kv.reserve(old + To)
            if len(kv.pages) > maxb:
                raise RuntimeError("listen graph block table too small")
            for i in range(To):
                r = b * To + i
                h[o + r] = old + i
                h[o + n + r] = kv.slot(old + i)
                h[o + 2 * n + r] = old + i + 1
            bt[b, :len(kv.pages)] = kv.pages
            kv.length = old + To
        f0 = items[0]["feats"]
        if f0.is_contiguous() and all(it["feats"].data_ptr() == f0.data_ptr() + b * self.R * 80 * 4
                                      for b, it in enumerate(items)):
            self.feats.copy_(f0.as_strided((B, self.R, 80), (self.R * 80, 80, 1)))  # one batched feature tensor
        else:
            for b, it in enumerate(items):
                self.feats[b].copy_(it["feats"])
        st = ops.stream(self.eng.device)
        self.meta_d.copy_(self.host[slot], non_blocking=True)
        _lib.call("fo_event_record", self.host_ev[slot], st)
        _lib.call("fo_graph_launch", self.exec, st)
        enc.advance(caches, self.T)
        probs = None
        if self.predict:
            self.probs_host.copy_(self.probs, non_blocking=False)
            probs = self.probs_host.numpy()
        res = []
        for b, it in enumerate(items):
            r = {"enc_cache": it["enc_cache"], "ada_cache": it["ada_cache"], "pe_index": new_pe[b],
                 "hidden_row": (self.x, b * To + To - 1), "probs": None}
            if probs is not None:
                r["probs"] = {"state_1": float(probs[b, 1]), "state_2": float(probs[b, 2])}
            res.append(r)
        return res

    def destroy(self):
        if self.exec is not None:
            _lib.call("fo_graph_destroy", self.exec)
            self.exec = None
        for e in self.host_ev:
            _lib.call("fo_event_destroy", e)
        self.host_ev = []
