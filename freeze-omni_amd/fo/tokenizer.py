"""Tokenizer loading for AudioLLM (models/audioLLM.py:73-74 AutoTokenizer.from_pretrained(llm_path)).

When llm_path carries tokenizer files the transformers tokenizer is used (host-side string work,
exactly like the reference).  Synthetic-weight runs at Qwen2-7B geometry have no tokenizer files
offline; ByteFallbackTokenizer then maps the chat special tokens and the chat template's words to
Qwen2's ids (so the prompts have Qwen2's token counts) and every other UTF-8 byte to a fixed id,
which is enough for the benchmark's fixed prompts.
"""
import os
import re

QWEN2_SPECIAL = {"<|endoftext|>": 151643, "<|im_start|>": 151644, "<|im_end|>": 151645}
# Qwen2 BPE ids of the pieces of the chat template and default system prompt, so the benchmark's
# prompts have the real tokenizer's lengths (e.g. "<|im_end|>\n<|im_start|>assistant\n" = 5 tokens)
QWEN2_WORDS = {"\n": 198, "system": 8948, "user": 872, "assistant": 77091, "You": 2610, " are": 525, " a": 264,
               " helpful": 10950, " assistant": 17847, ".": 13}
_BYTE_BASE = 1000  # byte b -> id b + _BYTE_BASE (inside Qwen2's 152064 vocabulary)
_PIECES = re.compile(r" ?[A-Za-z]+| ?[0-9]| ?[^\sA-Za-z0-9]+|\s+")  # GPT-style pre-tokenisation (ASCII subset)


class ByteFallbackTokenizer:
    def __init__(self, vocab_size=152064):
        self.vocab_size = vocab_size
        self.special = {k: v for k, v in QWEN2_SPECIAL.items() if v < vocab_size}
        self.words = {k: v for k, v in QWEN2_WORDS.items() if v < vocab_size}
        self.inv = {v: k for k, v in self.special.items()}
        self.inv_words = {v: k for k, v in self.words.items()}
        self.eos_token_id = self.special.get("<|endoftext|>", 0)
        self._split = re.compile("(" + "|".join(re.escape(s) for s in self.special) + ")")

    def encode(self, text):
        ids = []
        for part in self._split.split(text):
            if not part:
                continue
            if part in self.special:
                ids.append(self.special[part])
                continue
            for piece in _PIECES.findall(part) if part.isascii() else [part]:
                if piece in self.words:
                    ids.append(self.words[piece])
                else:
                    ids.extend(b + _BYTE_BASE for b in piece.encode("utf-8"))
        return ids

    def __call__(self, texts, return_tensors=None):
        if isinstance(texts, str):
            return {"input_ids": self.encode(texts)}
        ids = [self.encode(t) for t in texts]
        if return_tensors == "pt":
            import torch
            return {"input_ids": torch.tensor(ids)}
        return {"input_ids": ids}

    def decode(self, ids, skip_special_tokens=False):
        out, buf = [], bytearray()
        for i in ids:
            i = int(i)
            if _BYTE_BASE <= i < _BYTE_BASE + 256:
                buf.append(i - _BYTE_BASE)
                continue
            if buf:
                out.append(buf.decode("utf-8", errors="replace"))
                buf = bytearray()
            if i in self.inv_words:
                out.append(self.inv_words[i])
            elif i in self.inv and not skip_special_tokens:
                out.append(self.inv[i])
        if buf:
            out.append(buf.decode("utf-8", errors="replace"))
        return "".join(out)


def load_tokenizer(llm_path, vocab_size):
    if llm_path and (os.path.exists(os.path.join(llm_path, "tokenizer.json"))
                     or os.path.exists(os.path.join(llm_path, "vocab.json"))):
        from transformers import AutoTokenizer
        return AutoTokenizer.from_pretrained(llm_path, trust_remote_code=False)
    return ByteFallbackTokenizer(vocab_size)
