"""Tokenizers backed by the native C++ implementations (csrc/runtime/tokenizer.cpp).

* :class:`GPT2Tokenizer` — byte-level BPE from ``vocab.json`` + ``merges.txt`` (or ``tokenizer.json``);
  EOS = PAD = BOS = ``<|endoftext|>`` (reference core/tokenizer_bpe.h:29-32).
* :class:`GemmaTokenizer` — SentencePiece-BPE from Gemma's ``tokenizer.json`` with byte fallback and
  special tokens ``<bos> <eos> <pad> <unk>`` (reference core/tokenizer_gemma.h:18-31); add_bos
  default True like the reference.
"""
from __future__ import annotations

import os

from .._ext import native


class GPT2Tokenizer:
    def __init__(self, impl):
        self._t = impl

    @classmethod
    def from_pretrained(cls, path: str) -> "GPT2Tokenizer":
        rt = native().runtime
        if os.path.isdir(path):
            v, m = os.path.join(path, "vocab.json"), os.path.join(path, "merges.txt")
            if os.path.exists(v) and os.path.exists(m):
                return cls(rt.ByteLevelBPE.from_files(v, m))
            tj = os.path.join(path, "tokenizer.json")
            if os.path.exists(tj):
                return cls(rt.ByteLevelBPE.from_tokenizer_json(tj))
            raise FileNotFoundError(f"no vocab.json+merges.txt or tokenizer.json in {path}")
        return cls(rt.ByteLevelBPE.from_tokenizer_json(path))

    @classmethod
    def from_files(cls, vocab_json: str, merges_txt: str) -> "GPT2Tokenizer":
        return cls(native().runtime.ByteLevelBPE.from_files(vocab_json, merges_txt))

    def encode(self, text: str, add_bos: bool = False):
        ids = self._t.encode(text)
        return ([self.bos_id] + ids) if add_bos else ids

    def encode_batch(self, texts):
        return self._t.encode_batch(list(texts))

    def decode(self, ids, skip_special: bool = False) -> str:
        return self._t.decode(list(map(int, ids)), skip_special)

    def batch_encode(self, texts, max_len: int, pad: bool = True):
        """Reference GPT2BPETokenizer::batch_encode: truncate / right-pad with PAD, returns (ids, mask)."""
        out, mask = [], []
        for ids in self.encode_batch(texts):
            ids = ids[:max_len]
            m = [1] * len(ids)
            if pad:
                ids = ids + [self.pad_id] * (max_len - len(ids))
                m = m + [0] * (max_len - len(m))
            out.append(ids)
            mask.append(m)
        return out, mask

    def token_id(self, s):
        return self._t.token_id(s)

    @property
    def vocab_size(self):
        return self._t.vocab_size

    @property
    def eos_id(self):
        return self._t.eos_id

    @property
    def bos_id(self):
        return self._t.bos_id

    @property
    def pad_id(self):
        return self._t.pad_id

    @property
    def native(self):
        return self._t


class GemmaTokenizer:
    def __init__(self, impl):
        self._t = impl

    @classmethod
    def from_pretrained(cls, path: str) -> "GemmaTokenizer":
        tj = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
        return cls(native().runtime.SentencePieceBPE.from_tokenizer_json(tj))

    def encode(self, text: str, add_bos: bool = True):
        return self._t.encode(text, add_bos)

    def encode_batch(self, texts, add_bos: bool = False):
        return self._t.encode_batch(list(texts), add_bos)

    def decode(self, ids, skip_special: bool = True) -> str:
        return self._t.decode(list(map(int, ids)), skip_special)

    def token_id(self, s):
        return self._t.token_id(s)

    @property
    def vocab_size(self):
        return self._t.vocab_size

    @property
    def eos_id(self):
        return self._t.eos_id

    @property
    def bos_id(self):
        return self._t.bos_id

    @property
    def pad_id(self):
        return self._t.pad_id

    @property
    def native(self):
        return self._t


def load_tokenizer(kind: str, path: str):
    if kind in ("gpt2", "bytelevel"):
        return GPT2Tokenizer.from_pretrained(path)
    if kind in ("gemma", "gemma3", "sentencepiece"):
        return GemmaTokenizer.from_pretrained(path)
    raise ValueError(kind)
