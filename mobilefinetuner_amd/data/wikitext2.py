"""WikiText-2 (and any line-based text / pretokenized stream) datasets on the native C++ loader.

Reference: WikiText2Dataset (operators/finetune_ops/data/wikitext2_dataset.h:19-158); WT2Config
fields map 1:1 onto :class:`WT2Config`.  Batches come back as pinned CPU tensors:
``input_ids [B,S] int64``, ``targets [B,S] int64`` (already shifted next-token labels, -100 on padding
and on the last position of each chunk: the reference's labels=inputs + shift-in-loss semantics),
``attention_mask [B,S] float`` and ``lengths [B] int32``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from .._ext import native

SPLITS = {"train": 0, "valid": 1, "validation": 1, "test": 2}
FILES = {
    "train": ("wiki.train.raw", "wiki.train.tokens", "train.txt"),
    "valid": ("wiki.valid.raw", "wiki.valid.tokens", "valid.txt", "validation.txt"),
    "test": ("wiki.test.raw", "wiki.test.tokens", "test.txt"),
}


@dataclass
class WT2Config:
    data_dir: str = ""
    train_path: str = ""
    valid_path: str = ""
    test_path: str = ""
    pretokenized_path: str = ""
    pretokenized_meta: str = ""
    seq_len: int = 128
    stride: int = -1
    eos_id: int = 50256
    pad_id: int = 0
    insert_eos_between_lines: bool = True
    drop_last: bool = True
    seed: int = 2025
    shuffle_train: bool = True
    data_fraction: float = 1.0
    rank: int = 0
    world: int = 1

    def path_for(self, split: str) -> str:
        explicit = {"train": self.train_path, "valid": self.valid_path, "test": self.test_path}[split]
        if explicit:
            return explicit
        for name in FILES[split]:
            p = os.path.join(self.data_dir, name)
            if os.path.exists(p):
                return p
        raise FileNotFoundError(f"no {split} file under {self.data_dir!r} (tried {FILES[split]})")


def _resolve_meta(bin_path: str, meta: str) -> str:
    if meta:
        return meta
    cand = os.path.join(os.path.dirname(bin_path), "meta.json")
    if os.path.exists(cand):
        return cand
    raise FileNotFoundError(f"cannot locate meta.json for {bin_path}")


class LMDataset:
    """Chunked LM dataset over one token stream (one split)."""

    def __init__(self, cfg: WT2Config, split: str, tokens: torch.Tensor):
        rt = native().runtime
        self.cfg, self.split = cfg, split
        dc = rt.DataConfig()
        dc.seq_len, dc.stride = cfg.seq_len, cfg.stride
        dc.eos_id, dc.pad_id = cfg.eos_id, cfg.pad_id
        dc.insert_eos_between_lines = cfg.insert_eos_between_lines
        dc.drop_last = cfg.drop_last if split == "train" else cfg.drop_last
        dc.seed = cfg.seed
        dc.shuffle = cfg.shuffle_train if split == "train" else False
        dc.data_fraction = cfg.data_fraction
        dc.rank, dc.world = cfg.rank, cfg.world
        self._d = rt.TokenDataset(dc)
        self._d.set_tokens(tokens)

    # ---- construction helpers
    @classmethod
    def from_text(cls, cfg: WT2Config, split: str, tokenizer) -> "LMDataset":
        rt = native().runtime
        lines = rt.read_lines(cfg.path_for(split), cfg.insert_eos_between_lines)
        t = tokenizer.native
        if isinstance(t, rt.ByteLevelBPE):
            toks = rt.pack_lines_bytelevel(t, lines, cfg.eos_id, cfg.insert_eos_between_lines, cfg.data_fraction,
                                           cfg.seq_len)
        else:
            toks = rt.pack_lines_sentencepiece(t, lines, cfg.eos_id, cfg.insert_eos_between_lines,
                                               cfg.data_fraction, cfg.seq_len)
        return cls(cfg, split, toks)

    @classmethod
    def from_pretokenized(cls, cfg: WT2Config, split: str) -> "LMDataset":
        rt = native().runtime
        meta_path = _resolve_meta(cfg.pretokenized_path, cfg.pretokenized_meta)
        meta = rt.read_pretok_meta(meta_path)
        if meta["eos_token_id"] >= 0:
            cfg.eos_id = meta["eos_token_id"]
        if meta["pad_token_id"] >= 0:
            cfg.pad_id = meta["pad_token_id"]
        cfg.insert_eos_between_lines = meta["insert_eos_between_lines"]
        toks = rt.read_pretok_split(cfg.pretokenized_path, meta_path, SPLITS[split], cfg.data_fraction, cfg.seq_len)
        return cls(cfg, split, toks)

    @classmethod
    def synthetic(cls, cfg: WT2Config, split: str, vocab_size: int, n_tokens: int, seed: int = 0) -> "LMDataset":
        g = torch.Generator().manual_seed(seed + SPLITS[split])
        toks = torch.randint(0, vocab_size, (n_tokens,), generator=g, dtype=torch.int32)
        return cls(cfg, split, toks)

    @classmethod
    def load(cls, cfg: WT2Config, split: str, tokenizer=None) -> "LMDataset":
        if cfg.pretokenized_path:
            return cls.from_pretokenized(cfg, split)
        if tokenizer is None:
            raise ValueError("text datasets need a tokenizer")
        return cls.from_text(cfg, split, tokenizer)

    # ---- iteration
    def num_sequences(self) -> int:
        return self._d.num_sequences()

    def num_local(self) -> int:
        return self._d.num_local()

    def __len__(self):
        return self.num_local()

    def next_batch(self, batch_size: int, need_loop: bool = True):
        got, ids, tg, mk, ln = self._d.next_batch(batch_size, need_loop)
        if got == 0:
            return None
        return {"input_ids": ids, "targets": tg, "attention_mask": mk, "lengths": ln, "rows": got}

    def get_batch(self, chunk_indices):
        ids, tg, mk, ln = self._d.get_batch([int(i) for i in chunk_indices])
        return {"input_ids": ids, "targets": tg, "attention_mask": mk, "lengths": ln, "rows": len(chunk_indices)}

    def reset_cursor(self):
        self._d.reset_cursor()

    def shuffle(self):
        self._d.shuffle()

    def tokens(self) -> torch.Tensor:
        return self._d.tokens()

    def state(self) -> dict:
        return {"epoch": self._d.epoch(), "cursor": self._d.cursor(), "rng": bytes(self._d.rng_state()).hex()}

    def restore(self, st: dict):
        self._d.restore(int(st["epoch"]), int(st["cursor"]), bytes.fromhex(st.get("rng", "")))

    @property
    def epoch(self):
        return self._d.epoch()


def write_pretokenized(out_dir: str, splits: dict, eos_id: int, pad_id: int, vocab_size: int,
                       bos_id: int = -1, unk_id: int = -1, insert_eos: bool = True, name: str = "tokens.bin"):
    """Write {split: int32 tensor} as one stream + meta.json (scripts/pretokenize_wikitext2_gemma.py
    layout)."""
    import json
    os.makedirs(out_dir, exist_ok=True)
    off, meta_splits, parts = 0, {}, []
    for s in ("train", "valid", "test"):
        if s in splits:
            t = splits[s].to(torch.int32).contiguous()
            meta_splits[s] = {"offset": off, "length": int(t.numel())}
            off += int(t.numel())
            parts.append(t)
    allt = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int32)
    path = os.path.join(out_dir, name)
    allt.numpy().tofile(path)
    meta = {"total_tokens": int(allt.numel()), "eos_token_id": eos_id, "pad_token_id": pad_id, "bos_token_id": bos_id,
            "unk_token_id": unk_id, "vocab_size": vocab_size, "insert_eos_between_lines": insert_eos,
            "splits": meta_splits}
    with open(os.path.join(out_dir, "meta.json"), "w") as f:
        json.dump(meta, f, indent=2)
    return path
