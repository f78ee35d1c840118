"""Pretokenize WikiText-2 (or any train/valid/test text files) into ONE int32 token stream +
``meta.json`` -- the layout ``train_lora_gemma --pretokenized_path`` / ``eval_ppl`` read.

Reference: scripts/pretokenize_wikitext2_gemma.py:1-129 (HF tokenizer in Python, one stream, EOS
between lines, meta {total_tokens, eos/pad/bos/unk, vocab_size, insert_eos_between_lines,
splits{offset,length}}).  Here the tokenizers are the native C++ ones (csrc/runtime/tokenizer.cpp,
byte-level BPE for GPT-2, SentencePiece-BPE for Gemma-3) and the line packing is the native
multi-threaded ``pack_lines`` (EOS after every line, blank lines included, like the reference's
WikiText2Dataset), so training from the .bin sees exactly the tokens text mode would produce.

    python -m mobilefinetuner_amd.cli.pretokenize --data_dir wikitext-2-raw --tokenizer_dir gemma-3-270m \\
        --model_type gemma --out_dir data/wt2_gemma
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def build_parser():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--data_dir", required=True, help="directory with wiki.{train,valid,test}.raw (or *.tokens/*.txt)")
    ap.add_argument("--tokenizer_dir", required=True, help="vocab.json+merges.txt or tokenizer.json directory")
    ap.add_argument("--model_type", default="gpt2", choices=["gpt2", "gemma"])
    ap.add_argument("--out_dir", required=True)
    ap.add_argument("--name", default="", help="output file name (default wt2_<model_type>_tokens.bin)")
    ap.add_argument("--splits", default="train,valid,test")
    ap.add_argument("--no_eos_between_lines", action="store_true")
    return ap


def main(argv=None):
    a = build_parser().parse_args(argv)
    import torch
    from ..data.wikitext2 import FILES, LMDataset, WT2Config, write_pretokenized
    from ..tokenizers import load_tokenizer
    tok = load_tokenizer(a.model_type, a.tokenizer_dir)
    insert_eos = not a.no_eos_between_lines
    cfg = WT2Config(data_dir=a.data_dir, seq_len=1, eos_id=tok.eos_id, pad_id=tok.pad_id,
                    insert_eos_between_lines=insert_eos, shuffle_train=False, drop_last=False)
    streams = {}
    for split in [s.strip() for s in a.splits.split(",") if s.strip()]:
        try:
            path = cfg.path_for(split)
        except FileNotFoundError:
            print(f"[pretokenize] no {split} file under {a.data_dir} (tried {FILES[split]}), skipped")
            continue
        t0 = time.perf_counter()
        toks = LMDataset.from_text(cfg, split, tok).tokens()
        streams[split] = torch.as_tensor(toks, dtype=torch.int32)
        dt = time.perf_counter() - t0
        print(f"[pretokenize] {split}: {os.path.basename(path)} -> {streams[split].numel():,} tokens "
              f"({streams[split].numel() / max(dt, 1e-9):,.0f} tok/s)")
    if not streams:
        print("[pretokenize] nothing to do", file=sys.stderr)
        return 1
    unk = getattr(tok.native, "unk_id", -1)
    name = a.name or f"wt2_{a.model_type}_tokens.bin"
    out = write_pretokenized(a.out_dir, streams, eos_id=tok.eos_id, pad_id=tok.pad_id, vocab_size=tok.vocab_size,
                             bos_id=tok.bos_id, unk_id=unk, insert_eos=insert_eos, name=name)
    with open(os.path.join(a.out_dir, "meta.json")) as f:
        meta = json.load(f)
    print(f"[pretokenize] wrote {out} ({meta['total_tokens']:,} tokens) + meta.json")
    return 0


if __name__ == "__main__":
    sys.exit(main())
