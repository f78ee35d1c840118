"""eval_ppl — WikiText-2 perplexity of GPT-2 (optionally + a LoRA adapter), reference
gpt2_lora_finetune/eval_ppl.cpp:67-231.

Non-overlapping chunks (stride = seq_len, tail kept), token-weighted mean NLL over the predicted
tokens (exact, SURVEY §8 Q17: the reference weighted each batch's mean by all non-pad labels),
ppl = exp(nll), one JSONL record {"task":"wt2_ppl","split","tokens","nll","ppl","model","lora"}.
Evaluation runs under no_grad with the fused chunked CE (no logits materialisation); multi-GPU
runs shard the chunks and all-reduce the NLL/token sums.  ``--model_type gemma`` evaluates Gemma-3.
"""
from __future__ import annotations

import argparse
import json
import math
import time

import torch

from . import common


def build_parser():
    ap = argparse.ArgumentParser(prog="eval_ppl", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--data_root", default="")
    ap.add_argument("--split", default="valid", choices=["train", "valid", "test"])
    ap.add_argument("--seq_len", type=int, default=1024)
    ap.add_argument("--batch_size", type=int, default=1)
    ap.add_argument("--pretrained_dir", default="")
    ap.add_argument("--lora_path", default="")
    ap.add_argument("--lora_merge", type=int, default=1)
    ap.add_argument("--out", default="")
    ap.add_argument("--log_every", type=int, default=50)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--model_type", default="gpt2", choices=["gpt2", "gemma"])
    ap.add_argument("--pretokenized_path", default="")
    ap.add_argument("--pretokenized_meta", default="")
    ap.add_argument("--max_batches", type=int, default=0)
    common.add_runtime_args(ap)
    return ap


@torch.no_grad()
def evaluate(model, ds, batch_size, dev, log_every=0, max_batches=0):
    from ..parallel.ddp import allreduce_sum_
    from ..utils.logging import log0
    tot = torch.zeros(2, dtype=torch.float64, device=dev)
    nb = 0
    t0 = time.time()
    while True:
        b = ds.next_batch(batch_size, need_loop=False)
        if b is None or (max_batches and nb >= max_batches):
            break
        s, n = model.nll(b["input_ids"].to(dev), b["targets"].to(dev))
        tot[0] += s.double()
        tot[1] += n.double()
        nb += 1
        if log_every and nb % log_every == 0:
            log0(f"  [{nb}] running ppl {math.exp(float(tot[0] / tot[1].clamp(min=1))):.3f} ({time.time() - t0:.1f}s)")
    allreduce_sum_(tot)
    nll = float(tot[0] / tot[1].clamp(min=1))
    return nll, int(tot[1])


def main(argv=None):
    a = build_parser().parse_args(argv)
    from ..data.wikitext2 import LMDataset, WT2Config
    from ..io.lora_checkpoint import attach_lora, load_lora
    from ..peft.lora import merge_all, set_lora_enabled
    from ..utils.logging import log0
    rank, world, _, dev = common.init_distributed(a.device, getattr(a, 'dist_timeout_s', 600.0))
    dt = common.dtype_of(a)
    if a.model_type == "gpt2":
        model = common.load_gpt2(a.pretrained_dir, a.model, a.random_init, dev, dt)
        a.seq_len = min(a.seq_len, model.cfg.n_positions)
    else:
        model = common.load_gemma(a.pretrained_dir, a.model, a.random_init, dev, dt)
    model.eval()
    if a.lora_path:
        tensors, meta = load_lora(a.lora_path)
        spec = attach_lora(model, tensors, meta)
        log0(f"  ✓ LoRA attached: rank={spec.rank} alpha={spec.alpha:g}")
        if a.lora_merge:
            merge_all(model)
            set_lora_enabled(model, False)
            log0("  ✓ LoRA merged into base weights")
        elif dev.type == "cuda":
            # separate adapters: the fp32 A / B need their bf16 compute shadows (FlatParams)
            from ..peft.lora import lora_parameters
            from ..utils.params import FlatParams
            model._lora_flat = FlatParams(lora_parameters(model), dev)
    if a.model_type == "gemma":
        eos = model.cfg.eos_token_id
    else:
        eos = 50256
    cfg = WT2Config(data_dir=a.data_root, seq_len=a.seq_len, eos_id=eos, drop_last=False, shuffle_train=False,
                    rank=rank, world=world, pretokenized_path=a.pretokenized_path,
                    pretokenized_meta=a.pretokenized_meta)
    if a.synthetic_data or (not a.data_root and not a.pretokenized_path):
        vocab = model.cfg.vocab_size
        ds = LMDataset.synthetic(cfg, a.split, vocab, a.synthetic_tokens)
    elif a.pretokenized_path:
        ds = LMDataset.from_pretokenized(cfg, a.split)
    else:
        if a.model_type == "gpt2":
            from ..tokenizers import GPT2Tokenizer
            tok = GPT2Tokenizer.from_pretrained(a.pretrained_dir)
        else:
            from ..tokenizers import GemmaTokenizer
            tok = GemmaTokenizer.from_pretrained(a.pretrained_dir)
        cfg.eos_id = tok.eos_id
        ds = LMDataset.from_text(cfg, a.split, tok)
    log0(f"[eval_ppl] split={a.split} seq_len={a.seq_len} chunks={ds.num_sequences()} ranks={world}")
    t0 = time.time()
    nll, ntok = evaluate(model, ds, a.batch_size, dev, a.log_every, a.max_batches)
    ppl = math.exp(min(nll, 50.0))
    dt_s = time.time() - t0
    rec = {"task": "wt2_ppl", "split": a.split, "tokens": ntok, "nll": nll, "ppl": ppl,
           "model": a.pretrained_dir or a.model or a.model_type, "lora": a.lora_path, "seconds": dt_s,
           "tokens_per_sec": ntok / max(dt_s, 1e-9)}
    log0(json.dumps(rec))
    if rank == 0:
        common.jsonl_append(a.out, rec)
    return rec


if __name__ == "__main__":
    main()
