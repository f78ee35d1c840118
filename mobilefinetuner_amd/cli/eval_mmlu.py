"""eval_mmlu — MMLU accuracy of GPT-2 / Gemma-3 (+ optional LoRA), reference
gpt2_lora_finetune/eval_mmlu.cpp:60-167 (flags: --mmlu_root --split --fewshot --pretrained_dir
--lora_path --lora_merge --out --debug).  Writes per-subject + macro/micro records as JSONL."""
from __future__ import annotations

import argparse
import json

from . import common


def build_parser():
    ap = argparse.ArgumentParser(prog="eval_mmlu", description=__doc__)
    ap.add_argument("--mmlu_root", required=True)
    ap.add_argument("--split", default="dev", choices=["dev", "val", "test"])
    ap.add_argument("--fewshot", type=int, default=0)
    ap.add_argument("--pretrained_dir", default="")
    ap.add_argument("--lora_path", default="")
    ap.add_argument("--lora_merge", type=int, default=1)
    ap.add_argument("--out", default="")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--batch_size", type=int, default=16)
    ap.add_argument("--model_type", default="gpt2", choices=["gpt2", "gemma"])
    ap.add_argument("--tokenizer_dir", default="")
    common.add_runtime_args(ap)
    return ap


def main(argv=None):
    a = build_parser().parse_args(argv)
    from ..eval.mmlu import evaluate, read_split
    from ..io.lora_checkpoint import attach_lora, load_lora
    from ..peft.lora import merge_all, set_lora_enabled
    from ..utils.logging import log0
    _, _, _, dev = common.init_distributed(a.device, getattr(a, 'dist_timeout_s', 600.0))
    dt = common.dtype_of(a)
    if a.model_type == "gpt2":
        from ..tokenizers import GPT2Tokenizer
        model = common.load_gpt2(a.pretrained_dir, a.model, a.random_init, dev, dt)
        tok = GPT2Tokenizer.from_pretrained(a.tokenizer_dir or a.pretrained_dir)
        max_len = model.cfg.n_positions
    else:
        from ..tokenizers import GemmaTokenizer
        model = common.load_gemma(a.pretrained_dir, a.model, a.random_init, dev, dt)
        tok = GemmaTokenizer.from_pretrained(a.tokenizer_dir or a.pretrained_dir)
        max_len = None
    model.eval()
    if a.lora_path:
        t, m = load_lora(a.lora_path)
        attach_lora(model, t, m)
        if a.lora_merge:
            merge_all(model)
            set_lora_enabled(model, False)
    data = read_split(a.mmlu_root, a.split)
    log0(f"[eval_mmlu] {sum(len(v) for v in data.values())} questions in {len(data)} subjects (split={a.split}, "
         f"fewshot={a.fewshot})")
    res = evaluate(model, tok, data, dev, a.fewshot, a.batch_size, max_len)
    for r in res["per_subject"]:
        log0(f"  {r['subject']:<40} {r['correct']:>5}/{r['total']:<5} acc={r['acc']:.4f}")
    log0(f"[eval_mmlu] macro={res['macro']:.4f} micro={res['micro']:.4f} total={res['total']}")
    if a.out:
        for r in res["per_subject"]:
            common.jsonl_append(a.out, {"task": "mmlu", "split": a.split, **r})
        common.jsonl_append(a.out, {"task": "mmlu", "split": a.split, "macro": res["macro"], "micro": res["micro"],
                                    "total": res["total"], "fewshot": a.fewshot, "lora": a.lora_path})
    print(json.dumps({"macro": res["macro"], "micro": res["micro"], "total": res["total"]}))
    return res


if __name__ == "__main__":
    main()
