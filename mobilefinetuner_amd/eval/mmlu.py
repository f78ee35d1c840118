"""MMLU multiple-choice evaluation (reference MMLURunner, gpt2_lora_finetune/mmlu/mmlu_runner.cpp).

Same data layout (``<root>/<split>/*.csv`` with header subject,question,a,b,c,d,answer), same
prompt (``Question: ...\\nA. ...\\nB. ...\\nC. ...\\nD. ...\\nAnswer: `` with k-shot examples of the
same subject, each followed by its letter and a blank line), same scoring (log-softmax of the last
position over the tokens of "A".."D", argmax), macro/micro accuracy.  Differences: prompts are
evaluated in length-sorted right-padded batches on the GPU (causal attention makes padding
harmless for the last real position), the log-softmax+gather is one HIP kernel over only the last
rows (K15), and few-shot examples exclude the current item by index (the reference compared
addresses of copies, so an item among the first k could be its own example).
"""
from __future__ import annotations

import csv
import glob
import os
from collections import defaultdict
from dataclasses import dataclass

import torch

from ..ops import functional as Fx


@dataclass
class MCQ:
    subject: str
    question: str
    A: str
    B: str
    C: str
    D: str
    answer: str


def read_split(root: str, split: str):
    by_subj = defaultdict(list)
    for path in sorted(glob.glob(os.path.join(root, split, "*.csv"))):
        with open(path, newline="", encoding="utf-8") as f:
            rows = list(csv.reader(f))
        if not rows:
            continue
        head = [c.strip().lower() for c in rows[0]]
        idx = {k: head.index(k) if k in head else -1 for k in ("subject", "question", "a", "b", "c", "d", "answer")}
        if min(idx[k] for k in ("question", "a", "b", "c", "d", "answer")) < 0:
            # headerless Hendrycks layout: question,a,b,c,d,answer ; subject from the filename
            idx = {"subject": -1, "question": 0, "a": 1, "b": 2, "c": 3, "d": 4, "answer": 5}
            body = rows
        else:
            body = rows[1:]
        subj_from_file = os.path.basename(path).rsplit("_", 1)[0] if "_" in os.path.basename(path) else \
            os.path.splitext(os.path.basename(path))[0]
        for r in body:
            if len(r) <= max(idx.values()) or not any(x.strip() for x in r):
                continue
            ans = r[idx["answer"]].strip().upper()[:1] or "A"
            s = r[idx["subject"]].strip() if idx["subject"] >= 0 else subj_from_file
            by_subj[s].append(MCQ(s, r[idx["question"]].strip(), r[idx["a"]].strip(), r[idx["b"]].strip(),
                                  r[idx["c"]].strip(), r[idx["d"]].strip(), ans))
    return dict(by_subj)


def build_prompt(x: MCQ, shots=()):
    def one(q):
        return f"Question: {q.question}\nA. {q.A}\nB. {q.B}\nC. {q.C}\nD. {q.D}\nAnswer: "
    p = "".join(one(s) + s.answer + "\n\n" for s in shots)
    return p + one(x)


@torch.no_grad()
def score_prompts(model, tokenizer, prompts, letter_ids, device, batch_size=16, max_len=None):
    """Return [N, 4] log-probs of the letter tokens at the last prompt position."""
    from .._ext import native
    enc = [tokenizer.encode(p) if not hasattr(tokenizer, "bos_id") or tokenizer.__class__.__name__ != "GemmaTokenizer"
           else tokenizer.encode(p, add_bos=True) for p in prompts]
    if max_len:
        enc = [e[-max_len:] for e in enc]  # keep the tail (the question being asked)
    order = sorted(range(len(enc)), key=lambda i: len(enc[i]))
    out = torch.empty(len(enc), 4)
    w = Fx.cw(model.wte if hasattr(model, "wte") else model.embed)
    V = model.cfg.vocab_size
    idx = torch.tensor(letter_ids, dtype=torch.int64, device=device)
    for s in range(0, len(order), batch_size):
        chunk = order[s:s + batch_size]
        L = max(len(enc[i]) for i in chunk)
        ids = torch.zeros(len(chunk), L, dtype=torch.int64)
        last = []
        for r, i in enumerate(chunk):
            ids[r, : len(enc[i])] = torch.tensor(enc[i])
            last.append(r * L + len(enc[i]) - 1)
        h = model.hidden(ids.to(device))
        hl = h[torch.tensor(last, device=device)]
        logits = hl @ w.t()
        if logits.is_cuda and logits.dtype == torch.bfloat16:
            lp = native().logsoftmax_gather(logits.contiguous(), idx, V).float().cpu()
        else:
            lp = torch.log_softmax(logits[:, :V].float(), -1)[:, idx.cpu()].cpu()
        for r, i in enumerate(chunk):
            out[i] = lp[r]
    return out


def evaluate(model, tokenizer, data, device, fewshot=0, batch_size=16, max_len=None):
    letters = []
    for L in "ABCD":
        ids = tokenizer.encode(L) if tokenizer.__class__.__name__ != "GemmaTokenizer" else tokenizer.encode(L, add_bos=False)
        letters.append(ids[0] if ids else 0)
    per = []
    tc = tn = 0
    for subj in sorted(data):
        items = data[subj]
        prompts = []
        for i, x in enumerate(items):
            shots = [items[j] for j in range(min(fewshot, len(items))) if j != i] if fewshot > 0 else []
            prompts.append(build_prompt(x, shots))
        lp = score_prompts(model, tokenizer, prompts, letters, device, batch_size, max_len)
        pred = lp.argmax(-1).tolist()
        correct = sum(1 for x, p in zip(items, pred) if "ABCD"[p] == x.answer)
        per.append({"subject": subj, "correct": correct, "total": len(items), "acc": correct / max(1, len(items))})
        tc += correct
        tn += len(items)
    macro = sum(r["acc"] for r in per) / max(1, len(per))
    micro = tc / max(1, tn)
    return {"per_subject": per, "macro": macro, "micro": micro, "total": tn}
