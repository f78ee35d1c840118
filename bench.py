#!/usr/bin/env python3
"""Headline benchmark: GPT-2-124M LoRA r=8, seq 128, bf16 training throughput (tokens/s).

Metric/config from BASELINE.json ("tokens/sec GPT-2-124M LoRA r=8 seq128 at 1/2/4/8 GPU").
Synthetic token data + random-init GPT-2-124M weights (no network); one process per GPU
(launch with torch.distributed.run for N > 1; RCCL over xGMI).  Every timed step is a full
training step: forward, fused LM-head cross-entropy, backward through all 12 blocks, gradient
all-reduce (N > 1), global grad-norm clip and the fused AdamW update.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--seq 128] [--no-graph]

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# the reference publishes no tokens/s; its README epoch time (4-6 h / epoch of
# WikiText-2 on a mobile SoC, README.md:419) gives a derived 110-170 tokens/s.  We divide by the
# upper bound (170) so vs_baseline is conservative.
BASELINE_TOKENS_PER_SEC = 170.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    # 256 x 128 = 32k tokens per GPU per step: the M dimension every block GEMM sees.  Measured on
    # 1x MI355X: B=64 0.89M tok/s, B=128 1.02M, B=256 1.09M (block GEMMs reach higher MFMA
    # utilisation at M=32k; 288 GB HBM makes the activation footprint irrelevant).
    ap.add_argument("--batch", type=int, default=int(os.environ.get("MFT_BENCH_BATCH", 256)),
                    help="micro-batch (sequences) per GPU")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--rank", type=int, default=8)
    ap.add_argument("--alpha", type=float, default=16.0)
    ap.add_argument("--targets", default="AttnQKV,AttnProj")
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--grad_accum", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--profile", action="store_true", help="print a per-phase breakdown to stderr")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.optim.adamw import FusedAdamW
    from mobilefinetuner_amd.parallel.ddp import DataParallel
    from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2, lora_parameters, parse_gpt2_targets
    from mobilefinetuner_amd.train.engine import TrainStep
    from mobilefinetuner_amd.utils.params import FlatParams

    cfg = GPT2Config.preset(a.model)
    model = GPT2Model(cfg, dtype=torch.bfloat16, device=dev, seed=1234)  # identical on every rank
    spec = LoraSpec(rank=a.rank, alpha=a.alpha, targets=parse_gpt2_targets(a.targets))
    inject_gpt2(model, spec)
    flat = FlatParams(lora_parameters(model), dev)
    opt = FusedAdamW(flat, lr=2e-4, weight_decay=0.0, max_grad_norm=1.0)
    dp = DataParallel(flat) if world > 1 else None
    step = TrainStep(model, flat, opt, grad_accum=a.grad_accum, dp=dp, use_graph=not a.no_graph)

    # synthetic WikiText-shaped data: per-rank disjoint random token streams, labels = next token
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    nbuf = 4
    data = []
    for _ in range(nbuf):
        mb = []
        for _ in range(a.grad_accum):
            toks = torch.randint(0, cfg.vocab_size, (a.batch, a.seq + 1), generator=g)
            mb.append((toks[:, :-1].contiguous().to(dev), toks[:, 1:].contiguous().to(dev)))
        data.append(mb)

    for i in range(a.warmup):
        step(data[i % nbuf])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(data[i % nbuf])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    final_loss = float(loss.item())
    tokens = world * a.batch * a.seq * a.grad_accum * a.steps
    value = tokens / dt
    if rank == 0:
        out = {
            "metric": "tokens/sec GPT-2-124M LoRA r=8 seq128 (training, whole job)",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * dt / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_TOKENS_PER_SEC, 1),
            "dtype": "bf16",
            "data": "synthetic (random tokens, random-init weights)",
            "config": {
                "model": f"{a.model} (124M) LoRA r={a.rank} alpha={a.alpha:g} targets={a.targets}",
                "global_batch": world * a.batch * a.grad_accum,
                "micro_batch_per_gpu": a.batch,
                "seq_len": a.seq,
                "parallelism": f"dp{world}",
                "hipgraph": not a.no_graph,
                "final_loss": round(final_loss, 4),
                "baseline_tokens_per_sec": BASELINE_TOKENS_PER_SEC,
            },
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
