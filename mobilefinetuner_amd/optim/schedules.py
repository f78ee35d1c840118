"""Learning-rate schedules reproducing the reference's three variants exactly.

(a) GPT-2 CLIs (gpt2_lora_finetune/main.cpp:470-488, gpt2_full_finetune/main.cpp:394-407):
    linear warmup lr*(step+1)/W for step < W, then cosine from lr down to 10% of lr.
(b) Gemma trainer (optim/gemma_trainer.cpp:63-82): warmup = ceil(ratio * total_updates);
    1-indexed step; lr*step/warmup while step <= warmup, then linear (default) or cosine to 0.
(c) LoRATrainer (optim/trainer.cpp:44-64): linear or cosine decay after warmup.
"""
from __future__ import annotations

import math


def gpt2_cli_lr(step: int, base_lr: float, warmup_steps: int, total_steps: int, min_ratio: float = 0.1) -> float:
    """step is 0-indexed (reference main loop variable)."""
    if warmup_steps > 0 and step < warmup_steps:
        return base_lr * float(step + 1) / float(warmup_steps)
    if total_steps <= warmup_steps:
        return base_lr
    progress = float(step - warmup_steps) / float(max(1, total_steps - warmup_steps))
    progress = min(max(progress, 0.0), 1.0)
    cosine = 0.5 * (1.0 + math.cos(math.pi * progress))
    return base_lr * (min_ratio + (1.0 - min_ratio) * cosine)


def gemma_lr(step: int, base_lr: float, warmup_ratio: float, total_updates: int, kind: str = "linear") -> float:
    """step is 1-indexed (GemmaLoRATrainer::get_lr)."""
    warmup = int(math.ceil(warmup_ratio * total_updates)) if warmup_ratio > 0 else 0
    if warmup > 0 and step <= warmup:
        return base_lr * float(step) / float(warmup)
    if total_updates <= warmup:
        return base_lr
    progress = float(step - warmup) / float(max(1, total_updates - warmup))
    progress = min(max(progress, 0.0), 1.0)
    if kind == "cosine":
        return base_lr * 0.5 * (1.0 + math.cos(math.pi * progress))
    return base_lr * (1.0 - progress)


def trainer_lr(step: int, base_lr: float, warmup_steps: int, total_steps: int, kind: str = "linear") -> float:
    if warmup_steps > 0 and step < warmup_steps:
        return base_lr * float(step) / float(warmup_steps)
    progress = float(step - warmup_steps) / float(max(1, total_steps - warmup_steps))
    progress = min(max(progress, 0.0), 1.0)
    if kind == "cosine":
        return base_lr * 0.5 * (1.0 + math.cos(math.pi * progress))
    return base_lr * (1.0 - progress)


def constant_lr(step: int, base_lr: float, *_, **__) -> float:
    return base_lr
