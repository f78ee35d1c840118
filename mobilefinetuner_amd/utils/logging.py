"""Rank-aware console logging (rank 0 prints; every rank can append JSONL metrics)."""
from __future__ import annotations

import sys

import torch.distributed as dist


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def rank0() -> bool:
    return rank() == 0


def log0(*a, **k):
    if rank0():
        print(*a, **k, flush=True)


def logall(*a, **k):
    print(f"[rank{rank()}]", *a, **k, file=sys.stderr, flush=True)
