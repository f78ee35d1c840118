"""RoPE cos / sin tables (model setup, computed once per model on its device)."""
from __future__ import annotations

import torch


def rope_tables(seq_len, dim, theta, device=None, scaling_factor=1.0):
    """cos/sin tables [seq_len, dim/2] fp32 (HF default rope; linear scaling divides positions)."""
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float64) / dim))
    pos = torch.arange(seq_len, dtype=torch.float64) / scaling_factor
    f = torch.outer(pos, inv)
    return f.cos().float().to(device), f.sin().float().to(device)
