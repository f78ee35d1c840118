"""Flat parameter / gradient / bf16-shadow storage for the trainable parameters.

All trainable parameters of a model are re-homed into three contiguous device buffers:

* ``master`` fp32 — the parameters themselves (``p.data`` becomes a view),
* ``grad``   fp32 — ``p.grad`` is a persistent view; kernels accumulate into it (``+=``),
* ``shadow`` bf16 — ``p.shadow``, the compute copy read by the GEMMs, refreshed by the fused AdamW
  kernel in the same pass that updates the master (no separate cast pass).

One flat buffer means: one fused AdamW launch, one grad-norm reduction, one zero-fill, and one
RCCL all-reduce / reduce-scatter per bucket for data parallelism.  This replaces the reference's
per-tensor ``std::unordered_map<TensorPtr, AdamState>`` (optim/adam.h:99) and per-tensor
``zero_grad`` loops.  Each parameter starts on a 64-element boundary (16-B aligned vector access
for both fp32 and bf16 views).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

ALIGN = 64


def _round(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


@dataclass
class ParamSlot:
    name: str
    param: torch.nn.Parameter
    offset: int
    numel: int


class FlatParams:
    def __init__(self, named_params, device, shadow: bool = True, shadow_dtype=torch.bfloat16,
                 pad_multiple: int = 1):
        named_params = [(n, p) for n, p in named_params if p.requires_grad]
        self.slots: list[ParamSlot] = []
        off = 0
        for n, p in named_params:
            self.slots.append(ParamSlot(n, p, off, p.numel()))
            off += _round(p.numel())
        # pad_multiple: ZeRO needs world_size equal, ALIGN-aligned shards
        self.numel = _round(max(off, ALIGN), ALIGN * max(1, pad_multiple))
        self.device = torch.device(device)
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.shadow = torch.zeros(self.numel, dtype=shadow_dtype, device=self.device) if shadow else None
        for s in self.slots:
            p = s.param
            mv = self.master[s.offset:s.offset + s.numel].view(p.shape)
            mv.copy_(p.data.to(device=self.device, dtype=torch.float32))
            p.data = mv
            p.grad = self.grad[s.offset:s.offset + s.numel].view(p.shape)
            # norm weights compute in fp32 straight from the master (no bf16 rounding)
            if self.shadow is not None and not getattr(p, "_mft_fp32_compute", False):
                p.shadow = self.shadow[s.offset:s.offset + s.numel].view(p.shape)
        self.refresh_shadow()

    @property
    def params(self):
        return [s.param for s in self.slots]

    def refresh_shadow(self):
        if self.shadow is None:
            return
        if self.master.is_cuda:
            from .._ext import native
            native().cast_f32_bf16(self.master, self.shadow)
        else:
            self.shadow.copy_(self.master.to(self.shadow.dtype))

    def zero_grad(self):
        self.grad.zero_()
        # torch may have replaced a .grad (e.g. by an out-of-place op); restore the views
        for s in self.slots:
            g = s.param.grad
            if g is None or g.data_ptr() != self.grad[s.offset:].data_ptr():
                s.param.grad = self.grad[s.offset:s.offset + s.numel].view(s.param.shape)

    def named(self):
        return [(s.name, s.param) for s in self.slots]

    def state_dict_master(self):
        return {s.name: s.param.detach().float().cpu().clone() for s in self.slots}

    def __len__(self):
        return len(self.slots)
