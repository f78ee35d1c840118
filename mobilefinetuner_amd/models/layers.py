"""Building-block modules whose forward calls the fused ops of ``ops/functional.py``.

Weight layouts: linear weights are ``[out, in]`` (nn.Linear convention; GPT-2's HF Conv1D
``[in, out]`` weights are transposed once at load time, models/gpt2.py).  Linear/embedding weights
are stored in the compute dtype (bf16 on GPU) when frozen; trainable ones become fp32 masters with
a bf16 ``shadow`` once handed to ``utils.params.FlatParams``.  Norm weights are fp32.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from ..ops import functional as Fx


def _salt(name: str) -> int:
    """Stable per-adapter salt for the dropout hash (zlib.crc32: not randomised per process)."""
    import zlib
    return zlib.crc32(name.encode())


@dataclass
class LoRASlice:
    """One LoRA adapter on columns [col0, col0 + ncols) of a (possibly fused) linear output.
    A: [r, in] (PEFT lora_A.weight layout), B: [r, ncols] (reference lora_B layout).  The reference
    checkpoint stores A as [in, r] (graph/lora_saver.cpp:123-126); io/lora_checkpoint.py transposes."""
    col0: int
    ncols: int
    A: nn.Parameter
    B: nn.Parameter
    name: str = ""


class Linear(nn.Module):
    def __init__(self, in_features, out_features, bias=True, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, dtype=dtype, device=device),
                                   requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=dtype, device=device),
                                 requires_grad=False) if bias else None
        self.lora_slices: list[LoRASlice] = []
        self.lora_scale = 0.0
        self.lora_dropout = 0.0
        self.lora_enabled = True
        self._lora_params = nn.ParameterList()

    def add_lora(self, col0, ncols, rank, scale, init_A, name=""):
        dev = self.weight.device
        A = nn.Parameter(init_A.to(device=dev, dtype=torch.float32))
        B = nn.Parameter(torch.zeros(rank, ncols, dtype=torch.float32, device=dev))
        self._lora_params.append(A)
        self._lora_params.append(B)
        self.lora_slices.append(LoRASlice(col0, ncols, A, B, name))
        self.lora_scale = float(scale)
        return A, B

    def clear_lora(self):
        self.lora_slices = []
        self._lora_params = nn.ParameterList()
        self.__dict__.pop("_waug", None)

    def aug_cols(self) -> int:
        """Input width the producer should allocate for the augmented-K LoRA forward
        (ops.functional._LoRALinearAug), or 0 when this Linear takes a plain input: no active
        adapter, a trainable base weight, CPU tensors, in_features not a multiple of 32, or
        MFT_LORA_AUG=0."""
        import os
        if not (self.lora_slices and self.lora_enabled) or self.weight.requires_grad or not self.weight.is_cuda:
            return 0
        if getattr(self.weight, "_mft_sharded", False):  # no resident W copy for offloaded weights
            return 0
        if self.in_features % 32 or os.environ.get("MFT_LORA_AUG", "1") == "0":
            return 0
        return Fx.lora_aug_cols(self.in_features, [sl.A.shape[0] for sl in self.lora_slices])

    def _aug_weight(self, ka: int):
        """[out, ka] bf16 buffer = [W | (s B^T per slice, written each forward) | 0]; W copied once
        (dropped by merge_lora / clear_lora so a changed base weight is re-copied)."""
        wa = self.__dict__.get("_waug")
        wc = Fx.cw(self.weight)
        if wa is None or wa.shape[1] != ka or wa.device != wc.device:
            wa = torch.zeros(self.out_features, ka, dtype=wc.dtype, device=wc.device)
            wa[:, : self.in_features].copy_(wc)
            self.__dict__["_waug"] = wa
        return wa

    def forward(self, x):
        if self.lora_slices and self.lora_enabled:
            sl = [(s.col0, s.ncols, s.A, s.B, self.lora_dropout, _salt(s.name)) for s in self.lora_slices]
            if x.is_cuda and x.shape[-1] != self.in_features:
                ka = self.aug_cols()
                assert x.shape[-1] == ka, f"augmented input width {x.shape[-1]} != {ka}"
                return Fx.lora_linear_aug(x, self.weight, self.bias, sl, self.lora_scale, self._aug_weight(ka),
                                          self.training)
            return Fx.lora_linear(x, self.weight, self.bias, sl, self.lora_scale, self.training)
        return Fx.linear(x, self.weight, self.bias)

    @torch.no_grad()
    def merge_lora(self, sign: float = 1.0):
        """W[col0:col0+n, :] += sign * s * B^T A  (merge; sign=-1 unmerges) — K10."""
        for sl in self.lora_slices:
            A, B = sl.A.detach().float().contiguous(), sl.B.detach().float().contiguous()   # [r, in], [r, n]
            w = self.weight.data
            if w.is_cuda and w.is_contiguous() and w.dtype in (torch.bfloat16, torch.float32):
                # K10 lora_merge kernel (lora.hip): W[col0 + n, k] += sign * s * sum_r A[r, k] B[r, n]
                from .._ext import native
                native().lora_merge(w[sl.col0:sl.col0 + sl.ncols], 1, self.in_features, A, B,
                                    float(sign * self.lora_scale))
            else:
                delta = (B.t() @ A) * (sign * self.lora_scale)          # [n, in]
                w[sl.col0:sl.col0 + sl.ncols] = (w[sl.col0:sl.col0 + sl.ncols].float() + delta).to(w.dtype)
            if getattr(self.weight, "shadow", None) is not None:
                self.weight.shadow.copy_(self.weight.data.to(self.weight.shadow.dtype))
        Fx.drop_weight_t(self.weight)
        self.__dict__.pop("_waug", None)

    def extra_repr(self):
        return f"in={self.in_features}, out={self.out_features}, lora_slices={len(self.lora_slices)}"


class LayerNorm(nn.Module):
    def __init__(self, n, eps=1e-5, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(n, device=device), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(n, device=device), requires_grad=False)
        self.weight._mft_fp32_compute = True
        self.bias._mft_fp32_compute = True
        self.eps = eps
        self.__dict__["_consumer"] = None  # Linear fed by this norm (not a submodule)

    def set_consumer(self, lin):
        """Register the Linear this norm feeds so the output can be widened for its LoRA
        augmented-K input (Linear.aug_cols)."""
        self.__dict__["_consumer"] = lin

    def _out_cols(self):
        c = self.__dict__["_consumer"]
        return c.aug_cols() if c is not None else 0

    def forward(self, x):
        return Fx.layer_norm(x, self.weight, self.bias, self.eps, self._out_cols())

    def add_forward(self, x, delta):
        return Fx.add_layer_norm(x, delta, self.weight, self.bias, self.eps, self._out_cols())


class RMSNorm(nn.Module):
    """Gemma-style RMSNorm: y = x * rstd * (offset + w), offset 1 (reference core/ops.cpp:1515)."""

    def __init__(self, n, eps=1e-6, offset=1.0, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(n, device=device), requires_grad=False)
        self.weight._mft_fp32_compute = True
        self.eps, self.offset = eps, offset
        self.__dict__["_consumer"] = None

    def set_consumer(self, lin):
        self.__dict__["_consumer"] = lin

    def _out_cols(self):
        c = self.__dict__["_consumer"]
        return c.aug_cols() if c is not None else 0

    def forward(self, x):
        return Fx.rms_norm(x, self.weight, self.eps, self.offset, self._out_cols())

    def add_forward(self, x, delta):
        return Fx.add_rms_norm(x, delta, self.weight, self.eps, self.offset, self._out_cols())
