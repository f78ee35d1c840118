"""Tracing / profiling hooks (SURVEY §5.1 "MI355X equivalent").

* ``trace_range(name)`` — a roctx range (``torch.cuda.nvtx`` is backed by roctx on ROCm) around a
  phase, visible in ``rocprofv3 --marker-trace`` timelines; a no-op unless tracing is enabled
  (``MFT_TRACE=1`` or ``enable_tracing()``), so the hot loop pays nothing by default.
* ``PhaseTimer`` — hipEvent-based per-phase GPU timers (fwd+bwd / comm / optimizer / data), read
  back once per log interval (no per-step host sync).
* ``ProfileWindow("a:b")`` — calls hipProfilerStart at step a and hipProfilerStop after step b
  (``--profile_steps``), for ``rocprofv3 --selected-regions`` captures of a steady-state window.
"""
from __future__ import annotations

import contextlib
import os

import torch

_ENABLED = {"on": os.environ.get("MFT_TRACE", "0") == "1"}


def enable_tracing(on: bool = True):
    _ENABLED["on"] = bool(on)


def tracing_enabled() -> bool:
    return _ENABLED["on"]


@contextlib.contextmanager
def trace_range(name: str):
    if not _ENABLED["on"] or not torch.cuda.is_available():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


class PhaseTimer:
    """Accumulates GPU time per named phase with hipEvents; ``report()`` syncs once."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self.pending: list[tuple[str, torch.cuda.Event, torch.cuda.Event]] = []
        self.totals: dict[str, float] = {}
        self.counts: dict[str, int] = {}

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            with trace_range(name):
                yield
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        with trace_range(name):
            yield
        e.record()
        self.pending.append((name, s, e))

    def report(self, reset: bool = True) -> dict:
        """{phase: mean ms} over the phases recorded since the last report."""
        if self.pending:
            self.pending[-1][2].synchronize()
        for name, s, e in self.pending:
            self.totals[name] = self.totals.get(name, 0.0) + s.elapsed_time(e)
            self.counts[name] = self.counts.get(name, 0) + 1
        self.pending.clear()
        out = {k: self.totals[k] / max(1, self.counts[k]) for k in self.totals}
        if reset:
            self.totals.clear()
            self.counts.clear()
        return out


class ProfileWindow:
    """``spec`` = "a:b" (1-based global steps, inclusive): profiler on for steps a..b."""

    def __init__(self, spec: str = ""):
        self.a = self.b = None
        if spec:
            a, b = spec.split(":")
            self.a, self.b = int(a), int(b)
        self.active = False

    def before_step(self, step: int):
        if self.a is not None and step == self.a and torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.profiler.start()
            enable_tracing(True)
            self.active = True

    def after_step(self, step: int):
        if self.active and step == self.b:
            torch.cuda.synchronize()
            torch.cuda.profiler.stop()
            self.active = False


def model_flops_per_token(n_params: int, n_trainable: int, n_layer: int, seq: int, d_model: int) -> float:
    """Training FLOPs per token: forward 2N, data-grad backward 2N, weight-grad 2N_trainable, plus
    the attention score/value matmuls (causal: half of 4 * S * d per layer each direction)."""
    attn = n_layer * 2 * seq * d_model * 3  # fwd (QK^T, PV; causal half of 4Sd) + bwd (2x)
    return 4.0 * n_params + 2.0 * n_trainable + attn


# CDNA4 dense bf16 matrix peak of one MI355X (no 2:1 sparsity), the MFU denominator
MI355X_BF16_DENSE_TFLOPS = 2500.0


def model_flops_per_token_cfg(cfg, seq: int, n_params: int, n_trainable: int) -> float:
    """`model_flops_per_token` from a GPT2Config / Gemma3Config (attention width = heads x head_dim,
    so Gemma-3's 4 x 256 query width is counted, not its 640 residual width)."""
    n_layer = getattr(cfg, "n_layer", None) or cfg.num_hidden_layers
    if hasattr(cfg, "n_embd"):
        d_attn = cfg.n_embd
    else:
        d_attn = cfg.num_attention_heads * cfg.head_dim
    return model_flops_per_token(n_params, n_trainable, n_layer, seq, d_attn)


def mfu(tokens_per_sec_per_gpu: float, flops_per_token: float) -> tuple[float, float]:
    """(achieved model TFLOP/s per GPU, fraction of the bf16 dense peak)."""
    tf = tokens_per_sec_per_gpu * flops_per_token / 1e12
    return tf, tf / MI355X_BF16_DENSE_TFLOPS
