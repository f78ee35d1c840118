"""Data parallelism over RCCL (xGMI) / gloo: bucketed gradient all-reduce on the flat grad buffer.

The reference has no parallelism at all.  Design for MI355X:

* one process per GPU, ``torch.distributed`` backend ``nccl`` (= RCCL on ROCm) over xGMI;
* gradients live in ONE flat fp32 buffer (utils/params.py), so a bucket is just a contiguous
  slice — no packing/unpacking copies;
* buckets are laid out in reverse-forward order and launched asynchronously from the
  ``grad_ready`` hook that the fused backward kernels call, so the all-reduce of late layers
  overlaps the backward of early layers;
* bucket size defaults to 64 MiB: xGMI is point-to-point (7 links x ~153 GB/s per MI355X), ring
  collectives are per-link bound and latency-dominated below a few MB, so fewer, larger buckets
  win; LoRA grads (1.8-7.6 MB) always fit one bucket and are reduced once after backward.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import functional as Fx
from ..utils.params import FlatParams


def is_dist():
    return dist.is_available() and dist.is_initialized()


def world():
    return dist.get_world_size() if is_dist() else 1


def rank():
    return dist.get_rank() if is_dist() else 0


def _supports_avg(group=None):
    try:
        return dist.get_backend(group) == "nccl"
    except Exception:
        return False


def allreduce_mean_(t: torch.Tensor, group=None, async_op=False):
    if not is_dist() or dist.get_world_size(group) == 1:
        return None
    if _supports_avg(group):
        return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group, async_op=async_op)
    w = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=False)
    t.div_(dist.get_world_size(group))
    return None if not async_op else w


def allreduce_sum_(t: torch.Tensor, group=None):
    if is_dist() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


class DataParallel:
    """Bucketed, overlapped gradient averaging for a FlatParams grad buffer."""

    def __init__(self, flat: FlatParams, group=None, bucket_mb: float = 64.0, overlap: bool = True,
                 broadcast_from: int | None = 0):
        self.flat, self.group = flat, group
        self.world = dist.get_world_size(group) if is_dist() else 1
        self.overlap = overlap and self.world > 1
        cap = int(bucket_mb * (1 << 20) / 4)
        # buckets over slots in REVERSE order (last layer's grads are ready first)
        self.buckets = []
        cur, lo = [], None
        for s in reversed(flat.slots):
            if lo is None:
                lo = s.offset
            cur.append(s)
            span = (cur[0].offset + cur[0].numel) - s.offset
            if span >= cap:
                self.buckets.append(self._mk(cur))
                cur, lo = [], None
        if cur:
            self.buckets.append(self._mk(cur))
        self.param_bucket = {}
        for bi, b in enumerate(self.buckets):
            for s in b["slots"]:
                self.param_bucket[id(s.param)] = bi
        self._works = []
        self._pending = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._seen = set()
        # with gradient accumulation a bucket may only be reduced once its params received the
        # LAST micro-batch's contribution: TrainStep clears this flag for earlier micro-batches
        self.last_micro = True
        self._hook = None
        if self.overlap and len(self.buckets) > 1:
            self._hook = Fx.register_grad_ready_hook(self._on_ready)
        if broadcast_from is not None and self.world > 1:
            dist.broadcast(flat.master, src=broadcast_from, group=group)
            flat.refresh_shadow()

    @staticmethod
    def _mk(slots):
        lo = min(s.offset for s in slots)
        hi = max(s.offset + s.numel for s in slots)
        return {"slots": slots, "lo": lo, "hi": hi, "n": len(slots)}

    def begin_step(self):
        self._pending = [b["n"] for b in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._seen = set()
        self._works = []

    def _launch(self, bi):
        if self._launched[bi]:
            return
        b = self.buckets[bi]
        self._launched[bi] = True
        w = allreduce_mean_(self.flat.grad[b["lo"]:b["hi"]], self.group, async_op=True)
        if w is not None:
            self._works.append(w)

    def _on_ready(self, p):
        # inside a hipGraph capture (TrainStep use_graph) no collective may be enqueued: the bucket
        # stays pending and finish() reduces every bucket after the replay
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return
        if not self.last_micro:
            return
        bi = self.param_bucket.get(id(p))
        if bi is None or id(p) in self._seen:
            return
        self._seen.add(id(p))  # a param counts once per step (its LAST contribution fires the hook)
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def finish(self):
        """Make sure every bucket is reduced (launch the ones no hook completed) and wait."""
        if self.world == 1:
            return
        if not self.overlap or len(self.buckets) == 1:
            allreduce_mean_(self.flat.grad, self.group)
            return
        for bi in range(len(self.buckets)):
            self._launch(bi)
        for w in self._works:
            w.wait()
        self._works = []

    def close(self):
        if self._hook is not None:
            Fx.remove_grad_ready_hook(self._hook)
            self._hook = None
