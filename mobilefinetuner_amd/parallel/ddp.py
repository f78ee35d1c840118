"""Data parallelism over RCCL (xGMI) / gloo: bucketed gradient reduction on the flat grad buffer.

The reference has no parallelism at all.  Design for MI355X:

* one process per GPU, ``torch.distributed`` backend ``nccl`` (= RCCL on ROCm) over xGMI;
* gradients live in ONE flat fp32 buffer (utils/params.py), so a bucket is just a contiguous
  slice — no packing/unpacking copies;
* buckets are laid out in reverse-forward order and launched asynchronously from the
  ``grad_ready`` hook that the fused backward kernels call, so the reduction of late layers
  overlaps the backward of early layers (eager steps) and, on RCCL (``MFT_GRAPH_COMM``, default 1), inside the
  step's hipGraph: the hooks enqueue their RCCL collectives while the step is being captured, so
  the replay runs each bucket's collective on RCCL's stream as soon as the kernels producing it are
  done (``capturable``, see __init__);
* reductions: ``all_reduce`` (DDP, ZeRO-1), ``reduce_scatter_tensor`` per bucket into this rank's
  chunk (ZeRO-2, ``chunked``), or (legacy contiguous shards) ``reduce`` to the owning rank -- bucketed
  and overlapped, while the owned shard stays one contiguous range for the fused AdamW;
* optional bf16 reduction (``reduce_dtype=torch.bfloat16``): the bucket is cast into a bf16 comm
  buffer, reduced at half the xGMI bytes and cast back (full fine-tuning: 498 MB -> 249 MB per
  GPT-2 step);
* bucket size defaults to 64 MiB: xGMI is point-to-point (7 links x ~153 GB/s per MI355X), ring
  collectives are per-link bound and latency-dominated below a few MB, so fewer, larger buckets
  win; LoRA grads (1.8-7.6 MB) always fit one bucket and are reduced once after backward.
``MFT_DP_FORCE_COMM=1`` keeps the collectives on a 1-rank RCCL group (profiling the overlap on
one GPU).
"""
from __future__ import annotations

import os

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


# Averages are SUM + divide, never ReduceOp.AVG: RCCL 2.26's AVG (its PreMulSum kernels) returns
# wrong values in the last 4-8 elements of some lengths (66304, 66240 of fp32 on a 1-rank group;
# SUM exact at every length and offset -- scripts/probes/rs_tail.py, profiles/r3_rccl_avg_tail.txt)
def allreduce_mean_(t: torch.Tensor, group=None, async_op=False):
    if not is_dist() or dist.get_world_size(group) == 1:
        return None
    w = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=False)
    t.div_(dist.get_world_size(group))
    return None if not async_op else w


def allreduce_sum_(t: torch.Tensor, group=None):
    if is_dist() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


class DataParallel:
    """Bucketed, overlapped gradient averaging for a FlatParams grad buffer: all-reduce, or (ZeRO-2,
    ``chunked=True``) one ``reduce_scatter_tensor`` per bucket into this rank's chunk of it --
    bucket b = [lo, hi) splits into ``world`` equal chunks, rank r owns [lo + r c, lo + (r+1) c),
    and the chunks land back to back in ``own_grad`` (the rank's contiguous optimizer view).
    ``shard`` (legacy contiguous ZeRO-2 shards) reduces each bucket to its owner(s) instead."""

    def __init__(self, flat: FlatParams, group=None, bucket_mb: float = 64.0, overlap: bool = True,
                 broadcast_from: int | None = 0, reduce_dtype=None, shard: int | None = None,
                 chunked: bool = False):
        self.flat, self.group = flat, group
        self.world = dist.get_world_size(group) if is_dist() else 1
        self.rank = dist.get_rank(group) if is_dist() else 0
        self.force = is_dist() and os.environ.get("MFT_DP_FORCE_COMM", "0") == "1"
        self.active = self.world > 1 or self.force
        self.nccl = _supports_avg(group)
        self.overlap = overlap and self.active
        # collectives recorded into the step's hipGraph from the backward's grad-ready hooks: the
        # default on RCCL (MFT_GRAPH_COMM=0 reduces the buckets eagerly after the replay instead).
        # Round 2 kept it opt-in after captures aborted intermittently at capture end on a 1-rank
        # group; round 3 re-ran the recorded-collective tests (DDP, bf16, ZeRO-2:
        # tests/test_dp_graph_gpu.py::test_reducer_with_graph_step_matches_no_dp, part of the 184 GPU
        # tests passing in profiles/r3_final_gpu_tests.log) without an abort and found RCCL's AVG
        # inexact at some lengths (profiles/r3_rccl_avg_tail.txt), which is
        # no longer used (sum + divide).  The capture runs in thread_local mode so RCCL's watchdog
        # thread polling earlier events cannot invalidate it (train/engine.py).
        self.capturable = self.nccl and os.environ.get("MFT_GRAPH_COMM", "1") == "1"
        self.shard = shard
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
        if self.buckets:
            # the buckets tile the whole buffer (alignment gaps and the padding tail included), so
            # every element -- in particular every element of a ZeRO-2 shard -- is reduced once
            self.buckets[0]["hi"] = flat.numel
            self.buckets[-1]["lo"] = 0
            for k in range(len(self.buckets) - 1):
                self.buckets[k]["lo"] = self.buckets[k + 1]["hi"]
        self.param_bucket = {}
        for bi, b in enumerate(self.buckets):
            for s in b["slots"]:
                self.param_bucket[id(s.param)] = bi
        # ZeRO-2 chunk layout: every bucket length divides by world (slot offsets are 64-aligned and
        # the buffer is padded to ALIGN * world), chunk b of this rank at own_off[b] in own_grad
        self.chunked = bool(chunked)
        self.own_off, self.own_numel = [], 0
        if self.chunked:
            for b in self.buckets:
                assert (b["hi"] - b["lo"]) % self.world == 0, "ZeRO-2 chunks need bucket lengths divisible by world"
                b["c"] = (b["hi"] - b["lo"]) // self.world
                self.own_off.append(self.own_numel)
                self.own_numel += b["c"]
            self.own_grad = torch.zeros(self.own_numel, dtype=flat.grad.dtype, device=flat.grad.device)
            self.own_buf = None  # bf16 landing buffer of the reduced chunks
            if reduce_dtype is not None and reduce_dtype != flat.grad.dtype:
                self.own_buf = torch.empty(self.own_numel, dtype=reduce_dtype, device=flat.grad.device)
        self.comm_buf = None
        if reduce_dtype is not None and reduce_dtype != flat.grad.dtype and self.active:
            self.comm_buf = torch.empty(flat.numel, dtype=reduce_dtype, device=flat.grad.device)
        self._works = []
        self._pending = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._seen = set()
        # with gradient accumulation a bucket may only be reduced once its params received the
        # LAST micro-batch's contribution: TrainStep clears this flag for earlier micro-batches
        self.last_micro = True
        self._hook = None
        if self.overlap and (len(self.buckets) > 1 or shard is not None):
            self._hook = Fx.register_grad_ready_hook(self._on_ready)
        if broadcast_from is not None and self.world > 1:
            dist.broadcast(flat.master, src=broadcast_from, group=group)
            flat.refresh_shadow()

    @staticmethod
    def _mk(slots):
        lo = min(s.offset for s in slots)
        hi = max(s.offset + s.numel for s in slots)
        return {"slots": slots, "lo": lo, "hi": hi, "n": len(slots)}

    def _owner_segments(self, lo, hi):
        """[(owner rank, a, b)] cover [lo, hi) by the ranks' contiguous ZeRO-2 shards."""
        out, a = [], lo
        while a < hi:
            r = min(a // self.shard, self.world - 1)
            b = min(hi, (r + 1) * self.shard) if r < self.world - 1 else hi
            out.append((r, a, b))
            a = b
        return out

    def _dst(self, r):
        return dist.get_global_rank(self.group, r) if self.group is not None else r

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
        if not self.active:
            return
        lo, hi = b["lo"], b["hi"]
        t = self.flat.grad[lo:hi]
        if self.comm_buf is not None:
            c = self.comm_buf[lo:hi]
            c.copy_(t)
            t = c
        op = dist.ReduceOp.SUM  # (averaged in finish(): RCCL's AVG is inexact, allreduce_mean_ above)
        if self.chunked:
            c, o = b["c"], self.own_off[bi]
            out = (self.own_buf if self.comm_buf is not None else self.own_grad)[o:o + c]
            self._works.append(dist.reduce_scatter_tensor(out, t, op=op, group=self.group, async_op=True))
        elif self.shard is None:
            self._works.append(dist.all_reduce(t, op=op, group=self.group, async_op=True))
        else:
            for r, a, z in self._owner_segments(lo, hi):
                self._works.append(dist.reduce(t[a - lo:z - lo], dst=self._dst(r), op=op, group=self.group,
                                               async_op=True))

    def _on_ready(self, p):
        # while a hipGraph is captured the collective is recorded into it only if the backend can
        # (RCCL); otherwise the bucket stays pending and finish() reduces it after the replay
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing() and not self.capturable:
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

    def wants_graph_comm(self):
        """Record the reduction (and the optimizer step) into the step's hipGraph: only when the
        backward hooks overlap several buckets on RCCL; a single bucket (LoRA) is reduced by one
        eager collective after the replay."""
        return self.capturable and self._hook is not None

    def owned(self):
        """(lo, hi) of the reduced gradient this rank's optimizer reads (contiguous layouts)."""
        if self.shard is None:
            return 0, self.flat.numel
        lo = self.rank * self.shard
        return lo, (self.flat.numel if self.rank == self.world - 1 else lo + self.shard)

    def finish(self):
        """Launch every bucket no hook completed, wait, and finish the average (gloo: /world;
        bf16: cast back)."""
        if not self.active:
            return
        for bi in range(len(self.buckets)):
            self._launch(bi)
        for w in self._works:
            if w is not None:
                w.wait()
        self._works = []
        if self.chunked:
            if self.own_buf is not None:
                self.own_grad.copy_(self.own_buf)
            if self.world > 1:
                self.own_grad.div_(self.world)
            return
        lo, hi = self.owned()
        if self.comm_buf is not None:
            self.flat.grad[lo:hi].copy_(self.comm_buf[lo:hi])
        if self.world > 1:
            self.flat.grad[lo:hi].div_(self.world)

    def close(self):
        if self._hook is not None:
            Fx.remove_grad_ready_hook(self._hook)
            self._hook = None
