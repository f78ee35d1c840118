"""ZeRO-1 / ZeRO-2 partitioning of the flat parameter buffer across data-parallel ranks.

The reference's "ZeRO-inspired" sharder is a single-device disk LRU.  This is
the real cross-GPU version for full fine-tuning (gpt2_full_finetune, GPT-2 XL on 8 x MI355X):

* the flat fp32 grad / master buffers are split into ``world`` equal contiguous shards (padded);
* ZeRO-1: grads are all-reduced (averaged), each rank updates only its shard of the AdamW moments
  (optimizer memory / world);
* ZeRO-2: every gradient bucket is ``reduce``-d to the rank(s) owning its elements — the traffic of
  a reduce-scatter (half an all-reduce on the per-link-bound xGMI ring), but bucketed and launched
  from the backward's grad-ready hooks, so it overlaps the backward (and is recorded into the
  step's hipGraph with RCCL; parallel/ddp.py);
* the updated bf16 compute weights (the ``shadow``) are ``all_gather``-ed into every rank, so the
  next forward sees the full model;
* the global grad norm for clipping is the all-reduced sum of per-shard squares.

Collectives run on the flat buffers directly (no packing).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..optim.adamw import FusedAdamW
from ..utils.params import FlatParams
from .ddp import DataParallel, is_dist


class ZeroOptimizer:
    def __init__(self, flat: FlatParams, stage: int, group=None, bucket_mb: float = 64.0, overlap: bool = True,
                 reduce_dtype=None, **adamw_kwargs):
        assert stage in (1, 2)
        self.flat, self.stage, self.group = flat, stage, group
        self.world = dist.get_world_size(group) if is_dist() else 1
        self.rank = dist.get_rank(group) if is_dist() else 0
        n = flat.numel
        assert n % self.world == 0, "FlatParams must be created with pad_multiple=world_size"
        self.shard = n // self.world
        self.lo, self.hi = self.rank * self.shard, (self.rank + 1) * self.shard
        self.inner = FusedAdamW(flat, param_range=(self.lo, self.hi), **adamw_kwargs)
        if self.world > 1:
            # each rank scans only its shard for NaN/Inf: OR the flags so all ranks skip together
            self.inner.reduce_flag = lambda f: dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
        # parameters that compute straight from the fp32 master (norm weights/biases: no bf16
        # shadow) are not covered by the shadow all-gather; their owned slices are re-assembled
        # with one masked all-reduce of a packed index list (tiny: LN/RMSNorm parameters only)
        self._fp32_idx = self._fp32_own = None
        if flat.shadow is not None:
            loose = [s for s in flat.slots if getattr(s.param, "shadow", None) is None]
            if loose:
                idx = torch.cat([torch.arange(s.offset, s.offset + s.numel) for s in loose]).to(flat.master.device)
                self._fp32_idx = idx
                self._fp32_own = ((idx >= self.lo) & (idx < self.hi)).to(flat.master.dtype)
        if self.world > 1:  # identical starting weights everywhere
            dist.broadcast(flat.master, src=0, group=group)
            flat.refresh_shadow()
        # bucketed, backward-overlapped gradient reduction (all-reduce for stage 1, reduce to the
        # owning rank for stage 2)
        self.reducer = DataParallel(flat, group=group, bucket_mb=bucket_mb, overlap=overlap, broadcast_from=None,
                                    reduce_dtype=reduce_dtype, shard=self.shard if stage == 2 else None)

    # expose the FusedAdamW control surface used by Trainer/TrainStep
    def __getattr__(self, k):
        return getattr(self.inner, k)

    def reduce_gradients(self):
        """Finish this step's reduction (buckets the backward hooks did not launch are launched
        now) and re-arm the reducer for the next step."""
        self.reducer.finish()
        self.reducer.begin_step()

    def step(self, sumsq_ready: bool = False):
        if self.inner.max_grad_norm is not None:
            def allreduce_sumsq(t):
                if self.world > 1:
                    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            self.inner.compute_grad_sumsq(allreduce_sumsq)
        self.inner.step(sumsq_ready=True)
        if self.world > 1:
            # masters outside this shard are only read through the shadow; gather_master() refreshes
            # them for checkpointing
            sh = self.flat.shadow if self.flat.shadow is not None else self.flat.master
            dist.all_gather_into_tensor(sh, sh[self.lo:self.hi].clone(), group=self.group)
            if self._fp32_idx is not None:
                v = self.flat.master.index_select(0, self._fp32_idx) * self._fp32_own
                dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.group)
                self.flat.master.index_copy_(0, self._fp32_idx, v)

    def gather_master(self):
        """All-gather the fp32 master (for checkpointing on every rank)."""
        if self.world > 1:
            m = self.flat.master
            dist.all_gather_into_tensor(m, m[self.lo:self.hi].clone(), group=self.group)

    def state_dict(self):
        sd = self.inner.state_dict()
        sd["zero_stage"] = self.stage
        sd["zero_rank"] = self.rank
        return sd


class ZeroReducer:
    """Adapter with the DataParallel interface used by train.engine.TrainStep."""

    def __init__(self, zero: ZeroOptimizer):
        self.zero = zero
        self.world = zero.world
        self.group = zero.group

    @property
    def capturable(self):
        return self.zero.reducer.capturable

    def wants_graph_comm(self):
        return self.zero.reducer.wants_graph_comm()

    @property
    def last_micro(self):
        return self.zero.reducer.last_micro

    @last_micro.setter
    def last_micro(self, v):
        self.zero.reducer.last_micro = v

    def begin_step(self):
        self.zero.reducer.begin_step()

    def finish(self):
        self.zero.reducer.finish()

    def close(self):
        self.zero.reducer.close()
