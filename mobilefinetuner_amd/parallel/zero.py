"""ZeRO-1 / ZeRO-2 partitioning of the flat parameter buffer across data-parallel ranks.

The reference's "ZeRO-inspired" sharder is a single-device disk LRU.  This is
the real cross-GPU version for full fine-tuning (gpt2_full_finetune, GPT-2 XL on 8 x MI355X):

* the flat fp32 grad / master buffers are split into ``world`` equal contiguous shards (padded);
* ZeRO-1: grads are all-reduced (averaged), each rank updates only its shard of the AdamW moments
  (optimizer memory / world);
* ZeRO-2: ownership is per gradient BUCKET -- bucket [lo, hi) splits into ``world`` equal chunks and
  rank r owns chunk r of every bucket (the native engine's layout, engine/dist.h) -- so each bucket
  is ONE ``reduce_scatter_tensor`` (half the bytes of an all-reduce on the per-link-bound xGMI
  ring) launched from the backward's grad-ready hooks, overlapping the backward; the reduced
  chunks land back to back in a contiguous per-rank buffer that the fused AdamW updates (with its
  own contiguous fp32 master / bf16 shadow chunks), and one ``all_gather_into_tensor`` per bucket
  rebuilds the full bf16 shadow;
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


class _Owned:
    """This rank's ZeRO-2 chunks as one contiguous flat (master / grad / shadow): what FusedAdamW updates."""

    def __init__(self, master, grad, shadow):
        self.master, self.grad, self.shadow = master, grad, shadow
        self.numel = master.numel()


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
        if self.world > 1:  # identical starting weights everywhere
            dist.broadcast(flat.master, src=0, group=group)
            flat.refresh_shadow()
        # bucketed, backward-overlapped gradient reduction: all-reduce (stage 1) or one
        # reduce-scatter per bucket into this rank's chunks (stage 2)
        self.reducer = DataParallel(flat, group=group, bucket_mb=bucket_mb, overlap=overlap, broadcast_from=None,
                                    reduce_dtype=reduce_dtype, chunked=stage == 2)
        # element ranges this rank updates: [lo, hi) (stage 1) or chunk r of every bucket (stage 2)
        if stage == 2:
            R = self.reducer
            self.ranges = [(b["lo"] + self.rank * b["c"], b["lo"] + (self.rank + 1) * b["c"], R.own_off[i])
                           for i, b in enumerate(R.buckets)]
            master = torch.cat([flat.master[a:z] for a, z, _ in self.ranges]) if self.ranges else flat.master[:0].clone()
            shadow = master.to(flat.shadow.dtype) if flat.shadow is not None else None
            self.own = _Owned(master, R.own_grad, shadow)
            self.inner = FusedAdamW(self.own, **adamw_kwargs)
        else:
            self.ranges = [(self.lo, self.hi, 0)]
            self.own = None
            self.inner = FusedAdamW(flat, param_range=(self.lo, self.hi), **adamw_kwargs)
        if self.world > 1:
            # each rank scans only its elements for NaN/Inf: OR the flags so all ranks skip together
            self.inner.reduce_flag = lambda f: dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
        # parameters that compute straight from the fp32 master (norm weights/biases: no bf16
        # shadow) are not covered by the shadow all-gather; their owned elements are re-assembled
        # with one masked all-reduce of a packed index list (tiny: LN/RMSNorm parameters only)
        self._fp32_idx = self._fp32_own = None
        if flat.shadow is not None:
            loose = [s for s in flat.slots if getattr(s.param, "shadow", None) is None]
            if loose:
                idx = torch.cat([torch.arange(s.offset, s.offset + s.numel) for s in loose]).to(flat.master.device)
                own = torch.zeros_like(idx, dtype=torch.bool)
                for a, z, _ in self.ranges:
                    own |= (idx >= a) & (idx < z)
                self._fp32_idx = idx
                self._fp32_own = own.to(flat.master.dtype)

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
        fl = self.flat
        if self.stage == 2:
            # the updated chunks back into the full buffers: own master locally, the bf16 shadow by
            # one all-gather per bucket (every rank's chunk of it)
            for (a, z, o), b in zip(self.ranges, self.reducer.buckets):
                fl.master[a:z].copy_(self.own.master[o:o + (z - a)])
                if fl.shadow is not None:
                    if self.world > 1:
                        dist.all_gather_into_tensor(fl.shadow[b["lo"]:b["hi"]], self.own.shadow[o:o + (z - a)],
                                                    group=self.group)
                    else:
                        fl.shadow[a:z].copy_(self.own.shadow[o:o + (z - a)])
            if self.world > 1 and fl.shadow is None:
                self.gather_master()
        elif self.world > 1:
            # masters outside this shard are only read through the shadow; gather_master() refreshes
            # them for checkpointing
            sh = fl.shadow if fl.shadow is not None else fl.master
            dist.all_gather_into_tensor(sh, sh[self.lo:self.hi].clone(), group=self.group)
        if self.world > 1 and self._fp32_idx is not None:
            v = fl.master.index_select(0, self._fp32_idx) * self._fp32_own
            dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.group)
            fl.master.index_copy_(0, self._fp32_idx, v)

    def gather_master(self):
        """All-gather the fp32 master (for checkpointing on every rank)."""
        if self.world <= 1:
            return
        m = self.flat.master
        if self.stage == 2:
            for (a, z, o), b in zip(self.ranges, self.reducer.buckets):
                dist.all_gather_into_tensor(m[b["lo"]:b["hi"]], self.own.master[o:o + (z - a)], group=self.group)
        else:
            dist.all_gather_into_tensor(m, m[self.lo:self.hi].clone(), group=self.group)

    def load_state_dict(self, sd):
        # (the trainer restored the full fp32 master into the flat first: re-take this rank's chunks)
        if self.own is not None and self.ranges:
            self.own.master.copy_(torch.cat([self.flat.master[a:z] for a, z, _ in self.ranges]))
            if self.own.shadow is not None:
                self.own.shadow.copy_(self.own.master.to(self.own.shadow.dtype))
        self.inner.load_state_dict(sd)

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
