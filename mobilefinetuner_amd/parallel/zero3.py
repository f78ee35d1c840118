"""ZeRO-3: parameters, gradients and optimizer state all partitioned over the data-parallel ranks.

SURVEY §2.13 lists ZeRO-3 (per-layer ``all_gather`` of the parameters with prefetch + per-layer
``reduce_scatter`` of the gradients) as required by the north-star; the reference only has the
single-device disk sharder (opt_ops/sharding/parameter_sharder.h:1-21).

Layout.  The model is split into *units*: ``outer`` (token/position embeddings — the tied LM head
— used at both ends of the step) and one unit per transformer block.  Each unit's parameters are
laid out contiguously (64-element aligned) and padded to a multiple of ``64 * world``; rank r owns
the r-th contiguous slice of every unit.  The rank-local flat buffers are

    [ unit0 shard | unit1 shard | ... | replicated ]     fp32 master, fp32 grad, bf16 shadow

so ONE fused AdamW launch updates every owned element and writes the bf16 shadow shard that the
next step's all-gathers read.  Norm weights/biases (which compute in fp32 straight from the master,
``_mft_fp32_compute``) are tiny and stay replicated: their grads are all-reduced once per step.

Per step (GPU, bf16 compute):
  forward  block i : all_gather(shadow shards of unit i) -> unit's full bf16 buffer, prefetching
                     unit i+1 on the communication stream; the gathered buffers are two fixed
                     slots shared by the even / odd blocks (+ one for the outer unit): a block's
                     slot is overwritten by the block two ahead, and views captured by autograd
                     are refilled in place before the block's backward.  No allocation or
                     storage resize ever happens inside a step, so the whole ZeRO-3 step --
                     gathers, prefetches on the side stream, reduce-scatters, sharded AdamW --
                     is recorded into ONE hipGraph like the other configurations;
  backward block i : an autograd gate at the block OUTPUT re-gathers unit i (prefetching i-1) and
                     materialises a zeroed fp32 gradient buffer that the kernels accumulate into;
                     a gate at the block INPUT fires once the whole block's backward is done:
                     reduce_scatter(grad buffer) -> += the rank's grad shard, buffer released;
  end of step      : the ``outer`` unit's grads are reduce-scattered, replicated grads
                     all-reduced, then the sharded AdamW (grad norm = all-reduced sum of the
                     shard squares + the replicated part counted once).

Peak parameter memory per rank = shards (1/world of everything) + three gathered units (two block
slots and the outer unit) + their three fp32 gradient slots.  On the CPU (gloo, tests) the gathered copy is the fp32
master itself and autograd accumulates straight into the gradient buffer views.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch.autograd import Function

from ..optim.adamw import FusedAdamW
from .ddp import is_dist

ALIGN = 64


def _round(n, a):
    return (n + a - 1) // a * a


class _ShardFlat:
    """FlatParams-compatible view of one rank's partition (what FusedAdamW / TrainStep touch)."""

    def __init__(self, numel, device, shadow: bool):
        self.numel = numel
        self.device = torch.device(device)
        self.master = torch.zeros(numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(numel, dtype=torch.float32, device=self.device)
        self.shadow = torch.zeros(numel, dtype=torch.bfloat16, device=self.device) if shadow else None
        self.slots = []

    def refresh_shadow(self):
        if self.shadow is not None:
            self.shadow.copy_(self.master)

    def zero_grad(self):
        self.grad.zero_()

    def named(self):
        return [("__zero3_shard__", self.master)]


class _Unit:
    def __init__(self, name, params):
        self.name = name
        self.params = params          # [(name, Parameter)] sharded in this unit
        self.offsets = []
        off = 0
        for _, p in params:
            self.offsets.append(off)
            off += _round(p.numel(), ALIGN)
        self.used = off
        self.n = self.s = self.off = 0
        self.full = None              # gathered compute copy (a view of the unit's slot)
        self.gwork = None             # full-size fp32 gradient buffer (backward only; slot view)
        self.slot = None              # [owner] cell shared by the units of one slot
        self.gathered = False
        self.g_live = False
        self.event = None             # comm-stream event of an in-flight prefetch


class _Z3Gate(Function):
    """Identity on (x, h) whose backward runs exactly once, after both gradients are complete."""

    @staticmethod
    def forward(ctx, z3, i, kind, x, h):
        ctx.z3, ctx.i, ctx.kind = z3, i, kind
        return x.view_as(x), h.view_as(h)

    @staticmethod
    def backward(ctx, gx, gh):
        if ctx.kind == "enter":
            ctx.z3._pre_backward(ctx.i)
        else:
            ctx.z3._post_backward(ctx.i)
        return None, None, None, gx, gh


class Zero3:
    """Partition ``units`` = [(name, [(param_name, Parameter)])] (unit 0 must be the outer unit)."""

    always_finish = True  # TrainStep: run finish() even on a single rank
    sharded = True        # Trainer.save_state: optimizer + master are per-rank partitions

    def wants_graph_comm(self):
        # the step's Python bookkeeping (gathered / live flags) runs once, at capture: the
        # reduction and the sharded optimizer step must be recorded into the same graph
        return True

    def graph_ok(self):
        """A captured ZeRO-3 step records its all-gathers / reduce-scatters into the graph: on one
        rank there are none; across ranks unless MFT_GRAPH_COMM=0 (recorded RCCL collectives,
        parallel/ddp.py) -- then the step runs eagerly."""
        import os
        return self.world == 1 or os.environ.get("MFT_GRAPH_COMM", "1") == "1"

    def __init__(self, units, device, group=None, prefetch: bool = True, **adamw_kwargs):
        self.group = group
        self.world = dist.get_world_size(group) if is_dist() else 1
        self.rank = dist.get_rank(group) if is_dist() else 0
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        # one rank: the "shard" of every unit is the whole unit, so the compute copies alias the
        # shard (shadow / master) and the kernels accumulate straight into the shard's gradient --
        # no gather copies, no gradient buffers to zero and fold in (MFT_Z3_FORCE_COPY=1 keeps the
        # multi-rank gather / slot / reduce path, for testing it on one GPU)
        import os
        self.direct = self.world == 1 and os.environ.get("MFT_Z3_FORCE_COPY", "0") != "1"
        self.prefetch = prefetch and self.cuda and not self.direct
        self.comm = torch.cuda.Stream(device=self.device) if self.prefetch else None
        self.rep: list = []
        self.units: list[_Unit] = []
        seen = set()
        for uname, named in units:
            sh = []
            for n, p in named:
                if id(p) in seen or not p.requires_grad:
                    continue
                seen.add(id(p))
                (self.rep if getattr(p, "_mft_fp32_compute", False) else sh).append((n, p))
            self.units.append(_Unit(uname, sh))
        # rank-local flat layout
        off = 0
        for u in self.units:
            u.n = _round(max(u.used, ALIGN), ALIGN * self.world)
            u.s = u.n // self.world
            u.off = off
            off += u.s
        self.rep_off = off
        rep_offs = []
        for _, p in self.rep:
            rep_offs.append(off)
            off += _round(p.numel(), ALIGN)
        self.flat = _ShardFlat(max(off, ALIGN), self.device, shadow=self.cuda)
        gdt = torch.bfloat16 if self.cuda else torch.float32
        # slots: the outer unit's own, and two shared by the even / odd block units
        slots = []
        if not self.direct:
            nb = max([u.n for u in self.units[1:]] + [ALIGN])
            slots = [(torch.empty(self.units[0].n, dtype=gdt, device=self.device),
                      torch.empty(self.units[0].n, dtype=torch.float32, device=self.device), [None])]
            slots += [(torch.empty(nb, dtype=gdt, device=self.device),
                       torch.empty(nb, dtype=torch.float32, device=self.device), [None]) for _ in range(2)]
        with torch.no_grad():
            for ui, u in enumerate(self.units):
                full32 = torch.zeros(u.n, dtype=torch.float32, device=self.device)
                for (n, p), o in zip(u.params, u.offsets):
                    full32[o:o + p.numel()].copy_(p.data.reshape(-1).float())
                if self.world > 1:  # identical starting weights on every rank
                    dist.broadcast(full32, src=0, group=group)
                self.flat.master[u.off:u.off + u.s].copy_(full32[self.rank * u.s:(self.rank + 1) * u.s])
                del full32
                if self.direct:
                    src = self.flat.shadow if self.cuda else self.flat.master
                    u.full, u.gwork, u.slot = src[u.off:u.off + u.n], self.flat.grad[u.off:u.off + u.n], [None]
                else:
                    full, gwork, owner = slots[0] if ui == 0 else slots[1 + (ui & 1)]
                    u.full, u.gwork, u.slot = full[:u.n], gwork[:u.n], owner
                for (n, p), o in zip(u.params, u.offsets):
                    k = p.numel()
                    view = u.full[o:o + k].view(p.shape)
                    if self.cuda:
                        p.shadow = view
                        # the fp32 parameter itself is never materialised on a GPU rank: a
                        # zero-stride placeholder keeps shape/dtype for autograd bookkeeping
                        p.data = torch.empty_strided(p.shape, [0] * p.dim(), dtype=torch.float32,
                                                     device=self.device)
                    else:
                        p.data = view
                    p.grad = u.gwork[o:o + k].view(p.shape)
            for (n, p), o in zip(self.rep, rep_offs):
                mv = self.flat.master[o:o + p.numel()].view(p.shape)
                mv.copy_(p.data.to(self.device, torch.float32))
                if self.world > 1:
                    dist.broadcast(mv, src=0, group=group)
                p.data = mv
                p.grad = self.flat.grad[o:o + p.numel()].view(p.shape)
        self.flat.refresh_shadow()
        self.opt = FusedAdamW(self.flat, **adamw_kwargs)
        self.stats = {"all_gather": 0, "reduce_scatter": 0}

    # ------------------------------------------------------------------ gather / release
    def _src(self, u):
        src = self.flat.shadow if self.cuda else self.flat.master
        return src[u.off:u.off + u.s]

    def _take_slot(self, u):
        """u becomes the occupant of its slot; a previous occupant's gathered copy is gone."""
        prev = u.slot[0]
        if prev is not None and prev is not u:
            self._release(prev)
        u.slot[0] = u

    def _issue_gather(self, u, on_comm: bool):
        if u.gathered:
            return
        self._take_slot(u)
        cur = torch.cuda.current_stream(self.device) if self.cuda else None
        if on_comm:
            self.comm.wait_stream(cur)  # the shard is current (optimizer step done)
            ctx = torch.cuda.stream(self.comm)
        else:
            ctx = torch.no_grad()
        if self.direct:  # the compute copy IS the shard
            self.stats["all_gather"] += 1
            u.gathered = True
            return
        with ctx, torch.no_grad():
            if self.world > 1:
                dist.all_gather_into_tensor(u.full, self._src(u), group=self.group)
            else:
                u.full.copy_(self._src(u))
            if on_comm:
                u.event = torch.cuda.Event()
                u.event.record(self.comm)
        self.stats["all_gather"] += 1
        u.gathered = True

    def _ensure(self, u):
        """Make unit u usable on the current stream."""
        if not u.gathered:
            self._issue_gather(u, False)
        if u.event is not None:
            torch.cuda.current_stream(self.device).wait_event(u.event)
            u.event = None

    def _release(self, u):
        if u.gathered:
            if u.event is not None:  # prefetched but never consumed
                torch.cuda.current_stream(self.device).wait_event(u.event)
                u.event = None
            u.gathered = False

    def _prefetch(self, j):
        if 0 <= j < len(self.units) and self.prefetch:
            self._issue_gather(self.units[j], True)

    # ------------------------------------------------------------------ model hooks
    def begin_forward(self):
        self._ensure(self.units[0])

    def pre_block(self, i, x, h):
        u = self.units[i + 1]
        self._ensure(u)
        self._prefetch(i + 2)
        if torch.is_grad_enabled() and (x.requires_grad or h.requires_grad):
            return _Z3Gate.apply(self, i, "exit", x, h)
        return x, h

    def post_block(self, i, x, h):
        self._release(self.units[i + 1])
        if torch.is_grad_enabled() and (x.requires_grad or h.requires_grad):
            return _Z3Gate.apply(self, i, "enter", x, h)
        return x, h

    def _pre_backward(self, i):
        u = self.units[i + 1]
        self._ensure(u)
        self._prefetch(i)  # unit of block i-1 (index i in self.units)
        if not u.g_live:
            if not self.direct:
                u.gwork.zero_()
            u.g_live = True

    def _post_backward(self, i):
        u = self.units[i + 1]
        self._reduce_scatter(u)
        self._release(u)

    def _reduce_scatter(self, u):
        if not u.g_live:
            return
        if self.direct:  # the kernels accumulated into the shard's gradient already
            self.stats["reduce_scatter"] += 1
            u.g_live = False
            return
        with torch.no_grad():
            dst = self.flat.grad[u.off:u.off + u.s]
            if self.world > 1:
                tmp = torch.empty(u.s, dtype=torch.float32, device=self.device)
                dist.reduce_scatter_tensor(tmp, u.gwork, op=dist.ReduceOp.SUM, group=self.group)
                dst.add_(tmp, alpha=1.0 / self.world)
            else:
                dst.add_(u.gwork)
        self.stats["reduce_scatter"] += 1
        u.g_live = False

    # ------------------------------------------------------------------ DataParallel-style reducer
    def begin_step(self):
        """Host bookkeeping before a step (runs eagerly, also before each graph replay)."""
        self.units[0].g_live = True

    def zero_grad_buffers(self):
        """Device side of the step start, issued by TrainStep inside the (captured) step: the outer
        unit's gradient buffer starts every step at zero.  (Zeroing it from begin_step instead ran
        outside the graph and, keyed on g_live, was skipped from the second replay on -- the outer
        unit's gradients then kept adding up across steps on the copy path.)"""
        if not self.direct:
            self.units[0].gwork.zero_()

    def finish(self):
        """After the last micro-batch's backward: outer-unit grads, replicated grads."""
        self._reduce_scatter(self.units[0])
        self._release(self.units[0])  # stale after the optimizer step
        if self.world > 1 and self.rep_off < self.flat.numel:
            g = self.flat.grad[self.rep_off:]
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
            g.div_(self.world)

    def close(self):
        pass

    # ------------------------------------------------------------------ optimizer surface
    def step(self, sumsq_ready: bool = False):
        o = self.opt
        if o.max_grad_norm is not None:
            g = self.flat.grad
            if g.is_cuda:
                from .._ext import native
                native().sumsq(g[:self.rep_off], o.sumsq_dev, False)
            else:
                o.sumsq_dev.copy_(g[:self.rep_off].double().pow(2).sum().float().reshape(1))
            if self.world > 1:
                dist.all_reduce(o.sumsq_dev, op=dist.ReduceOp.SUM, group=self.group)
            if self.rep_off < self.flat.numel:  # replicated part: identical everywhere, count once
                o.sumsq_dev.add_(g[self.rep_off:].double().pow(2).sum().float().reshape(1))
        if self.world > 1 and o.reduce_flag is None:
            o.reduce_flag = lambda f: dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
        o.step(sumsq_ready=True)

    def __getattr__(self, k):  # set_lr, grad_norm, skipped_last, lr, step_count, m, v, ...
        if k == "opt":
            raise AttributeError(k)
        return getattr(self.opt, k)

    def state_dict(self):
        sd = self.opt.state_dict()
        sd["zero_stage"] = 3
        sd["zero_rank"] = self.rank
        return sd

    def load_state_dict(self, sd):
        self.opt.load_state_dict(sd)

    # ------------------------------------------------------------------ consolidation
    @torch.no_grad()
    def full_state(self, names=None) -> dict:
        """{param_name: fp32 CPU tensor} of every trainable parameter (collective: call on all
        ranks).  Used for checkpoints / export; the training layout is untouched."""
        out = {}
        for u in self.units:
            full = torch.empty(u.n, dtype=torch.float32, device=self.device)
            if self.world > 1:
                dist.all_gather_into_tensor(full, self.flat.master[u.off:u.off + u.s].contiguous(), group=self.group)
            else:
                full.copy_(self.flat.master[u.off:u.off + u.s])
            for (n, p), o in zip(u.params, u.offsets):
                out[n] = full[o:o + p.numel()].view(p.shape).cpu()
        for n, p in self.rep:
            out[n] = p.detach().float().cpu().clone()
        return out

    def materialize(self):
        """Context manager: inside, every sharded parameter's ``.data`` holds its full fp32 value
        (e.g. for an HF-format export that reads module parameters); restored on exit."""
        z3 = self

        class _Ctx:
            def __enter__(self_):
                st = z3.full_state()
                self_.saved = []
                for u in z3.units:
                    for n, p in u.params:
                        self_.saved.append((p, p.data))
                        p.data = st[n].to(z3.device)
                return st

            def __exit__(self_, *exc):
                for p, d in self_.saved:
                    p.data = d
                return False

        return _Ctx()

    def load_full_state(self, state: dict):
        """Inverse of full_state (every rank passes the same dict)."""
        with torch.no_grad():
            for u in self.units:
                full = torch.zeros(u.n, dtype=torch.float32, device=self.device)
                for (n, p), o in zip(u.params, u.offsets):
                    full[o:o + p.numel()].copy_(state[n].reshape(-1).to(self.device, torch.float32))
                self.flat.master[u.off:u.off + u.s].copy_(full[self.rank * u.s:(self.rank + 1) * u.s])
            for n, p in self.rep:
                p.data.copy_(state[n].to(self.device, torch.float32))
            self.flat.refresh_shadow()
            for u in self.units:
                self._release(u)


def gpt2_units(model):
    units = [("outer", [("wte", model.wte), ("wpe", model.wpe)] +
              [(f"ln_f.{n}", p) for n, p in model.ln_f.named_parameters()])]
    for i, b in enumerate(model.blocks):
        units.append((f"block{i}", [(f"blocks.{i}.{n}", p) for n, p in b.named_parameters()]))
    return units


def gemma_units(model):
    units = [("outer", [("embed", model.embed)] + [(f"norm.{n}", p) for n, p in model.norm.named_parameters()])]
    for i, L in enumerate(model.layers):
        units.append((f"block{i}", [(f"layers.{i}.{n}", p) for n, p in L.named_parameters()]))
    return units


def attach_zero3(model, device, group=None, prefetch: bool = True, **adamw_kwargs) -> Zero3:
    """Partition a full-fine-tuning model's parameters (call after set_full_finetune())."""
    units = gemma_units(model) if hasattr(model, "layers") else gpt2_units(model)
    z3 = Zero3(units, device, group=group, prefetch=prefetch, **adamw_kwargs)
    model.zero3 = z3
    return z3
