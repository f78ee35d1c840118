"""Parameter residency manager ("--shard_enable"): frozen weights live in pinned host memory and are
brought onto the GPU per transformer block under a device byte budget (LRU eviction), with the
next block prefetched on the copy stream while the current one computes.

Reference: ParameterSharder (operators/opt_ops/sharding/parameter_sharder.h:36-93, .cpp:86-276):
register_parameter -> offload to disk (optionally fp16), require(name) -> LRU eviction to fit the
budget + reload + refill the owner pointer, mark_dirty -> rewrite on eviction, offload_all; hooks
called from the model forward per block (graph/gpt2_model.cpp:536-554).  The reference's evicted
tensors stayed alive while the autograd graph referenced them ("real savings are bounded").

MI355X design: the native HostTier (csrc/runtime/offload.cpp) holds the bytes in pinned DRAM (and
optionally spills to ``--shard_dir`` files), copies run as hipMemcpyAsync on a high-priority copy
stream ordered with hipEvents; eviction frees the DEVICE STORAGE in place (``storage.resize_(0)``),
so tensors captured by autograd are released too and are re-filled in place before the backward of
their block (a gate autograd node at each block boundary calls ``require`` on the way back).
Frozen weights are bf16 already, so the host copy keeps the device dtype (the reference's
fp16-on-disk quantisation of fp32 weights has nothing to halve here; ``--shard_fp16_disk`` instead
halves the host-offloaded optimizer state, optim/adamw.py).  Eviction never synchronises the device
(stream-ordered release, see _evict), and the backward prefetches the preceding block.
"""
from __future__ import annotations

import torch

from .._ext import native


class _Group:
    def __init__(self, name, tensors):
        self.name = name
        self.tensors = tensors
        self.nbytes = [t.numel() * t.element_size() for t in tensors]


class ParameterSharder:
    def __init__(self, budget_bytes: int, disk_dir: str = "", prefetch: bool = True):
        self.tier = native().runtime.HostTier(int(budget_bytes), disk_dir, 0)
        self.groups: dict[str, _Group] = {}
        self.order: list[str] = []
        self.prefetch = prefetch
        self.stats = {"fetches": 0, "evictions": 0}

    def register_group(self, name: str, tensors):
        tensors = [t for t in tensors if t is not None]
        for t in tensors:
            if not (t.is_cuda and t.is_contiguous()):
                raise ValueError(f"{name}: sharded tensors must be contiguous GPU tensors")
        g = _Group(name, tensors)
        total = sum(g.nbytes)
        if self.tier.device_budget and total > self.tier.device_budget:
            raise RuntimeError(f"group {name} ({total} B) exceeds the shard budget ({self.tier.device_budget} B)")
        for i, t in enumerate(tensors):
            self.tier.add(f"{name}#{i}", g.nbytes[i])
            self.tier.offload(f"{name}#{i}", t)  # host copy now (weights are frozen: never dirty)
        self.groups[name] = g
        self.order.append(name)
        # register_parameter(keep_in_memory=false): drop the device copy until first require()
        for i in range(len(tensors)):
            self.tier.synchronize(f"{name}#{i}")
        self._evict(name)

    def _evict(self, name):
        g = self.groups[name]
        for i, t in enumerate(g.tensors):
            key = f"{name}#{i}"
            if not self.tier.resident(key):
                continue
            if self.tier.dirty(key):
                self.tier.offload(key, t)
                self.tier.synchronize(key)  # the write-back reads the storage on the copy stream
            # No device sync: the storage returns to the caching allocator on the compute stream,
            # which hands it out again only to later work of that stream (ordered after the
            # already-queued kernels still reading it), and every refill's H2D copy is ordered
            # after the compute stream by the tier (order event, csrc/runtime/offload.cpp).
            t.untyped_storage().resize_(0)
            self.tier.mark_resident(key, False)
        self.stats["evictions"] += 1

    def _fetch(self, name):
        g = self.groups[name]
        for i, t in enumerate(g.tensors):
            key = f"{name}#{i}"
            if self.tier.resident(key):
                self.tier.touch(key)
                continue
            t.untyped_storage().resize_(g.nbytes[i])
            self.tier.fetch(key, t)
            self.tier.mark_resident(key, True)
        self.stats["fetches"] += 1

    def _make_room(self, name, keep):
        """Evict least-recently-used groups (never those in ``keep``) until ``name`` fits."""
        g = self.groups[name]
        need = sum(b for i, b in enumerate(g.nbytes) if not self.tier.resident(f"{name}#{i}"))
        if not need:
            return
        victims = []
        for key in self.tier.victims(need, ""):
            gname = key.split("#")[0]
            if gname not in keep and gname not in victims:
                victims.append(gname)
        for v in victims:
            self._evict(v)

    def require(self, name: str, backward: bool = False):
        """Make ``name`` resident; prefetch the group used next -- the following block in the
        forward (after the last block: the embedding, which the tied LM head reads next), the
        preceding one in the backward (before block 0: the embedding, which the next step's forward
        reads first) -- evicting least-recently-used groups to make room, so the copy of the next
        group always overlaps the compute of this one (the reference's require() loads on demand)."""
        g = self.groups.get(name)
        if g is None:
            return
        self._make_room(name, {name})
        self._fetch(name)
        if self.prefetch and len(self.order) > 1:
            idx = self.order.index(name)
            nxt = self.order[(idx - 1) % len(self.order)] if backward else self.order[(idx + 1) % len(self.order)]
            both = sum(self.groups[name].nbytes) + sum(self.groups[nxt].nbytes)
            if nxt != name and (not self.tier.device_budget or both <= self.tier.device_budget):
                self._make_room(nxt, {name, nxt})
                self._fetch(nxt)

    def offload_all(self):
        for n in self.order:
            self._evict(n)

    def resident_bytes(self) -> int:
        return self.tier.resident_bytes


class _Gate(torch.autograd.Function):
    """Identity whose backward makes `name` resident before gradients enter that block."""

    @staticmethod
    def forward(ctx, x, sharder, name):
        ctx.sharder, ctx.name = sharder, name
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.sharder.require(ctx.name, backward=True)
        return g, None, None


def gate(x, sharder, name):
    if sharder is None or not torch.is_grad_enabled():
        return x
    return _Gate.apply(x, sharder, name)


def shard_gpt2(model, budget_bytes: int, disk_dir: str = "") -> ParameterSharder:
    """Register GPT-2's frozen weights per block (plus embeddings) and attach to the model."""
    sh = ParameterSharder(budget_bytes, disk_dir)
    sh.register_group("embed", [model.wte.data, model.wpe.data])
    for i, b in enumerate(model.blocks):
        for lin in (b.c_attn, b.c_proj, b.c_fc, b.mlp_proj):
            lin.weight._mft_sharded = True  # no cached transposed copies of offloaded weights
        ts = [b.c_attn.weight.data, b.c_attn.bias.data, b.c_proj.weight.data, b.c_proj.bias.data,
              b.c_fc.weight.data, b.c_fc.bias.data, b.mlp_proj.weight.data, b.mlp_proj.bias.data]
        sh.register_group(f"block{i}", [t for t in ts if not t.requires_grad])
    model.sharder = sh
    return sh


def shard_gemma(model, budget_bytes: int, disk_dir: str = "") -> ParameterSharder:
    sh = ParameterSharder(budget_bytes, disk_dir)
    sh.register_group("embed", [model.embed.data])
    for i, L in enumerate(model.layers):
        for lin in (L.qkv_proj, L.o_proj, L.gate_up_proj, L.down_proj):
            lin.weight._mft_sharded = True
        ts = [L.qkv_proj.weight.data, L.o_proj.weight.data, L.gate_up_proj.weight.data, L.down_proj.weight.data]
        sh.register_group(f"block{i}", ts)
    model.sharder = sh
    return sh
