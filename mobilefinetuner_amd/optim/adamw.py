"""Fused AdamW over the flat parameter buffer + global grad-norm clipping.

Reference: Adam (operators/finetune_ops/optim/adam.h:23-104, adam.cpp:25-140) — bias-corrected Adam
with *coupled* L2 weight decay (adam.cpp:65-67), AMSGrad option, save_state/load_state (stub) — and
the clip_grad_norm copies (gpt2_lora_finetune/main.cpp:491-516: global L2 norm, scale
max/(norm+1e-6) when norm > max).

Here: decoupled AdamW by default (the PyTorch/PEFT alignment scripts' semantics,
pytorch_alignment/gpt2_lora_finetune.py:239), ``l2_coupled=True`` reproduces the reference.  One
kernel launch updates every trainable parameter, applies the clip factor computed on device, skips
the step when any grad is non-finite, and writes the bf16 shadow weights.  lr / step / grad-norm
live in device memory so the whole optimizer step can be replayed from a hipGraph.
"""
from __future__ import annotations

import math
import os

import torch

from .._ext import native
from ..utils.params import FlatParams


class FusedAdamW:
    def __init__(self, flat: FlatParams, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 max_grad_norm: float | None = 1.0, l2_coupled: bool = False, skip_nonfinite: bool = True,
                 param_range: tuple[int, int] | None = None, offload: bool = False,
                 offload_chunk: int = 1 << 26, offload_dtype=torch.float32, offload_slots: int = 3):
        self.flat = flat
        self.beta1, self.beta2 = betas
        self.eps, self.weight_decay = eps, weight_decay
        self.max_grad_norm = max_grad_norm if (max_grad_norm or 0) > 0 else None
        self.l2_coupled = l2_coupled
        self.skip_nonfinite = skip_nonfinite
        dev = flat.master.device
        # optional sub-range (ZeRO-1/2: this rank owns [lo, hi) of the flat buffer)
        self.lo, self.hi = param_range if param_range is not None else (0, flat.numel)
        n = self.hi - self.lo
        # offload: the AdamW moments live in pinned host DRAM (native HostTier, csrc/runtime/
        # offload.cpp; SURVEY §2.13 "host-DRAM offload tier for optimizer state", the reference's
        # analogue is the disk sharder).  Default "zerocopy": the fused AdamW kernel reads and
        # writes them in place over PCIe (both directions at once, nothing staged): GPT-2 XL
        # ZeRO-3 offload 226.5 ms/step vs 314 ms streaming chunks through K device slots
        # ("stream", MFT_OFFLOAD_MODE=stream; profiles/r2_offload_zerocopy_vs_stream.txt)
        # offload_dtype=bf16 (the reference's --shard_fp16_disk default): the host copies of the
        # moments are 16-bit -- half the PCIe bytes each way -- and the kernel updates them in
        # place with stochastic rounding (optim.hip), the fp32 master weights stay fp32
        self.offload = bool(offload) and dev.type == "cuda"
        offload_chunk = int(os.environ.get("MFT_OFFLOAD_CHUNK", offload_chunk))
        offload_slots = int(os.environ.get("MFT_OFFLOAD_SLOTS", offload_slots))
        self.mdt = torch.bfloat16 if offload_dtype in (torch.bfloat16, torch.float16, "bf16", "fp16") else torch.float32
        # offload_mode: "stream" copies chunks through K device slots on two copy streams;
        # "zerocopy" lets the AdamW kernel read and write the pinned host moments directly over
        # PCIe (full duplex, no staging copies, no device slots)
        self.zerocopy = self.offload and os.environ.get("MFT_OFFLOAD_MODE", "zerocopy") == "zerocopy"
        if self.offload and self.zerocopy:
            self._tier = native().runtime.HostTier(0, "", 0)
            esz = torch.tensor([], dtype=self.mdt).element_size()
            for k in ("m", "v"):
                self._tier.add(f"{k}#0", n * esz)
                self._tier.host_tensor(f"{k}#0", self.mdt, [n]).zero_()
            self._chunks = [(0, n)]
            self._zm = self._tier.device_tensor("m#0", self.mdt, [n])
            self._zv = self._tier.device_tensor("v#0", self.mdt, [n])
            self.m = self.v = None
        elif self.offload:
            self._tier = native().runtime.HostTier(0, "", 0)
            self._chunks = []
            esz = torch.tensor([], dtype=self.mdt).element_size()
            for c0 in range(0, n, offload_chunk):
                c1 = min(n, c0 + offload_chunk)
                for k in ("m", "v"):
                    self._tier.add(f"{k}#{c0}", (c1 - c0) * esz)
                    self._tier.host_tensor(f"{k}#{c0}", self.mdt, [c1 - c0]).zero_()
                self._chunks.append((c0, c1))
            cmax = min(n, offload_chunk)
            # K device slots: the fetch of chunk c+K-1 only waits for the write-back of chunk c-1,
            # so H2D and D2H (PCIe is full duplex) stay busy together
            self._ns = max(2, int(offload_slots))
            self._slots = [(torch.empty(cmax, dtype=self.mdt, device=dev),
                            torch.empty(cmax, dtype=self.mdt, device=dev)) for _ in range(self._ns)]
            self.m = self.v = None
        else:
            self.m = torch.zeros(n, dtype=torch.float32, device=dev)
            self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        self.lr_dev = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
        # step_dev counts APPLIED updates (a NaN/Inf-skipped step does not advance the bias
        # correction); the kernel uses t = step_dev + 1 and adamw_commit advances it
        self.step_dev = torch.zeros(1, dtype=torch.float32, device=dev)
        self.sumsq_dev = torch.zeros(1, dtype=torch.float32, device=dev)
        self.nonfinite_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        # running count of skipped updates, kept on device (read only when a log line is due)
        self.skipped_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.lr = float(lr)
        self.attempts = 0
        # set by the ZeRO optimizers: all-reduces the skip flag (MAX) so every rank skips together
        self.reduce_flag = None

    # ---- host-side control (outside any captured graph)
    def set_lr(self, lr: float):
        self.lr = float(lr)
        self.lr_dev.fill_(self.lr)  # value travels as a kernel argument: no host-buffer race

    def grad_norm(self) -> float:
        """Global grad L2 norm of the last step (host sync)."""
        return math.sqrt(max(float(self.sumsq_dev.item()), 0.0))

    def skipped_last(self) -> bool:
        return bool(self.nonfinite_dev.item())

    @property
    def step_count(self) -> int:
        """Applied (non-skipped) updates (host sync)."""
        return int(self.step_dev.item())

    # ---- device work (graph-capturable)
    def compute_grad_sumsq(self, extra_sumsq=None):
        g = self.flat.grad[self.lo:self.hi]
        if g.is_cuda:
            native().sumsq(g, self.sumsq_dev, False)
        else:
            self.sumsq_dev.copy_(g.double().pow(2).sum().float().reshape(1))
        if extra_sumsq is not None:  # sharded (ZeRO) norm: caller all-reduces
            extra_sumsq(self.sumsq_dev)

    def step(self, sumsq_ready: bool = False):
        self.attempts += 1
        p = self.flat.master[self.lo:self.hi]
        g = self.flat.grad[self.lo:self.hi]
        if (self.max_grad_norm is not None) and not sumsq_ready:
            self.compute_grad_sumsq()
        if self.skip_nonfinite:
            self.nonfinite_dev.zero_()
            if p.is_cuda:
                native().nonfinite_check(g, self.nonfinite_dev)
            else:
                self.nonfinite_dev.fill_(int(not bool(torch.isfinite(g).all())))
            if self.reduce_flag is not None:
                self.reduce_flag(self.nonfinite_dev)
        sumsq = self.sumsq_dev if self.max_grad_norm is not None else None
        nonfinite = self.nonfinite_dev if self.skip_nonfinite else None
        if p.is_cuda:
            C = native()
            sh = self.flat.shadow[self.lo:self.hi] if self.flat.shadow is not None else None
            if self.offload and self.zerocopy:
                C.adamw_step(p, g, self._zm, self._zv, self.lr_dev, self.step_dev,
                             self.sumsq_dev if self.max_grad_norm is not None else None,
                             self.beta1, self.beta2, self.eps, self.weight_decay,
                             float(self.max_grad_norm or 0.0), self.l2_coupled, sh,
                             self.nonfinite_dev if self.skip_nonfinite else None, self.lo)
            elif self.offload:
                self._step_offloaded(C, p, g, sh)
            else:
                C.adamw_step(p, g, self.m, self.v, self.lr_dev, self.step_dev, sumsq,
                             self.beta1, self.beta2, self.eps, self.weight_decay,
                             float(self.max_grad_norm or 0.0), self.l2_coupled, sh, nonfinite, self.lo)
            C.adamw_commit(self.step_dev, nonfinite, sumsq)
        else:
            self._step_reference(p, g)
        if nonfinite is not None:
            self.skipped_dev.add_(self.nonfinite_dev)

    def _step_offloaded(self, C, p, g, sh):
        """Chunk c: H2D on one copy stream, update on the compute stream, D2H on another copy
        stream (PCIe is full duplex: write-back of chunk c-1 and fetch of chunk c+1 run at once).
        A device slot is refilled only after its previous chunk's write-back (slot_free event)."""
        cur = torch.cuda.current_stream(p.device)
        if not hasattr(self, "_h2d"):
            self._h2d = torch.cuda.Stream(device=p.device)
            self._d2h = torch.cuda.Stream(device=p.device)
            self._free = [torch.cuda.Event() for _ in range(self._ns)]
            self._host = [(self._tier.host_tensor(f"m#{c0}", self.mdt, [c1 - c0]),
                           self._tier.host_tensor(f"v#{c0}", self.mdt, [c1 - c0])) for c0, c1 in self._chunks]
        # every cross-stream dependency of the step is created inside it (hipGraph-capturable):
        # the previous step's write-backs precede this step's refills, both copy streams fork
        # from the compute stream, and a captured step joins its write-back stream at the end
        cur.wait_stream(self._d2h)
        for e in self._free:
            e.record(cur)
        self._h2d.wait_stream(cur)
        ns = self._ns
        fetched = [torch.cuda.Event() for _ in range(ns)]

        def fetch(i):
            c0, c1 = self._chunks[i]
            mb, vb = self._slots[i % ns]
            self._h2d.wait_event(self._free[i % ns])
            with torch.cuda.stream(self._h2d):
                mb[:c1 - c0].copy_(self._host[i][0], non_blocking=True)
                vb[:c1 - c0].copy_(self._host[i][1], non_blocking=True)
            fetched[i % ns].record(self._h2d)

        for i in range(min(ns - 1, len(self._chunks))):
            fetch(i)
        for i, (c0, c1) in enumerate(self._chunks):
            mb, vb = self._slots[i % ns]
            if i + ns - 1 < len(self._chunks):
                fetch(i + ns - 1)
            cur.wait_event(fetched[i % ns])
            C.adamw_step(p[c0:c1], g[c0:c1], mb[:c1 - c0], vb[:c1 - c0], self.lr_dev, self.step_dev,
                         self.sumsq_dev if self.max_grad_norm is not None else None,
                         self.beta1, self.beta2, self.eps, self.weight_decay,
                         float(self.max_grad_norm or 0.0), self.l2_coupled,
                         sh[c0:c1] if sh is not None else None,
                         self.nonfinite_dev if self.skip_nonfinite else None, self.lo + c0)
            self._d2h.wait_stream(cur)
            with torch.cuda.stream(self._d2h):
                self._host[i][0].copy_(mb[:c1 - c0], non_blocking=True)
                self._host[i][1].copy_(vb[:c1 - c0], non_blocking=True)
            self._free[i % ns].record(self._d2h)
        if torch.cuda.is_current_stream_capturing():
            cur.wait_stream(self._d2h)

    def _moments_host(self):
        if hasattr(self, "_d2h"):
            self._d2h.synchronize()
        if self.zerocopy:
            torch.cuda.current_stream(self.flat.master.device).synchronize()
        m = torch.cat([self._tier.host_tensor(f"m#{c0}", self.mdt, [c1 - c0]) for c0, c1 in self._chunks]).float()
        v = torch.cat([self._tier.host_tensor(f"v#{c0}", self.mdt, [c1 - c0]) for c0, c1 in self._chunks]).float()
        return m, v

    @torch.no_grad()
    def _step_reference(self, p, g):
        if self.skip_nonfinite and (bool(self.nonfinite_dev.item()) or not math.isfinite(float(self.sumsq_dev))):
            return
        clip = 1.0
        if self.max_grad_norm is not None:
            norm = float(self.sumsq_dev.sqrt())
            if norm > self.max_grad_norm:
                clip = self.max_grad_norm / (norm + 1e-6)
        self.step_dev.add_(1.0)
        t = float(self.step_dev)
        lr = float(self.lr_dev)
        gg = g * clip
        if self.l2_coupled:
            gg = gg + self.weight_decay * p
        self.m.mul_(self.beta1).add_(gg, alpha=1 - self.beta1)
        self.v.mul_(self.beta2).addcmul_(gg, gg, value=1 - self.beta2)
        bc1 = 1 - self.beta1 ** t
        bc2 = 1 - self.beta2 ** t
        denom = self.v.sqrt() / math.sqrt(bc2) + self.eps
        if not self.l2_coupled:
            p.mul_(1 - lr * self.weight_decay)
        p.addcdiv_(self.m, denom, value=-lr / bc1)
        if self.flat.shadow is not None:
            self.flat.shadow[self.lo:self.hi].copy_(p.to(self.flat.shadow.dtype))

    # ---- state (full training-state checkpoint)
    def state_dict(self):
        if self.offload:
            m, v = self._moments_host()
        else:
            m, v = self.m.detach().cpu(), self.v.detach().cpu()
        return {"m": m, "v": v, "step": self.step_count,
                "lr": self.lr, "betas": (self.beta1, self.beta2), "eps": self.eps,
                "weight_decay": self.weight_decay, "range": (self.lo, self.hi)}

    def load_state_dict(self, sd):
        if self.offload:
            if hasattr(self, "_d2h"):
                self._d2h.synchronize()
            torch.cuda.current_stream(self.flat.master.device).synchronize()
            for c0, c1 in self._chunks:
                self._tier.host_tensor(f"m#{c0}", self.mdt, [c1 - c0]).copy_(sd["m"][c0:c1])
                self._tier.host_tensor(f"v#{c0}", self.mdt, [c1 - c0]).copy_(sd["v"][c0:c1])
        else:
            self.m.copy_(sd["m"].to(self.m.device))
            self.v.copy_(sd["v"].to(self.v.device))
        self.step_dev.fill_(float(int(sd["step"])))
        self.set_lr(sd.get("lr", self.lr))
