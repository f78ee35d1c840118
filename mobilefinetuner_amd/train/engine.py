"""Training-step engine: eager or hipGraph-captured, with gradient accumulation, data parallelism,
global grad-norm clipping and the fused AdamW step.

Reference call stack: per step, `accum` micro-batches of forward -> lm_cross_entropy
-> loss*(1/accum) -> backward, then clip_and_get_grad_norm, lr_schedule, Adam::step, zero_grad,
MemoryManager::force_cleanup (gpt2_lora_finetune/main.cpp:561-684).  The reference reads the loss
back to the host on every micro-step (main.cpp:573); here the loss is accumulated on device and
only read when a log line is due, and with ``use_graph`` the whole sequence (zero-grad, every
micro-batch fwd+bwd, all-reduce, clip, AdamW) is one hipGraph replay — no per-kernel launch cost,
which matters at GPT-2-124M / seq 128 sizes where a step is a few milliseconds.
"""
from __future__ import annotations

import torch

from ..optim.adamw import FusedAdamW
from ..utils.trace import trace_range
from ..parallel.ddp import DataParallel
from ..utils.params import FlatParams



class TrainStep:
    def __init__(self, model, flat: FlatParams, opt: FusedAdamW, grad_accum: int = 1,
                 dp: DataParallel | None = None, use_graph: bool = False, graph_comm: bool | None = None,
                 loss_fn=None):
        self.model, self.flat, self.opt = model, flat, opt
        self.accum = max(1, int(grad_accum))
        self.dp = dp
        # a reducer whose step can only be captured with its collectives (ZeRO-3) may veto the graph
        self.use_graph = use_graph and (dp is None or not hasattr(dp, "graph_ok") or dp.graph_ok())
        # graph_comm: the gradient reduction and the optimizer step are recorded into the hipGraph
        # too (the reducer's collectives then overlap the captured backward); default: as the
        # reducer asks (multi-bucket RCCL data parallelism, ZeRO-3)
        if graph_comm is None:
            graph_comm = dp is not None and hasattr(dp, "wants_graph_comm") and dp.wants_graph_comm()
        self.graph_comm = bool(graph_comm)
        self.loss_fn = loss_fn or (lambda m, ids, lab, scale: m(ids, lab, loss_scale=scale))
        self.loss_dev = None
        self.graph = None
        self._static = None
        self._eager_warm = 0

    # ----------------------------------------------------------------- eager pieces
    def _fwd_bwd(self, batches):
        scale = 1.0 / self.accum
        if self.loss_dev is None or self.loss_dev.device != self.flat.grad.device:
            self.loss_dev = torch.zeros(1, device=self.flat.grad.device, dtype=torch.float32)
        self.loss_dev.zero_()
        self.flat.grad.zero_()
        if self.dp is not None and hasattr(self.dp, "zero_grad_buffers"):
            self.dp.zero_grad_buffers()  # reducer-owned gradient buffers (ZeRO-3 slots): in the graph
        from ..ops.functional import dropout_counter
        dropout_counter(self.flat.grad.device).add_(1)  # fresh LoRA-dropout masks every step
        for i, (ids, lab) in enumerate(batches):
            if self.dp is not None and hasattr(self.dp, "last_micro"):
                self.dp.last_micro = i == len(batches) - 1
            loss = self.loss_fn(self.model, ids, lab, scale)
            (loss * scale).backward()
            self.loss_dev.add_(loss.detach().float().reshape(1), alpha=scale)

    def _reduce(self):
        # ZeRO-3 must always finish (its outer-unit grads reach the shard there, even on 1 rank);
        # a DataParallel reducer decides itself (1-rank profiling groups)
        if self.dp is not None:
            self.dp.finish()

    def _opt(self):
        self.opt.step()

    def _eager_step(self, batches):
        if self.dp is not None:
            self.dp.begin_step()
        with trace_range("fwd_bwd"):
            self._fwd_bwd(batches)
        with trace_range("grad_allreduce"):
            self._reduce()
        with trace_range("optimizer"):
            self._opt()

    # ----------------------------------------------------------------- graph capture
    def _capture(self, batches):
        dev = self.flat.grad.device
        self._static = [(ids.clone(), lab.clone()) for ids, lab in batches]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            if self.dp is not None:
                self.dp.begin_step()
            # thread_local: RCCL's watchdog thread keeps polling the events of earlier collectives
            # while this thread captures; under the default "global" mode those hipEventQuery
            # calls fail (hipErrorStreamCaptureUnsupported) and abort the process group
            with torch.cuda.graph(self.graph, stream=side, capture_error_mode="thread_local"):
                self._fwd_bwd(self._static)
                if self.graph_comm:
                    self._reduce()
                    self._opt()
        torch.cuda.current_stream(dev).wait_stream(side)

    def __call__(self, batches):
        """batches: list (len = grad_accum) of (input_ids [B,S] int64, labels [B,S] int64) on device.
        Returns the device tensor holding the mean micro-batch loss (no host sync)."""
        assert len(batches) == self.accum, f"expected {self.accum} micro-batches"
        if not self.use_graph or not self.flat.grad.is_cuda:
            self._eager_step(batches)
            return self.loss_dev
        if self.graph is None:
            # warm-up eagerly (lazy kernel/attribute init, hipBLASLt workspaces) before capture;
            # these are real optimizer steps on real batches.
            if self._eager_warm < 2:
                self._eager_warm += 1
                self._eager_step(batches)
                return self.loss_dev
            self._capture(batches)
            # the capture did not execute the work; fall through to a replay on these batches
        for (sid, slab), (ids, lab) in zip(self._static, batches):
            if sid.data_ptr() != ids.data_ptr():
                sid.copy_(ids, non_blocking=True)
                slab.copy_(lab, non_blocking=True)
        if self.dp is not None:
            self.dp.begin_step()
        with trace_range("fwd_bwd_graph"):
            self.graph.replay()
        if not self.graph_comm:
            with trace_range("grad_allreduce"):
                self._reduce()
            with trace_range("optimizer"):
                self._opt()
        return self.loss_dev
