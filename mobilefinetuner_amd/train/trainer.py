"""Model-agnostic training loop shared by the three training CLIs.

Reference orchestration: the gpt2_lora_finetune main loop (gpt2_lora_finetune/main.cpp:561-684),
GemmaLoRATrainer (optim/gemma_trainer.cpp:104-227) and LoRATrainer (optim/trainer.cpp:18-235):
micro-batch loop with 1/accum loss scaling, global grad-norm clip, LR schedule per update,
optimizer step, zero-grad, log line, EMA loss, periodic token-weighted validation PPL with JSONL
records, periodic adapter checkpoints, energy-aware sleep.

MI355X additions: the step runs through ``TrainStep`` (hipGraph capture, device-side loss
accumulation, fused AdamW), data-parallel gradient averaging + per-rank data shards, global
metrics all-reduced over ranks, NaN/Inf skip-step accounting, HBM stats and tokens/s in the log,
and a full training-state checkpoint (weights + AdamW moments + schedule step + data cursor/RNG +
EMA) so ``--resume_from`` continues exactly (the reference restored adapter weights only, Q19).
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from ..optim import schedules
from ..optim.adamw import FusedAdamW
from ..parallel.ddp import DataParallel, allreduce_sum_, is_dist
from ..utils.logging import log0, rank0
from ..utils.params import FlatParams
from ..utils import trace
from ..utils.trace import PhaseTimer, ProfileWindow, enable_tracing, trace_range
from .engine import TrainStep


@dataclass
class TrainConfig:
    epochs: int = 0
    steps: int = 0
    max_steps: int = -1
    batch_size: int = 1
    grad_accum: int = 1
    lr: float = 1e-4
    weight_decay: float = 0.0
    warmup_steps: int = 0
    warmup_ratio: float = 0.0
    schedule: str = "gpt2"          # gpt2 (warmup + cosine to 10%) | linear | cosine | constant
    clip_grad_norm: float = 1.0
    l2_coupled: bool = False        # reference Adam semantics (coupled L2)
    offload_optimizer: bool = False  # AdamW moments in pinned host DRAM, streamed per chunk
    offload_bf16: bool = True        # ... as bf16 (stochastic rounding; the reference's --shard_fp16_disk 1)
    log_interval: int = 1
    eval_interval: int = 0
    eval_batches: int = 50
    eval_batch_size: int = 2
    eval_out: str = ""
    save_every: int = 0
    ema_beta: float = 0.9
    use_graph: bool = True
    log_style: str = "gpt2"         # gpt2 | gemma
    state_dir: str = ""             # full training-state checkpoint directory
    profile_steps: str = ""         # "a:b" window for roctx ranges / torch profiler markers
    metrics_out: str = ""           # JSONL per-log-step metrics
    extra: dict = field(default_factory=dict)


def rng_state(device) -> dict:
    """Every RNG stream a resumed run must continue: torch CPU / HIP generators and the device
    step counter that keys the counter-based LoRA dropout masks."""
    from ..ops.functional import dropout_counter
    st = {"cpu": torch.get_rng_state().tolist()}
    if device.type == "cuda":
        st["cuda"] = torch.cuda.get_rng_state(device).tolist()
        st["dropout_ctr"] = int(dropout_counter(device).item())
    return st


def set_rng_state(st: dict, device):
    from ..ops.functional import dropout_counter
    if "cpu" in st:
        torch.set_rng_state(torch.tensor(st["cpu"], dtype=torch.uint8))
    if device.type == "cuda" and "cuda" in st:
        torch.cuda.set_rng_state(torch.tensor(st["cuda"], dtype=torch.uint8), device)
        dropout_counter(device).fill_(int(st.get("dropout_ctr", 0)))


class Trainer:
    @staticmethod
    def _odt(cfg):
        return torch.bfloat16 if cfg.offload_bf16 else torch.float32

    def __init__(self, model, flat: FlatParams, train_ds, valid_ds, cfg: TrainConfig, device,
                 save_fn=None, power_monitor=None, dp: DataParallel | None = None, loss_fn=None,
                 zero_stage: int = 0):
        self.model, self.flat, self.train_ds, self.valid_ds = model, flat, train_ds, valid_ds
        if device.type == "cuda":
            from ..utils.gemm_tuning import enable_tuned_gemms
            enable_tuned_gemms()
        self.cfg, self.device = cfg, device
        self.save_fn = save_fn
        self.pm = power_monitor
        self.dp = dp
        if zero_stage == 3:
            # parallel/zero3.py: attach_zero3(model, ...) already partitioned the model; ``flat`` is
            # its rank-local shard view.  The Zero3 object is both the optimizer and the reducer.
            z3 = model.zero3
            z3.opt.set_lr(cfg.lr)
            z3.opt.weight_decay = cfg.weight_decay
            z3.opt.max_grad_norm = cfg.clip_grad_norm if (cfg.clip_grad_norm or 0) > 0 else None
            z3.opt.l2_coupled = cfg.l2_coupled
            self.opt = z3
            dp = self.dp = z3
        elif zero_stage > 0:
            from ..parallel.zero import ZeroOptimizer, ZeroReducer
            self.opt = ZeroOptimizer(flat, zero_stage, lr=cfg.lr, weight_decay=cfg.weight_decay,
                                     max_grad_norm=cfg.clip_grad_norm, l2_coupled=cfg.l2_coupled,
                                     offload=cfg.offload_optimizer, offload_dtype=self._odt(cfg))
            dp = ZeroReducer(self.opt)
            self.dp = dp
        else:
            self.opt = FusedAdamW(flat, lr=cfg.lr, weight_decay=cfg.weight_decay,
                                  max_grad_norm=cfg.clip_grad_norm, l2_coupled=cfg.l2_coupled,
                                  offload=cfg.offload_optimizer, offload_dtype=self._odt(cfg))
        # every configuration -- ZeRO-3's gathers / prefetches / reduce-scatters included -- runs as
        # one hipGraph replay per step, except a host-offloaded optimizer (PCIe-bound chunk copies:
        # eager copies on the copy streams beat graph memcpy nodes, 306 vs 369 ms on GPT-2 XL)
        self.step_fn = TrainStep(model, flat, self.opt, grad_accum=cfg.grad_accum, dp=dp,
                                 use_graph=cfg.use_graph and device.type == "cuda" and not cfg.offload_optimizer,
                                 loss_fn=loss_fn)
        world = dist.get_world_size() if is_dist() else 1
        micro, accum = cfg.batch_size, max(1, cfg.grad_accum)
        n_local = train_ds.num_local()
        self.steps_per_epoch = max(1, (n_local + micro * accum - 1) // (micro * accum))
        self.total_steps = cfg.steps
        if cfg.epochs > 0:
            self.total_steps = self.steps_per_epoch * cfg.epochs
        if cfg.max_steps and cfg.max_steps > 0:
            self.total_steps = min(self.total_steps, cfg.max_steps) if self.total_steps else cfg.max_steps
        self.world = world
        self.global_step = 0
        self.ema_loss = None
        self.total_tokens = 0
        self.skipped = 0
        self._skipped_base = 0
        # EMA of the loss kept on device (no per-step host sync); read at log time only
        self._ema_dev = torch.zeros(1, dtype=torch.float32, device=device)
        self._ema_init = torch.zeros(1, dtype=torch.float32, device=device)
        self.history = []

    # ------------------------------------------------------------------ schedule
    def lr_at(self, step: int) -> float:
        c = self.cfg
        if c.schedule == "gpt2":
            return schedules.gpt2_cli_lr(step, c.lr, c.warmup_steps, self.total_steps)
        if c.schedule in ("linear", "cosine"):
            return schedules.gemma_lr(step + 1, c.lr, c.warmup_ratio, self.total_steps, c.schedule)
        return c.lr

    # ------------------------------------------------------------------ data
    def _to_dev(self, t):
        if self.device.type == "cuda":
            return t.pin_memory().to(self.device, non_blocking=True)
        return t.to(self.device)

    def _next_micro(self):
        b = self.train_ds.next_batch(self.cfg.batch_size, need_loop=True)
        return self._to_dev(b["input_ids"]), self._to_dev(b["targets"]), int(b["attention_mask"].sum().item())

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate(self, max_batches=None, batch_size=None) -> dict:
        """Token-weighted NLL over the validation split (exact: sum NLL / #predicted tokens,
        SURVEY §8 Q17); all-reduced over data-parallel ranks."""
        ds = self.valid_ds
        if ds is None:
            return {}
        ds.reset_cursor()
        nb = max_batches if max_batches is not None else self.cfg.eval_batches
        bs = batch_size or self.cfg.eval_batch_size
        self.model.eval()
        tot = torch.zeros(2, dtype=torch.float64, device=self.device)
        done = 0
        while nb <= 0 or done < nb:
            b = ds.next_batch(bs, need_loop=False)
            if b is None:
                break
            s, n = self.model.nll(self._to_dev(b["input_ids"]), self._to_dev(b["targets"]))
            tot[0] += s.double()
            tot[1] += n.double()
            done += 1
        self.model.train()
        allreduce_sum_(tot)
        nll = float(tot[0] / tot[1].clamp(min=1))
        return {"nll": nll, "ppl": math.exp(min(nll, 50.0)), "tokens": int(tot[1])}

    # ------------------------------------------------------------------ checkpoint / resume
    def _moments(self):
        sd = self.opt.state_dict()  # host copies (also for host-offloaded moments)
        return {"m": sd["m"], "v": sd["v"]}

    def save_state(self, path: str):
        """Everything goes into ``<path>.tmp`` first; rank 0 then swaps it in (``path`` ->
        ``path.old``, ``path.tmp`` -> ``path``) after all ranks wrote, so a crash mid-save never
        leaves a torn checkpoint (``load_state`` falls back to ``path.old``)."""
        import shutil

        from ..io import safetensors as st
        final, old = path, path + ".old"
        path = path + ".tmp"
        r = dist.get_rank() if is_dist() else 0
        if r == 0:
            shutil.rmtree(path, ignore_errors=True)
            os.makedirs(path, exist_ok=True)
        if is_dist():
            dist.barrier()
        if getattr(self.opt, "sharded", False):
            # ZeRO-3: every rank writes its own partition (master shard + AdamW moments)
            st.save_file(os.path.join(path, f"trainable.rank{r}.safetensors"),
                         {n: p.detach() for n, p in self.flat.named()})
            st.save_file(os.path.join(path, f"optimizer.rank{r}.safetensors"), self._moments())
        elif hasattr(self.opt, "stage"):
            # ZeRO-1/2: every rank updated only its shard of the fp32 master (other shards reach it
            # only through the bf16 shadow all-gather): consolidate the masters first (collective,
            # all ranks), then rank 0 writes them; moments are per-rank shards
            self.opt.gather_master()
            if r == 0:
                st.save_file(os.path.join(path, "trainable.safetensors"),
                             {n: p.detach() for n, p in self.flat.named()})
            st.save_file(os.path.join(path, f"optimizer.rank{r}.safetensors"), self._moments())
        elif r == 0:
            st.save_file(os.path.join(path, "trainable.safetensors"),
                         {n: p.detach() for n, p in self.flat.named()})
            st.save_file(os.path.join(path, "optimizer.safetensors"),
                         self._moments())
        self._sync_metrics()
        state = {"global_step": self.global_step, "opt_step": self.opt.step_count, "lr": self.opt.lr,
                 "ema_loss": self.ema_loss, "total_tokens": self.total_tokens, "skipped": self.skipped,
                 "data": self.train_ds.state(), "world": self.world, "total_steps": self.total_steps,
                 "rng": rng_state(self.device)}
        with open(os.path.join(path, f"trainer_state.rank{r}.json"), "w") as f:
            json.dump(state, f)
        if is_dist():
            dist.barrier()
        if r == 0:
            shutil.rmtree(old, ignore_errors=True)
            if os.path.exists(final):
                os.rename(final, old)
            os.rename(path, final)
            shutil.rmtree(old, ignore_errors=True)
        if is_dist():
            dist.barrier()

    def load_state(self, path: str):
        from ..io import safetensors as st
        r = dist.get_rank() if is_dist() else 0
        if not os.path.exists(path) and os.path.exists(path + ".old"):  # crash between the swap's renames
            path = path + ".old"
        def pick(stem):
            per_rank = os.path.join(path, f"{stem}.rank{r}.safetensors")
            return per_rank if os.path.exists(per_rank) else os.path.join(path, f"{stem}.safetensors")

        w = st.load_file(pick("trainable"))
        for n, p in self.flat.named():
            p.data.copy_(w[n].to(p.device, p.dtype))
        self.flat.refresh_shadow()
        if getattr(self.opt, "sharded", False):
            for u in self.model.zero3.units:  # gathered copies are stale now
                self.model.zero3._release(u)
        o = st.load_file(pick("optimizer"))
        sp = os.path.join(path, f"trainer_state.rank{r}.json")
        if not os.path.exists(sp):
            sp = os.path.join(path, "trainer_state.rank0.json")
        with open(sp) as f:
            s = json.load(f)
        self.opt.load_state_dict({"m": o["m"], "v": o["v"], "step": s["opt_step"], "lr": s["lr"]})
        self.global_step = int(s["global_step"])
        self.ema_loss = s["ema_loss"]
        self.total_tokens = int(s["total_tokens"])
        self.skipped = int(s.get("skipped", 0))
        self._skipped_base = self.skipped
        if getattr(self.opt, "skipped_dev", None) is not None:
            self.opt.skipped_dev.zero_()
        if self.ema_loss is not None:
            self._ema_dev.fill_(float(self.ema_loss))
            self._ema_init.fill_(1.0)
        if "rng" in s:
            set_rng_state(s["rng"], self.device)
        self.train_ds.restore(s["data"])
        log0(f"[Resume] restored full training state from {path} at global step {self.global_step}")

    # ------------------------------------------------------------------ device-side metrics
    def _ema_update(self, loss_dev, beta):
        """ema = beta * ema + (1 - beta) * loss on device; a non-finite loss leaves it unchanged.
        Each rank keeps the EMA of its local loss; the EMA is linear, so the all-reduced mean of the
        per-rank EMAs (taken at log time) equals the EMA of the rank-mean loss."""
        beta = max(0.0, min(0.9999, float(beta)))
        l = loss_dev.detach().float().reshape(1)
        ok = torch.isfinite(l)
        new = torch.where(self._ema_init > 0, beta * self._ema_dev + (1 - beta) * l, l)
        self._ema_dev.copy_(torch.where(ok, new, self._ema_dev))
        self._ema_init.copy_(torch.where(ok, torch.ones_like(self._ema_init), self._ema_init))

    def _sync_metrics(self):
        """Host copies of the device-side EMA and skipped-step counter (one sync, log time)."""
        if self.cfg.ema_beta > 0:
            # rank-invariant: every rank joins the all-reduce whether or not its own EMA has seen a
            # finite loss yet (branching on the local init flag first could leave some ranks out of
            # the collective and hang the job); the EMA is the mean over the initialised ranks
            e = torch.cat([(self._ema_dev * self._ema_init).reshape(1), self._ema_init.reshape(1)]).float()
            if is_dist():
                allreduce_sum_(e)
            n = float(e[1].item())
            if n > 0:
                self.ema_loss = float(e[0].item()) / n
        sk = getattr(self.opt, "skipped_dev", None)
        if sk is not None:
            self.skipped = self._skipped_base + int(sk.item())

    # ------------------------------------------------------------------ loop
    def _mfu(self, tps_per_gpu: float, seq: int):
        """Model TFLOP/s per GPU and MFU vs the MI355X bf16 dense peak (SURVEY §5.1 counters)."""
        cfg = getattr(self.model, "cfg", None)
        if cfg is None:
            return 0.0, 0.0
        if getattr(self, "_fpt", None) is None or self._fpt[0] != seq:
            n_params = sum(p.numel() for p in self.model.parameters())
            n_train = sum(p.numel() for p in self.model.parameters() if p.requires_grad)
            self._fpt = (seq, trace.model_flops_per_token_cfg(cfg, seq, n_params, n_train))
        return trace.mfu(tps_per_gpu, self._fpt[1])

    def train(self):
        c = self.cfg
        if self.total_steps <= 0:
            log0("[Train] nothing to do (steps=0)")
            return self.history
        accum = max(1, c.grad_accum)
        t_last = time.perf_counter()
        tok_last = self.total_tokens
        window = ProfileWindow(c.profile_steps)
        if c.extra.get("trace"):
            enable_tracing(True)
        timer = PhaseTimer(enabled=self.device.type == "cuda")
        fault = c.extra.get("inject_fault", "")
        fault_step, fault_rank = (int(v) for v in fault.split(":")) if fault else (-1, -1)
        my_rank = dist.get_rank() if is_dist() else 0
        for step in range(self.global_step, self.total_steps):
            window.before_step(step + 1)
            if step + 1 == fault_step and my_rank == fault_rank:
                raise RuntimeError(f"injected fault at step {step + 1} on rank {my_rank} (--inject_fault)")
            cur_epoch = step // self.steps_per_epoch + 1
            step_in_epoch = step % self.steps_per_epoch + 1
            lr = self.lr_at(step)
            self.opt.set_lr(lr)
            batches, ntok = [], 0
            for _ in range(accum):
                ids, tg, nt = self._next_micro()
                batches.append((ids, tg))
                ntok += nt
            with timer.phase("train_step"):
                loss_dev = self.step_fn(batches)
            window.after_step(step + 1)
            self.global_step = step + 1
            ntok_all = ntok * self.world
            self.total_tokens += ntok_all
            do_log = (step + 1) % max(1, c.log_interval) == 0 or step + 1 == self.total_steps
            if c.ema_beta > 0:
                self._ema_update(loss_dev, c.ema_beta)
            if do_log:
                lt = loss_dev.detach().clone()
                if is_dist():
                    allreduce_sum_(lt)
                    lt /= self.world
                loss = float(lt.item())
                skipped = self.opt.skipped_last()
                self._sync_metrics()
                step_ms = timer.report().get("train_step", 0.0)
                gn = self.opt.grad_norm()
                gn_clip = min(gn, c.clip_grad_norm) if c.clip_grad_norm > 0 else gn
                now = time.perf_counter()
                tps = (self.total_tokens - tok_last) / max(now - t_last, 1e-9)
                t_last, tok_last = now, self.total_tokens
                ppl = math.exp(min(loss, 50.0))
                mem = torch.cuda.max_memory_allocated(self.device) / 2 ** 30 if self.device.type == "cuda" else 0.0
                tflops, mfu_frac = self._mfu(tps / self.world, batches[0][0].shape[1])
                if c.log_style == "gemma":
                    log0(f"[Step {step + 1}] Loss={loss:.4f} PPL={ppl:.2f} LR={lr:.6g} "
                         f"grad_norm={gn_clip:.3f} tokens/s={tps:.0f}")
                else:
                    log0(f"[Train] epoch {cur_epoch}/{c.epochs} | step {step_in_epoch}/{self.steps_per_epoch} "
                         f"(global {step + 1}/{self.total_steps}) | lr {lr:.6f} | loss {loss:.4f} | ppl {ppl:.2f} "
                         f"| grad_norm {gn_clip:.3f} | tokens {ntok_all} | tokens_per_sec {tps:.0f} "
                         f"| hbm_peak_gb {mem:.2f} | step_ms {step_ms:.2f} | tflops {tflops:.1f} | mfu {mfu_frac:.3f}" + (" | skipped_nonfinite" if skipped else ""))
                rec = {"step": step + 1, "epoch": cur_epoch, "loss": loss, "lr": lr, "grad_norm": gn,
                       "tokens_per_sec": tps, "hbm_peak_gb": mem, "step_ms": step_ms, "skipped_total": self.skipped,
                       "tflops_per_gpu": tflops, "mfu": mfu_frac}
                self.history.append(rec)
                if c.metrics_out and rank0():
                    with open(c.metrics_out, "a") as f:
                        f.write(json.dumps(rec) + "\n")
            if c.eval_interval > 0 and (step + 1) % c.eval_interval == 0:
                ev = self.evaluate()
                self._sync_metrics()
                log0(f"\n[Eval] epoch {cur_epoch} | step {step + 1} | valid_ppl {ev['ppl']:.2f} | ema_loss "
                     f"{(self.ema_loss or 0):.4f} | total_tokens {self.total_tokens}\n")
                if c.eval_out and rank0():
                    with open(c.eval_out, "a") as f:
                        f.write(json.dumps({"step": step + 1, "epoch": cur_epoch, "valid_ppl": ev["ppl"],
                                            "ema_loss": self.ema_loss, "total_tokens": self.total_tokens}) + "\n")
            if c.save_every > 0 and (step + 1) % c.save_every == 0:
                # ZeRO checkpoints consolidate with collectives: every rank enters save_fn (which
                # writes on rank 0 only); otherwise only rank 0 calls it
                collective = hasattr(self.opt, "gather_master") or getattr(self.opt, "sharded", False)
                if self.save_fn is not None and (collective or rank0()):
                    self.save_fn(step + 1)
                if c.state_dir:
                    self.save_state(c.state_dir)
            if self.pm is not None:
                ms = self.pm.suggest_sleep_ms(step + 1)
                if ms > 0:
                    # the step is queued asynchronously: drain it first so the GPU really idles for
                    # the whole pause (a host-only sleep would overlap the running kernels and save
                    # no energy -- the reference's CPU engine slept after finishing its step)
                    if self.device.type == "cuda":
                        torch.cuda.synchronize(self.device)
                    time.sleep(ms / 1000.0)
        return self.history
