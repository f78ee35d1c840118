#!/usr/bin/env python3
"""Headline benchmark: GPT-2-124M LoRA r=8, seq 128, bf16 training throughput (tokens/s).

Metric/config from BASELINE.json ("tokens/sec GPT-2-124M LoRA r=8 seq128 at 1/2/4/8 GPU").
Synthetic token data + random-init GPT-2-124M weights (no network); one process per GPU
(launch with torch.distributed.run for N > 1; RCCL over xGMI).  Every timed step is a full
training step: forward, fused LM-head cross-entropy, backward through all 12 blocks, gradient
all-reduce (N > 1), global grad-norm clip and the fused AdamW update.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config gpt2-lora|gemma3-270m-lora|gpt2-full|gpt2-xl-zero|gpt2-xl-zero3] [--zero S]
                  [--batch B] [--seq S] [--no-graph] [--cpu_smoke]

``--gpus N`` with N > 1 and no ``WORLD_SIZE`` in the environment: this process becomes a launcher
(``mobilefinetuner_amd.launch``) that starts N fresh rank processes (one per GPU, RCCL) and exits
with their exit code; it never touches the GPU itself.  Under ``torch.distributed.run`` (WORLD_SIZE
set) every process is one rank and ``--gpus`` must equal the world size.
``--cpu_smoke``: gpt2-tiny on the CPU over gloo, for the GPU-less multi-rank test of this path.

Prints ONE JSON line on rank 0.

Engines (``--engine``):
  native  (default for gpt2-lora, gemma3-270m-lora, gpt2-full) -- the torch-free libmft C++ engine:
          this process starts the native CLI (mobilefinetuner_amd/bin/gpt2_lora_finetune,
          train_lora_gemma, gpt2_full_finetune) as a fresh child with --random_init --synthetic_data
          --bench_steps K --bench_warmup W; the child runs the C++ autograd tape + hipGraph-captured
          step, times exactly K steps between device synchronizes and cross-rank barriers, takes the
          MAX over ranks (RCCL) and prints one MFT_BENCH line, which this process turns into the
          driver's JSON record.  Under torch.distributed.run each rank process starts its own child
          (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* pass through; the native communicator
          bootstraps on MASTER_PORT + 1).  This process never touches the GPU and never imports torch.
  torch   the PyTorch-driven Python package path (kept as the test oracle; the ZeRO configs).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# the reference publishes no tokens/s; its README epoch time (4-6 h / epoch of
# WikiText-2 on a mobile SoC, README.md:419) gives a derived 110-170 tokens/s.  We divide by the
# upper bound (170) so vs_baseline is conservative.
BASELINE_TOKENS_PER_SEC = 170.0


# BASELINE.json "configs" -> (model preset, mode, default micro-batch, seq, metric label)
CONFIGS = {
    # headline: GPT-2 small LoRA r=8 seq 128 (BASELINE.json "metric")
    "gpt2-lora": dict(model="gpt2", mode="lora", batch=1024, seq=128, targets="AttnQKV,AttnProj", engine="native",
                      metric="tokens/sec GPT-2-124M LoRA r=8 seq128 (training, whole job)"),
    # Gemma-3 270M LoRA r=8 seq 256 (RMSNorm / QK-norm+RoPE / GQA / sliding-window kernels)
    "gemma3-270m-lora": dict(model="gemma3-270m", mode="lora", batch=256, seq=256, targets="full", engine="native",
                             metric="tokens/sec Gemma-3-270M LoRA r=8 seq256 (training, whole job)"),
    # Gemma-3 1B LoRA r=8 seq 256 (the reference's larger Gemma preset, README.md:411: 26 layers,
    # d 1152, 4 q-heads / 1 KV head of 256, vocab 262144)
    "gemma3-1b-lora": dict(model="gemma3-1b", mode="lora", batch=128, seq=256, targets="full", engine="native",
                           metric="tokens/sec Gemma-3-1B LoRA r=8 seq256 (training, whole job)"),
    # GPT-2 small full fine-tuning, DP over RCCL (bucketed, backward-overlapped all-reduce).  Micro-
    # batches (profiles/r3_fullbatch_ab.txt, one MI355X): gpt2-full 512 x 128 1.046M tok/s, 1024 x 128
    # 1.075M (97 GB peak); GPT-2 XL ZeRO-3 64 x 128 70.6K, 128 x 128 84.8K, 256 x 128 87.1K (210 GB
    # peak on ONE GPU -- 1/N of the 25 GB optimizer state at N ranks); + host AdamW 64 x 128 34.2K,
    # 256 x 128 65.0K (the PCIe-bound optimizer step amortised over 4x the tokens)
    "gpt2-full": dict(model="gpt2", mode="full", batch=1024, seq=128, zero=0, engine="native",
                      metric="tokens/sec GPT-2-124M full fine-tune seq128 (training, whole job)"),
    # GPT-2 XL (1.5B) full fine-tuning with ZeRO-2 partitioned optimizer / reduce-scattered grads
    "gpt2-xl-zero": dict(model="gpt2-xl", mode="full", batch=256, seq=128, zero=2, engine="native",
                         metric="tokens/sec GPT-2-XL full fine-tune ZeRO-2 seq128 (training, whole job)"),
    # same with ZeRO-3: parameters partitioned too, all-gathered per block (prefetched one block
    # ahead on a communication stream), gradients reduce-scattered per block during backward
    "gpt2-xl-zero3": dict(model="gpt2-xl", mode="full", batch=256, seq=128, zero=3, engine="native",
                          metric="tokens/sec GPT-2-XL full fine-tune ZeRO-3 seq128 (training, whole job)"),
    # BASELINE config 5: ZeRO partition + host-DRAM tier (AdamW moments in pinned host memory,
    # streamed through the GPU per chunk on the native HostTier's copy stream)
    "gpt2-xl-zero3-offload": dict(model="gpt2-xl", mode="full", batch=256, seq=128, zero=3, offload=True, engine="native",
                                  metric="tokens/sec GPT-2-XL full fine-tune ZeRO-3 + host-offloaded AdamW "
                                         "seq128 (training, whole job)"),
}


# (layers, attention width) for the model-FLOPs formula (utils/trace.model_flops_per_token_cfg)
_ATTN_DIMS = {"gpt2": (12, 768), "gpt2-medium": (24, 1024), "gpt2-large": (36, 1280), "gpt2-xl": (48, 1600),
              "gemma3-270m": (18, 4 * 256), "gemma3-1b": (26, 4 * 256)}
MI355X_BF16_DENSE_TFLOPS = 2500.0


def _flops_per_token(model, seq, n_params, n_train):
    n_layer, d_attn = _ATTN_DIMS[model]
    return 4.0 * n_params + 2.0 * n_train + n_layer * 2 * seq * d_attn * 3


def _native_cmd(a, cfgd):
    """argv of the native CLI for this config (random-init weights, synthetic tokens)."""
    here = os.path.dirname(os.path.abspath(__file__))
    bindir = os.path.join(here, "mobilefinetuner_amd", "bin")
    total = a.steps + a.warmup
    # enough distinct synthetic tokens for a few different batches per rank (the stream wraps)
    ntok = max(2_000_000, 4 * a.batch * (a.seq + 1) * a.grad_accum)
    common = ["--random_init", "--synthetic_data", "--synthetic_tokens", str(ntok), "--seq_len", str(a.seq),
              "--bench_steps", str(a.steps), "--bench_warmup", str(a.warmup)]
    if a.no_graph:
        common.append("--no_graph")
    if cfgd["model"].startswith("gemma"):
        return [os.path.join(bindir, "train_lora_gemma"), "--model", cfgd["model"], "--batch", str(a.batch),
                "--grad_accum", str(a.grad_accum), "--rank", str(a.rank), "--alpha", str(a.alpha),
                "--lora_dropout", "0", "--targets", a.targets or cfgd["targets"], "--lr", "2e-4",
                "--max_steps", str(total), "--log_interval", "0"] + common
    exe = "gpt2_full_finetune" if cfgd["mode"] == "full" else "gpt2_lora_finetune"
    cmd = [os.path.join(bindir, exe), "--model", cfgd["model"], "--batch_size", str(a.batch),
           "--grad_accum_steps", str(a.grad_accum), "--steps", str(total), "--log_interval", "0"]
    if cfgd["mode"] == "full":
        cmd += ["--lr", "1e-5", "--weight_decay", "0.01"]
        zero = cfgd.get("zero", 0) if a.zero < 0 else a.zero
        if zero:  # on one GPU too: the partitioned path (1-rank communicator) is what runs
            cmd += ["--zero_stage", str(zero)]
        if cfgd.get("offload", False) or a.offload_optimizer:
            cmd += ["--offload", "host"]
            if a.offload_fp32:
                cmd += ["--offload_moments", "fp32"]
            if a.offload_mode:
                cmd += ["--offload_mode", a.offload_mode]
        if a.bf16_grads:
            cmd += ["--bf16_grads"]
    else:
        cmd += ["--rank", str(a.rank), "--alpha", str(a.alpha), "--lr", "2e-4",
                "--lora_targets", a.targets or cfgd["targets"]]
    return cmd + common


def run_native(a, cfgd) -> int:
    """Start the native CLI as a child (never exec: this process stays the parent), relay its
    exit code; rank 0 turns the child's MFT_BENCH line into the driver's JSON record."""
    import subprocess
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks")
    cmd = _native_cmd(a, cfgd)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env["MFT_BENCH_MARKS"] = "1"
    # the child's log goes to our stderr as it comes (progress), its MFT_BENCH line is kept; rank 0
    # integrates its GPU's socket power over the timed steps (MFT_BENCH_T0 .. T1) -- sysfs hwmon reads
    # in this process, which never touches the GPU runtime
    from mobilefinetuner_amd.energy import EnergyMeter, pci_power_reader
    meter = None
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    rec = None
    for line in p.stdout:
        if line.startswith("MFT_BENCH "):
            rec = json.loads(line[len("MFT_BENCH "):])
        elif line.startswith("MFT_BENCH_T0"):
            reader = pci_power_reader(line[len("MFT_BENCH_T0"):]) if rank == 0 else None
            if reader:  # the GPU this rank's engine runs on, by PCI address
                meter = EnergyMeter(interval=0.02, reader=reader)
                meter.__enter__()
        elif line.startswith("MFT_BENCH_T1"):
            if meter and meter._thr is not None:
                meter.__exit__(None, None, None)
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = p.wait()
    if rc != 0:
        sys.stderr.write(f"bench.py: native engine exited with {rc}: {' '.join(cmd)}\n")
        return rc
    if rank != 0:
        return 0
    if rec is None:
        sys.stderr.write("bench.py: the native engine printed no MFT_BENCH line\n")
        return 1
    dt = rec["seconds"]
    tokens = rec["world"] * rec["batch"] * rec["seq"] * rec["accum"] * rec["steps"]
    value = tokens / dt
    fpt = _flops_per_token(cfgd["model"], rec["seq"], rec["n_params"], rec["n_trainable"])
    tflops = value / rec["world"] * fpt / 1e12
    zero = (cfgd.get("zero", 0) if a.zero < 0 else a.zero) if cfgd["mode"] == "full" else 0
    mode = "LoRA r=%d alpha=%g targets=%s" % (a.rank, a.alpha, a.targets or cfgd["targets"]) \
        if cfgd["mode"] == "lora" else "full fine-tune" + (f" ZeRO-{zero}" if zero else "") + \
        (" + host-offloaded AdamW (bf16 moments)" if (cfgd.get("offload", False) or a.offload_optimizer) else "")
    # physical devices, not ranks: the loopback backend runs every rank on one GPU (tests)
    cbe = os.environ.get("MFT_COMM_BACKEND", "rccl")
    phys = 1 if cbe == "loopback" else rec["world"]
    out_rec = {
        "metric": cfgd["metric"],
        "value": round(value, 1),
        "unit": "tokens/s",
        "n_gpus": phys,
        "steps": rec["steps"],
        "warmup": rec["warmup"],
        "ms_per_step": round(1000 * dt / rec["steps"], 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / BASELINE_TOKENS_PER_SEC, 1) if a.config == "gpt2-lora" else None,
        "dtype": "bf16",
        "data": "synthetic (random tokens, random-init weights)",
        "config": {
            "model": f"{cfgd['model']} {mode} ({rec['n_params'] / 1e6:.0f}M params)",
            "global_batch": rec["world"] * rec["batch"] * rec["accum"],
            "micro_batch_per_gpu": rec["batch"],
            "seq_len": rec["seq"],
            "parallelism": f"dp{rec['world']}",
            "engine": "native libmft (C++ autograd tape, " + ("hipGraph-captured step)" if rec.get("hipgraph")
                                                               else "eager step, no hipGraph)"),
            "ranks": rec["world"],
            "backend": cbe if (rec["world"] > 1 or zero) else "none",
            "hipgraph": bool(rec.get("hipgraph", False)),  # what the engine ran, not what was asked
            "final_loss": round(rec["final_loss"], 4),
            "model_tflops_per_gpu": round(tflops, 1),
            "mfu_bf16_dense": round(tflops / MI355X_BF16_DENSE_TFLOPS, 4),
            "baseline_tokens_per_sec": BASELINE_TOKENS_PER_SEC if a.config == "gpt2-lora" else None,
            "peak_hbm_gb_rank0": rec.get("peak_reserved_gb"),
            "gpu_energy_rank0": _energy(meter, rec["batch"] * rec["seq"] * rec["accum"] * rec["steps"]),
        },
    }
    print(json.dumps(out_rec), flush=True)
    return 0


def _energy(meter, tokens_rank0):
    """rank 0's GPU over the timed steps: mean / peak socket power and joules per token of that GPU's
    own tokens (None when the sensors are not readable)"""
    if meter is None or meter._thr is None:
        return None
    r = meter.report(tokens_rank0)
    if not r.get("ok"):
        return None
    return {"mean_w": round(r["mean_w"], 1), "peak_w": round(r["peak_w"], 1),
            "joules_per_token": round(r["joules_per_token"], 6), "samples": r["samples"]}


def _odesc(a):
    return " + host-offloaded AdamW (" + ("fp32" if a.offload_fp32 else "bf16 stochastic-rounded") + " moments)"


def _force_comm():
    import torch.distributed as dist
    return dist.is_initialized() and os.environ.get("MFT_DP_FORCE_COMM", "0") == "1"


def build(a, cfgd, dev, world):
    import torch
    from mobilefinetuner_amd.optim.adamw import FusedAdamW
    from mobilefinetuner_amd.parallel.ddp import DataParallel
    from mobilefinetuner_amd.train.engine import TrainStep
    from mobilefinetuner_amd.utils.params import FlatParams

    name = cfgd["model"]
    if name.startswith("gemma"):
        from mobilefinetuner_amd.models.gemma3 import Gemma3Config, Gemma3Model
        mcfg = Gemma3Config.preset(name)
        model = Gemma3Model(mcfg, dtype=torch.bfloat16, device=dev, seed=1234)
        vocab = mcfg.vocab_size
    else:
        from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
        mcfg = GPT2Config.preset(name)
        model = GPT2Model(mcfg, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32, device=dev,
                          seed=1234)  # identical on every rank
        vocab = mcfg.vocab_size
    if cfgd["mode"] == "lora":
        from mobilefinetuner_amd.peft import lora as L
        if name.startswith("gemma"):
            spec = L.LoraSpec(rank=a.rank, alpha=a.alpha, targets=L.parse_gemma_targets(a.targets or cfgd["targets"]))
            L.inject_gemma(model, spec)
        else:
            spec = L.LoraSpec(rank=a.rank, alpha=a.alpha, targets=L.parse_gpt2_targets(a.targets or cfgd["targets"]))
            L.inject_gpt2(model, spec)
        flat = FlatParams(L.lora_parameters(model), dev)
        opt = FusedAdamW(flat, lr=2e-4, weight_decay=0.0, max_grad_norm=1.0)
        dp = DataParallel(flat) if (world > 1 or _force_comm()) else None
        desc = f"{name} LoRA r={a.rank} alpha={a.alpha:g} targets={a.targets or cfgd['targets']}"
    else:
        model.set_full_finetune()
        # the config's ZeRO stage also on 1 GPU (the stage's own collectives / gather-release work
        # is then measured even with nothing to shard across), so a config's label is what ran
        zero = cfgd.get("zero", 0)
        if a.zero >= 0:  # explicit override
            zero = a.zero
        offload = bool(cfgd.get("offload", False) or a.offload_optimizer)
        # host-offloaded AdamW moments in bf16 (the reference's --shard_fp16_disk default 1)
        okw = dict(offload=offload, offload_dtype=torch.float32 if a.offload_fp32 else torch.bfloat16)
        if zero == 3:
            from mobilefinetuner_amd.parallel.zero3 import attach_zero3
            z3 = attach_zero3(model, dev, lr=1e-5, weight_decay=0.01, max_grad_norm=1.0, **okw)
            desc = f"{name} full fine-tune ZeRO-3" + (_odesc(a) if offload else "")
            step = TrainStep(model, z3.flat, z3, grad_accum=a.grad_accum, dp=z3, use_graph=not (a.no_graph or offload))
            return model, step, vocab, desc, sum(p.numel() for p in model.parameters())
        flat = FlatParams(model.named_parameters(), dev, pad_multiple=max(1, world))
        if zero:
            from mobilefinetuner_amd.parallel.zero import ZeroOptimizer, ZeroReducer
            opt = ZeroOptimizer(flat, zero, lr=1e-5, weight_decay=0.01, max_grad_norm=1.0, **okw)
            dp = ZeroReducer(opt)
        else:
            opt = FusedAdamW(flat, lr=1e-5, weight_decay=0.01, max_grad_norm=1.0, **okw)
            dp = DataParallel(flat, reduce_dtype=torch.bfloat16 if a.bf16_grads else None) \
                if (world > 1 or _force_comm()) else None
        desc = f"{name} full fine-tune" + (f" ZeRO-{zero}" if zero else "") + (_odesc(a) if offload else "")
    # a host-offloaded optimizer step is PCIe-bound: it runs eagerly (as graph memcpy nodes its
    # chunk copies were slower, 369 vs 306 ms/step on GPT-2 XL ZeRO-3)
    offload = cfgd["mode"] == "full" and bool(cfgd.get("offload", False) or a.offload_optimizer)
    step = TrainStep(model, flat, opt, grad_accum=a.grad_accum, dp=dp, use_graph=not (a.no_graph or offload))
    nparams = sum(p.numel() for p in model.parameters())
    return model, step, vocab, desc, nparams


def _spawn_ranks(n: int) -> int:
    """Parent of an N-rank run started without torch.distributed.run: fresh subprocesses (never
    exec, never a GPU call here), rank-failure propagation by the launcher."""
    from mobilefinetuner_amd.launch import launch
    return launch([os.path.abspath(__file__)] + sys.argv[1:], n, timeout=float(os.environ.get("MFT_BENCH_TIMEOUT", 0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="gpt2-lora", choices=sorted(CONFIGS),
                    help="benchmark configuration (BASELINE.json configs); default = the headline metric")
    ap.add_argument("--engine", default="", choices=["", "native", "torch"],
                    help="native = the libmft C++ engine (default where the config has one), torch = the Python path")
    # micro-batch default per config; for the headline 1024 x 128 = 128k tokens per GPU per step: the
    # M dimension every block GEMM sees.  Measured on 1x MI355X, round 2 (profiles/r2_batch_ab.txt,
    # interleaved): B=512 1.537 / 1.544M tok/s, B=768 1.502 / 1.498M, B=1024 1.574 / 1.575M -- the
    # N = 768 / 2304 GEMMs tile into whole waves of 256 CUs at M = 64k and 128k (not at 96k), and
    # the per-step fixed costs (optimizer, LM-head finalize, small LoRA kernels) halve per token;
    # 288 GB HBM makes the activation footprint irrelevant.
    ap.add_argument("--batch", type=int, default=int(os.environ.get("MFT_BENCH_BATCH", 0)),
                    help="micro-batch (sequences) per GPU (0 = the config's default)")
    ap.add_argument("--seq", type=int, default=0)
    ap.add_argument("--offload_optimizer", action="store_true", help="full fine-tune: AdamW state in pinned host DRAM")
    ap.add_argument("--offload_fp32", action="store_true", help="offloaded AdamW moments in fp32 (default bf16)")
    ap.add_argument("--offload_mode", choices=["stream", "zerocopy"], default=None,
                    help="native ZeRO-3 offload: per-unit updates during the next forward (stream, default) or one "
                         "update after the backward (zerocopy)")
    ap.add_argument("--zero", type=int, default=-1, choices=[-1, 0, 1, 2, 3],
                    help="full fine-tune configs: ZeRO stage override (-1 = the config's, used when N > 1)")
    ap.add_argument("--rank", type=int, default=8)
    ap.add_argument("--alpha", type=float, default=16.0)
    ap.add_argument("--targets", default="")
    ap.add_argument("--grad_accum", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--bf16_grads", action="store_true", help="full fine-tune DP: all-reduce gradients in bf16")
    ap.add_argument("--cpu_smoke", action="store_true",
                    help="gpt2-tiny on the CPU over gloo (tests the multi-rank bench path without a GPU)")
    a = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(_spawn_ranks(a.gpus))
    cfgd = dict(CONFIGS[a.config])
    if a.cpu_smoke:
        cfgd["model"] = "gpt2-tiny"
    a.batch = a.batch or (4 if a.cpu_smoke else cfgd["batch"])
    a.seq = a.seq or (32 if a.cpu_smoke else cfgd["seq"])
    engine = a.engine or ("torch" if a.cpu_smoke else cfgd.get("engine", "torch"))
    if engine == "native":
        if a.cpu_smoke:
            raise SystemExit("bench.py: --cpu_smoke runs the torch path (the native engine is GPU-only)")
        sys.exit(run_native(a, cfgd))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if a.cpu_smoke:
        # host tensors run through the test-suite's fp32 oracle (the op layer itself is GPU-only)
        os.environ.setdefault("MFT_HOST_ORACLE", os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests",
                                                              "oracle"))
        dev = torch.device("cpu")
        a.no_graph = True
        if world > 1:
            dist.init_process_group("gloo")
    else:
        force_comm = os.environ.get("MFT_DP_FORCE_COMM", "0") == "1"
        if world > 1 or force_comm:
            if os.environ.get("MFT_DIST_BACKEND", "nccl") != "nccl":
                local_rank = 0  # every rank shares the one GPU
            torch.cuda.set_device(local_rank)
            if world == 1:  # 1-rank RCCL group: profile the reducer's collectives on one GPU
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 2000))
                os.environ.setdefault("RANK", "0")
                os.environ.setdefault("WORLD_SIZE", "1")
            backend = os.environ.get("MFT_DIST_BACKEND", "nccl")  # gloo: several ranks on one GPU (tests)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            else:
                dist.init_process_group(backend)
        dev = torch.device("cuda", local_rank)
        torch.cuda.set_device(dev)
    if world > 1:
        assert dist.get_world_size() == a.gpus, (dist.get_world_size(), a.gpus)
    sync = (lambda: None) if a.cpu_smoke else torch.cuda.synchronize
    if not a.cpu_smoke:
        # library GEMMs with the offline-tuned solutions shipped in the package (no tuning here)
        from mobilefinetuner_amd.utils.gemm_tuning import enable_tuned_gemms
        enable_tuned_gemms()

    model, step, vocab, desc, nparams = build(a, cfgd, dev, world)

    # synthetic WikiText-shaped data: per-rank disjoint random token streams, labels = next token
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    nbuf = 4
    data = []
    for _ in range(nbuf):
        mb = []
        for _ in range(a.grad_accum):
            toks = torch.randint(0, vocab, (a.batch, a.seq + 1), generator=g)
            mb.append((toks[:, :-1].contiguous().to(dev), toks[:, 1:].contiguous().to(dev)))
        data.append(mb)

    for i in range(a.warmup):
        step(data[i % nbuf])
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(data[i % nbuf])
    if world > 1:
        dist.barrier()
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    final_loss = float(loss.item())
    from mobilefinetuner_amd.utils import trace
    n_train = sum(p.numel() for p in model.parameters() if p.requires_grad)
    fpt = trace.model_flops_per_token_cfg(model.cfg, a.seq, nparams, n_train)
    tokens = world * a.batch * a.seq * a.grad_accum * a.steps
    value = tokens / dt
    tflops, mfu = trace.mfu(value / world, fpt)
    # physical devices, not ranks: gloo ranks share GPU 0 (tests), the CPU smoke uses none
    tbe = ("gloo" if a.cpu_smoke else os.environ.get("MFT_DIST_BACKEND", "nccl")) if world > 1 else "none"
    phys = 0 if a.cpu_smoke else (1 if tbe not in ("nccl", "none") else world)
    if rank == 0:
        out = {
            "metric": cfgd["metric"],
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": phys,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * dt / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            # the reference publishes no throughput; only the GPT-2 small figure can be derived
            "vs_baseline": round(value / BASELINE_TOKENS_PER_SEC, 1) if (a.config == "gpt2-lora" and not a.cpu_smoke) else None,
            "dtype": "fp32" if a.cpu_smoke else "bf16",
            "data": "synthetic (random tokens, random-init weights)" + (" [cpu smoke]" if a.cpu_smoke else ""),
            "config": {
                "model": f"{desc} ({nparams / 1e6:.0f}M params)",
                "global_batch": world * a.batch * a.grad_accum,
                "micro_batch_per_gpu": a.batch,
                "seq_len": a.seq,
                "parallelism": f"dp{world}",
                "ranks": world,
                "backend": "rccl" if tbe == "nccl" else tbe,
                "hipgraph": bool(getattr(step, "use_graph", False)),
                "final_loss": round(final_loss, 4),
                "model_tflops_per_gpu": round(tflops, 1),
                "mfu_bf16_dense": round(mfu, 4),
                "baseline_tokens_per_sec": BASELINE_TOKENS_PER_SEC if a.config == "gpt2-lora" else None,
            },
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
