"""Shared CLI plumbing: process-group bootstrap, model/tokenizer/data loading, energy and shard flags.

Flag names and defaults follow the reference CLIs (gpt2_lora_finetune/main.cpp:32-171,
optim/train_lora_gemma.cpp:173-350, eval_ppl.cpp:23-65, eval_mmlu.cpp:18-58).  Added:
``--dtype``, ``--random_init``/``--model`` preset, ``--synthetic_data``, ``--no_graph``,
``--compat_l2_adam``, ``--zero_stage``, ``--state_dir``, ``--metrics_out``, ``--device``.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..utils.logging import log0


def init_distributed(device_pref: str = "auto", timeout_s: float = 600.0):
    """One process per GPU (mft_launch / torchrun env).  Backend nccl (= RCCL over xGMI) on GPUs,
    gloo on CPU.  ``timeout_s`` bounds every collective: with TORCH_NCCL_ASYNC_ERROR_HANDLING the
    RCCL watchdog aborts a rank whose peer died instead of hanging, and mft_launch
    then stops the job."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() and device_pref != "cpu"
    dev = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        import datetime
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        to = datetime.timedelta(seconds=float(timeout_s))
        if use_cuda:
            dist.init_process_group("nccl", device_id=dev, timeout=to)
        else:
            dist.init_process_group("gloo", timeout=to)
    return rank, world, local, dev


def add_energy_args(ap):
    g = ap.add_argument_group("energy-aware throttling (reference PowerMonitor)")
    g.add_argument("--pm_interval", type=int, default=0)
    g.add_argument("--pm_batt_thresh", type=float, default=20.0)
    g.add_argument("--pm_temp_thresh", type=float, default=42.0)
    g.add_argument("--pm_fb_high", type=float, default=2.0)
    g.add_argument("--pm_fb_low", type=float, default=0.5)
    g.add_argument("--pm_ft_high", type=float, default=2.0)
    g.add_argument("--pm_ft_low", type=float, default=0.5)
    g.add_argument("--pm_manual_batt", type=float, default=100.0)
    g.add_argument("--pm_manual_temp", type=float, default=30.0)
    g.add_argument("--pm_disable_batt", action="store_true")
    g.add_argument("--pm_disable_temp", action="store_true")
    g.add_argument("--pm_schedule", default="")
    g.add_argument("--pm_gpu_telemetry", action="store_true",
                   help="read MI355X junction temperature / power headroom instead of manual readings")


def add_shard_args(ap):
    g = ap.add_argument_group("parameter sharding / offload")
    g.add_argument("--shard_enable", action="store_true",
                   help="LoRA: frozen weights in a pinned host tier, fetched per block under --shard_budget_mb; "
                        "full fine-tune: AdamW state in pinned host DRAM (same as --offload_optimizer)")
    g.add_argument("--offload_optimizer", action="store_true",
                   help="AdamW moments in pinned host DRAM, streamed through the GPU per chunk on a copy stream")
    g.add_argument("--shard_dir", default="")
    g.add_argument("--shard_budget_mb", type=int, default=512)
    g.add_argument("--shard_fp16_disk", type=int, default=1,
                   help="16-bit host/disk copies: host-offloaded AdamW moments in bf16 with stochastic rounding "
                        "(half the PCIe bytes); sharded frozen weights are bf16 already")
    g.add_argument("--zero_stage", type=int, default=0, choices=[0, 1, 2, 3],
                   help="ZeRO partitioning across ranks: optimizer state (1), + gradients (2), + parameters "
                        "with per-block all-gather / reduce-scatter (3)")


def add_runtime_args(ap):
    g = ap.add_argument_group("MI355X runtime")
    g.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    g.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    g.add_argument("--model", default="", help="architecture preset for --random_init (e.g. gpt2, gemma3-270m)")
    g.add_argument("--random_init", action="store_true", help="random-init weights (no checkpoint needed)")
    g.add_argument("--synthetic_data", action="store_true", help="random token data (no dataset needed)")
    g.add_argument("--synthetic_tokens", type=int, default=2_000_000)
    g.add_argument("--no_graph", action="store_true", help="disable hipGraph capture of the train step")
    g.add_argument("--compat_l2_adam", action="store_true", help="reference Adam: coupled L2 weight decay")
    g.add_argument("--state_dir", default="", help="full training-state checkpoint dir (resume target)")
    g.add_argument("--metrics_out", default="")
    g.add_argument("--activation_checkpointing", action="store_true")
    g.add_argument("--profile_steps", default="", help="a:b — hipProfilerStart/Stop + roctx ranges for steps a..b "
                   "(rocprofv3 --selected-regions)")
    g.add_argument("--trace", action="store_true", help="roctx ranges around every step phase (MFT_TRACE=1)")
    g.add_argument("--inject_fault", default="", help="step:rank — raise on that rank at that step (failure tests)")
    g.add_argument("--dist_timeout_s", type=float, default=600.0, help="collective timeout (RCCL watchdog)")


def runtime_train_kwargs(a) -> dict:
    """TrainConfig fields fed from the runtime flag block."""
    return dict(profile_steps=getattr(a, "profile_steps", ""),
                extra={"inject_fault": getattr(a, "inject_fault", ""), "trace": bool(getattr(a, "trace", False))})


def build_power_monitor(a):
    from .._ext import native
    rt = native().runtime
    c = rt.PowerConfig()
    c.check_interval_steps = a.pm_interval
    c.battery_threshold = a.pm_batt_thresh
    c.temp_threshold = a.pm_temp_thresh
    c.freq_b_high, c.freq_b_low = a.pm_fb_high, a.pm_fb_low
    c.freq_t_high, c.freq_t_low = a.pm_ft_high, a.pm_ft_low
    c.enable_battery = not a.pm_disable_batt
    c.enable_temp = not a.pm_disable_temp
    c.use_gpu_telemetry = bool(getattr(a, "pm_gpu_telemetry", False))
    c.gpu_index = int(os.environ.get("LOCAL_RANK", "0"))
    pm = rt.PowerMonitor(c)
    pm.set_manual_readings(a.pm_manual_batt, a.pm_manual_temp)
    if a.pm_schedule:
        pm.set_schedule(a.pm_schedule)
    if a.pm_interval <= 0 and not a.pm_schedule:
        return None
    return pm


def dtype_of(a):
    return torch.bfloat16 if a.dtype == "bf16" else torch.float32


def load_gpt2(pretrained_dir: str, preset: str, random_init: bool, device, dtype, seed: int = 0):
    from ..io import safetensors as st
    from ..models import hf_io
    from ..models.gpt2 import GPT2Config, GPT2Model
    cfg_path = os.path.join(pretrained_dir, "config.json") if pretrained_dir else ""
    if cfg_path and os.path.exists(cfg_path):
        cfg = GPT2Config.from_json(cfg_path)
        log0(f"  ✓ Loaded GPT-2 config: layers={cfg.n_layer}, hidden={cfg.n_embd}, heads={cfg.n_head}")
    else:
        cfg = GPT2Config.preset(preset or "gpt2")
        log0(f"  GPT-2 preset {preset or 'gpt2'}: layers={cfg.n_layer}, hidden={cfg.n_embd}, heads={cfg.n_head}")
    model = GPT2Model(cfg, dtype=dtype, device=device, init=random_init or not pretrained_dir, seed=seed)
    if pretrained_dir and not random_init:
        sd = st.load_model_dir(pretrained_dir)
        hf_io.load_gpt2_state(model, sd)
        log0("  ✓ Model load complete")
    else:
        log0("  ✓ Random-initialised weights")
    return model


def load_gemma(model_dir: str, preset: str, random_init: bool, device, dtype, seed: int = 0):
    from ..io import safetensors as st
    from ..models import hf_io
    from ..models.gemma3 import Gemma3Config, Gemma3Model
    cfg_path = os.path.join(model_dir, "config.json") if model_dir else ""
    if cfg_path and os.path.exists(cfg_path):
        cfg = Gemma3Config.from_json(cfg_path)
    else:
        cfg = Gemma3Config.preset(preset or "gemma3-270m")
    log0(f"  Gemma-3 config: layers={cfg.num_hidden_layers} hidden={cfg.hidden_size} heads={cfg.num_attention_heads}"
         f"/{cfg.num_key_value_heads} head_dim={cfg.head_dim} vocab={cfg.vocab_size}")
    model = Gemma3Model(cfg, dtype=dtype, device=device, init=random_init or not model_dir, seed=seed)
    if model_dir and not random_init:
        hf_io.load_gemma_state(model, st.load_model_dir(model_dir))
        log0("  ✓ Gemma weights loaded")
    else:
        log0("  ✓ Random-initialised weights")
    return model


def jsonl_append(path: str, rec: dict):
    import json
    if not path:
        return
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")
