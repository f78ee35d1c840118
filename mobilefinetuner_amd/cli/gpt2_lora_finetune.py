"""gpt2_lora_finetune — LoRA fine-tuning of GPT-2 on WikiText-2 (reference
gpt2_lora_finetune/main.cpp:189-710), on MI355X.

    python -m mobilefinetuner_amd.cli.gpt2_lora_finetune --data_dir DATA --pretrained_dir gpt2 \
        --lora_out out/lora.safetensors --epochs 1 --batch_size 4 --grad_accum_steps 2 --lr 2e-4
    torchrun --nproc-per-node 8 -m mobilefinetuner_amd.cli.gpt2_lora_finetune ...   # data parallel

Defaults follow the reference CmdArgs; targets are the reference's fused c_attn + attn.c_proj
(``--lora_targets`` extends to the MLP, ``--split_qkv`` gives per-q/k/v adapters).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

from . import common


def build_parser():
    ap = argparse.ArgumentParser(prog="gpt2_lora_finetune", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--data_dir", default="")
    ap.add_argument("--pretrained_dir", default="")
    ap.add_argument("--lora_out", default="")
    ap.add_argument("--resume_from", default="")
    ap.add_argument("--eval_out", default="")
    ap.add_argument("--epochs", type=int, default=0)
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--batch_size", type=int, default=1)
    ap.add_argument("--grad_accum_steps", type=int, default=1)
    ap.add_argument("--seq_len", type=int, default=128)
    ap.add_argument("--rank", type=int, default=8)
    ap.add_argument("--alpha", type=float, default=16.0)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--weight_decay", type=float, default=0.0)
    ap.add_argument("--warmup_steps", type=int, default=0)
    ap.add_argument("--clip_grad_norm", type=float, default=1.0)
    ap.add_argument("--lora_dropout", type=float, default=0.0)
    ap.add_argument("--data_fraction", type=float, default=1.0)
    ap.add_argument("--log_interval", type=int, default=1)
    ap.add_argument("--eval_interval", type=int, default=0)
    ap.add_argument("--eval_batches", type=int, default=50)
    ap.add_argument("--eval_batch_size", type=int, default=2)
    ap.add_argument("--save_every", type=int, default=0)
    ap.add_argument("--ema_beta", type=float, default=0.9)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--lora_targets", default="AttnQKV,AttnProj")
    ap.add_argument("--split_qkv", action="store_true")
    ap.add_argument("--lora_init", default="reference", choices=["reference", "peft"])
    common.add_energy_args(ap)
    common.add_shard_args(ap)
    common.add_runtime_args(ap)
    return ap


def main(argv=None):
    a = build_parser().parse_args(argv)
    from ..data.wikitext2 import LMDataset, WT2Config
    from ..io.lora_checkpoint import attach_lora, load_lora, make_checkpoint_path, save_lora
    from ..parallel.ddp import DataParallel
    from ..peft.lora import LoraSpec, inject_gpt2, lora_parameters, parse_gpt2_targets
    from ..tokenizers import GPT2Tokenizer
    from ..train.trainer import TrainConfig, Trainer
    from ..utils.logging import log0
    from ..utils.params import FlatParams

    rank, world, _, dev = common.init_distributed(a.device, getattr(a, 'dist_timeout_s', 600.0))
    torch.manual_seed(a.seed)
    log0("\n========== GPT-2 LoRA Finetune (MI355X) ==========\n")
    log0("[Config]")
    for k in ("data_dir", "pretrained_dir", "lora_out", "resume_from", "eval_out", "epochs", "steps", "batch_size",
              "grad_accum_steps", "seq_len", "rank", "alpha", "lr", "weight_decay", "warmup_steps", "clip_grad_norm",
              "lora_dropout", "data_fraction", "log_interval", "eval_interval", "save_every", "ema_beta", "seed"):
        log0(f"  {k:<15}: {getattr(a, k)}")
    log0(f"  world_size     : {world} ({'RCCL/xGMI' if dev.type == 'cuda' and world > 1 else dev.type})")

    log0("\n[1/6] Loading pretrained model...")
    model = common.load_gpt2(a.pretrained_dir, a.model, a.random_init, dev, common.dtype_of(a), seed=1234)
    if a.seq_len > model.cfg.n_positions:
        log0(f"  ⚠️ seq_len({a.seq_len}) exceeds n_positions({model.cfg.n_positions}), clamped")
        a.seq_len = model.cfg.n_positions
    model.activation_checkpointing = a.activation_checkpointing

    log0("\n[2/6] LoRA adapters...")
    if a.resume_from and os.path.isfile(a.resume_from):
        tensors, meta = load_lora(a.resume_from)
        spec = attach_lora(model, tensors, meta)
        log0(f"  ✓ Resumed adapter from {a.resume_from} (rank={spec.rank}, targets={spec.targets})")
    else:
        spec = LoraSpec(rank=a.rank, alpha=a.alpha, dropout=a.lora_dropout, split_qkv=a.split_qkv,
                        targets=parse_gpt2_targets(a.lora_targets), init=a.lora_init, seed=42)
        added = inject_gpt2(model, spec)
        log0(f"  ✓ Injected {len(added)} adapters (rank={a.rank}, alpha={a.alpha:g}, targets={spec.targets})")
    if a.shard_enable and dev.type == "cuda":
        from ..parallel.sharder import shard_gpt2
        sh = shard_gpt2(model, a.shard_budget_mb << 20, a.shard_dir)
        log0(f"  ✓ Parameter sharding ON: budget={a.shard_budget_mb} MB, host tier {sh.tier.host_bytes >> 20} MB")
    flat = FlatParams(lora_parameters(model), dev)
    log0(f"  trainable params: {flat.numel:,} (padded)  |  total: {model.num_parameters():,}")

    log0("\n[3/6] Loading dataset...")
    dcfg = WT2Config(data_dir=a.data_dir, seq_len=a.seq_len, eos_id=50256, seed=a.seed,
                     data_fraction=a.data_fraction, rank=rank, world=world)
    vcfg = WT2Config(**{**dcfg.__dict__, "drop_last": False, "shuffle_train": False})
    if a.synthetic_data or not a.data_dir:
        train = LMDataset.synthetic(dcfg, "train", model.cfg.vocab_size, a.synthetic_tokens)
        valid = LMDataset.synthetic(vcfg, "valid", model.cfg.vocab_size, max(a.synthetic_tokens // 20, 4 * a.seq_len))
        log0("  (synthetic token data)")
    else:
        tok = GPT2Tokenizer.from_pretrained(a.pretrained_dir)
        dcfg.eos_id = vcfg.eos_id = tok.eos_id
        train = LMDataset.from_text(dcfg, "train", tok)
        valid = LMDataset.from_text(vcfg, "valid", tok)
    log0(f"  ✓ Train set: {train.num_sequences()} sequences ({train.num_local()} on this rank)")
    log0(f"  ✓ Validation set: {valid.num_sequences()} sequences")

    dp = DataParallel(flat) if world > 1 else None
    tc = TrainConfig(epochs=a.epochs, steps=a.steps, batch_size=a.batch_size, grad_accum=a.grad_accum_steps,
                     lr=a.lr, weight_decay=a.weight_decay, warmup_steps=a.warmup_steps, schedule="gpt2",
                     clip_grad_norm=a.clip_grad_norm, l2_coupled=a.compat_l2_adam, log_interval=a.log_interval,
                     eval_interval=a.eval_interval, eval_batches=a.eval_batches, eval_batch_size=a.eval_batch_size,
                     eval_out=a.eval_out, save_every=a.save_every, ema_beta=a.ema_beta, use_graph=not a.no_graph,
                     state_dir=a.state_dir, metrics_out=a.metrics_out,
                     **common.runtime_train_kwargs(a))

    def save(step):
        if a.lora_out:
            p = make_checkpoint_path(a.lora_out, step)
            save_lora(p, model)
            log0(f"\n[Checkpoint] Saved {p}\n")

    trainer = Trainer(model, flat, train, valid, tc, dev, save_fn=save, power_monitor=common.build_power_monitor(a),
                      dp=dp)
    if a.resume_from and (os.path.isdir(a.resume_from) or os.path.isdir(a.resume_from + ".old")):
        trainer.load_state(a.resume_from)
    log0("\n[Training plan]")
    log0(f"  epochs         : {a.epochs}\n  steps_per_epoch: {trainer.steps_per_epoch}\n  total_steps    : "
         f"{trainer.total_steps}\n  effective_batch: {a.batch_size * a.grad_accum_steps * world} (micro="
         f"{a.batch_size} × accum={a.grad_accum_steps} × ranks={world})")
    log0("\n[4/6] Optimizer: fused AdamW (" + ("coupled L2, reference" if a.compat_l2_adam else "decoupled") + ")")
    log0("\n[5/6] Starting training...\n========================================\n")
    trainer.train()
    log0("\n[6/6] Saving final LoRA weights...")
    if a.lora_out and rank == 0:
        save_lora(a.lora_out, model)
        log0(f"  ✓ LoRA saved to: {a.lora_out}")
    if a.state_dir:
        trainer.save_state(a.state_dir)
    log0("\n========================================\n✅ Training complete!")
    log0(f"  Total steps: {trainer.total_steps}\n  Total tokens: {trainer.total_tokens}\n  Final EMA loss: "
         f"{(trainer.ema_loss or 0):.4f}\n  Skipped (non-finite) steps: {trainer.skipped}")
    log0("========================================\n")
    if dp is not None:
        dp.close()
    return trainer


if __name__ == "__main__":
    try:
        main()
    except KeyboardInterrupt:
        sys.exit(130)
