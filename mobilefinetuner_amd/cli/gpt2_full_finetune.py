"""gpt2_full_finetune — full-parameter fine-tuning of GPT-2 (reference gpt2_full_finetune/main.cpp:
251-583; the reference never wired it into CMake).  All parameters train: fp32 masters + bf16 compute
shadows in one flat buffer, fused AdamW (weight decay 0.01 default like the reference), gradients
averaged over ranks with bucketed RCCL all-reduce overlapped with backward, or partitioned with
``--zero_stage 1|2|3`` (reduce-scatter + all-gather over xGMI; 3 also partitions the parameters,
gathered per block, parallel/zero3.py).  Saves an HF-keyed safetensors
checkpoint (Conv1D [in,out] layout) at ``--save_every`` and at the end.
"""
from __future__ import annotations

import argparse
import os

import torch

from . import common


def build_parser():
    ap = argparse.ArgumentParser(prog="gpt2_full_finetune", description=__doc__)
    ap.add_argument("--data_dir", default="")
    ap.add_argument("--pretrained_dir", default="")
    ap.add_argument("--output_path", default="")
    ap.add_argument("--resume_from", default="")
    ap.add_argument("--eval_out", default="")
    ap.add_argument("--epochs", type=int, default=0)
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--batch_size", type=int, default=1)
    ap.add_argument("--grad_accum_steps", type=int, default=1)
    ap.add_argument("--seq_len", type=int, default=128)
    ap.add_argument("--lr", type=float, default=5e-5)
    ap.add_argument("--weight_decay", type=float, default=0.01)
    ap.add_argument("--warmup_steps", type=int, default=0)
    ap.add_argument("--clip_grad_norm", type=float, default=1.0)
    ap.add_argument("--data_fraction", type=float, default=1.0)
    ap.add_argument("--log_interval", type=int, default=1)
    ap.add_argument("--eval_interval", type=int, default=0)
    ap.add_argument("--eval_batches", type=int, default=50)
    ap.add_argument("--eval_batch_size", type=int, default=2)
    ap.add_argument("--save_every", type=int, default=0)
    ap.add_argument("--ema_beta", type=float, default=0.9)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--bucket_mb", type=float, default=64.0)
    common.add_energy_args(ap)
    common.add_shard_args(ap)
    common.add_runtime_args(ap)
    return ap


def save_full(path, model):
    from ..io import safetensors as st
    from ..models import hf_io
    st.save_file(path, hf_io.export_gpt2_state(model), {"format": "pt", "writer": "mobilefinetuner_amd"})


def main(argv=None):
    a = build_parser().parse_args(argv)
    from ..data.wikitext2 import LMDataset, WT2Config
    from ..io import safetensors as st
    from ..io.lora_checkpoint import make_checkpoint_path
    from ..models import hf_io
    from ..parallel.ddp import DataParallel
    from ..tokenizers import GPT2Tokenizer
    from ..train.trainer import TrainConfig, Trainer
    from ..utils.logging import log0
    from ..utils.params import FlatParams

    rank, world, _, dev = common.init_distributed(a.device, getattr(a, 'dist_timeout_s', 600.0))
    torch.manual_seed(a.seed)
    log0("\n========== GPT-2 Full Finetune (MI355X) ==========\n")
    model = common.load_gpt2(a.pretrained_dir, a.model, a.random_init, dev, common.dtype_of(a), seed=1234)
    if a.resume_from:
        hf_io.load_gpt2_state(model, st.load_file(a.resume_from))
        log0(f"  ✓ Resumed weights from {a.resume_from}")
    a.seq_len = min(a.seq_len, model.cfg.n_positions)
    model.activation_checkpointing = a.activation_checkpointing
    model.set_full_finetune()
    z3 = None
    # full fine-tuning has no frozen weights to shard: --shard_enable moves the optimizer state to
    # the pinned host tier instead (BASELINE config "ZeRO-style param shard + host-DRAM offload")
    offload = bool(a.offload_optimizer or a.shard_enable) and dev.type == "cuda"
    if a.zero_stage == 3:
        from ..parallel.zero3 import attach_zero3
        z3 = attach_zero3(model, dev, lr=a.lr, weight_decay=a.weight_decay, max_grad_norm=a.clip_grad_norm,
                          l2_coupled=a.compat_l2_adam, offload=offload,
                          offload_dtype=torch.bfloat16 if a.shard_fp16_disk else torch.float32)
        flat = z3.flat
    else:
        flat = FlatParams(model.named_parameters(), dev, pad_multiple=world if a.zero_stage else 1)
    log0(f"  trainable params: {model.num_parameters(True):,}  (flat buffer {flat.numel:,}, "
         f"zero_stage={a.zero_stage}, ranks={world})")
    dcfg = WT2Config(data_dir=a.data_dir, seq_len=a.seq_len, seed=a.seed, data_fraction=a.data_fraction,
                     rank=rank, world=world)
    vcfg = WT2Config(**{**dcfg.__dict__, "drop_last": False, "shuffle_train": False})
    if a.synthetic_data or not a.data_dir:
        train = LMDataset.synthetic(dcfg, "train", model.cfg.vocab_size, a.synthetic_tokens)
        valid = LMDataset.synthetic(vcfg, "valid", model.cfg.vocab_size, max(a.synthetic_tokens // 20, 4 * a.seq_len))
    else:
        tok = GPT2Tokenizer.from_pretrained(a.pretrained_dir)
        dcfg.eos_id = vcfg.eos_id = tok.eos_id
        train = LMDataset.from_text(dcfg, "train", tok)
        valid = LMDataset.from_text(vcfg, "valid", tok)
    log0(f"  ✓ Train set: {train.num_sequences()} sequences; valid {valid.num_sequences()}")
    dp = DataParallel(flat, bucket_mb=a.bucket_mb) if (world > 1 and not a.zero_stage) else None
    tc = TrainConfig(epochs=a.epochs, steps=a.steps, batch_size=a.batch_size, grad_accum=a.grad_accum_steps,
                     lr=a.lr, weight_decay=a.weight_decay, warmup_steps=a.warmup_steps, schedule="gpt2",
                     clip_grad_norm=a.clip_grad_norm, l2_coupled=a.compat_l2_adam, log_interval=a.log_interval,
                     eval_interval=a.eval_interval, eval_batches=a.eval_batches, eval_batch_size=a.eval_batch_size,
                     eval_out=a.eval_out, save_every=a.save_every, ema_beta=a.ema_beta,
                     use_graph=not a.no_graph, state_dir=a.state_dir, metrics_out=a.metrics_out,
                     offload_optimizer=offload, offload_bf16=bool(a.shard_fp16_disk),
                     **common.runtime_train_kwargs(a))

    trainer = None

    def save_final(path):
        """Collective for ZeRO (every rank calls it); rank 0 writes."""
        if z3 is not None:
            with z3.materialize():
                if rank == 0:
                    save_full(path, model)
            return
        if a.zero_stage:
            trainer.opt.gather_master()
        if rank == 0:
            save_full(path, model)

    def save(step):
        if a.output_path:
            save_final(make_checkpoint_path(a.output_path, step))

    trainer = Trainer(model, flat, train, valid, tc, dev, save_fn=save, power_monitor=common.build_power_monitor(a),
                      dp=dp, zero_stage=a.zero_stage)
    if a.state_dir and (os.path.isdir(a.state_dir) or os.path.isdir(a.state_dir + ".old")):
        trainer.load_state(a.state_dir)  # full-state resume (weights, moments, step, data cursor, RNG)
    log0(f"[Training plan] steps_per_epoch={trainer.steps_per_epoch} total_steps={trainer.total_steps}\n")
    trainer.train()
    if a.output_path:
        save_final(a.output_path)
        log0(f"  ✓ Full model saved to {a.output_path}")
    if a.state_dir:
        trainer.save_state(a.state_dir)
    log0(f"✅ Training complete! total_tokens={trainer.total_tokens} final_ema_loss={(trainer.ema_loss or 0):.4f}")
    if dp is not None:
        dp.close()
    return trainer


if __name__ == "__main__":
    main()
