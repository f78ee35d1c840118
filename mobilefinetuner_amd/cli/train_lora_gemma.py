"""train_lora_gemma — LoRA fine-tuning of Gemma-3 (270M / 1B) on WikiText-2 (reference
operators/finetune_ops/optim/train_lora_gemma.cpp:352-975 + GemmaLoRATrainer).

Flags follow the reference CliOptions (``--k v`` and ``--k=v``, unambiguous prefixes accepted);
unknown flags are reported and ignored like the reference parser.  The README-style aliases
``--learning_rate --lora_r --lora_alpha`` (which the reference silently ignored) are honoured.
``--targets full|attn|light`` picks the preset, ``--lora_targets q,k,v,o,gate,up,down`` overrides.
Schedule: warmup = ceil(ratio * updates), 1-indexed, then linear (default) or cosine to 0.
Saves ``<output_dir>/gemma_lora.safetensors`` (reference key layout, MLP adapters included).

Alignment mode (``--align_dump_dir``): one fixed batch forward/backward (+ ``--align_do_step``),
dumping inputs, per-layer hidden states, loss, LoRA grads and post-step weights as .npy, plus
finite-difference checks of selected attention LoRA gradients (``--align_numeric_attn``), like the
reference's cross-framework alignment harness (train_lora_gemma.cpp:609-922).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

from . import common


def build_parser():
    ap = argparse.ArgumentParser(prog="train_lora_gemma", description=__doc__, allow_abbrev=True,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model_dir", default="")
    ap.add_argument("--data_dir", default="")
    ap.add_argument("--pretokenized_path", default="")
    ap.add_argument("--pretokenized_meta", default="")
    ap.add_argument("--output_dir", default="runs/gemma_lora")
    ap.add_argument("--targets", default="full")
    ap.add_argument("--lora_targets", default="")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--max_steps", type=int, default=-1)
    ap.add_argument("--seq_len", type=int, default=256)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--grad_accum", type=int, default=1)
    ap.add_argument("--lr", "--learning_rate", dest="lr", type=float, default=2e-4)
    ap.add_argument("--rank", "--lora_r", dest="rank", type=int, default=8)
    ap.add_argument("--alpha", "--lora_alpha", dest="alpha", type=float, default=32.0)
    ap.add_argument("--lora_dropout", type=float, default=0.1)
    ap.add_argument("--warmup_ratio", type=float, default=0.03)
    ap.add_argument("--max_grad_norm", type=float, default=1.0)
    ap.add_argument("--weight_decay", type=float, default=0.0)
    ap.add_argument("--loss_reduction", default="mean", choices=["mean", "sum"])
    ap.add_argument("--lr_schedule", default="linear", choices=["linear", "cosine", "constant"])
    ap.add_argument("--data_fraction", type=float, default=1.0)
    ap.add_argument("--log_interval", type=int, default=1)
    ap.add_argument("--eval_steps", type=int, default=0)
    ap.add_argument("--eval_batches", type=int, default=50)
    ap.add_argument("--save_every", type=int, default=0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--preview_tokens", type=int, default=0)
    ap.add_argument("--interleaved_rope", action="store_true", help="reference RoPE pairing (SURVEY §8 Q9)")
    ap.add_argument("--dump_embedding_dir", default="")
    # alignment harness
    ap.add_argument("--align_dump_dir", default="")
    ap.add_argument("--align_layers", default="0,1,17")
    ap.add_argument("--align_dump_grads", action="store_true")
    ap.add_argument("--align_do_step", action="store_true")
    ap.add_argument("--align_disable_debug", action="store_true")
    ap.add_argument("--align_no_retain_grad", action="store_true")
    ap.add_argument("--align_pt_weights_dir", default="")
    ap.add_argument("--align_numeric_attn", action="store_true")
    ap.add_argument("--align_numeric_eps", type=float, default=1e-3)
    ap.add_argument("--align_numeric_count", type=int, default=4)
    ap.add_argument("--align_numeric_targets", default="q,v")
    common.add_energy_args(ap)
    common.add_shard_args(ap)
    common.add_runtime_args(ap)
    return ap


def _np_dump(d, name, t):
    import numpy as np
    os.makedirs(d, exist_ok=True)
    np.save(os.path.join(d, name + ".npy"), t.detach().float().cpu().numpy())


def alignment_mode(a, model, flat, train, dev):
    """Single fixed batch: dumps + optional one optimizer step + finite-difference grad checks."""
    from ..optim.adamw import FusedAdamW
    from ..utils.logging import log0
    d = a.align_dump_dir
    b = train.get_batch(list(range(min(a.batch, train.num_sequences()))))
    ids, tg = b["input_ids"].to(dev), b["targets"].to(dev)
    _np_dump(d, "input_ids", ids)
    layers = [int(x) for x in a.align_layers.split(",") if x.strip() != ""]
    caps = {}
    hooks = []
    for li in layers:
        if li < len(model.layers):
            L = model.layers[li]

            def mk(li):
                def hook(mod, inp, out):
                    caps[li] = out.detach()
                return hook
            hooks.append(L.post_feedforward_layernorm.register_forward_hook(mk(li)))
    loss = model(ids, tg)
    loss.backward()
    for h in hooks:
        h.remove()
    for li, t in caps.items():
        _np_dump(d, f"layer{li}_mlp_out", t)
    _np_dump(d, "loss", loss.detach().reshape(1))
    log0(f"[align] loss={loss.item():.6f}")
    if a.align_dump_grads:
        for n, p in flat.named():
            _np_dump(os.path.join(d, "grads"), n, p.grad)
    if a.align_numeric_attn:
        tg_names = [f".attn.{t.strip()}.lora_" for t in a.align_numeric_targets.split(",")]
        eps = a.align_numeric_eps
        checked = 0
        for n, p in flat.named():
            if not any(t in n for t in tg_names) or checked >= a.align_numeric_count:
                continue
            i = int(torch.argmax(p.grad.abs().reshape(-1)))
            ana = float(p.grad.reshape(-1)[i])
            with torch.no_grad():
                orig = float(p.data.reshape(-1)[i])
                vals = []
                for sgn in (1, -1):
                    p.data.reshape(-1)[i] = orig + sgn * eps
                    flat.refresh_shadow()
                    vals.append(float(model(ids, tg)))
                p.data.reshape(-1)[i] = orig
                flat.refresh_shadow()
            num = (vals[0] - vals[1]) / (2 * eps)
            log0(f"[align] {n}[{i}] analytic={ana:.6e} numeric={num:.6e} rel={abs(ana - num) / max(abs(num), 1e-12):.3e}")
            checked += 1
    if a.align_do_step:
        opt = FusedAdamW(flat, lr=a.lr, weight_decay=a.weight_decay, max_grad_norm=a.max_grad_norm)
        opt.step()
        for n, p in flat.named():
            _np_dump(os.path.join(d, "post_step"), n, p)
        log0(f"[align] one AdamW step done, grad_norm={opt.grad_norm():.6f}")
    log0(f"[align] dumps written to {d}")


def main(argv=None):
    ap = build_parser()
    a, unknown = ap.parse_known_args(argv)
    from ..data.wikitext2 import LMDataset, WT2Config
    from ..io.lora_checkpoint import make_checkpoint_path, save_lora
    from ..parallel.ddp import DataParallel
    from ..peft.lora import LoraSpec, inject_gemma, lora_parameters, parse_gemma_targets
    from ..tokenizers import GemmaTokenizer
    from ..train.trainer import TrainConfig, Trainer
    from ..utils.logging import log0
    from ..utils.params import FlatParams
    if unknown:
        log0(f"[train_lora_gemma] ignoring unknown arguments: {unknown}")
    rank, world, _, dev = common.init_distributed(a.device, getattr(a, 'dist_timeout_s', 600.0))
    torch.manual_seed(a.seed)
    log0("\n========== Gemma-3 LoRA Finetune (MI355X) ==========")
    model = common.load_gemma(a.model_dir, a.model, a.random_init, dev, common.dtype_of(a), seed=1234)
    model.set_interleaved_rope(a.interleaved_rope)
    model.activation_checkpointing = a.activation_checkpointing
    targets = parse_gemma_targets(a.lora_targets) if a.lora_targets else parse_gemma_targets(a.targets)
    spec = LoraSpec(rank=a.rank, alpha=a.alpha, dropout=a.lora_dropout, targets=targets, init="peft", seed=42)
    added = inject_gemma(model, spec)
    log0(f"  ✓ LoRA: {len(added)} adapters rank={a.rank} alpha={a.alpha:g} targets={targets}")
    if a.shard_enable and dev.type == "cuda":
        from ..parallel.sharder import shard_gemma
        largest = max(p.numel() * p.element_size() for p in model.parameters())
        budget = max(a.shard_budget_mb << 20, 2 * largest)  # reference raises the budget to the largest param
        sh = shard_gemma(model, budget, a.shard_dir)
        log0(f"  ✓ Parameter sharding ON: budget={budget >> 20} MB")
    flat = FlatParams(lora_parameters(model), dev)
    cfg = model.cfg
    dcfg = WT2Config(data_dir=a.data_dir, seq_len=a.seq_len, eos_id=cfg.eos_token_id, pad_id=cfg.pad_token_id,
                     seed=a.seed, data_fraction=a.data_fraction, rank=rank, world=world,
                     pretokenized_path=a.pretokenized_path, pretokenized_meta=a.pretokenized_meta)
    vcfg = WT2Config(**{**dcfg.__dict__, "drop_last": False, "shuffle_train": False})
    if a.synthetic_data or (not a.data_dir and not a.pretokenized_path):
        train = LMDataset.synthetic(dcfg, "train", cfg.vocab_size, a.synthetic_tokens)
        valid = LMDataset.synthetic(vcfg, "valid", cfg.vocab_size, max(a.synthetic_tokens // 20, 4 * a.seq_len))
    elif a.pretokenized_path:
        train = LMDataset.from_pretokenized(dcfg, "train")
        valid = LMDataset.from_pretokenized(vcfg, "valid")
    else:
        tok = GemmaTokenizer.from_pretrained(a.model_dir)
        dcfg.eos_id = vcfg.eos_id = tok.eos_id
        dcfg.pad_id = vcfg.pad_id = tok.pad_id
        train = LMDataset.from_text(dcfg, "train", tok)
        valid = LMDataset.from_text(vcfg, "valid", tok)
    if a.preview_tokens:
        log0(f"  preview: {train.tokens()[: a.preview_tokens].tolist()}")
    log0(f"  ✓ Train {train.num_sequences()} seqs, valid {valid.num_sequences()} seqs (seq_len={a.seq_len})")
    if a.align_dump_dir:
        alignment_mode(a, model, flat, train, dev)
        return None
    dp = DataParallel(flat) if world > 1 else None
    tc = TrainConfig(epochs=a.epochs, max_steps=a.max_steps, batch_size=a.batch, grad_accum=a.grad_accum, lr=a.lr,
                     weight_decay=a.weight_decay, warmup_ratio=a.warmup_ratio, schedule=a.lr_schedule,
                     clip_grad_norm=a.max_grad_norm, l2_coupled=a.compat_l2_adam, log_interval=a.log_interval,
                     eval_interval=a.eval_steps, eval_batches=a.eval_batches, eval_batch_size=a.batch,
                     save_every=a.save_every, use_graph=not a.no_graph, log_style="gemma", state_dir=a.state_dir,
                     metrics_out=a.metrics_out, **common.runtime_train_kwargs(a))
    out = os.path.join(a.output_dir, "gemma_lora.safetensors")

    def save(step):
        save_lora(make_checkpoint_path(out, step), model)

    trainer = Trainer(model, flat, train, valid, tc, dev, save_fn=save, power_monitor=common.build_power_monitor(a),
                      dp=dp)
    if a.state_dir and (os.path.isdir(a.state_dir) or os.path.isdir(a.state_dir + ".old")):
        trainer.load_state(a.state_dir)  # full-state resume (weights, moments, step, data cursor, RNG)
    log0(f"[Plan] steps/epoch={trainer.steps_per_epoch} total={trainer.total_steps}")
    trainer.train()
    if rank == 0:
        save_lora(out, model)
        log0(f"  ✓ Saved LoRA to {out}")
    if a.state_dir:
        trainer.save_state(a.state_dir)
    ev = trainer.evaluate()
    if ev:
        log0(f"[Eval] valid_loss={ev['nll']:.4f} valid_ppl={ev['ppl']:.2f}")
    if dp is not None:
        dp.close()
    return trainer


if __name__ == "__main__":
    main(sys.argv[1:])
