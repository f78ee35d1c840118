"""LoRA adapter checkpoints.

Reference formats (both F32 safetensors, sorted keys, compact header, ``__metadata__`` last):

* GPT-2 (LoraSaver, graph/lora_saver.cpp:123-280): keys ``layer.{i}.{attn.qkv|attn.q|attn.k|attn.v|
  attn.proj|mlp.fc_in|mlp.fc_out}.lora_{A,B}``, A ``[in, r]``, B ``[r, out]``; metadata
  {rank, alpha, dropout, split_qkv, targets} as strings (targets = "AttnQKV,AttnProj", ...).
  :func:`save_lora` reproduces this file byte for byte.
* Gemma (GemmaLoraInjector::save_lora_safetensors, graph/gemma_lora_injector.cpp:129-216): keys
  ``layer.{i}.attn.{q,k,v,proj}.lora_{A,B}``, PEFT layout A ``[r, in]``, B ``[out, r]``; metadata
  {rank, alpha, dropout, targets}.  We also export the MLP adapters (``mlp.gate/up/down``) when they
  were trained.

Plus a PEFT-native export (``adapter_model.safetensors`` + ``adapter_config.json``).
Internally A is ``[r, in]`` and B ``[r, out]`` (models/layers.py).
"""
from __future__ import annotations

import json
import os

import torch

from ..peft.lora import LoraSpec
from . import safetensors as st


def _fmt(x) -> str:
    """C++ ostream formatting of a float/int (default precision 6, %g-like)."""
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, int):
        return str(x)
    return f"{float(x):g}"


def _is_gemma(model) -> bool:
    return hasattr(model, "layers") and not hasattr(model, "blocks")


def lora_state(model) -> tuple[dict, dict]:
    """(tensors, metadata) in the reference layout for this model family."""
    spec: LoraSpec = getattr(model, "lora_spec", LoraSpec())
    tensors = {}
    gemma = _is_gemma(model)
    for m in model.modules():
        for sl in getattr(m, "lora_slices", []):
            A = sl.A.detach().float().cpu()
            B = sl.B.detach().float().cpu()
            if gemma:
                tensors[sl.name + ".lora_A"] = A.contiguous()           # [r, in]
                tensors[sl.name + ".lora_B"] = B.t().contiguous()       # [out, r]
            else:
                tensors[sl.name + ".lora_A"] = A.t().contiguous()       # [in, r]
                tensors[sl.name + ".lora_B"] = B.contiguous()           # [r, out]
    if gemma:
        present = sorted({k.split(".", 2)[2].rsplit(".lora_", 1)[0] for k in tensors})
        order = ["attn.q", "attn.k", "attn.v", "attn.proj", "mlp.gate", "mlp.up", "mlp.down"]
        meta = [("rank", _fmt(spec.rank)), ("alpha", _fmt(float(spec.alpha))), ("dropout", _fmt(float(spec.dropout))),
                ("targets", ",".join(t for t in order if t in present))]
    else:
        meta = [("rank", _fmt(spec.rank)), ("alpha", _fmt(float(spec.alpha))), ("dropout", _fmt(float(spec.dropout))),
                ("split_qkv", _fmt(bool(spec.split_qkv))), ("targets", ",".join(spec.targets))]
    return tensors, dict(meta)


def save_lora(path: str, model):
    """Write the adapter in the reference format (byte-compatible with graph/lora_saver.cpp)."""
    tensors, meta = lora_state(model)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    st.save_file(path, tensors, meta, sort_keys=True, align8=False)


def make_checkpoint_path(stem_path: str, step: int) -> str:
    """`<stem>_step<N><ext>` (gpt2_lora_finetune/main.cpp:180-187)."""
    root, ext = os.path.splitext(stem_path)
    return f"{root}_step{step}{ext or '.safetensors'}"


def load_lora(path: str) -> tuple[dict, dict]:
    return st.load_file(path), st.load_metadata(path)


def spec_from_metadata(meta: dict, tensors: dict) -> LoraSpec:
    rank = int(meta.get("rank", 0) or 0)
    if rank <= 0:
        a = next(v for k, v in tensors.items() if k.endswith("lora_A"))
        rank = min(a.shape)
    spec = LoraSpec(rank=rank, alpha=float(meta.get("alpha", 2 * rank)), dropout=float(meta.get("dropout", 0.0)))
    spec.split_qkv = meta.get("split_qkv", "false") == "true" or any(".attn.q.lora" in k for k in tensors)
    t = meta.get("targets", "")
    if t and "attn." not in t:
        spec.targets = [x for x in t.split(",") if x]
    else:
        tg = []
        for k in tensors:
            part = k.split(".", 2)[2].rsplit(".lora_", 1)[0]
            name = {"attn.qkv": "AttnQKV", "attn.q": "AttnQKV", "attn.k": "AttnQKV", "attn.v": "AttnQKV",
                    "attn.proj": "AttnProj", "mlp.fc_in": "MlpFcIn", "mlp.fc_out": "MlpFcOut"}.get(part)
            if name and name not in tg:
                tg.append(name)
        spec.targets = tg
    return spec


@torch.no_grad()
def attach_lora(model, tensors: dict, meta: dict) -> LoraSpec:
    """Clear existing adapters and re-attach from a checkpoint (LoraSaver::attach_from_state,
    graph/lora_saver.cpp:389-452).  Returns the spec."""
    from ..peft.lora import inject_gemma, inject_gpt2, parse_gemma_targets
    for m in model.modules():
        if hasattr(m, "clear_lora"):
            m.clear_lora()
    spec = spec_from_metadata(meta, tensors)
    gemma = _is_gemma(model)
    if gemma:
        parts = {k.split(".", 2)[2].rsplit(".lora_", 1)[0] for k in tensors}
        names = {"attn.q": "q_proj", "attn.k": "k_proj", "attn.v": "v_proj", "attn.proj": "o_proj",
                 "mlp.gate": "gate_proj", "mlp.up": "up_proj", "mlp.down": "down_proj"}
        spec.targets = parse_gemma_targets(",".join(names[p] for p in sorted(parts) if p in names))
        layers = sorted({int(k.split(".")[1]) for k in tensors})
        spec.layers = layers
        inject_gemma(model, spec)
    else:
        layers = sorted({int(k.split(".")[1]) for k in tensors})
        spec.layers = layers
        inject_gpt2(model, spec)
    for m in model.modules():
        for sl in getattr(m, "lora_slices", []):
            A = tensors[sl.name + ".lora_A"].float()
            B = tensors[sl.name + ".lora_B"].float()
            sl.A.data.copy_(A if gemma else A.t())
            sl.B.data.copy_(B.t() if gemma else B)
            for p in (sl.A, sl.B):
                if getattr(p, "shadow", None) is not None:
                    p.shadow.copy_(p.data.to(p.shadow.dtype))
    return spec


def export_peft(out_dir: str, model, base_model_name_or_path: str = ""):
    """PEFT-native adapter directory (adapter_model.safetensors + adapter_config.json)."""
    spec: LoraSpec = model.lora_spec
    gemma = _is_gemma(model)
    tensors, targets = {}, set()
    for mod_name, lin in model.linear_modules().items():
        for sl in lin.lora_slices:
            A = sl.A.detach().float().cpu()        # [r, in]
            B = sl.B.detach().float().cpu().t()    # [n, r]
            if gemma:
                sub = sl.name.split(".")[-1]
                full = {"q": "self_attn.q_proj", "k": "self_attn.k_proj", "v": "self_attn.v_proj",
                        "proj": "self_attn.o_proj", "gate": "mlp.gate_proj", "up": "mlp.up_proj",
                        "down": "mlp.down_proj"}[sub]
                layer = int(sl.name.split(".")[1])
                key = f"base_model.model.model.layers.{layer}.{full}"
                targets.add(full.split(".")[-1])
            else:
                if sl.ncols != lin.out_features:
                    raise ValueError(f"{sl.name}: partial-column adapters (split_qkv) have no PEFT equivalent")
                key = f"base_model.model.transformer.{mod_name}"
                targets.add(mod_name.split(".")[-1])
            tensors[key + ".lora_A.weight"] = A.contiguous()
            tensors[key + ".lora_B.weight"] = B.contiguous()
    os.makedirs(out_dir, exist_ok=True)
    st.save_file(os.path.join(out_dir, "adapter_model.safetensors"), tensors, {"format": "pt"})
    cfg = {"peft_type": "LORA", "task_type": "CAUSAL_LM", "r": spec.rank, "lora_alpha": spec.alpha,
           "lora_dropout": spec.dropout, "target_modules": sorted(targets), "bias": "none",
           "fan_in_fan_out": not gemma, "base_model_name_or_path": base_model_name_or_path,
           "inference_mode": True}
    with open(os.path.join(out_dir, "adapter_config.json"), "w") as f:
        json.dump(cfg, f, indent=2)
