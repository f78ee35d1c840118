"""LoRA specification and injection for GPT-2 and Gemma-3.

Reference: LoraSpec / LoraInjector (operators/finetune_ops/graph/lora_injector.h:19-191,
lora_injector.cpp:48-148) for GPT-2 — targets {AttnQKV, AttnProj, MlpFcIn, MlpFcOut}, optional
split_qkv, scale alpha/r, A ~ U(+-sqrt(6/(in+r))) seeded 42+in+out, B = 0 — and
GemmaLoraSpec / GemmaLoraInjector (graph/gemma_lora_injector.h:9-56, .cpp:30-46) — targets
{q,k,v,o,gate,up,down}, presets full_attn_mlp / attention_only / attention_light, A ~ U(+-1/sqrt(in)).

On our side an adapter is a ``LoRASlice`` on a (possibly fused) Linear: Gemma's q|k|v and gate|up
projections are single fused GEMMs, so each adapter owns a column slice of the fused output.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

GPT2_TARGETS = ("AttnQKV", "AttnProj", "MlpFcIn", "MlpFcOut")
GEMMA_TARGETS = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj")
GEMMA_PRESETS = {
    "full": GEMMA_TARGETS,
    "full_attn_mlp": GEMMA_TARGETS,
    "attn": ("q_proj", "k_proj", "v_proj", "o_proj"),
    "attention_only": ("q_proj", "k_proj", "v_proj", "o_proj"),
    "light": ("q_proj", "v_proj"),
    "attention_light": ("q_proj", "v_proj"),
}
_ALIASES = {
    "attnqkv": "AttnQKV", "attn_qkv": "AttnQKV", "c_attn": "AttnQKV", "qkv": "AttnQKV",
    "attnproj": "AttnProj", "attn_proj": "AttnProj", "proj": "AttnProj",
    "mlpfcin": "MlpFcIn", "mlp_fc_in": "MlpFcIn", "c_fc": "MlpFcIn", "fc_in": "MlpFcIn",
    "mlpfcout": "MlpFcOut", "mlp_fc_out": "MlpFcOut", "fc_out": "MlpFcOut",
}


def parse_gpt2_targets(csv: str):
    out = []
    for item in csv.split(","):
        item = item.strip()
        if not item:
            continue
        t = _ALIASES.get(item.lower())
        if t is None:
            raise ValueError(f"unknown GPT-2 LoRA target {item!r}")
        if t not in out:
            out.append(t)
    return out


def parse_gemma_targets(csv_or_preset: str):
    key = csv_or_preset.strip().lower()
    if key in GEMMA_PRESETS:
        return list(GEMMA_PRESETS[key])
    out = []
    for item in csv_or_preset.split(","):
        item = item.strip().lower()
        if not item:
            continue
        if not item.endswith("_proj"):
            item = item + "_proj"
        if item not in GEMMA_TARGETS:
            raise ValueError(f"unknown Gemma LoRA target {item!r}")
        if item not in out:
            out.append(item)
    return out


@dataclass
class LoraSpec:
    rank: int = 8
    alpha: float = 16.0
    dropout: float = 0.0
    split_qkv: bool = False
    targets: list = field(default_factory=lambda: ["AttnQKV", "AttnProj"])
    layers: list | None = None  # None = all layers
    init: str = "reference"     # "reference" (seeded uniform as above) or "peft" (kaiming-uniform)
    seed: int = 42

    @property
    def scale(self):
        return self.alpha / self.rank


def _gpt2_init_A(in_f, out_f, r, seed_base):
    """Reference init (graph/lora_injector.cpp:70-85): A[in, r] ~ U(+-sqrt(6/(in+r))); returned as [r, in]."""
    g = torch.Generator().manual_seed(seed_base + in_f + out_f)
    bound = math.sqrt(6.0 / (in_f + r))
    return ((torch.rand(in_f, r, generator=g) * 2 - 1) * bound).t().contiguous()


def _peft_init_A(in_f, r, g):
    """PEFT kaiming_uniform(a=sqrt(5)) on lora_A.weight [r, in] == U(+-1/sqrt(in))."""
    bound = 1.0 / math.sqrt(in_f)
    return (torch.rand(r, in_f, generator=g) * 2 - 1) * bound


def inject_gpt2(model, spec: LoraSpec):
    """Attach adapters; freeze everything else.  Returns list of (name, A, B)."""
    for p in model.parameters():
        p.requires_grad_(False)
    C = model.cfg.n_embd
    added = []
    layers = spec.layers if spec.layers is not None else range(len(model.blocks))
    g = torch.Generator().manual_seed(spec.seed)
    for i in layers:
        b = model.blocks[i]
        plan = []
        if "AttnQKV" in spec.targets:
            if spec.split_qkv:
                plan += [(b.c_attn, 0, C, f"layer.{i}.attn.q"), (b.c_attn, C, C, f"layer.{i}.attn.k"),
                         (b.c_attn, 2 * C, C, f"layer.{i}.attn.v")]
            else:
                plan.append((b.c_attn, 0, 3 * C, f"layer.{i}.attn.qkv"))
        if "AttnProj" in spec.targets:
            plan.append((b.c_proj, 0, C, f"layer.{i}.attn.proj"))
        if "MlpFcIn" in spec.targets:
            plan.append((b.c_fc, 0, 4 * C, f"layer.{i}.mlp.fc_in"))
        if "MlpFcOut" in spec.targets:
            plan.append((b.mlp_proj, 0, C, f"layer.{i}.mlp.fc_out"))
        for lin, c0, n, name in plan:
            if spec.init == "peft":
                A0 = _peft_init_A(lin.in_features, spec.rank, g)
            else:
                A0 = _gpt2_init_A(lin.in_features, n, spec.rank, spec.seed)
            A, B = lin.add_lora(c0, n, spec.rank, spec.scale, A0, name)
            lin.lora_dropout = float(spec.dropout)
            added.append((name, A, B))
    model.lora_spec = spec
    return added


def inject_gemma(model, spec: LoraSpec):
    for p in model.parameters():
        p.requires_grad_(False)
    cfg = model.cfg
    qd, kd = cfg.num_attention_heads * cfg.head_dim, cfg.num_key_value_heads * cfg.head_dim
    I = cfg.intermediate_size
    g = torch.Generator().manual_seed(spec.seed)
    added = []
    layers = spec.layers if spec.layers is not None else range(len(model.layers))
    for i in layers:
        L = model.layers[i]
        plan = []
        t = spec.targets
        if "q_proj" in t:
            plan.append((L.qkv_proj, 0, qd, f"layer.{i}.attn.q"))
        if "k_proj" in t:
            plan.append((L.qkv_proj, qd, kd, f"layer.{i}.attn.k"))
        if "v_proj" in t:
            plan.append((L.qkv_proj, qd + kd, kd, f"layer.{i}.attn.v"))
        if "o_proj" in t:
            plan.append((L.o_proj, 0, cfg.hidden_size, f"layer.{i}.attn.proj"))
        if "gate_proj" in t:
            plan.append((L.gate_up_proj, 0, I, f"layer.{i}.mlp.gate"))
        if "up_proj" in t:
            plan.append((L.gate_up_proj, I, I, f"layer.{i}.mlp.up"))
        if "down_proj" in t:
            plan.append((L.down_proj, 0, cfg.hidden_size, f"layer.{i}.mlp.down"))
        for lin, c0, n, name in plan:
            A0 = _peft_init_A(lin.in_features, spec.rank, g)
            A, B = lin.add_lora(c0, n, spec.rank, spec.scale, A0, name)
            lin.lora_dropout = float(spec.dropout)
            added.append((name, A, B))
    model.lora_spec = spec
    return added


def lora_parameters(model):
    out = []
    for m in model.modules():
        for sl in getattr(m, "lora_slices", []):
            out.append((sl.name + ".lora_A", sl.A))
            out.append((sl.name + ".lora_B", sl.B))
    return out


def lora_slices(model):
    out = []
    for m in model.modules():
        for sl in getattr(m, "lora_slices", []):
            out.append((m, sl))
    return out


@torch.no_grad()
def merge_all(model, sign=1.0):
    for m in model.modules():
        if getattr(m, "lora_slices", None):
            m.merge_lora(sign)


def set_lora_enabled(model, enabled: bool):
    for m in model.modules():
        if hasattr(m, "lora_enabled"):
            m.lora_enabled = enabled
