"""HF-checkpoint key mapping for GPT-2 and Gemma-3 (load + export).

Reference: GPT2KeyMapper (graph/safetensors_loader.cpp:294-336), GemmaKeyMapper (:345-376),
load_tensors_mapped with the 'transformer.' prefix fallback (:250-253), and the full-model writer
collect_named_parameters / save (gpt2_full_finetune/main.cpp:122-237).

GPT-2 HF Conv1D weights are [in, out]; we store [out, in] (transposed here, once).  Gemma's q/k/v
and gate/up projections are fused into one weight each ([q;k;v], [gate;up]) for single GEMMs.
"""
from __future__ import annotations

import torch


def _strip(sd):
    out = {}
    for k, v in sd.items():
        if k.startswith("transformer."):
            k = k[len("transformer."):]
        out[k] = v
    return out


@torch.no_grad()
def _put(param, value):
    param.data.copy_(value.to(device=param.device, dtype=param.dtype).reshape(param.shape))


@torch.no_grad()
def load_gpt2_state(model, sd: dict):
    """sd: HF GPT2 state dict (torch tensors); missing keys raise."""
    sd = _strip(sd)
    V, C = model.cfg.vocab_size, model.cfg.n_embd
    wte = sd["wte.weight"]
    model.wte.data.zero_()
    model.wte.data[:V].copy_(wte.to(model.wte.dtype))
    _put(model.wpe, sd["wpe.weight"][: model.cfg.n_positions])
    for i, b in enumerate(model.blocks):
        p = f"h.{i}."
        _put(b.ln_1.weight, sd[p + "ln_1.weight"])
        _put(b.ln_1.bias, sd[p + "ln_1.bias"])
        _put(b.c_attn.weight, sd[p + "attn.c_attn.weight"].t())
        _put(b.c_attn.bias, sd[p + "attn.c_attn.bias"])
        _put(b.c_proj.weight, sd[p + "attn.c_proj.weight"].t())
        _put(b.c_proj.bias, sd[p + "attn.c_proj.bias"])
        _put(b.ln_2.weight, sd[p + "ln_2.weight"])
        _put(b.ln_2.bias, sd[p + "ln_2.bias"])
        _put(b.c_fc.weight, sd[p + "mlp.c_fc.weight"].t())
        _put(b.c_fc.bias, sd[p + "mlp.c_fc.bias"])
        _put(b.mlp_proj.weight, sd[p + "mlp.c_proj.weight"].t())
        _put(b.mlp_proj.bias, sd[p + "mlp.c_proj.bias"])
    _put(model.ln_f.weight, sd["ln_f.weight"])
    _put(model.ln_f.bias, sd["ln_f.bias"])


@torch.no_grad()
def export_gpt2_state(model, prefix: str = "") -> dict:
    """HF-keyed fp32 state dict (Conv1D [in,out] layout) — the full-FT checkpoint format."""
    V = model.cfg.vocab_size
    f = lambda t: t.detach().float().cpu().contiguous()  # noqa: E731
    sd = {prefix + "wte.weight": f(model.wte[:V]), prefix + "wpe.weight": f(model.wpe)}
    for i, b in enumerate(model.blocks):
        p = f"{prefix}h.{i}."
        sd[p + "ln_1.weight"] = f(b.ln_1.weight)
        sd[p + "ln_1.bias"] = f(b.ln_1.bias)
        sd[p + "attn.c_attn.weight"] = f(b.c_attn.weight.t())
        sd[p + "attn.c_attn.bias"] = f(b.c_attn.bias)
        sd[p + "attn.c_proj.weight"] = f(b.c_proj.weight.t())
        sd[p + "attn.c_proj.bias"] = f(b.c_proj.bias)
        sd[p + "ln_2.weight"] = f(b.ln_2.weight)
        sd[p + "ln_2.bias"] = f(b.ln_2.bias)
        sd[p + "mlp.c_fc.weight"] = f(b.c_fc.weight.t())
        sd[p + "mlp.c_fc.bias"] = f(b.c_fc.bias)
        sd[p + "mlp.c_proj.weight"] = f(b.mlp_proj.weight.t())
        sd[p + "mlp.c_proj.bias"] = f(b.mlp_proj.bias)
    sd[prefix + "ln_f.weight"] = f(model.ln_f.weight)
    sd[prefix + "ln_f.bias"] = f(model.ln_f.bias)
    return sd


@torch.no_grad()
def load_gemma_state(model, sd: dict):
    """sd: HF Gemma3ForCausalLM / Gemma3TextModel state dict."""
    def g(k):
        for cand in (k, "model." + k, "model.language_model." + k, "language_model.model." + k):
            if cand in sd:
                return sd[cand]
        raise KeyError(k)

    cfg = model.cfg
    emb = g("embed_tokens.weight")
    model.embed.data.zero_()
    model.embed.data[: cfg.vocab_size].copy_(emb[: cfg.vocab_size].to(model.embed.dtype))
    for i, L in enumerate(model.layers):
        p = f"layers.{i}."
        qkv = torch.cat([g(p + "self_attn.q_proj.weight"), g(p + "self_attn.k_proj.weight"),
                         g(p + "self_attn.v_proj.weight")], 0)
        _put(L.qkv_proj.weight, qkv)
        _put(L.o_proj.weight, g(p + "self_attn.o_proj.weight"))
        _put(L.q_norm.weight, g(p + "self_attn.q_norm.weight"))
        _put(L.k_norm.weight, g(p + "self_attn.k_norm.weight"))
        gu = torch.cat([g(p + "mlp.gate_proj.weight"), g(p + "mlp.up_proj.weight")], 0)
        _put(L.gate_up_proj.weight, gu)
        _put(L.down_proj.weight, g(p + "mlp.down_proj.weight"))
        _put(L.input_layernorm.weight, g(p + "input_layernorm.weight"))
        _put(L.post_attention_layernorm.weight, g(p + "post_attention_layernorm.weight"))
        _put(L.pre_feedforward_layernorm.weight, g(p + "pre_feedforward_layernorm.weight"))
        _put(L.post_feedforward_layernorm.weight, g(p + "post_feedforward_layernorm.weight"))
    _put(model.norm.weight, g("norm.weight"))


@torch.no_grad()
def export_gemma_state(model, prefix: str = "model.") -> dict:
    cfg = model.cfg
    f = lambda t: t.detach().float().cpu().contiguous()  # noqa: E731
    qd, kd = cfg.num_attention_heads * cfg.head_dim, cfg.num_key_value_heads * cfg.head_dim
    I = cfg.intermediate_size
    sd = {prefix + "embed_tokens.weight": f(model.embed[: cfg.vocab_size])}
    for i, L in enumerate(model.layers):
        p = f"{prefix}layers.{i}."
        w = L.qkv_proj.weight
        sd[p + "self_attn.q_proj.weight"] = f(w[:qd])
        sd[p + "self_attn.k_proj.weight"] = f(w[qd:qd + kd])
        sd[p + "self_attn.v_proj.weight"] = f(w[qd + kd:])
        sd[p + "self_attn.o_proj.weight"] = f(L.o_proj.weight)
        sd[p + "self_attn.q_norm.weight"] = f(L.q_norm.weight)
        sd[p + "self_attn.k_norm.weight"] = f(L.k_norm.weight)
        sd[p + "mlp.gate_proj.weight"] = f(L.gate_up_proj.weight[:I])
        sd[p + "mlp.up_proj.weight"] = f(L.gate_up_proj.weight[I:])
        sd[p + "mlp.down_proj.weight"] = f(L.down_proj.weight)
        for n in ("input_layernorm", "post_attention_layernorm", "pre_feedforward_layernorm",
                  "post_feedforward_layernorm"):
            sd[p + n + ".weight"] = f(getattr(L, n).weight)
    sd[prefix + "norm.weight"] = f(model.norm.weight)
    return sd
