"""Gemma-3 text models (270M / 1B) on the fused gfx950 ops.

Reference: GemmaTextConfig / GemmaModel (operators/finetune_ops/graph/gemma_model.h:17-178,
gemma_model.cpp:138-944): embedding x sqrt(H); per layer RMSNorm(1+w) -> attention (q/k/v, q_norm /
k_norm over head_dim, RoPE with theta 1e6 on global / 1e4 on local layers, GQA, scale
query_pre_attn_scalar^-1/2, causal or sliding-window mask) -> post-attn norm -> residual ->
pre-ffn norm -> GeGLU MLP -> post-ffn norm -> residual; final norm; LM head tied to the embedding.

MI355X design: q|k|v and gate|up are single fused GEMMs; q_norm/k_norm + RoPE is one fused kernel
reading the packed projection in place (rotate-half, HF layout; the reference's interleaved RoPE,
SURVEY §8 Q9, is available with ``interleaved_rope=True``); GQA (4:1 for 270M/1B) is handled inside
the flash-attention kernel without materialising repeated K/V (reference core/ops.cpp:2072-2149);
the LM head reuses the (padded) embedding with the fused chunked CE — no transposed 671 MB copy
(Q10).
"""
from __future__ import annotations

import json
import math
from dataclasses import asdict, dataclass, field

import torch
import torch.nn as nn

from ..ops import functional as Fx
from ..ops.rope_tables import rope_tables
from ..parallel.sharder import gate
from .layers import Linear, RMSNorm


def _pattern_layer_types(n_layers: int, pattern: int = 6):
    return ["full_attention" if (i + 1) % pattern == 0 else "sliding_attention" for i in range(n_layers)]


@dataclass
class Gemma3Config:
    vocab_size: int = 262144
    hidden_size: int = 640
    intermediate_size: int = 2048
    num_hidden_layers: int = 18
    num_attention_heads: int = 4
    num_key_value_heads: int = 1
    head_dim: int = 256
    rms_norm_eps: float = 1e-6
    rope_theta: float = 1_000_000.0
    rope_local_base_freq: float = 10_000.0
    rope_scaling_factor: float = 1.0      # linear scaling on global layers
    sliding_window: int = 512
    query_pre_attn_scalar: float = 256.0
    max_position_embeddings: int = 32768
    hidden_activation: str = "gelu_pytorch_tanh"
    layer_types: list = field(default_factory=list)
    tie_word_embeddings: bool = True
    initializer_range: float = 0.02
    bos_token_id: int = 2
    eos_token_id: int = 1
    pad_token_id: int = 0

    def __post_init__(self):
        if not self.layer_types:
            self.layer_types = _pattern_layer_types(self.num_hidden_layers)

    @property
    def vocab_padded(self):
        return (self.vocab_size + 127) // 128 * 128

    @classmethod
    def preset(cls, name: str) -> "Gemma3Config":
        name = name.lower().replace("_", "-")
        table = {
            "gemma3-270m": dict(hidden_size=640, intermediate_size=2048, num_hidden_layers=18,
                                num_attention_heads=4, num_key_value_heads=1),
            "gemma3-1b": dict(hidden_size=1152, intermediate_size=6912, num_hidden_layers=26,
                              num_attention_heads=4, num_key_value_heads=1),
            "gemma3-tiny": dict(vocab_size=1024, hidden_size=128, intermediate_size=256, num_hidden_layers=3,
                                num_attention_heads=4, num_key_value_heads=2, head_dim=64, sliding_window=16,
                                max_position_embeddings=512, query_pre_attn_scalar=64.0,
                                layer_types=["sliding_attention", "sliding_attention", "full_attention"]),
        }
        for alias, key in (("gemma-3-270m", "gemma3-270m"), ("gemma-3-1b", "gemma3-1b"), ("gemma3", "gemma3-270m")):
            table[alias] = table[key]
        if name not in table:
            raise ValueError(f"unknown Gemma-3 preset {name!r}; choose from {sorted(table)}")
        return cls(**table[name])

    @classmethod
    def from_dict(cls, d: dict) -> "Gemma3Config":
        d = dict(d.get("text_config", d))
        c = cls(layer_types=list(d.get("layer_types") or []),
                num_hidden_layers=d.get("num_hidden_layers", 18))
        for k in ("vocab_size", "hidden_size", "intermediate_size", "num_attention_heads", "num_key_value_heads",
                  "head_dim", "rms_norm_eps", "sliding_window", "query_pre_attn_scalar", "max_position_embeddings",
                  "hidden_activation", "tie_word_embeddings", "initializer_range", "bos_token_id", "eos_token_id",
                  "pad_token_id"):
            if d.get(k) is not None:
                setattr(c, k, d[k])
        if d.get("rope_theta") is not None:
            c.rope_theta = float(d["rope_theta"])
        if d.get("rope_local_base_freq") is not None:
            c.rope_local_base_freq = float(d["rope_local_base_freq"])
        rs = d.get("rope_scaling")
        if isinstance(rs, dict) and rs.get("rope_type", rs.get("type")) == "linear":
            c.rope_scaling_factor = float(rs.get("factor", 1.0))
        rp = d.get("rope_parameters")  # transformers >= 5 layout
        if isinstance(rp, dict):
            if "full_attention" in rp:
                full = rp["full_attention"]
                c.rope_theta = float(full.get("rope_theta", c.rope_theta))
                if full.get("rope_type") == "linear":
                    c.rope_scaling_factor = float(full.get("factor", 1.0))
            if "sliding_attention" in rp:
                c.rope_local_base_freq = float(rp["sliding_attention"].get("rope_theta", c.rope_local_base_freq))
        if not c.layer_types or len(c.layer_types) != c.num_hidden_layers:
            c.layer_types = _pattern_layer_types(c.num_hidden_layers, d.get("sliding_window_pattern", 6))
        return c

    @classmethod
    def from_json(cls, path: str) -> "Gemma3Config":
        with open(path) as f:
            return cls.from_dict(json.load(f))

    def to_dict(self):
        return asdict(self)


class Gemma3Layer(nn.Module):
    def __init__(self, cfg: Gemma3Config, idx: int, dtype, device):
        super().__init__()
        H, D = cfg.hidden_size, cfg.head_dim
        self.nq, self.nkv, self.D = cfg.num_attention_heads, cfg.num_key_value_heads, D
        self.sliding = cfg.layer_types[idx] == "sliding_attention"
        self.window = cfg.sliding_window if self.sliding else 0
        self.scale = cfg.query_pre_attn_scalar ** -0.5
        eps = cfg.rms_norm_eps
        self.input_layernorm = RMSNorm(H, eps, 1.0, device)
        self.qkv_proj = Linear(H, (self.nq + 2 * self.nkv) * D, False, dtype, device)
        self.o_proj = Linear(self.nq * D, H, False, dtype, device)
        self.q_norm = RMSNorm(D, eps, 1.0, device)
        self.k_norm = RMSNorm(D, eps, 1.0, device)
        self.post_attention_layernorm = RMSNorm(H, eps, 1.0, device)
        self.pre_feedforward_layernorm = RMSNorm(H, eps, 1.0, device)
        self.gate_up_proj = Linear(H, 2 * cfg.intermediate_size, False, dtype, device)
        self.down_proj = Linear(cfg.intermediate_size, H, False, dtype, device)
        self.post_feedforward_layernorm = RMSNorm(H, eps, 1.0, device)
        self.input_layernorm.set_consumer(self.qkv_proj)
        self.pre_feedforward_layernorm.set_consumer(self.gate_up_proj)
        self.act = cfg.hidden_activation
        self.interleaved_rope = False

    def attn(self, h, B, S, cos, sin, kv_lens):
        qkv = self.qkv_proj(h).view(B, S, self.nq + 2 * self.nkv, self.D)
        # O goes straight into o_proj's augmented-K input when it carries a LoRA adapter
        o = Fx.qk_norm_rope_attention(qkv, self.nq, self.nkv, self.q_norm.weight, self.k_norm.weight, cos, sin,
                                      self.q_norm.eps, self.k_norm.eps, 1.0, self.interleaved_rope, self.scale,
                                      self.window, kv_lens, self.o_proj.aug_cols())
        return self.o_proj(o.view(B * S, -1))

    def mlp(self, h):
        return self.down_proj(Fx.gated_act(self.gate_up_proj(h), self.act, self.down_proj.aug_cols()))


class Gemma3Model(nn.Module):
    def __init__(self, cfg: Gemma3Config, dtype=torch.bfloat16, device="cuda", init: bool = True, seed: int = 0,
                 rope_len: int | None = None):
        super().__init__()
        self.cfg, self.dtype = cfg, dtype
        self.embed = nn.Parameter(torch.zeros(cfg.vocab_padded, cfg.hidden_size, dtype=dtype, device=device),
                                  requires_grad=False)
        self.embed._mft_tied = True  # embedding + LM head (ops.functional grad_ready ordering)
        self.layers = nn.ModuleList([Gemma3Layer(cfg, i, dtype, device) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, 1.0, device)
        s = math.sqrt(cfg.hidden_size)
        self.embed_scale = float(torch.tensor(s, dtype=dtype).float()) if dtype != torch.float32 else s
        self._rope = {}
        self._rope_len = rope_len or min(cfg.max_position_embeddings, 4096)
        self.activation_checkpointing = False
        if init:
            self.init_weights(seed)

    def rope(self, kind: str, S: int, device):
        n = max(S, self._rope_len)
        key = (kind, str(device))
        t = self._rope.get(key)
        if t is None or t[0].shape[0] < S:
            if kind == "global":
                t = rope_tables(n, self.cfg.head_dim, self.cfg.rope_theta, device, self.cfg.rope_scaling_factor)
            else:
                t = rope_tables(n, self.cfg.head_dim, self.cfg.rope_local_base_freq, device)
            self._rope[key] = t
        return t

    def set_interleaved_rope(self, flag: bool):
        for L in self.layers:
            L.interleaved_rope = flag

    @torch.no_grad()
    def init_weights(self, seed=0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        std = self.cfg.initializer_range
        for n, p in self.named_parameters():
            if p.dim() == 2:
                p.data.copy_((torch.randn(p.shape, generator=g) * std).to(p.dtype))
        self.embed.data[self.cfg.vocab_size:].zero_()

    def linear_modules(self):
        out = {}
        for i, L in enumerate(self.layers):
            out[f"layers.{i}.self_attn.qkv_proj"] = L.qkv_proj
            out[f"layers.{i}.self_attn.o_proj"] = L.o_proj
            out[f"layers.{i}.mlp.gate_up_proj"] = L.gate_up_proj
            out[f"layers.{i}.mlp.down_proj"] = L.down_proj
        return out

    def hidden(self, input_ids, kv_lens=None):
        B, S = input_ids.shape
        dev = input_ids.device
        gcos, gsin = self.rope("global", S, dev)
        lcos, lsin = self.rope("local", S, dev)
        sh = getattr(self, "sharder", None)
        z3 = getattr(self, "zero3", None)  # parallel/zero3.py: per-layer gather / reduce-scatter
        if sh is not None:
            sh.require("embed")
        if z3 is not None:
            z3.begin_forward()
        x = Fx.embedding(input_ids, self.embed, None, self.embed_scale)
        h = self.layers[0].input_layernorm(x)
        n = len(self.layers)
        for i, L in enumerate(self.layers):
            nxt = self.layers[i + 1].input_layernorm if i + 1 < n else self.norm
            cos, sin = (lcos, lsin) if L.sliding else (gcos, gsin)
            if sh is not None:
                sh.require(f"block{i}")
            if z3 is not None:
                x, h = z3.pre_block(i, x, h)
            if self.activation_checkpointing and self.training and torch.is_grad_enabled():
                x, h = torch.utils.checkpoint.checkpoint(self._layer, L, nxt, x, h, B, S, cos, sin, kv_lens,
                                                         use_reentrant=False)
            else:
                x, h = self._layer(L, nxt, x, h, B, S, cos, sin, kv_lens)
            if z3 is not None:
                x, h = z3.post_block(i, x, h)
            if sh is not None:
                x, h = gate(x, sh, f"block{i}"), gate(h, sh, f"block{i}")
        if sh is not None:
            sh.require("embed")
        return h

    @staticmethod
    def _layer(L, nxt, x, h, B, S, cos, sin, kv_lens):
        a = L.post_attention_layernorm(L.attn(h, B, S, cos, sin, kv_lens))
        x, h = L.pre_feedforward_layernorm.add_forward(x, a)
        f = L.post_feedforward_layernorm(L.mlp(h))
        return nxt.add_forward(x, f)

    def forward(self, input_ids, labels=None, kv_lens=None, loss_scale=1.0):
        h = self.hidden(input_ids, kv_lens)
        if labels is None:
            return h
        return Fx.lm_head_cross_entropy(h, self.embed, labels.reshape(-1), self.cfg.vocab_size,
                                        w_grad_scale=loss_scale)

    def logits(self, input_ids, kv_lens=None):
        h = self.hidden(input_ids, kv_lens)
        w = Fx.cw(self.embed)
        return (h @ w.t())[:, : self.cfg.vocab_size].view(*input_ids.shape, -1)

    def nll(self, input_ids, labels, kv_lens=None):
        h = self.hidden(input_ids, kv_lens)
        return Fx.lm_head_token_nll(h, self.embed, labels.reshape(-1), self.cfg.vocab_size)

    def num_parameters(self, trainable_only=False):
        ps = [p for p in self.parameters() if (p.requires_grad or not trainable_only)]
        n = sum(p.numel() for p in ps)
        if not trainable_only:
            n -= (self.cfg.vocab_padded - self.cfg.vocab_size) * self.cfg.hidden_size
        return n

    def set_full_finetune(self):
        for p in self.parameters():
            p.requires_grad_(True)
