"""GPT-2 (small / medium / large / xl) on the fused gfx950 ops.

Reference: GPT2Model (operators/finetune_ops/graph/gpt2_model.h:77-186, gpt2_model.cpp:142-861),
GPT2Config (gpt2_model.h:50-66, config parsing gpt2_model.cpp:121-140).

Differences by design: Q/K/V are NOT split with memcpy — the packed c_attn output
[B,S,3,H,D] feeds the flash-attention kernel in place and its backward writes one packed dqkv
(Q2/Q3 fixed: attention-side LoRA gets real gradients); embeddings have a backward (Q5); the
residual add is fused into the following LayerNorm; the tied LM head + cross entropy is one fused,
vocab-chunked op that never materialises fp32 logits; the token table is padded to a multiple of
128 rows so logits rows are 16-B aligned (padded rows are zero and never trained).
"""
from __future__ import annotations

import json
import math
from dataclasses import asdict, dataclass

import torch
import torch.nn as nn

from ..ops import functional as Fx
from ..parallel.sharder import gate
from .layers import LayerNorm, Linear


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    layer_norm_epsilon: float = 1e-5
    tie_word_embeddings: bool = True
    initializer_range: float = 0.02

    @property
    def head_dim(self):
        return self.n_embd // self.n_head

    @property
    def vocab_padded(self):
        return (self.vocab_size + 127) // 128 * 128

    @classmethod
    def preset(cls, name: str) -> "GPT2Config":
        name = name.lower().replace("_", "-")
        table = {
            "gpt2": dict(n_embd=768, n_layer=12, n_head=12),
            "gpt2-small": dict(n_embd=768, n_layer=12, n_head=12),
            "gpt2-124m": dict(n_embd=768, n_layer=12, n_head=12),
            "gpt2-medium": dict(n_embd=1024, n_layer=24, n_head=16),
            "gpt2-large": dict(n_embd=1280, n_layer=36, n_head=20),
            "gpt2-xl": dict(n_embd=1600, n_layer=48, n_head=25),
            "gpt2-tiny": dict(n_embd=128, n_layer=2, n_head=2, vocab_size=1000, n_positions=256),
        }
        if name not in table:
            raise ValueError(f"unknown GPT-2 preset {name!r}; choose from {sorted(table)}")
        return cls(**table[name])

    @classmethod
    def from_json(cls, path: str) -> "GPT2Config":
        with open(path) as f:
            d = json.load(f)
        c = cls()
        c.vocab_size = d.get("vocab_size", c.vocab_size)
        c.n_positions = d.get("n_positions", d.get("n_ctx", c.n_positions))
        c.n_embd = d.get("n_embd", c.n_embd)
        c.n_layer = d.get("n_layer", c.n_layer)
        c.n_head = d.get("n_head", c.n_head)
        c.layer_norm_epsilon = d.get("layer_norm_epsilon", c.layer_norm_epsilon)
        c.tie_word_embeddings = d.get("tie_word_embeddings", True)
        c.initializer_range = d.get("initializer_range", c.initializer_range)
        return c

    def to_dict(self):
        return asdict(self)


class GPT2Block(nn.Module):
    def __init__(self, cfg: GPT2Config, dtype, device):
        super().__init__()
        C = cfg.n_embd
        self.ln_1 = LayerNorm(C, cfg.layer_norm_epsilon, device)
        self.c_attn = Linear(C, 3 * C, True, dtype, device)
        self.c_proj = Linear(C, C, True, dtype, device)
        self.ln_2 = LayerNorm(C, cfg.layer_norm_epsilon, device)
        self.c_fc = Linear(C, 4 * C, True, dtype, device)
        self.mlp_proj = Linear(4 * C, C, True, dtype, device)
        self.H, self.D = cfg.n_head, cfg.head_dim
        # norms write straight into their consumer's augmented LoRA input when it has one
        self.ln_1.set_consumer(self.c_attn)
        self.ln_2.set_consumer(self.c_fc)

    def attn(self, h, B, S, kv_lens):
        qkv = self.c_attn(h).view(B, S, 3, self.H, self.D)
        # c_proj with an active LoRA adapter takes the attention output widened to its augmented-K
        # input (Linear.aug_cols); the attention kernel writes O straight into that buffer.
        o = Fx.flash_attention_qkvpacked(qkv, 1.0 / math.sqrt(self.D), True, 0, kv_lens, self.c_proj.aug_cols())
        return self.c_proj(o.reshape(B * S, o.shape[-1] if o.dim() == 3 else self.H * self.D))

    def mlp(self, h):
        return Fx.mlp_gelu(h, self.c_fc, self.mlp_proj)


class GPT2Model(nn.Module):
    """forward(input_ids[B,S], labels[B,S] shifted targets) -> mean loss; or final hidden."""

    def __init__(self, cfg: GPT2Config, dtype=torch.bfloat16, device="cuda", init: bool = True, seed: int = 0):
        super().__init__()
        self.cfg = cfg
        self.dtype = dtype
        C = cfg.n_embd
        self.wte = nn.Parameter(torch.zeros(cfg.vocab_padded, C, dtype=dtype, device=device), requires_grad=False)
        self.wpe = nn.Parameter(torch.zeros(cfg.n_positions, C, dtype=dtype, device=device), requires_grad=False)
        self.wte._mft_tied = True  # embedding + LM head (ops.functional grad_ready ordering)
        self.blocks = nn.ModuleList([GPT2Block(cfg, dtype, device) for _ in range(cfg.n_layer)])
        self.ln_f = LayerNorm(C, cfg.layer_norm_epsilon, device)
        self.activation_checkpointing = False
        if init:
            self.init_weights(seed)

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """HF GPT-2 init: N(0, 0.02), residual projections N(0, 0.02/sqrt(2L)), zero biases."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        std = self.cfg.initializer_range

        def nrm(p, s):
            p.data.copy_((torch.randn(p.shape, generator=g) * s).to(p.dtype))

        nrm(self.wte, std)
        self.wte.data[self.cfg.vocab_size:].zero_()
        nrm(self.wpe, 0.01)
        proj_std = std / math.sqrt(2 * self.cfg.n_layer)
        for b in self.blocks:
            nrm(b.c_attn.weight, std)
            nrm(b.c_fc.weight, std)
            nrm(b.c_proj.weight, proj_std)
            nrm(b.mlp_proj.weight, proj_std)

    def linear_modules(self):
        """name -> Linear (HF-style names, used by LoRA injection and checkpoint IO)."""
        out = {}
        for i, b in enumerate(self.blocks):
            out[f"h.{i}.attn.c_attn"] = b.c_attn
            out[f"h.{i}.attn.c_proj"] = b.c_proj
            out[f"h.{i}.mlp.c_fc"] = b.c_fc
            out[f"h.{i}.mlp.c_proj"] = b.mlp_proj
        return out

    def hidden(self, input_ids, kv_lens=None):
        B, S = input_ids.shape
        assert S <= self.cfg.n_positions, f"sequence {S} exceeds n_positions {self.cfg.n_positions}"
        sh = getattr(self, "sharder", None)
        z3 = getattr(self, "zero3", None)  # parallel/zero3.py: per-block gather / reduce-scatter
        if sh is not None:
            sh.require("embed")
        if z3 is not None:
            z3.begin_forward()
        x = Fx.embedding(input_ids, self.wte, self.wpe)  # [B*S, C]
        h = self.blocks[0].ln_1(x)
        n = len(self.blocks)
        for i, blk in enumerate(self.blocks):
            nxt = self.blocks[i + 1].ln_1 if i + 1 < n else self.ln_f
            if sh is not None:
                sh.require(f"block{i}")
            if z3 is not None:
                x, h = z3.pre_block(i, x, h)
            if self.activation_checkpointing and self.training and torch.is_grad_enabled():
                x, h = torch.utils.checkpoint.checkpoint(self._block, blk, nxt, x, h, B, S, kv_lens,
                                                         use_reentrant=False)
            else:
                x, h = self._block(blk, nxt, x, h, B, S, kv_lens)
            if z3 is not None:
                x, h = z3.post_block(i, x, h)
            if sh is not None:  # backward re-fetches this block's weights before its dgrad
                x, h = gate(x, sh, f"block{i}"), gate(h, sh, f"block{i}")
        if sh is not None:
            sh.require("embed")  # tied LM head
        return h  # = ln_f(x) [B*S, C]

    @staticmethod
    def _block(blk, nxt, x, h, B, S, kv_lens):
        a = blk.attn(h, B, S, kv_lens)
        x, h = blk.ln_2.add_forward(x, a)
        f = blk.mlp(h)
        return nxt.add_forward(x, f)

    def forward(self, input_ids, labels=None, kv_lens=None, loss_scale=1.0):
        h = self.hidden(input_ids, kv_lens)
        if labels is None:
            return h
        return Fx.lm_head_cross_entropy(h, self.wte, labels.reshape(-1), self.cfg.vocab_size,
                                        w_grad_scale=loss_scale)

    def logits(self, input_ids, kv_lens=None):
        h = self.hidden(input_ids, kv_lens)
        w = Fx.cw(self.wte)
        return (h @ w.t())[:, : self.cfg.vocab_size].view(*input_ids.shape, -1)

    def nll(self, input_ids, labels, kv_lens=None):
        """(sum NLL, #tokens) over shifted labels — token-weighted eval."""
        h = self.hidden(input_ids, kv_lens)
        return Fx.lm_head_token_nll(h, self.wte, labels.reshape(-1), self.cfg.vocab_size)

    def num_parameters(self, trainable_only=False):
        ps = [p for p in self.parameters() if (p.requires_grad or not trainable_only)]
        n = sum(p.numel() for p in ps)
        if not trainable_only:
            n -= (self.cfg.vocab_padded - self.cfg.vocab_size) * self.cfg.n_embd
        return n

    def set_full_finetune(self):
        for p in self.parameters():
            p.requires_grad_(True)
