"""Host (CPU, fp32) implementations of the public fused ops of ``mobilefinetuner_amd.ops.functional``
(same names / signatures), built on ``reference``.  Trainable parameters are used directly (autograd
fills their ``.grad``), frozen ones through their compute view."""
from __future__ import annotations

import math

import torch

from mobilefinetuner_amd.ops.functional import rw

from . import reference as ref


def layer_norm(x, w, b, eps=1e-5, out_cols=0):
    return ref.layer_norm(x, rw(w), rw(b), eps).to(x.dtype)


def add_layer_norm(x, delta, w, b, eps=1e-5, out_cols=0):
    s = x + delta
    return s, ref.layer_norm(s, rw(w), rw(b), eps).to(x.dtype)


def rms_norm(x, w, eps=1e-6, offset=1.0, out_cols=0):
    return ref.rms_norm(x, rw(w), eps, offset).to(x.dtype)


def add_rms_norm(x, delta, w, eps=1e-6, offset=1.0, out_cols=0):
    s = x + delta
    return s, ref.rms_norm(s, rw(w), eps, offset).to(x.dtype)


def gelu(x):
    return ref.gelu_tanh(x).to(x.dtype)


def gated_act(gu, act="gelu", out_cols=0):
    a = 0 if act in ("gelu", "gelu_tanh", "gelu_pytorch_tanh") else 1
    return ref.gated(gu, a).to(gu.dtype)


def embedding(ids, wte, wpe=None, scale=1.0):
    B, S = ids.shape
    e = rw(wte)[ids.reshape(-1)].float()
    if scale != 1.0:
        e = e * scale
    if wpe is not None:
        e = e + rw(wpe)[:S].float().repeat(B, 1)
    return e.to(rw(wte).dtype)


def flash_attention(q, k, v, scale=None, causal=True, window=0, kv_lens=None):
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    return ref.attention(q, k, v, scale, causal, window, kv_lens)[0].to(q.dtype).contiguous()


def flash_attention_qkvpacked(qkv, scale=None, causal=True, window=0, kv_lens=None, out_cols=0):
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    return ref.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], scale, causal, window,
                         kv_lens)[0].to(qkv.dtype).contiguous()


def qk_norm_rope(x, w, cos, sin, eps=1e-6, offset=1.0, interleaved=False):
    y = ref.rms_norm(x, rw(w), eps, offset).to(x.dtype)
    return ref.rope(y, cos, sin, 0, interleaved).to(x.dtype)


def qk_norm_rope_attention(qkv, nq, nkv, wq, wk, cos, sin, eps_q, eps_k, offset=1.0, interleaved=False, scale=None,
                           window=0, kv_lens=None, out_cols=0):
    D = qkv.shape[-1]
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    q = qk_norm_rope(qkv[:, :, :nq], wq, cos, sin, eps_q, offset, interleaved)
    k = qk_norm_rope(qkv[:, :, nq:nq + nkv], wk, cos, sin, eps_k, offset, interleaved)
    return flash_attention(q, k, qkv[:, :, nq + nkv:], scale, True, window, kv_lens)


def linear(x, w, b=None):
    y = x.float() @ rw(w).float().t()
    if b is not None:
        y = y + rw(b).float()
    return y.to(x.dtype)


def lora_linear(x, w, b, slices, scale, training: bool = True):
    xf = x.float()
    y = xf @ rw(w).float().t()
    if b is not None:
        y = y + rw(b).float()
    parts = []
    for sl in slices:
        c0, n, A, B = sl[:4]
        p = float(sl[4]) if len(sl) > 4 else 0.0
        if not (training and torch.is_grad_enabled()):
            p = 0.0
        xd = torch.nn.functional.dropout(xf, p) if p > 0 else xf
        parts.append((c0, n, scale * ((xd @ rw(A).float().t()) @ rw(B).float())))
    if parts:
        y = y.clone()
        for c0, n, d in parts:
            y[..., c0:c0 + n] = y[..., c0:c0 + n] + d
    return y.to(x.dtype)


def lm_head_cross_entropy(h, w, labels, vocab_size, chunk=None, w_grad_scale=1.0):
    logits = (h.float() @ rw(w).float().t())[:, :vocab_size]
    return torch.nn.functional.cross_entropy(logits, labels.reshape(-1), ignore_index=-100)


def lm_head_token_nll(h, w, labels, vocab_size, chunk=None):
    with torch.no_grad():
        logits = (h.float() @ rw(w).float().t())[:, :vocab_size]
        nll = torch.nn.functional.cross_entropy(logits, labels.reshape(-1), ignore_index=-100, reduction="sum")
        return nll, (labels >= 0).sum()
