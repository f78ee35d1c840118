"""Plain-PyTorch fp32 reference implementations of every fused op: the numerics oracle the HIP
kernels are tested against, and (through ``host_ops``) the host-tensor path of the GPU-less CI.
They mirror the semantics of the reference engine's ops where SURVEY §8 says we keep them, and
HF/PEFT semantics elsewhere."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def layer_norm(x, w, b, eps):
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)


def rms_norm(x, w, eps, offset):
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return xf * r * (w.float() + offset)


def gelu_tanh(x):
    return F.gelu(x.float(), approximate="tanh")


def gated(gu, act):
    g, u = gu.float().chunk(2, dim=-1)
    a = F.gelu(g, approximate="tanh") if act == 0 else F.silu(g)
    return a * u


def attention(q, k, v, scale, causal=True, window=0, kv_lens=None):
    """q [B,Sq,H,D], k/v [B,Sk,Hkv,D] -> o [B,Sq,H,D] (fp32), lse [B,H,Sq]."""
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    G = H // Hkv
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3).repeat_interleave(G, dim=1)
    vf = v.float().permute(0, 2, 1, 3).repeat_interleave(G, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    i = torch.arange(Sq, device=q.device)[:, None] + (Sk - Sq)
    j = torch.arange(Sk, device=q.device)[None, :]
    allowed = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device)
    if causal:
        allowed &= j <= i
    if window and window > 0:
        allowed &= (i - j) < window
    allowed = allowed[None, None].expand(B, H, Sq, Sk).clone()
    if kv_lens is not None:
        allowed &= (j[None, None] < kv_lens.view(B, 1, 1, 1).to(q.device))
    s = s.masked_fill(~allowed, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    o = torch.matmul(p, vf).permute(0, 2, 1, 3)
    return o, lse


from mobilefinetuner_amd.ops.rope_tables import rope_tables  # noqa: E402,F401  (model setup helper)


def rope(x, cos, sin, pos0=0, interleaved=False):
    """x [B,S,H,D]; rotate-half (HF) or interleaved pairs (reference compat)."""
    S, D = x.shape[1], x.shape[-1]
    c = cos[pos0:pos0 + S].view(1, S, 1, D // 2)
    s = sin[pos0:pos0 + S].view(1, S, 1, D // 2)
    xf = x.float()
    if interleaved:
        a, b = xf[..., 0::2], xf[..., 1::2]
        out = torch.empty_like(xf)
        out[..., 0::2] = a * c - b * s
        out[..., 1::2] = b * c + a * s
        return out
    a, b = xf[..., : D // 2], xf[..., D // 2:]
    return torch.cat([a * c - b * s, b * c + a * s], dim=-1)


def cross_entropy_rows(logits, labels, V):
    lf = logits[:, :V].float()
    lse = torch.logsumexp(lf, dim=-1)
    valid = (labels >= 0) & (labels < V)
    lab = labels.clamp(0, V - 1)
    tgt = lf.gather(1, lab[:, None]).squeeze(1)
    return torch.where(valid, lse - tgt, torch.zeros_like(lse))


def lm_cross_entropy(logits, labels, ignore_index=-100, reduction="mean"):
    """HF-style shifted LM loss (core/lm_loss.cpp:106-210): logits[:, :-1] vs labels[:, 1:]."""
    lg = logits[:, :-1].reshape(-1, logits.shape[-1]).float()
    lb = labels[:, 1:].reshape(-1)
    return F.cross_entropy(lg, lb, ignore_index=ignore_index, reduction=reduction)


def perplexity(loss):
    return math.exp(loss)


def adam_step(p, g, m, v, vhat, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
              decoupled=True, amsgrad=False):
    """One Adam(W) step in fp32, in place, the reference's formulas (operators/finetune_ops/optim/adam.cpp:
    56-87): bias-corrected moments and, with AMSGrad, v_hat = max(v_hat, v / bc2) used directly in the
    denominator (torch instead keeps the max of the RAW v and divides by the current bc2).  decoupled=False
    is the reference's coupled L2 (grad += wd * p); True is AdamW's decay p *= 1 - lr * wd.  step: the
    1-based index of this step."""
    if not decoupled and weight_decay:
        g = g + weight_decay * p
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1, bc2 = 1 - beta1 ** step, 1 - beta2 ** step
    vc = v / bc2
    if amsgrad:
        torch.maximum(vhat, vc, out=vhat)
        vc = vhat
    if decoupled and weight_decay:
        p.mul_(1 - lr * weight_decay)
    p.sub_(lr * (m / bc1) / (vc.sqrt() + eps))
    return p
