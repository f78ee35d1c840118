"""Autograd-aware fused ops -- ONE device path: the gfx950 HIP kernels of ``_C`` (no silent
fallback: a missing extension raises).

CPU tensors are not a second backend of this layer.  Every public op is wrapped by
``_device_op``: a call on host tensors is routed to an externally installed host implementation
(``install_host_ops``) or raises.  The only such implementation is the fp32 PyTorch oracle of the
test-suite (``tests/oracle``), installed by ``tests/conftest.py`` / ``MFT_HOST_ORACLE`` for the
GPU-less CI tests (HF parity, gloo data-parallel, CLI smoke runs).

Gradient convention (replaces the reference's overwrite-on-backward): every trainable
parameter's ``.grad`` is a persistent view into a flat fp32 grad buffer (see
``utils/params.py``).  The GPU backward kernels ACCUMULATE straight into ``p.grad`` and return
``None`` for that input; if a parameter has no grad buffer yet a fresh gradient is returned and
autograd's AccumulateGrad adds it.  Each accumulation calls ``grad_ready(p)`` so data-parallel
engines can launch bucket all-reduces while backward is still running.
"""
from __future__ import annotations

import functools
import math
import os

import torch
from torch.autograd import Function

from .._ext import native

GEMM_EPI_NONE, GEMM_EPI_BIAS, GEMM_EPI_BIAS_GELU, GEMM_EPI_DGELU, GEMM_EPI_F32ACC, GEMM_EPI_LORA = 0, 1, 2, 3, 4, 5
GEMM_EPI_BIAS_GELU_D, GEMM_EPI_MUL_AUX = 9, 10

# ---------------------------------------------------------------- host tensors (test oracle only)
_HOST_OPS = [None]


def install_host_ops(mod):
    """Route public ops called on CPU tensors to ``mod`` (functions of the same names and
    signatures).  Only the test-suite's fp32 oracle (tests/oracle) does this."""
    _HOST_OPS[0] = mod


def _load_env_oracle():
    path = os.environ.get("MFT_HOST_ORACLE", "")
    if not path or _HOST_OPS[0] is not None:
        return
    import importlib.util
    import sys
    init = os.path.join(path, "__init__.py")
    spec = importlib.util.spec_from_file_location("mft_host_oracle", init, submodule_search_locations=[path])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["mft_host_oracle"] = mod
    spec.loader.exec_module(mod)
    install_host_ops(mod.host_ops)


def _device_op(fn):
    name = fn.__name__

    @functools.wraps(fn)
    def op(*args, **kwargs):
        t = next((a for a in args if isinstance(a, torch.Tensor)), None)
        if t is not None and not t.is_cuda:
            if _HOST_OPS[0] is None:
                _load_env_oracle()
            if _HOST_OPS[0] is None:
                raise RuntimeError(f"mobilefinetuner_amd.ops.{name}: the fused ops run on the GPU (gfx950 HIP "
                                   f"kernels); host tensors need the test-suite oracle (tests/oracle, "
                                   f"MFT_HOST_ORACLE=<repo>/tests/oracle)")
            return getattr(_HOST_OPS[0], name)(*args, **kwargs)
        return fn(*args, **kwargs)

    return op


# ---------------------------------------------------------------- parameter helpers

_ready_hooks: list = []


def register_grad_ready_hook(fn):
    _ready_hooks.append(fn)
    return fn


def remove_grad_ready_hook(fn):
    if fn in _ready_hooks:
        _ready_hooks.remove(fn)


def grad_ready(p):
    for h in _ready_hooks:
        h(p)


def cw(p):
    """Compute view of a parameter: its bf16 shadow if it has one, else the tensor itself."""
    if p is None:
        return None
    return getattr(p, "shadow", None) if getattr(p, "shadow", None) is not None else p


def rw(p):
    """Weight view for the host oracle (tests/oracle): the autograd-tracked parameter itself when trainable
    (so AccumulateGrad fills p.grad), else its compute view."""
    if p is None:
        return None
    return p if p.requires_grad else cw(p)


def _needs(p):
    return p is not None and p.requires_grad


def _sink(p, g):
    """Accumulate fp32 gradient g into p.grad; returns what backward must return for p."""
    if not _needs(p):
        return None
    if p.grad is not None:
        p.grad.add_(g.view_as(p.grad).to(p.grad.dtype))
        grad_ready(p)
        return None
    return g.to(p.dtype).view_as(p)


def _grad_buf(p):
    """fp32 buffer the kernels accumulate into directly (p.grad), or None."""
    if _needs(p) and p.grad is not None and p.grad.dtype == torch.float32 and p.grad.is_contiguous():
        return p.grad
    return None


# ---------------------------------------------------------------- normalisation
class _Norm(Function):
    @staticmethod
    def forward(ctx, x, delta, w, b, eps, rms, offset, out_cols):
        C = native()
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        d2 = delta.reshape(-1, shape[-1]).contiguous() if delta is not None else None
        wc = cw(w).float() if cw(w).dtype != torch.float32 else cw(w)
        if rms:
            y, s, rstd = C.rmsnorm_fwd(x2, d2, wc, eps, offset, out_cols)
            mean = None
        else:
            bc = cw(b).float() if cw(b).dtype != torch.float32 else cw(b)
            y, s, mean, rstd = C.layernorm_fwd(x2, d2, wc, bc, eps, out_cols)
        xs = s if d2 is not None else x2
        ctx.save_for_backward(xs, wc, mean if mean is not None else rstd, rstd)
        ctx.params = (w, b)
        ctx.rms, ctx.offset, ctx.has_delta, ctx.shape = rms, offset, d2 is not None, shape
        yshape = (*shape[:-1], y.shape[-1])  # wider than x when out_cols > N (appended columns)
        if d2 is not None:
            return s.view(shape), y.view(yshape)
        return y.view(yshape)

    @staticmethod
    def backward(ctx, *grads):
        C = native()
        xs, wc, mean, rstd = ctx.saved_tensors
        w, b = ctx.params
        N = ctx.shape[-1]
        if ctx.has_delta:
            ds, dy = grads
        else:
            ds, dy = None, grads[0]
        if dy is not None:
            dy2 = dy.reshape(-1, dy.shape[-1])
            if dy2.stride(-1) != 1 or dy2.stride(0) % 8:
                dy2 = dy2.contiguous()
        else:
            dy2 = torch.zeros_like(xs)
        if ds is not None and dy is None:
            dy2 = torch.zeros_like(xs)
        ds2 = ds.reshape(-1, N).contiguous() if ds is not None else None
        dwb = _grad_buf(w)
        tmp_w = torch.zeros(N, device=xs.device, dtype=torch.float32) if (_needs(w) and dwb is None) else None
        dw_t = dwb if dwb is not None else tmp_w
        if ctx.rms:
            dx = C.rmsnorm_bwd(xs, dy2, wc, rstd, ds2, ctx.offset, dw_t)
            gb = None
        else:
            dbb = _grad_buf(b)
            tmp_b = torch.zeros(N, device=xs.device, dtype=torch.float32) if (_needs(b) and dbb is None) else None
            db_t = dbb if dbb is not None else tmp_b
            dx = C.layernorm_bwd(xs, dy2, wc, mean, rstd, ds2, dw_t, db_t)
            gb = tmp_b if tmp_b is not None else None
            if dbb is not None:
                grad_ready(b)
        gw = tmp_w if tmp_w is not None else None
        if dwb is not None:
            grad_ready(w)
        dx = dx.view(ctx.shape)
        gwr = gw.to(w.dtype).view_as(w) if gw is not None else None
        gbr = gb.to(b.dtype).view_as(b) if gb is not None else None
        return dx, (dx if ctx.has_delta else None), gwr, gbr, None, None, None, None


# out_cols > width: the GPU output is allocated [.., out_cols] with the normalised values in the first
# `width` columns and the rest left for the consumer (a LoRA Linear appends its rank-r projections
# there, _LoRALinearAug).  CPU paths ignore it.
@_device_op
def layer_norm(x, w, b, eps=1e-5, out_cols=0):
    return _Norm.apply(x, None, w, b, eps, False, 0.0, int(out_cols))


@_device_op
def add_layer_norm(x, delta, w, b, eps=1e-5, out_cols=0):
    """s = x + delta; y = LayerNorm(s)  -> (s, y) (fused residual + norm)."""
    return _Norm.apply(x, delta, w, b, eps, False, 0.0, int(out_cols))


@_device_op
def rms_norm(x, w, eps=1e-6, offset=1.0, out_cols=0):
    return _Norm.apply(x, None, w, None, eps, True, offset, int(out_cols))


@_device_op
def add_rms_norm(x, delta, w, eps=1e-6, offset=1.0, out_cols=0):
    return _Norm.apply(x, delta, w, None, eps, True, offset, int(out_cols))


# ---------------------------------------------------------------- activations
class _Gelu(Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        ctx.save_for_backward(x)
        return native().gelu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return native().gelu_bwd(x, dy.contiguous())


class _Gated(Function):
    @staticmethod
    def forward(ctx, gu, act, out_cols):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        ctx.act = act
        return native().gated_fwd(gu, act, out_cols)

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        if dy.dim() != 2 or dy.stride(-1) != 1:
            dy = dy.contiguous()
        return native().gated_bwd(gu, dy, ctx.act), None, None


@_device_op
def gelu(x):
    return _Gelu.apply(x)


@_device_op
def gated_act(gu, act="gelu", out_cols=0):
    """gelu_tanh(gate) * up (GeGLU, Gemma) or silu(gate) * up (SwiGLU); gu = [gate | up].
    out_cols > I (GPU): returns [M, out_cols] with the activation in the first I columns and zeros
    after, the augmented-K input of a LoRA consumer (Linear.aug_cols)."""
    a = 0 if act in ("gelu", "gelu_tanh", "gelu_pytorch_tanh") else 1
    I = gu.shape[-1] // 2
    oc = int(out_cols) if out_cols and out_cols > I else 0
    if oc:
        gu = gu.reshape(-1, 2 * I)
    return _Gated.apply(gu, a, oc)


# ---------------------------------------------------------------- embedding
class _Embedding(Function):
    @staticmethod
    def forward(ctx, ids, wte, wpe, S, scale):
        ids = ids.reshape(-1).contiguous()
        out = native().embed_fwd(ids, cw(wte), cw(wpe) if wpe is not None else None, S, 0, scale)
        ctx.save_for_backward(ids)
        ctx.params = (wte, wpe)
        ctx.S, ctx.scale = S, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        (ids,) = ctx.saved_tensors
        wte, wpe = ctx.params
        dout = dout.contiguous()
        gte = gpe = None
        if _needs(wte) or _needs(wpe):
            bte = _grad_buf(wte)
            bpe = _grad_buf(wpe)
            tte = torch.zeros(wte.shape, device=dout.device) if (_needs(wte) and bte is None) else None
            tpe = torch.zeros(wpe.shape, device=dout.device) if (_needs(wpe) and bpe is None) else None
            native().embed_bwd(ids, dout, bte if bte is not None else tte, bpe if bpe is not None else tpe, ctx.S, 0,
                               ctx.scale)
            if bte is not None:
                grad_ready(wte)
            if bpe is not None:
                grad_ready(wpe)
            gte = tte.to(wte.dtype) if tte is not None else None
            gpe = tpe.to(wpe.dtype) if tpe is not None else None
        return None, gte, gpe, None, None


@_device_op
def embedding(ids, wte, wpe=None, scale=1.0):
    """ids [B,S] -> [B*S, C]: wte[ids]*scale (+ wpe[pos])."""
    B, S = ids.shape
    return _Embedding.apply(ids, wte, wpe, S, float(scale))


# ---------------------------------------------------------------- attention
class _FlashAttn(Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal, window, kv_lens):
        o, lse, _ = native().attn_fwd(q, k, v, scale, causal, window, kv_lens, 0)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.cfg = (scale, causal, window, kv_lens)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        scale, causal, window, kv_lens = ctx.cfg
        dq = torch.empty(q.shape, device=q.device, dtype=q.dtype)
        dk = torch.empty(k.shape, device=k.device, dtype=k.dtype)
        dv = torch.empty(v.shape, device=v.device, dtype=v.dtype)
        native().attn_bwd(q, k, v, o, do.contiguous(), lse, dq, dk, dv, scale, causal, window, kv_lens)
        return dq, dk, dv, None, None, None, None


class _FlashAttnPacked(Function):
    """qkv [B,S,3,H,D] packed GEMM output consumed in place; backward writes one packed dqkv."""

    @staticmethod
    def forward(ctx, qkv, scale, causal, window, kv_lens, out_cols):
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        o_full, lse, o = native().attn_fwd(q, k, v, scale, causal, window, kv_lens, out_cols)
        ctx.save_for_backward(qkv, o, lse)
        ctx.cfg = (scale, causal, window, kv_lens)
        ctx.wide = out_cols > 0 and o_full.dim() == 3
        return o_full

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        scale, causal, window, kv_lens = ctx.cfg
        dqkv = torch.empty_like(qkv)
        B, S, _, H, D = qkv.shape
        if ctx.wide:  # [B, S, out_cols] gradient of the widened output: O's columns come first
            do = do[..., :H * D].view(B, S, H, D)
        if do.stride(-1) != 1:
            do = do.contiguous()
        native().attn_bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], o, do, lse, dqkv[:, :, 0],
                          dqkv[:, :, 1], dqkv[:, :, 2], scale, causal, window, kv_lens)
        return dqkv, None, None, None, None, None


@_device_op
def flash_attention(q, k, v, scale=None, causal=True, window=0, kv_lens=None):
    """q [B,Sq,H,D], k/v [B,Sk,Hkv,D] (strided views OK) -> o [B,Sq,H,D]."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    return _FlashAttn.apply(q, k, v, float(scale), bool(causal), int(window or 0), kv_lens)


@_device_op
def flash_attention_qkvpacked(qkv, scale=None, causal=True, window=0, kv_lens=None, out_cols=0):
    """qkv [B,S,3,H,D] -> o [B,S,H,D]; with out_cols > H*D (GPU) -> [B,S,out_cols] whose first H*D
    columns hold O (room for the consumer's appended LoRA columns, _LoRALinearAug)."""
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    H, D = qkv.shape[3], qkv.shape[4]
    oc = int(out_cols) if out_cols and out_cols > H * D else 0
    return _FlashAttnPacked.apply(qkv, float(scale), bool(causal), int(window or 0), kv_lens, oc)


# ---------------------------------------------------------------- fused per-head RMSNorm + RoPE
class _QKNormRoPE(Function):
    @staticmethod
    def forward(ctx, x, w, cos, sin, eps, offset, interleaved):
        wc = cw(w)
        y, rstd = native().qknorm_rope_fwd(x, wc, cos, sin, 0, eps, offset, interleaved)
        ctx.save_for_backward(x, rstd, wc, cos, sin)
        ctx.w = w
        ctx.cfg = (offset, interleaved)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, rstd, wc, cos, sin = ctx.saved_tensors
        w = ctx.w
        offset, interleaved = ctx.cfg
        dx = torch.empty(x.shape, device=x.device, dtype=x.dtype)
        buf = _grad_buf(w)
        tmp = torch.zeros(w.shape, device=x.device) if (_needs(w) and buf is None) else None
        native().qknorm_rope_bwd(x, dy.contiguous(), rstd, wc, dx, buf if buf is not None else tmp, cos, sin, 0,
                                 offset, interleaved)
        if buf is not None:
            grad_ready(w)
        return dx, (tmp.to(w.dtype) if tmp is not None else None), None, None, None, None, None


@_device_op
def qk_norm_rope(x, w, cos, sin, eps=1e-6, offset=1.0, interleaved=False):
    """x [B,S,H,D] strided view -> rope(rmsnorm(x) * (w + offset)) contiguous [B,S,H,D]."""
    return _QKNormRoPE.apply(x, w, cos, sin, float(eps), float(offset), bool(interleaved))


# ---------------------------------------------------------------- Gemma attention block
class _QKNormRoPEAttn(Function):
    """Gemma-3 attention core on the packed qkv GEMM output [B, S, nq + 2 nkv, D]: per-head q/k
    RMSNorm + RoPE, then causal (sliding-window) GQA flash attention.  Replaces the reference's
    separate q_norm / k_norm / rope / attention graph nodes (models/gemma_model.cpp attention
    block).  One Function owns all three slices of qkv so the backward writes a single packed
    dqkv: the attention backward stores dV straight into its slice and the q/k norm-RoPE backward
    kernels store dQ / dK into theirs -- no zero-filled per-view gradients summed by autograd.
    out_cols > nq*D: O is written into a [B, S, out_cols] buffer (augmented-K input of o_proj)."""

    @staticmethod
    def forward(ctx, qkv, wq, wk, cos, sin, eps_q, eps_k, offset, interleaved, nq, nkv, scale, window, kv_lens,
                out_cols):
        C = native()
        wqc, wkc = cw(wq), cw(wk)
        q, rq = C.qknorm_rope_fwd(qkv[:, :, :nq], wqc, cos, sin, 0, eps_q, offset, interleaved)
        k, rk = C.qknorm_rope_fwd(qkv[:, :, nq:nq + nkv], wkc, cos, sin, 0, eps_k, offset, interleaved)
        o_full, lse, o = C.attn_fwd(q, k, qkv[:, :, nq + nkv:], scale, True, window, kv_lens, out_cols)
        ctx.save_for_backward(qkv, q, k, o, lse, rq, rk, wqc, wkc, cos, sin)
        ctx.w = (wq, wk)
        ctx.cfg = (offset, interleaved, nq, nkv, scale, window, kv_lens)
        ctx.wide = out_cols > 0 and o_full.dim() == 3
        return o_full

    @staticmethod
    def backward(ctx, do):
        qkv, q, k, o, lse, rq, rk, wqc, wkc, cos, sin = ctx.saved_tensors
        offset, interleaved, nq, nkv, scale, window, kv_lens = ctx.cfg
        C = native()
        B, S, _, D = qkv.shape
        if ctx.wide:
            do = do[..., :nq * D].view(B, S, nq, D)
        if do.stride(-1) != 1 or not ctx.wide:
            do = do.contiguous()
        dqkv = torch.empty_like(qkv)
        dq = torch.empty_like(q)
        dk = torch.empty_like(k)
        C.attn_bwd(q, k, qkv[:, :, nq + nkv:], o, do, lse, dq, dk, dqkv[:, :, nq + nkv:], scale, True, window,
                   kv_lens)
        grads = []
        for w, wc, x, dy, r, dst in ((ctx.w[0], wqc, qkv[:, :, :nq], dq, rq, dqkv[:, :, :nq]),
                                     (ctx.w[1], wkc, qkv[:, :, nq:nq + nkv], dk, rk, dqkv[:, :, nq:nq + nkv])):
            buf = _grad_buf(w)
            tmp = torch.zeros(w.shape, device=qkv.device) if (_needs(w) and buf is None) else None
            C.qknorm_rope_bwd(x, dy, r, wc, dst, buf if buf is not None else tmp, cos, sin, 0, offset, interleaved)
            if buf is not None:
                grad_ready(w)
            grads.append(tmp.to(w.dtype) if tmp is not None else None)
        return (dqkv, grads[0], grads[1]) + (None,) * 12


@_device_op
def qk_norm_rope_attention(qkv, nq, nkv, wq, wk, cos, sin, eps_q, eps_k, offset=1.0, interleaved=False, scale=None,
                           window=0, kv_lens=None, out_cols=0):
    """qkv [B,S,nq+2nkv,D] -> o [B,S,nq,D] = attention(rope(rmsnorm_q(q)), rope(rmsnorm_k(k)), v);
    with out_cols > nq*D (GPU) -> [B,S,out_cols] whose first nq*D columns hold O."""
    D = qkv.shape[-1]
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    oc = int(out_cols) if out_cols and out_cols > nq * D else 0
    return _QKNormRoPEAttn.apply(qkv, wq, wk, cos, sin, float(eps_q), float(eps_k), float(offset), bool(interleaved),
                                 int(nq), int(nkv), float(scale), int(window or 0), kv_lens, oc)


# ---------------------------------------------------------------- linear layers
# GEMM routing (measured per shape at M = 65536 on MI355X, scripts/bench_gemm_t.py, in one process):
#   * every FUSED GEMM runs on the hand-written 8-phase MFMA kernel (csrc/kernels/gemm8.hip): fc +
#     bias + GELU (writes pre-activation and activation), mlp_proj data-grad x GELU'(pre), LoRA
#     data-grads with the rank-r update in the epilogue;
#   * plain data-grads dx = dy W run on gemm8's NN form (W read k-major with ds_read_b64_tr_b16, no
#     transposed weight copies): 0.95-1.0x hipBLASLt (fc dx 276 vs 264 us, qkv dx 208 vs 206,
#     LM-head dx 3.91 vs 3.77 ms);
#   * plain forward GEMMs y = x W^T + b and fp32 weight-gradient accumulation are "plain library
#     GEMMs" and stay on hipBLASLt where it is measurably faster (NT forward: gemm8 0.79-0.87x;
#     TN weight-grads: gemm8 0.69-1.40x in isolation, slower inside the full-FT step).  MFT_GEMM8_ALL=1 routes them through gemm8 too, and
#     --deterministic (set_deterministic) always uses gemm8's split-K TN form, whose fixed-order
#     slab reduction makes weight gradients bitwise reproducible.
# Shapes outside gemm8's contract (reduction dim % 64, output columns % 8) fall back to torch.mm
# with a one-time notice.
_NOTED = set()
_DETERMINISTIC = [os.environ.get("MFT_DETERMINISTIC", "0") == "1"]


def set_deterministic(on: bool = True):
    """Deterministic-reduction mode: fixed-order two-stage reductions instead of
    float atomics in every kernel that has both forms (LoRA weight-grads, embedding grad, attention
    dQ) and gemm8's split-K weight gradients instead of hipBLASLt's."""
    _DETERMINISTIC[0] = bool(on)
    native().set_deterministic(bool(on))


def deterministic() -> bool:
    return _DETERMINISTIC[0]


def _gemm8_all() -> bool:
    return os.environ.get("MFT_GEMM8_ALL", "0") == "1"


def _note(what):
    if what not in _NOTED:
        _NOTED.add(what)
        import sys
        print(f"[mobilefinetuner_amd] {what}: shape outside gemm8's contract, using torch.mm", file=sys.stderr)


def _g8_ok(x2, *ts) -> bool:
    return all(t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(-1) == 1 and t.stride(0) % 8 == 0
               for t in (x2, *ts))


def gemm_linear(x2, wc, bc=None):
    """y = x W^T (+ b), W [out, in]."""
    M, K = x2.shape
    N = wc.shape[0]
    if _gemm8_all() and _g8_ok(x2, wc) and K % 64 == 0 and N % 8 == 0 and (bc is None or bc.dtype == torch.bfloat16):
        if bc is None:
            return native().gemm_t(x2, wc, False, False, GEMM_EPI_NONE)[0]
        return native().gemm_t(x2, wc, False, False, GEMM_EPI_BIAS, bias=bc)[0]
    return torch.addmm(bc, x2, wc.t()) if bc is not None else torch.mm(x2, wc.t())


def gemm_dx(dy2, wc, out=None):
    """dx = dy W (W [out, in], possibly a row-strided view) -- gemm8 NN."""
    N = wc.shape[0]
    if _g8_ok(dy2, wc) and N % 64 == 0 and wc.shape[1] % 8 == 0 and (out is None or _g8_ok(out)):
        return native().gemm_t(dy2, wc, False, True, GEMM_EPI_NONE, out=out)[0]
    _note("data-grad")
    if out is not None:
        return torch.mm(dy2, wc, out=out)
    return torch.mm(dy2, wc)


def _mm_wgrad_into(buf, dy2, x2, alpha=1.0):
    """buf (fp32 [N, K]) += alpha * dy2^T @ x2, accumulated in place in the fp32 grad buffer: the TN gemm8
    (split-K slabs + a fixed-order reduce, bitwise reproducible) where its shape rules hold, else torch."""
    M = dy2.shape[0]
    if (_g8_ok(dy2, x2) and buf.is_contiguous() and M % 64 == 0 and dy2.shape[1] % 8 == 0
            and x2.shape[1] % 8 == 0):
        native().gemm_t(dy2, x2, True, True, GEMM_EPI_F32ACC, alpha=float(alpha), out=buf.view(dy2.shape[1], -1))
        return
    buf.add_(torch.mm(dy2.t(), x2, out_dtype=torch.float32), alpha=alpha)


def _bias_grad(b, dy2):
    """Accumulate the bias gradient (column sums of dy) into b.grad; returns what backward must
    return for b.  GPU: colsum kernel straight into the fp32 grad buffer."""
    if not _needs(b):
        return None
    buf = _grad_buf(b)
    if (buf is not None and dy2.is_cuda and dy2.dtype == torch.bfloat16 and dy2.dim() == 2 and dy2.stride(-1) == 1
            and dy2.shape[-1] % 8 == 0 and dy2.stride(0) % 8 == 0):
        native().colsum_acc(dy2, buf.view(-1), True)
        grad_ready(b)
        return None
    return _sink(b, dy2.float().sum(0))


class _Linear(Function):
    @staticmethod
    def forward(ctx, x, w, b):
        wc, bc = cw(w), cw(b)
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        y = gemm_linear(x2, wc, bc)
        ctx.save_for_backward(x2 if _needs(w) else None)
        ctx.params = (w, b)
        ctx.wc = wc
        ctx.shape = shape
        return y.view(*shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        (x2,) = ctx.saved_tensors
        w, b = ctx.params
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = gemm_dx(dy2, ctx.wc).view(ctx.shape)
        gw = gb = None
        if _needs(w):
            buf = _grad_buf(w)
            if buf is not None:
                _mm_wgrad_into(buf, dy2, x2)
                grad_ready(w)
            else:
                gw = torch.zeros(w.shape, device=dy2.device, dtype=torch.float32)
                _mm_wgrad_into(gw, dy2, x2)
                gw = gw.to(w.dtype)
        if _needs(b):
            gb = _bias_grad(b, dy2)
        return dx, gw, gb


@_device_op
def linear(x, w, b=None):
    """y = x W^T + b with W [out, in] (nn.Linear layout)."""
    return _Linear.apply(x, w, b)


def frozen_weight_t(p):
    """Cached row-major [in, out] copy of a FROZEN [out, in] weight, or None.  The fused data-grad
    GEMMs (x GELU'(pre), + rank-r LoRA update) run ~8% faster in gemm8's NT form than in its NN form
    (mlp_proj dx + dGELU 454 vs 481 us, LoRA qkv/proj dx 138 vs 152 us avg, MI355X), so frozen
    weights -- whose copy is built once (85 M params -> 170 MB of 288 GB) -- use NT; trainable or
    sharded weights use NN and need no copy at all (no per-step transposes)."""
    if _needs(p) or getattr(p, "_mft_sharded", False):
        return None
    wc = cw(p)
    c = getattr(p, "_mft_wt", None)
    if c is None or c.data_ptr() == 0 or c.shape != (wc.shape[1], wc.shape[0]):
        c = wc.t().contiguous()
        p._mft_wt = c
    return c


def drop_weight_t(p):
    if hasattr(p, "_mft_wt"):
        del p._mft_wt


def _fused_dx(dy2, w, epi, **kw):
    """dx = epi(dy W): gemm8 NT on the cached transposed copy of a frozen W, NN otherwise."""
    wt = frozen_weight_t(w)
    if wt is not None:
        return native().gemm_t(dy2, wt, False, False, epi, **kw)
    return native().gemm_t(dy2, cw(w), False, True, epi, **kw)


class _MLPGelu(Function):
    """y = GELU(x W1^T + b1) W2^T + b2 with both GELU passes fused into the hand-written MFMA GEMM
    (csrc/kernels/gemm8.hip): the fc GEMM's epilogue adds the bias and writes BOTH GELU(pre) and
    GELU'(pre) (one sigmoid for both; saved for backward instead of pre); the mlp_proj data-grad
    GEMM's epilogue multiplies by it, so no separate GELU pass touches the [M, 4C] activations in
    either direction and the backward does no transcendental work.  Reference MLP: graph/gpt2_model.cpp (c_fc matmul, gelu_new, c_proj matmul as three
    separate ops)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        C = native()
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        w1c, b1c, w2c, b2c = cw(w1), cw(b1), cw(w2), cw(b2)
        h, dgl = C.gemm_t(x2, w1c, False, False, GEMM_EPI_BIAS_GELU_D, bias=b1c)  # dgl = GELU'(pre)
        y = gemm_linear(h, w2c, b2c)
        ctx.save_for_backward(x2 if _needs(w1) else None, dgl, h if _needs(w2) else None)
        ctx.params = (w1, b1, w2, b2)
        ctx.wc = w1c
        ctx.shape = shape
        return y.view(*shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x2, dgl, h = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        w1c = ctx.wc
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dpre = _fused_dx(dy2, w2, GEMM_EPI_MUL_AUX, aux=dgl)[0]
        grads = [None] * 5
        if ctx.needs_input_grad[0]:
            grads[0] = gemm_dx(dpre, w1c).view(ctx.shape)
        for i, (p, g_out, g_in) in enumerate(((w2, dy2, h), (w1, dpre, x2))):
            if not _needs(p):
                continue
            buf = _grad_buf(p)
            if buf is not None:
                _mm_wgrad_into(buf, g_out, g_in)
                grad_ready(p)
            else:
                gt = torch.zeros(p.shape, device=g_out.device, dtype=torch.float32)
                _mm_wgrad_into(gt, g_out, g_in)
                grads[3 if i == 0 else 1] = gt.to(p.dtype)
        if _needs(b2):
            grads[4] = _bias_grad(b2, dy2)
        if _needs(b1):
            grads[2] = _bias_grad(b1, dpre)
        return tuple(grads)


def fused_mlp_available() -> bool:
    """Fused-epilogue MLP on the 8-phase gemm8.hip kernel (MFT_FUSED_MLP=0 disables).  Measured in
    the GPT-2 LoRA bench step on MI355X (A/B in one call): 1.338M vs 1.321M tok/s unfused; isolated
    at M=32k: fc+GELU 198 us vs 215 (hipBLASLt addmm + GELU kernel), mlp_proj dx+dGELU 209 us vs
    275 (hipBLASLt mm + GELU-backward kernel)."""
    import os
    return os.environ.get("MFT_FUSED_MLP", "1") != "0"


def mlp_gelu(x, fc, proj):
    """GPT-2 MLP: proj(GELU(fc(x))).  Fused-epilogue path when neither Linear carries an active
    LoRA adapter (the adapter's rank-r update lands between the GEMM and the GELU)."""
    plain = not ((fc.lora_slices and fc.lora_enabled) or (proj.lora_slices and proj.lora_enabled))
    K = x.shape[-1]
    if (x.is_cuda and plain and fc.bias is not None and proj.bias is not None and fused_mlp_available()
            and K % 64 == 0 and fc.out_features % 64 == 0):
        return _MLPGelu.apply(x, fc.weight, fc.bias, proj.weight, proj.bias)
    return proj(gelu(fc(x)))


class _LoRALinear(Function):
    """y = x W^T + b + sum_i s * (x A_i^T) B_i placed in column slices [c0_i, c0_i + n_i) of y.

    W (and b) frozen; A_i [r, in] (PEFT lora_A layout), B_i [r, n_i] fp32 masters with bf16
    shadows (``p.shadow``).  One hipBLASLt base GEMM for the whole (possibly fused, e.g. q|k|v)
    weight, then the rank-r work per slice in lora.hip (reference: LoRALinear slices
    {A,B,scale,col0,cols}, nn/lora_linear.h:17-97)."""

    @staticmethod
    def forward(ctx, x, w, b, s, slices, *ab):
        C = native()
        wc, bc = cw(w), cw(b)
        shape = x.shape
        K, N = shape[-1], wc.shape[0]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        y = gemm_linear(x2, wc, bc)
        us = []
        ctr = dropout_counter(x.device)
        for i, (c0, n, dp, salt) in enumerate(slices):
            Ac, Bc = cw(ab[2 * i]), cw(ab[2 * i + 1])
            R = Ac.shape[0]
            u = torch.empty(x2.shape[0], R, device=x.device, dtype=x.dtype)
            C.lora_rowdot(x2, Ac, u, 1.0, dp, salt, ctr)      # u = dropout(x) A^T
            ys = y[:, c0:c0 + n]
            C.lora_update(ys, u, Bc, ys, float(s), 0.0, 0, None)  # y[:, slice] += s u B
            us.append(u)
        ctx.save_for_backward(x2, *us)
        ctx.params = ab
        ctx.slices, ctx.wc = slices, wc
        ctx.s, ctx.shape, ctx.N = float(s), shape, N
        return y.view(*shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x2, *us = ctx.saved_tensors
        ab = ctx.params
        s, N = ctx.s, ctx.N
        K = x2.shape[1]
        dy2 = dy.reshape(-1, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = gemm_dx(dy2, ctx.wc) if ctx.needs_input_grad[0] else None
        grads = []
        ctr = dropout_counter(dy.device)
        for i, (c0, n, dp, salt) in enumerate(ctx.slices):
            A, B = ab[2 * i], ab[2 * i + 1]
            Ac, Bc = cw(A), cw(B)
            R = Ac.shape[0]
            dys = dy2[:, c0:c0 + n]
            v = torch.empty(dy2.shape[0], R, device=dy.device, dtype=dy.dtype)
            db_done = _dy_pass(C, dy2, c0, n, B, us[i], 0, R, v, s)  # v = s dy B^T (+ dB in the same pass)
            if dx is not None:
                C.lora_update(dx, v, Ac, dx, 1.0, dp, salt, ctr)  # dx += mask * (v A)
            gA = gB = None
            if _needs(A):
                buf = _grad_buf(A)
                tgt = buf if buf is not None else torch.zeros(R, K, device=dy.device)
                C.lora_wgrad(x2, v, tgt, 1, K, 1.0, dp, salt, ctr)  # dA[r, k] += sum_m v[m, r] drop(x)[m, k]
                if buf is not None:
                    grad_ready(A)
                else:
                    gA = tgt
            if _needs(B):
                buf = _grad_buf(B)
                tgt = buf if buf is not None else torch.zeros(R, n, device=dy.device)
                if not db_done:
                    C.lora_wgrad(dys, us[i], tgt, 1, n, s, 0.0, 0, None)  # dB[r, n] += s sum_m u[m, r] dy[m, n]
                if buf is not None:
                    grad_ready(B)
                else:
                    gB = tgt
            grads += [gA, gB]
        if dx is not None:
            dx = dx.view(ctx.shape)
        return (dx, None, None, None, None, *grads)


class _LoRALinearAug(Function):
    """LoRA Linear whose forward is ONE GEMM over an augmented K dimension:

        y = [x | u_1 .. u_n | 0] . [W | s B_1^T .. s B_n^T | 0]^T + b,   u_i = dropout(x) A_i^T

    The producer of x (LayerNorm / attention) wrote it into the first K columns of a wider buffer
    ``xa`` [M, Ka] and ZEROED columns [K, Ka) (contract: padding meets zero weights, and 0 * NaN from
    uninitialised memory would not be 0); the rank-r projections u_i are written into the appended
    columns by lora_rowdot,
    and ``waug`` [N, Ka] (owned by the Linear) carries W once plus s B_i^T, refreshed every call, in
    each slice's rows.  This removes the per-slice rank-r update pass over y [M, N] (lora_update)
    from the forward: the rank-r work rides in the GEMM's K loop (Ka = K + 64 for r <= 64 total).
    Backward: dx = dy W (W part of waug) + mask * (v A) written straight into the wide grad
    buffer; dA/dB by lora_wgrad as in _LoRALinear.  Reference: LoRALinear, nn/lora_linear.h:17-97."""

    @staticmethod
    def forward(ctx, xa, w, b, s, slices, K, waug, *ab):
        C = native()
        shape = xa.shape
        Ka = shape[-1]
        xa2 = xa.reshape(-1, Ka)
        x2 = xa2[:, :K]
        ctr = dropout_counter(xa.device)
        off = K
        # several adapters on one input without dropout (q|k|v, gate|up): ONE pass over x for all
        # u_i (the u columns of consecutive slices are adjacent in xa)
        batched = len(slices) > 1 and all(dp == 0 for (_, _, dp, _) in slices)
        acat = None
        if batched:
            acat = torch.cat([cw(ab[2 * i]) for i in range(len(slices))])
            C.lora_rowdot(x2, acat, xa2[:, K:K + acat.shape[0]], 1.0, 0.0, 0, None)
        for i, (c0, n, dp, salt) in enumerate(slices):
            Ac, Bc = cw(ab[2 * i]), cw(ab[2 * i + 1])
            R = Ac.shape[0]
            if not batched:
                C.lora_rowdot(x2, Ac, xa2[:, off:off + R], 1.0, dp, salt, ctr)  # u_i -> appended columns
            torch.mul(Bc.t(), s, out=waug[c0:c0 + n, off:off + R])              # s B_i^T -> W' rows of slice i
            off += R
        bc = cw(b)
        y = gemm_linear(xa2, waug, bc)
        ctx.save_for_backward(xa)  # the input itself (a no-grad view of it must not be saved)
        ctx.params = ab
        ctx.slices, ctx.waug, ctx.K, ctx.w = slices, waug, K, w
        ctx.s, ctx.shape = float(s), shape
        ctx.acat = acat  # [A_1; ..; A_n] of this step's shadows, reused by the backward's LoRA epilogue
        return y.view(*shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        C = native()
        (xa,) = ctx.saved_tensors
        ab, s, K = ctx.params, ctx.s, ctx.K
        xa2 = xa.reshape(-1, xa.shape[-1])
        M, Ka = xa2.shape
        x2 = xa2[:, :K]
        N = ctx.waug.shape[0]
        dy2 = dy.reshape(-1, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dxa = None
        ranks = [cw(ab[2 * i]).shape[0] for i in range(len(ctx.slices))]
        fused = ctx.needs_input_grad[0] and _lora_epi_ok(ctx.slices, ranks, dy2, K)
        if ctx.needs_input_grad[0]:
            # columns [K, Ka) of the input gradient are never read (the producers' backward reads
            # only their own K columns through the row stride), so they are left unwritten
            dxa = torch.empty(M, Ka, device=dy.device, dtype=dy.dtype)
            if not fused:
                dx = gemm_dx(dy2, ctx.waug[:, :K])
        vs = []
        db_done = set()
        if fused:
            # every v_i = s dy_i B_i^T into one [M, sum r] buffer, then ONE gemm8 launch computes
            # dx = dy W + [v_1 .. v_n] [A_1; ..; A_n] with the rank-r update in its epilogue
            vall = torch.empty(M, sum(ranks), device=dy.device, dtype=dy.dtype)
            o = 0
            for i, (c0, n, dp, salt) in enumerate(ctx.slices):
                if _dy_pass(C, dy2, c0, n, ab[2 * i + 1], xa2, K + o, ranks[i], vall[:, o:o + ranks[i]], s):
                    db_done.add(i)  # dB_i came out of the same pass over dy_i (lora_dy)
                vs.append(vall[:, o:o + ranks[i]])
                o += ranks[i]
            acat = ctx.acat
            if acat is None:
                acat = torch.cat([cw(ab[2 * i]) for i in range(len(ranks))]) if len(ranks) > 1 else cw(ab[0])
            _fused_dx(dy2, ctx.w, GEMM_EPI_LORA, out=dxa[:, :K], lora_u=vall, lora_w=acat)
        grads = []
        ctr = dropout_counter(dy.device)
        off = K
        first = True
        # dA of every rank-8 adapter in ONE pass over x (segmented lora_wgrad) when all of them have
        # grad buffers and no dropout
        da_done = False
        if fused and len(ctx.slices) > 1 and all(r == 8 for r in ranks) and len(ranks) <= 8:
            bufs = [_grad_buf(ab[2 * i]) for i in range(len(ranks))]
            if all(b is not None for b in bufs) and all(dp == 0 for (_, _, dp, _) in ctx.slices):
                C.lora_wgrad_multi(x2, vall, bufs, 1.0)
                da_done = True
        for i, (c0, n, dp, salt) in enumerate(ctx.slices):
            A, B = ab[2 * i], ab[2 * i + 1]
            Ac, Bc = cw(A), cw(B)
            R = Ac.shape[0]
            dys = dy2[:, c0:c0 + n]
            if fused:
                v = vs[i]
            else:
                v = torch.empty(M, R, device=dy.device, dtype=dy.dtype)
                C.lora_rowdot(dys, Bc, v, s, 0.0, 0, None)  # v = s dy B^T
            if dxa is not None and not fused:
                # dx (+)= mask * (v A); the first slice also moves dx into the wide gradient buffer
                C.lora_update(dx if first else dxa[:, :K], v, Ac, dxa[:, :K], 1.0, dp, salt, ctr)
                first = False
            gA = gB = None
            if da_done:
                grad_ready(A)
            elif _needs(A):
                buf = _grad_buf(A)
                tgt = buf if buf is not None else torch.zeros(R, K, device=dy.device)
                C.lora_wgrad(x2, v, tgt, 1, K, 1.0, dp, salt, ctr)
                if buf is not None:
                    grad_ready(A)
                else:
                    gA = tgt
            if _needs(B):
                buf = _grad_buf(B)
                tgt = buf if buf is not None else torch.zeros(R, n, device=dy.device)
                if i not in db_done:
                    C.lora_wgrad(dys, xa2[:, off:off + R], tgt, 1, n, s, 0.0, 0, None)  # dB += s u^T dy
                if buf is not None:
                    grad_ready(B)
                else:
                    gB = tgt
            grads += [gA, gB]
            off += R
        if dxa is not None and first and not fused:  # no slices (cannot happen via Linear)
            dxa[:, :K].copy_(dx)
        if dxa is not None:
            dxa = dxa.view(ctx.shape)
        return (dxa, None, None, None, None, None, None, *grads)


def _dy_pass(C, dy2, c0, n, B, xa2, uoff, R, v, s) -> bool:
    """v = s dy[:, c0:c0+n] B^T into ``v``; when B's fp32 grad buffer exists and the shapes meet
    lora_dy's contract (rank 8, 8-column aligned slice, u columns 16-B aligned), dB += s u^T dy is
    produced by the SAME pass over dy (returns True); otherwise lora_rowdot only (False).
    MFT_LORA_DY=0 disables the fused pass (A/B switch)."""
    buf = _grad_buf(B)
    M, N = dy2.shape
    ok = (buf is not None and os.environ.get("MFT_LORA_DY", "1") != "0" and R == 8 and n % 8 == 0 and c0 % 8 == 0
          and N % 8 == 0 and uoff % 8 == 0 and xa2.stride(0) % 8 == 0)
    if ok:
        vpart = torch.empty(((n + 255) // 256) * M * 8, device=dy2.device, dtype=torch.float32)
        C.lora_dy(dy2[:, c0:c0 + n], cw(B), xa2[:, uoff:uoff + 8], buf, vpart, v, s)
        return True
    C.lora_rowdot(dy2[:, c0:c0 + n], cw(B), v, s, 0.0, 0, None)
    return False


def _lora_epi_ok(slices, ranks, dy2, K) -> bool:
    """The fused dx path (gemm8 GEMM_EPI_LORA) needs no LoRA dropout (the mask would apply to v A
    only), sum(r) a multiple of 8 up to 32, and gemm8's shape contract (reduction dim % 64)."""
    if os.environ.get("MFT_LORA_EPI", "1") == "0" or not dy2.is_cuda or dy2.dtype != torch.bfloat16:
        return False
    rt = sum(ranks)
    return (all(sl[2] == 0.0 for sl in slices) and 0 < rt <= 32 and rt % 8 == 0 and dy2.shape[1] % 64 == 0
            and K % 8 == 0)


def lora_aug_cols(in_features: int, ranks) -> int:
    """Width of the augmented LoRA input [x | u_1..u_n | 0]: K + sum(r), rounded up to 64 (hipBLASLt
    measured slower at K + 8 .. K + 32 than at K + 64 on gfx950, scripts/probe_kpad.py)."""
    return (in_features + sum(ranks) + 63) // 64 * 64


def lora_linear_aug(xa, w, b, slices, scale, waug, training: bool = True):
    """xa [.., Ka] holds x in its first w.shape[1] columns; see _LoRALinearAug."""
    K = w.shape[1]
    meta, ab = [], []
    for sl in slices:
        c0, n, A, B = sl[:4]
        p = float(sl[4]) if len(sl) > 4 else 0.0
        salt = int(sl[5]) if len(sl) > 5 else 0
        if not (training and torch.is_grad_enabled()):
            p = 0.0
        meta.append((int(c0), int(n), p, salt & 0xFFFFFFFF))
        ab += [A, B]
    return _LoRALinearAug.apply(xa, w, b, float(scale), tuple(meta), int(K), waug, *ab)


@_device_op
def lora_linear(x, w, b, slices, scale, training: bool = True):
    """slices: list of (col0, ncols, A, B[, dropout_p, salt]).  See _LoRALinear.  Dropout (PEFT
    semantics: on the LoRA input only) is active when ``training`` and grad mode are on."""
    norm = []
    for sl in slices:
        c0, n, A, B = sl[:4]
        p = float(sl[4]) if len(sl) > 4 else 0.0
        salt = int(sl[5]) if len(sl) > 5 else 0
        if not (training and torch.is_grad_enabled()):
            p = 0.0
        norm.append((c0, n, A, B, p, salt))
    meta = tuple((int(c0), int(n), float(p), int(salt) & 0xFFFFFFFF) for (c0, n, _, _, p, salt) in norm)
    ab = []
    for sl in norm:
        ab += [sl[2], sl[3]]
    return _LoRALinear.apply(x, w, b, float(scale), meta, *ab)


_DROP_CTR = {}


def dropout_counter(device):
    """Device-resident step counter feeding the counter-based LoRA dropout masks; the training
    engine bumps it once per step (inside the captured graph)."""
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = str(device)
    t = _DROP_CTR.get(key)
    if t is None:
        t = torch.zeros(1, dtype=torch.int64, device=device)
        _DROP_CTR[key] = t
    return t


# ---------------------------------------------------------------- fused LM head + cross entropy
def default_ce_chunk(vpad: int) -> int:
    """Rows of the LM-head CE processed per fused call (each call holds one [rows, Vpad] bf16 E
    workspace: exp(logit - tile max), the only vocab-wide tensor, never the logits themselves).

    Sized for 288 GB of HBM: a 32 GiB budget (MFT_CE_BUDGET_GB), at most 65536 rows -- the whole
    GPT-2 bench step (6.6 GB) and the whole Gemma-3 bench step (262144 columns, 32 GiB) in ONE
    call: the NN dgrad has only ceil(C / 256) column tiles, so row chunks smaller than the step
    leave CUs idle (Gemma, C = 640: 2 x 32768-row calls 57.5 ms vs one 65536-row call 52.9 ms;
    GPT-2 4096-row chunks were 9% slower per step in round 1, profiles/)."""
    import os
    env = os.environ.get("MFT_CE_CHUNK")
    if env:
        return int(env)
    budget = float(os.environ.get("MFT_CE_BUDGET_GB", "32")) * (1 << 30)
    rows = int(budget // (2 * vpad))
    return max(64, min(65536, rows // 64 * 64))


class _LMHeadCE(Function):
    """Fused LM head + CE (xent.hip ``lm_head_ce``): per chunk of rows ONE gemm8 forward whose
    epilogue reduces the fp32 logits tile to (max, sum-exp) and stores E = exp(logit - tile max),
    a row finalize, and -- for dh -- one gemm8 NN whose main loop rescales its accumulator per
    vocab tile, so neither logits nor dlogits are ever produced by an elementwise pass.  When the
    LM-head weight itself trains (full fine-tune, tied wte) E is turned into dlogits in place and
    also feeds the TN weight-gradient GEMM."""

    @staticmethod
    def forward(ctx, h, w, labels, V, chunk, w_grad_scale):
        C = native()
        wc = cw(w)
        M = h.shape[0]
        h = h.contiguous()
        labels = labels.reshape(-1).contiguous()
        valid = (labels >= 0).sum().float()
        scale = 1.0 / valid.clamp(min=1.0)
        loss_rows = torch.empty(M, device=h.device, dtype=torch.float32)
        need_grad = ctx.needs_input_grad[0] or _needs(w)
        dh = torch.empty_like(h) if need_grad else None
        wbuf = _grad_buf(w) if need_grad else None
        wtmp = torch.zeros(w.shape, device=h.device) if (need_grad and _needs(w) and wbuf is None) else None
        want_w = wbuf is not None or wtmp is not None
        for i in range(0, M, chunk):
            hc = h[i:i + chunk]
            E = torch.empty(hc.shape[0], wc.shape[0], device=h.device, dtype=torch.bfloat16) if need_grad else None
            C.lm_head_ce(hc, wc, labels[i:i + chunk], V, E, loss_rows[i:i + chunk], scale, 1.0,
                         dh[i:i + chunk] if need_grad else None, want_w)
            if want_w:
                tgt = wbuf if wbuf is not None else wtmp
                _mm_wgrad_into(tgt, E, hc, w_grad_scale)       # dW += dlogits^T h, gemm8 TN
        # a tied weight (GPT-2 wte) receives its final contribution later, from the embedding
        # backward, which fires the hook; announcing it here would let a DP bucket reduce early
        if wbuf is not None and not getattr(w, "_mft_tied", False):
            grad_ready(w)
        loss = loss_rows.sum() * scale
        ctx.save_for_backward(dh if dh is not None else torch.empty(0))
        ctx.wtmp = wtmp
        ctx.w = w
        return loss

    @staticmethod
    def backward(ctx, gout):
        (dh,) = ctx.saved_tensors
        dh = native().scale_bf16(dh, gout.float().reshape(1), 1.0)
        gw = ctx.wtmp.to(ctx.w.dtype) if ctx.wtmp is not None else None
        return dh, gw, None, None, None, None


@_device_op
def lm_head_cross_entropy(h, w, labels, vocab_size, chunk=None, w_grad_scale=1.0):
    """Mean token NLL of logits = h W^T (W [Vpad, C], first vocab_size rows real) vs labels
    (already shifted; -100 = ignore).  No raw / fp32 logits reach HBM: per chunk of rows the gemm8
    forward epilogue reduces them to per-tile softmax statistics and (training only) stores
    E = exp(logit - tile max) in bf16 -- one [rows, Vpad] bf16 buffer, the size of bf16 logits --
    which the NN dgrad consumes once with a per-tile accumulator rescale (see ``_LMHeadCE``).
    NOTE: the W gradient is produced during forward and scaled by ``w_grad_scale`` (pass the
    same factor the loss is later multiplied by, e.g. 1/grad_accum); dh honours grad_output."""
    if chunk is None:
        chunk = default_ce_chunk(cw(w).shape[0])
    return _LMHeadCE.apply(h, w, labels, int(vocab_size), int(chunk), float(w_grad_scale))


@_device_op
def lm_head_token_nll(h, w, labels, vocab_size, chunk=None):
    """Per-row NLL (no grad) for evaluation: returns (sum_nll, n_valid) device scalars."""
    with torch.no_grad():
        C = native()
        wc = cw(w)
        M = h.shape[0]
        if chunk is None:
            chunk = default_ce_chunk(wc.shape[0])
        labels = labels.reshape(-1).contiguous()
        loss_rows = torch.empty(M, device=h.device, dtype=torch.float32)
        for i in range(0, M, chunk):  # loss only: the fused forward stores no logits at all
            C.lm_head_ce(h[i:i + chunk].contiguous(), wc, labels[i:i + chunk], vocab_size, None, loss_rows[i:i + chunk],
                         None, 1.0, None, False)
        return loss_rows.sum(), (labels >= 0).sum()
