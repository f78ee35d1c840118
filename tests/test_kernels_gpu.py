"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"{msg} max abs err {err:.3e} > {tol:.3e}"


def _rel(a, b, tol, msg=""):
    """Relative L2 error: for reductions over many rows (weight / bias gradients), where a max-abs
    bound would have to scale with the row count."""
    a, b = a.float(), b.float()
    err = ((a - b).norm() / b.norm().clamp(min=1e-12)).item()
    assert err <= tol, f"{msg} rel L2 err {err:.3e} > {tol:.3e}"


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


def test_native_loaded():
    from mobilefinetuner_amd._ext import native
    C = native()
    assert "_C" in C.__file__ or C.__name__.endswith("_C")


@pytest.mark.parametrize("N", [768, 640, 1600, 256])
@pytest.mark.parametrize("resid", [False, True])
def test_layernorm(N, resid):
    from mobilefinetuner_amd.ops import functional as Fx
    M = 333
    x = torch.randn(M, N, device=DEV).bfloat16().requires_grad_()
    d = torch.randn(M, N, device=DEV).bfloat16().requires_grad_() if resid else None
    w = torch.nn.Parameter(torch.randn(N, device=DEV))
    b = torch.nn.Parameter(torch.randn(N, device=DEV))
    if resid:
        s, y = Fx.add_layer_norm(x, d, w, b)
    else:
        y = Fx.layer_norm(x, w, b)
    gy = torch.randn_like(y)
    gs = torch.randn_like(y) if resid else None
    loss = (y.float() * gy.float()).sum() + ((s.float() * gs.float()).sum() if resid else 0)
    loss.backward()
    xr = x.detach().float().requires_grad_()
    dr = d.detach().float().requires_grad_() if resid else None
    wr = w.detach().clone().requires_grad_()
    br = b.detach().clone().requires_grad_()
    sr = (xr + dr).bfloat16().float() if resid else xr
    yr = torch.nn.functional.layer_norm(sr, (N,), wr, br, 1e-5)
    lr_ = (yr * gy.float()).sum() + ((sr * gs.float()).sum() if resid else 0)
    lr_.backward()
    _close(y, yr, 0.05, msg="ln y")
    _close(x.grad, xr.grad, 0.08, 0.01, msg="ln dx")
    _rel(w.grad, wr.grad, 2e-3, msg="ln dw")
    _rel(b.grad, br.grad, 2e-3, msg="ln db")
    _close(w.grad, wr.grad, 0.02, 2e-3, msg="ln dw")
    if resid:
        _close(d.grad, dr.grad, 0.08, 0.01, msg="ln ddelta")


@pytest.mark.parametrize("N", [640, 1152, 256])
def test_rmsnorm(N):
    from mobilefinetuner_amd.ops import functional as Fx
    M = 257
    x = torch.randn(M, N, device=DEV).bfloat16().requires_grad_()
    w = torch.nn.Parameter(torch.randn(N, device=DEV) * 0.1)
    y = Fx.rms_norm(x, w, 1e-6, 1.0)
    gy = torch.randn_like(y)
    (y.float() * gy.float()).sum().backward()
    xr = x.detach().float().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * (1 + wr)
    (yr * gy.float()).sum().backward()
    _close(y, yr, 0.05, msg="rms y")
    _close(x.grad, xr.grad, 0.08, 0.01, msg="rms dx")
    _rel(w.grad, wr.grad, 2e-3, msg="rms dw")
    _close(w.grad, wr.grad, 0.02, 2e-3, msg="rms dw")


def test_gelu_and_gated():
    from mobilefinetuner_amd.ops import functional as Fx
    x = torch.randn(129, 3072, device=DEV).bfloat16().requires_grad_()
    y = Fx.gelu(x)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    xr = x.detach().float().requires_grad_()
    yr = torch.nn.functional.gelu(xr, approximate="tanh")
    (yr * g.float()).sum().backward()
    _close(y, yr, 0.03, msg="gelu")
    _close(x.grad, xr.grad, 0.05, msg="gelu dx")
    for act in ("gelu", "silu"):
        gu = torch.randn(77, 2 * 256, device=DEV).bfloat16().requires_grad_()
        y = Fx.gated_act(gu, act)
        g = torch.randn_like(y)
        (y.float() * g.float()).sum().backward()
        r = gu.detach().float().requires_grad_()
        a, u = r.chunk(2, -1)
        yr = (torch.nn.functional.gelu(a, approximate="tanh") if act == "gelu" else torch.nn.functional.silu(a)) * u
        (yr * g.float()).sum().backward()
        _close(y, yr, 0.05, msg=f"gated {act}")
        _close(gu.grad, r.grad, 0.1, 0.01, msg=f"gated {act} grad")


@pytest.mark.parametrize("M,K,N,nn,bm", [(300, 128, 264, False, 8), (1000, 192, 512, True, 8),
                                          (777, 256, 136, False, 8), (64, 64, 8, True, 8),
                                          (517, 320, 392, False, 8), (517, 320, 392, True, 8),
                                          (777, 320, 520, False, 8), (64, 64, 8, False, 8),
                                          (1000, 704, 1024, False, 8)])
def test_gemm_mfma(M, K, N, nn, bm):
    """gemm8 through the `gemm` binding (NT and NN operand layouts, M/N tails) and its epilogues vs fp32
    torch."""
    from mobilefinetuner_amd._ext import native
    C = native()
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(K, N, device=DEV) if nn else torch.randn(N, K, device=DEV)).mul(0.1).bfloat16()
    b = torch.randn(N, device=DEV).bfloat16()
    ref_ = x.float() @ (w.float() if nn else w.float().t())
    y = C.gemm(x, w, nn, 0, None, None, 1.0, bm, None)[0]
    _close(y, ref_, 0.02, 0.01, msg="gemm")
    y = C.gemm(x, w, nn, 1, b, None, 0.5, bm, None)[0]
    _close(y, 0.5 * ref_ + b.float(), 0.02, 0.01, msg="gemm bias")
    h, pre = C.gemm(x, w, nn, 2, b, None, 1.0, bm, None)
    pr = ref_ + b.float()
    _close(pre, pr, 0.02, 0.01, msg="gemm pre")
    _close(h, torch.nn.functional.gelu(pr, approximate="tanh"), 0.02, 0.01, msg="gemm gelu")
    g = C.gemm(x, w, nn, 3, None, pre, 1.0, bm, None)[0]
    pf = pre.float()
    xg = pf.clone().requires_grad_()
    torch.nn.functional.gelu(xg, approximate="tanh").sum().backward()
    _close(g, ref_ * xg.grad, 0.03, 0.01, msg="gemm dgelu")
    acc = torch.ones(M, N, device=DEV)
    C.gemm(x, w, nn, 4, None, None, 2.0, bm, acc)
    _close(acc, 1 + 2 * ref_, 0.05, 0.01, msg="gemm f32 acc")


@pytest.mark.parametrize("M,N,K,R", [(300, 768, 2304, 8), (512, 256, 128, 24), (1000, 200, 320, 32)])
def test_gemm8_lora_epilogue(M, N, K, R):
    """gemm8 GEMM_EPI_LORA: C = A B^T + U W (the fused LoRA data-grad) vs fp32 torch; strided C."""
    from mobilefinetuner_amd._ext import native
    C = native()
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    u = torch.randn(M, R, device=DEV).bfloat16()
    w = (torch.randn(R, N, device=DEV) * 0.1).bfloat16()
    wide = torch.full((M, N + 64), 7.0, device=DEV).bfloat16()
    out = wide[:, :N]
    C.gemm(a, b, False, 5, None, None, 1.0, 8, out, u, w)
    ref_ = a.float() @ b.float().t() + u.float() @ w.float()
    _close(out, ref_, 0.03, 0.01, msg="gemm8 lora")
    assert (wide[:, N:].float() == 7.0).all()


@pytest.mark.parametrize("dropout", [0.0, 0.2])
def test_lora_augmented_k_matches_plain(dropout):
    """_LoRALinearAug ([x | u] . [W | sB^T] single GEMM) == _LoRALinear (GEMM + rank-r update)."""
    from mobilefinetuner_amd.models.layers import Linear
    from mobilefinetuner_amd.ops import functional as Fx
    from mobilefinetuner_amd.utils.params import FlatParams
    M, K, N = 300, 256, 384
    lin = Linear(K, N, device=DEV)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(N, K) * 0.05)
        lin.bias.copy_(torch.randn(N) * 0.1)
    for i, (c0, n) in enumerate([(0, 128), (128, 128), (256, 128)]):
        A, B = lin.add_lora(c0, n, 8, 2.0, torch.randn(8, K) * 0.05, name=f"s{i}")
        with torch.no_grad():
            B.copy_(torch.randn_like(B) * 0.05)
    lin.lora_dropout = dropout
    flat = FlatParams([(f"p{i}", p) for i, p in enumerate(lin._lora_params)], DEV)
    ka = lin.aug_cols()
    assert ka == Fx.lora_aug_cols(K, [8, 8, 8]) == 320
    x = torch.randn(M, K, device=DEV).bfloat16()
    g = torch.randn(M, N, device=DEV).bfloat16()
    ctr = Fx.dropout_counter(DEV)
    outs = []
    for aug in (False, True):
        flat.zero_grad()
        if aug:
            xa = torch.zeros(M, ka, device=DEV).bfloat16()  # producers hand over zeroed padding
            xa[:, :K] = x
            xa.requires_grad_()
            y = lin(xa)
        else:
            xa = x.clone().requires_grad_()
            y = lin(xa)
        (y.float() * g.float()).sum().backward()
        outs.append((y.float(), xa.grad[:, :K].float(), flat.grad.clone()))
    (y0, dx0, gw0), (y1, dx1, gw1) = outs
    assert torch.isfinite(y1).all() and torch.isfinite(dx1).all()
    # producers honour the zero-padding contract even on recycled (garbage) memory
    from mobilefinetuner_amd.ops import functional as F2
    junk = torch.full((M, ka), float("nan"), device=DEV).bfloat16()
    del junk
    xn = F2.layer_norm(torch.randn(M, K, device=DEV).bfloat16(), torch.ones(K, device=DEV),
                       torch.zeros(K, device=DEV), 1e-5, ka)
    assert xn.shape[-1] == ka and (xn[:, K:] == 0).all()
    _close(y1, y0, 0.03, 0.01, msg="aug y")
    _close(dx1, dx0, 0.03, 0.01, msg="aug dx")
    _close(gw1, gw0, 0.05, 0.02, msg="aug lora grads")
    del ctr


@pytest.mark.parametrize("trainable", [False, True])
def test_fused_mlp_gelu_epilogues(trainable, monkeypatch):
    """gemm.hip BIAS_GELU / DGELU epilogue MLP vs the fp32 reference (tanh GELU)."""
    monkeypatch.setenv("MFT_FUSED_MLP", "1")
    from mobilefinetuner_amd.models.layers import Linear
    from mobilefinetuner_amd.ops import functional as Fx
    from oracle import reference as ref
    assert Fx.fused_mlp_available()
    M, C = 500, 256
    fc, proj = Linear(C, 4 * C, device=DEV), Linear(4 * C, C, device=DEV)
    with torch.no_grad():
        for lin in (fc, proj):
            lin.weight.copy_(torch.randn_like(lin.weight, dtype=torch.float32) * 0.05)
            lin.bias.copy_(torch.randn_like(lin.bias, dtype=torch.float32) * 0.5)
    if trainable:
        for lin in (fc, proj):
            lin.weight.requires_grad_(True)
            lin.bias.requires_grad_(True)
    x = torch.randn(M, C, device=DEV).bfloat16().requires_grad_()
    y = Fx.mlp_gelu(x, fc, proj)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    xr = x.detach().float().requires_grad_()
    ps = [t.detach().float().requires_grad_(trainable) for t in (fc.weight, fc.bias, proj.weight, proj.bias)]
    yr = ref.gelu_tanh(xr @ ps[0].t() + ps[1]) @ ps[2].t() + ps[3]
    (yr * g.float()).sum().backward()
    _close(y, yr, 0.03, 0.02, msg="mlp y")
    _close(x.grad, xr.grad, 0.03, 0.03, msg="mlp dx")
    if trainable:
        for p, r, n in zip((fc.weight, fc.bias, proj.weight, proj.bias), ps, ("w1", "b1", "w2", "b2")):
            _close(p.grad, r.grad, 0.05, 0.03, msg=f"mlp d{n}")


def _attn_ref(q, k, v, scale, causal, window, kv_lens=None):
    from oracle import reference as ref
    return ref.attention(q, k, v, scale, causal, window, kv_lens)


@pytest.mark.parametrize("B,S,H,Hkv,D,causal,window", [
    (2, 128, 4, 4, 64, True, 0),     # short path (one workgroup per (batch, head))
    (3, 100, 2, 2, 64, True, 0),     # short path, partial tile
    (2, 128, 4, 2, 64, True, 0),     # short path + GQA
    (2, 128, 2, 2, 64, False, 0),    # short path, non-causal
    (1, 17, 2, 2, 64, True, 0),      # short path, tiny S
    (2, 160, 4, 4, 64, True, 0),     # general path at D=64
    (2, 256, 4, 1, 256, True, 0),
    (1, 320, 4, 1, 256, True, 64),
    (2, 64, 4, 2, 128, False, 0),
    (1, 1024, 2, 2, 64, True, 0),
    (2, 200, 4, 1, 256, True, 0),    # split path, partial tile
    (1, 300, 4, 2, 128, True, 100),  # split path, sliding window
    (2, 96, 2, 1, 256, False, 0),    # split path, non-causal
])
def test_flash_attention(B, S, H, Hkv, D, causal, window):
    from mobilefinetuner_amd.ops import functional as Fx
    q = torch.randn(B, S, H, D, device=DEV).bfloat16().requires_grad_()
    k = torch.randn(B, S, Hkv, D, device=DEV).bfloat16().requires_grad_()
    v = torch.randn(B, S, Hkv, D, device=DEV).bfloat16().requires_grad_()
    scale = 1.0 / math.sqrt(D)
    o = Fx.flash_attention(q, k, v, scale, causal, window)
    go = torch.randn_like(o)
    (o.float() * go.float()).sum().backward()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf, _ = _attn_ref(qr, kr, vr, scale, causal, window)
    (orf * go.float()).sum().backward()
    _close(o, orf, 0.03, msg="attn o")
    _close(q.grad, qr.grad, 0.06, 0.02, msg="attn dq")
    _close(k.grad, kr.grad, 0.06, 0.02, msg="attn dk")
    _close(v.grad, vr.grad, 0.06, 0.02, msg="attn dv")


@pytest.mark.parametrize("B,S,H,Hkv,D,window", [
    (512, 128, 12, 12, 64, 0),   # GPT-2 124M heads at seq 128 (short path; the bench step runs 1024 such rows)
    (256, 256, 4, 1, 256, 0),    # Gemma-3 270M bench step, global layer (split path, GQA 4:1)
    (256, 256, 4, 1, 256, 128),  # ... sliding-window layer (window below S so the mask is exercised)
])
def test_flash_attention_production_shapes(B, S, H, Hkv, D, window):
    """Attention forward + backward at the benchmarked shapes vs the fp32 oracle (relative L2 over
    all elements plus a max-abs bound): the per-layer launch the training steps actually run."""
    from mobilefinetuner_amd.ops import functional as Fx
    g = torch.Generator(device=DEV).manual_seed(11)
    q = torch.randn(B, S, H, D, device=DEV, generator=g).bfloat16().requires_grad_()
    k = torch.randn(B, S, Hkv, D, device=DEV, generator=g).bfloat16().requires_grad_()
    v = torch.randn(B, S, Hkv, D, device=DEV, generator=g).bfloat16().requires_grad_()
    scale = 1.0 / math.sqrt(D)
    o = Fx.flash_attention(q, k, v, scale, True, window)
    go = torch.randn(o.shape, device=DEV, generator=g)
    (o.float() * go).sum().backward()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf, _ = _attn_ref(qr, kr, vr, scale, True, window)
    (orf * go).sum().backward()
    for name, a, b in (("o", o, orf), ("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        _rel(a, b, 1e-2, msg=f"attn {name}")
    _close(o, orf, 0.03, msg="attn o")
    _close(v.grad, vr.grad, 0.06, 0.02, msg="attn dv")


@pytest.mark.parametrize("nw", ["4", "8"])
def test_flash_attention_split_kvlens_rect(nw, monkeypatch):
    """Split kernels (D = 256, GQA 4:1) with right padding and Sq < Sk (bottom-right causal), at
    both workgroup sizes (MFT_ATTN_NW_*)."""
    from mobilefinetuner_amd._ext import native
    for var in ("MFT_ATTN_NW_FWD", "MFT_ATTN_NW_DKDV", "MFT_ATTN_NW_DQ"):
        monkeypatch.setenv(var, nw)
    B, Sq, Sk, H, Hkv, D = 2, 90, 210, 4, 1, 256
    q = torch.randn(B, Sq, H, D, device=DEV).bfloat16()
    k = torch.randn(B, Sk, Hkv, D, device=DEV).bfloat16()
    v = torch.randn(B, Sk, Hkv, D, device=DEV).bfloat16()
    kv = torch.tensor([210, 150], dtype=torch.int32, device=DEV)
    scale = D ** -0.5
    o, lse, _ = native().attn_fwd(q, k, v, scale, True, 0, kv, 0)
    go = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    native().attn_bwd(q, k, v, o, go, lse, dq, dk, dv, scale, True, 0, kv)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    orf, lser = _attn_ref(qr, kr, vr, scale, True, 0, kv)
    (orf * go.float()).sum().backward()
    valid = torch.isfinite(lser) & (lser < 1e29)
    _close(o, orf, 0.03, msg="split o")
    _close(lse[valid], lser[valid], 0.05, msg="split lse")
    _close(dq, qr.grad, 0.06, 0.02, msg="split dq")
    _close(dk, kr.grad, 0.06, 0.02, msg="split dk")
    _close(dv, vr.grad, 0.06, 0.02, msg="split dv")


def test_flash_attention_lse_and_spike():
    """Force the online-softmax rescale branch (guide §5.4 rule 26): spike one key."""
    from mobilefinetuner_amd._ext import native
    B, S, H, D = 1, 256, 2, 64
    q = torch.randn(B, S, H, D, device=DEV)
    k = torch.randn(B, S, H, D, device=DEV)
    v = torch.randn(B, S, H, D, device=DEV)
    k[0, 200] *= 30.0
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    o, lse, _ = native().attn_fwd(q, k, v, 0.125, True, 0, None, 0)
    orf, lser = _attn_ref(q.float(), k.float(), v.float(), 0.125, True, 0)
    _close(o, orf, 0.03, msg="spike o")
    _close(lse, lser, 0.05, msg="spike lse")


def test_flash_attention_packed_and_kvlens():
    from mobilefinetuner_amd.ops import functional as Fx
    B, S, H, D = 2, 128, 3, 64
    qkv = torch.randn(B, S, 3, H, D, device=DEV).bfloat16().requires_grad_()
    kv = torch.tensor([128, 77], dtype=torch.int32, device=DEV)
    o = Fx.flash_attention_qkvpacked(qkv, 0.125, True, 0, kv)
    go = torch.randn_like(o)
    (o.float() * go.float()).sum().backward()
    r = qkv.detach().float().requires_grad_()
    orf, _ = _attn_ref(r[:, :, 0], r[:, :, 1], r[:, :, 2], 0.125, True, 0, kv)
    (orf * go.float()).sum().backward()
    # rows >= kv_len of batch 1 still attend to keys < 77 (causal + padding)
    _close(o, orf, 0.03, msg="packed o")
    _close(qkv.grad, r.grad, 0.06, 0.02, msg="packed dqkv")
    # widened output for an augmented-K consumer: O in the first H*D columns, zeros after
    with torch.no_grad():
        ow = Fx.flash_attention_qkvpacked(qkv, 0.125, True, 0, kv, out_cols=H * D + 64)
    assert ow.shape == (B, S, H * D + 64)
    assert torch.equal(ow[..., :H * D], o.reshape(B, S, H * D)) and (ow[..., H * D:] == 0).all()


@pytest.mark.parametrize("V,C", [(50257, 768), (1000, 128), (70001, 64), (262144, 64)])
def test_lm_head_ce(V, C):
    from mobilefinetuner_amd.ops import functional as Fx
    M = 300
    Vp = (V + 127) // 128 * 128
    h = (torch.randn(M, C, device=DEV) * 0.5).bfloat16().requires_grad_()
    w = torch.zeros(Vp, C, device=DEV)
    w[:V] = torch.randn(V, C, device=DEV) * 0.05
    w = torch.nn.Parameter(w.bfloat16())
    lab = torch.randint(0, V, (M,), device=DEV)
    lab[::7] = -100
    loss = Fx.lm_head_cross_entropy(h, w, lab, V, chunk=128)
    (loss * 0.5).backward()
    hr = h.detach().float().requires_grad_()
    wr = w.detach().float()[:V].requires_grad_()
    lr_ = torch.nn.functional.cross_entropy(hr @ wr.t(), lab, ignore_index=-100)
    (lr_ * 0.5).backward()
    assert abs(loss.item() - lr_.item()) < 2e-2 * max(1.0, lr_.item())
    _close(h.grad, hr.grad, 2e-3, 0.03, msg="ce dh")


@pytest.mark.parametrize("R", [8, 16, 32])
def test_lora_linear(R):
    from mobilefinetuner_amd.ops import functional as Fx
    M, K, N = 250, 768, 2304
    x = (torch.randn(M, K, device=DEV) * 0.5).bfloat16().requires_grad_()
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    slices = []
    refs = []
    for (c0, n) in [(0, 768), (768, 768), (1536, 768)]:
        A = torch.nn.Parameter(torch.randn(R, K, device=DEV) * 0.05)
        B = torch.nn.Parameter(torch.randn(R, n, device=DEV) * 0.05)
        A.shadow = A.detach().bfloat16()
        B.shadow = B.detach().bfloat16()
        slices.append((c0, n, A, B))
    y = Fx.lora_linear(x, W, b, slices, 2.0)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    xr = x.detach().float().requires_grad_()
    yr = xr @ W.float().t() + b.float()
    parts = []
    for (c0, n, A, B) in slices:
        Ar = A.shadow.float().requires_grad_()
        Br = B.shadow.float().requires_grad_()
        refs.append((Ar, Br))
        parts.append(2.0 * (xr @ Ar.t()) @ Br)
    yr = yr + torch.cat(parts, dim=1)
    (yr * g.float()).sum().backward()
    _close(y, yr, 0.05, 0.01, msg="lora y")
    _close(x.grad, xr.grad, 0.1, 0.01, msg="lora dx")
    for (c0, n, A, B), (Ar, Br) in zip(slices, refs):
        _close(A.grad, Ar.grad, 0.05, 0.02, msg="lora dA")
        _close(B.grad, Br.grad, 0.05, 0.02, msg="lora dB")


def test_embedding():
    from mobilefinetuner_amd.ops import functional as Fx
    V, C, B, S = 1000, 128, 3, 17
    wte = torch.nn.Parameter(torch.randn(V, C, device=DEV).bfloat16().float())
    wte.shadow = wte.detach().bfloat16()
    wpe = torch.nn.Parameter(torch.randn(64, C, device=DEV).bfloat16().float())
    wpe.shadow = wpe.detach().bfloat16()
    wte.grad = torch.zeros_like(wte)
    wpe.grad = torch.zeros_like(wpe)
    ids = torch.randint(0, V, (B, S), device=DEV)
    out = Fx.embedding(ids, wte, wpe)
    ref = (wte.detach()[ids.reshape(-1)] + wpe.detach()[:S].repeat(B, 1))
    _close(out, ref, 0.05, msg="emb")
    g = torch.randn_like(out)
    (out.float() * g.float()).sum().backward()
    dwte = torch.zeros(V, C, device=DEV).index_add_(0, ids.reshape(-1), g.float())
    dwpe = g.float().view(B, S, C).sum(0)
    _close(wte.grad, dwte, 0.05, msg="emb dwte")
    _close(wpe.grad[:S], dwpe, 0.05, msg="emb dwpe")


@pytest.mark.parametrize("D,interleaved", [(256, False), (128, False), (64, False), (256, True)])
def test_qknorm_rope(D, interleaved):
    from mobilefinetuner_amd.ops import functional as Fx
    from oracle import reference as ref
    B, S, H = 2, 67, 3
    big = torch.randn(B, S, H + 2, D, device=DEV).bfloat16().requires_grad_()
    x = big[:, :, 1:1 + H]
    w = torch.nn.Parameter(torch.randn(D, device=DEV) * 0.1)
    cos, sin = ref.rope_tables(S, D, 10000.0, DEV)
    y = Fx.qk_norm_rope(x, w, cos, sin, 1e-6, 1.0, interleaved)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    r = big.detach().float().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    xr = r[:, :, 1:1 + H]
    yn = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * (1 + wr)
    yr = ref.rope(yn, cos, sin, 0, interleaved)
    (yr * g.float()).sum().backward()
    _close(y, yr, 0.06, msg="qkrope y")
    _close(big.grad, r.grad, 0.1, 0.01, msg="qkrope dx")
    _rel(w.grad, wr.grad, 5e-3, msg="qkrope dw")


def test_gated_widened_output():
    """gated_act(out_cols): activation in the first I columns, zeros after; wide row-strided dy."""
    from mobilefinetuner_amd.ops import functional as Fx
    I, OC = 256, 288
    gu = torch.randn(91, 2 * I, device=DEV).bfloat16().requires_grad_()
    y = Fx.gated_act(gu, "gelu", OC)
    assert y.shape == (91, OC)
    assert y[:, I:].abs().max().item() == 0
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    r = gu.detach().float().requires_grad_()
    a, u = r.chunk(2, -1)
    yr = torch.nn.functional.gelu(a, approximate="tanh") * u
    (yr * g[:, :I].float()).sum().backward()
    _close(y[:, :I], yr, 0.05, msg="gated wide y")
    _close(gu.grad, r.grad, 0.1, 0.01, msg="gated wide grad")


@pytest.mark.parametrize("nq,nkv,window,oc", [(4, 1, 0, 0), (4, 1, 48, 1056), (2, 2, 0, 544)])
def test_qknorm_rope_attention_fused(nq, nkv, window, oc):
    """Fused Gemma attention core (packed qkv -> O, one packed dqkv) vs the fp32 composition."""
    from mobilefinetuner_amd.ops import functional as Fx
    from oracle import reference as ref
    B, S, D = 2, 128, 256
    qkv = (torch.randn(B, S, nq + 2 * nkv, D, device=DEV)).bfloat16().requires_grad_()
    wq = torch.nn.Parameter(torch.randn(D, device=DEV) * 0.1)
    wk = torch.nn.Parameter(torch.randn(D, device=DEV) * 0.1)
    cos, sin = ref.rope_tables(S, D, 10000.0, DEV)
    scale = 256 ** -0.5
    o = Fx.qk_norm_rope_attention(qkv, nq, nkv, wq, wk, cos, sin, 1e-6, 1e-6, 1.0, False, scale, window, None, oc)
    if oc:
        assert o.shape == (B, S, oc) and o[..., nq * D:].abs().max().item() == 0
        o = o[..., :nq * D].reshape(B, S, nq, D)
    g = torch.randn_like(o)
    (o.float() * g.float()).sum().backward()
    r = qkv.detach().float().requires_grad_()
    wqr, wkr = wq.detach().clone().requires_grad_(), wk.detach().clone().requires_grad_()

    def nr(x, w):
        return ref.rope(x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-6) * (1 + w), cos, sin)

    q, k, v = nr(r[:, :, :nq], wqr), nr(r[:, :, nq:nq + nkv], wkr), r[:, :, nq + nkv:]
    orf = ref.attention(q, k, v, scale, True, window, None)[0]
    (orf * g.float()).sum().backward()
    _close(o, orf, 0.03, msg="fused attn o")
    _close(qkv.grad, r.grad, 0.05, 0.02, msg="fused attn dqkv")
    _rel(wq.grad, wqr.grad, 1e-2, msg="fused attn dwq")
    _rel(wk.grad, wkr.grad, 1e-2, msg="fused attn dwk")


def test_adamw_matches_reference():
    from mobilefinetuner_amd.optim.adamw import FusedAdamW
    from mobilefinetuner_amd.utils.params import FlatParams
    ps = [("a", torch.nn.Parameter(torch.randn(1000))), ("b", torch.nn.Parameter(torch.randn(37, 5)))]
    ps_cpu = [("a", torch.nn.Parameter(ps[0][1].detach().clone())), ("b", torch.nn.Parameter(ps[1][1].detach().clone()))]
    fg = FlatParams(ps, DEV)
    fc = FlatParams(ps_cpu, "cpu")
    og = FusedAdamW(fg, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    oc = FusedAdamW(fc, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    for it in range(5):
        grads = [torch.randn(1000), torch.randn(37, 5)]
        for (_, p), gr in zip(fg.named(), grads):
            p.grad.copy_(gr.to(DEV))
        for (_, p), gr in zip(fc.named(), grads):
            p.grad.copy_(gr)
        og.step()
        oc.step()
    _close(fg.master.cpu(), fc.master, 1e-5, 1e-5, msg="adamw master")
    _close(fg.shadow.cpu().float(), fc.master, 2e-2, msg="adamw shadow")
    assert abs(og.grad_norm() - oc.grad_norm()) < 1e-3 * oc.grad_norm()


def test_adamw_skips_nonfinite():
    from mobilefinetuner_amd.optim.adamw import FusedAdamW
    from mobilefinetuner_amd.utils.params import FlatParams
    fg = FlatParams([("a", torch.nn.Parameter(torch.randn(100)))], DEV)
    before = fg.master.clone()
    o = FusedAdamW(fg, lr=1e-1)
    fg.grad[3] = float("nan")
    o.step()
    assert torch.equal(fg.master, before) and o.skipped_last()


def test_casts_and_scale():
    from mobilefinetuner_amd._ext import native
    C = native()
    x = torch.randn(1001, device=DEV)
    y = torch.empty(1001, device=DEV, dtype=torch.bfloat16)
    C.cast_f32_bf16(x, y)
    assert torch.equal(y, x.bfloat16())
    z = torch.empty(1001, device=DEV)
    C.cast_bf16_f32(y, z)
    assert torch.equal(z, y.float())
    s = C.scale_bf16(y, torch.tensor([2.0], device=DEV), 0.5)
    _close(s, y.float(), 1e-2)


def test_gpt2_train_step_decreases_loss():
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.optim.adamw import FusedAdamW
    from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2, lora_parameters
    from mobilefinetuner_amd.train.engine import TrainStep
    from mobilefinetuner_amd.utils.params import FlatParams
    cfg = GPT2Config.preset("gpt2-tiny")
    m = GPT2Model(cfg, device=DEV)
    inject_gpt2(m, LoraSpec(rank=8, alpha=16, targets=["AttnQKV", "AttnProj", "MlpFcIn", "MlpFcOut"]))
    flat = FlatParams(lora_parameters(m), DEV)
    opt = FusedAdamW(flat, lr=3e-3)
    st = TrainStep(m, flat, opt, use_graph=True)
    ids = torch.randint(0, cfg.vocab_size, (4, 65), device=DEV)
    batch = [(ids[:, :-1].contiguous(), ids[:, 1:].contiguous())]
    losses = [float(st(batch).item()) for _ in range(30)]
    assert losses[-1] < losses[0] - 0.1, losses


def test_lora_dropout_consistent_fwd_bwd():
    """The hash mask must be identical in u = drop(x)A^T (fwd), dA and the dx term (bwd)."""
    from mobilefinetuner_amd._ext import native
    from mobilefinetuner_amd.ops import functional as Fx
    C = native()
    M, K, N, R, p, salt = 96, 64, 64, 8, 0.3, 1234
    ctr = Fx.dropout_counter(DEV)
    # recover the mask with A = I: u = drop(ones) -> mask/(1-p)
    ones = torch.ones(M, K, device=DEV, dtype=torch.bfloat16)
    eye = torch.eye(K, device=DEV, dtype=torch.bfloat16)
    um = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    C.lora_rowdot(ones, eye, um, 1.0, p, salt, ctr)
    mask = (um.float() * (1 - p)).round()
    assert set(mask.unique().tolist()) <= {0.0, 1.0}
    assert abs(1 - mask.mean().item() - p) < 0.05
    x = (torch.randn(M, K, device=DEV) * 0.5).bfloat16().requires_grad_()
    W = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    A = torch.nn.Parameter(torch.randn(R, K, device=DEV) * 0.1)
    B = torch.nn.Parameter(torch.randn(R, N, device=DEV) * 0.1)
    A.shadow, B.shadow = A.detach().bfloat16(), B.detach().bfloat16()
    y = Fx.lora_linear(x, W, None, [(0, N, A, B, p, salt)], 2.0, training=True)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    xr = x.detach().float().requires_grad_()
    Ar = A.shadow.float().requires_grad_()
    Br = B.shadow.float().requires_grad_()
    xd = xr * mask / (1 - p)
    yr = xr @ W.float().t() + 2.0 * (xd @ Ar.t()) @ Br
    (yr * g.float()).sum().backward()
    _close(y, yr, 0.03, 0.01, msg="drop y")
    _close(x.grad, xr.grad, 0.05, 0.01, msg="drop dx")
    _close(A.grad, Ar.grad, 0.05, 0.02, msg="drop dA")
    _close(B.grad, Br.grad, 0.05, 0.02, msg="drop dB")
    ctr.add_(1)
    um2 = torch.empty_like(um)
    C.lora_rowdot(ones, eye, um2, 1.0, p, salt, ctr)
    assert not torch.equal(um, um2), "a new step must draw a new mask"


def test_colsum_and_wgrad_accumulate():
    """Bias-grad column sums and the TN gemm8 weight-grad accumulation (beta = 1) into fp32 buffers."""
    from mobilefinetuner_amd._ext import native
    C = native()
    M, N, K = 1000, 264, 200
    dy = torch.randn(M, N, device=DEV).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    out = torch.full((N,), 2.0, device=DEV)
    C.colsum_acc(dy, out, True)
    _close(out, 2.0 + dy.float().sum(0), 0.02, 1e-3, msg="colsum")
    C.colsum_acc(dy[:, :256], out[:256], False)
    _close(out[:256], dy[:, :256].float().sum(0), 0.02, 1e-3, msg="colsum strided")
    w = torch.ones(N, K, device=DEV)
    Mw = M // 64 * 64  # (the TN form takes token counts in whole 64-row K-tiles)
    C.gemm_t(dy[:Mw], x[:Mw], True, True, 4, None, None, 0.5, w, None, None, 0)  # 4 = GEMM_EPI_F32ACC
    _close(w, 1.0 + 0.5 * dy[:Mw].float().t() @ x[:Mw].float(), 0.05, 1e-3, msg="wgrad acc")


def test_gated_row_pair_grid_stride():
    """gated kernels' row-pair mapping: an odd row count past the 16,384-block cap (grid-strided pairs, a
    lone last row) and I = 2056 > 256 lanes x 8 columns (a partial second column pass)."""
    from mobilefinetuner_amd.ops import functional as Fx
    M, I = 32771, 2056
    for act in ("gelu", "silu"):
        gu = torch.randn(M, 2 * I, device=DEV).bfloat16().requires_grad_()
        y = Fx.gated_act(gu, act)
        g = torch.randn_like(y)
        (y.float() * g.float()).sum().backward()
        r = gu.detach().float().requires_grad_()
        a, u = r.chunk(2, -1)
        yr = (torch.nn.functional.gelu(a, approximate="tanh") if act == "gelu" else torch.nn.functional.silu(a)) * u
        (yr * g.float()).sum().backward()
        # |y| reaches ~25 over 67M outputs: half a bf16 ulp there is ~0.06, so the bound scales with max |y|
        _close(y, yr, 0.02, 0.01, msg=f"gated {act} long")
        _close(gu.grad, r.grad, 0.1, 0.01, msg=f"gated {act} long grad")
        del gu, y, g, r, yr


def test_adamw_amsgrad_matches_reference():
    """AMSGrad, the reference's rule (optim/adam.cpp:52,75-80: v_hat = max(v_hat, v / bc2)): the fused kernel
    with a vmax buffer == the fp64 oracle tests/oracle/reference.py::adam_step over 6 steps (decoupled
    weight decay, fp32 moments, a large early gradient so the running max matters), tail path included."""
    from mobilefinetuner_amd._ext import native
    from oracle.reference import adam_step
    C = native()
    torch.manual_seed(0)
    n = 4099  # tail path too
    p0 = torch.randn(n, device="cuda")
    rp, rm, rv, rvh = (t.double().cpu() for t in (p0, torch.zeros(n), torch.zeros(n), torch.zeros(n)))
    p, m, v, vmax = p0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    lr = torch.full((1,), 1e-2, device="cuda")
    step = torch.zeros(1, device="cuda")
    for it in range(6):
        g = torch.randn(n, device="cuda") * (3.0 if it == 1 else 0.3)  # a large early step makes the max matter
        adam_step(rp, g.double().cpu(), rm, rv, rvh, it + 1, 1e-2, 0.9, 0.99, 1e-8, 0.05, True, True)
        C.adamw_step(p, g, m, v, lr, step, None, 0.9, 0.99, 1e-8, 0.05, 0.0, False, None, None, 0, vmax)
        C.adamw_commit(step, None, None)
    torch.cuda.synchronize()
    assert torch.allclose(p.cpu().double(), rp, rtol=1e-5, atol=1e-6), (p.cpu().double() - rp).abs().max()
    assert torch.allclose(vmax.cpu().double(), rvh, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("M,K,R,ldx", [(1000, 640, 8, 704), (77, 768, 32, 768), (4099, 2048, 16, 2112),
                                        (300, 200, 8, 264), (513, 2304, 8, 2304), (130, 1152, 64, 1152)])
def test_lora_rowdot_matches_fp32(M, K, R, ldx, monkeypatch):
    """u = s x A^T on the wave-per-16-rows MFMA kernel (default) against fp32, with X a strided column slice
    of a wider row (the augmented-K buffer), ragged row counts, K not a multiple of 32 (200: the masked tail
    chunk) and every rank-tile count (R 8 / 16 / 32 / 64)."""
    from mobilefinetuner_amd._ext import native
    C = native()
    g = torch.Generator(device=DEV).manual_seed(11)
    xbuf = (torch.randn(M, ldx, device=DEV, generator=g) * 0.5).bfloat16()
    x = xbuf[:, :K]
    A = (torch.randn(R, K, device=DEV, generator=g) * 0.05).bfloat16()
    u = torch.empty(M, R, device=DEV, dtype=torch.bfloat16)
    C.lora_rowdot(x, A, u, 1.5, 0.0, 0, None)
    ref = 1.5 * x.float() @ A.float().t()
    _close(u, ref, 0.02, 0.01, msg="rowdot")
