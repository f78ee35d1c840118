"""gemm8 in every operand layout (NT forward, NN data-grad, TN split-K weight-grad) at the
production M = 65536 GPT-2 and Gemma-3 shapes, against an fp32 PyTorch reference (relative
tolerances).  N = 640 / 8 / 120 exercise the N-tail path that skips the (A*, B1) quadrants."""
import pytest
import torch

pytestmark = pytest.mark.gpu

EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_DGELU, EPI_F32ACC, EPI_LORA = 0, 1, 2, 3, 4, 5
EPI_BIAS_GELU_D, EPI_MUL_AUX = 9, 10


def C():
    from mobilefinetuner_amd._ext import native
    return native()


def rnd(*shape, s=1.0, gen=None):
    return ((torch.rand(*shape, device="cuda", generator=gen) * 2 - 1) * s).bfloat16()


def relerr(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp(min=1e-12)).item()


@pytest.mark.parametrize("M,K,N", [(65536, 768, 2304), (65536, 3072, 768), (65536, 768, 50304), (1000, 832, 776),
                                   (300, 64, 8), (65536, 1024, 640), (777, 128, 120)])
def test_gemm8_nt(M, K, N):
    g = torch.Generator(device="cuda").manual_seed(1)
    x, w, b = rnd(M, K, gen=g), rnd(N, K, s=0.05, gen=g), rnd(N, s=0.5, gen=g)
    y = C().gemm_t(x, w, False, False, EPI_BIAS, bias=b)[0]
    ref = x.float() @ w.float().t() + b.float()
    assert relerr(y, ref) < 1e-2


@pytest.mark.parametrize("M,K,N", [(65536, 3072, 768), (65536, 768, 3072), (65536, 2304, 768), (8192, 50304, 768),
                                   (1000, 832, 776), (65536, 2048, 640), (8192, 262144, 640)])
def test_gemm8_nn(M, K, N):
    g = torch.Generator(device="cuda").manual_seed(2)
    dy, w = rnd(M, K, gen=g), rnd(K, N, s=0.05, gen=g)
    y = C().gemm_t(dy, w, False, True, EPI_NONE)[0]
    assert relerr(y, dy.float() @ w.float()) < 1e-2


def test_gemm8_nn_dgelu_and_lora():
    g = torch.Generator(device="cuda").manual_seed(3)
    M, K, N = 65536, 768, 3072
    dy, w, pre = rnd(M, K, gen=g), rnd(K, N, s=0.05, gen=g), rnd(M, N, s=3, gen=g)
    y = C().gemm_t(dy, w, False, True, EPI_DGELU, aux=pre)[0]
    pf = pre.float()
    t = torch.tanh(0.7978845608 * (pf + 0.044715 * pf ** 3))
    dg = 0.5 * (1 + t) + 0.5 * pf * (1 - t ** 2) * 0.7978845608 * (1 + 3 * 0.044715 * pf ** 2)
    assert relerr(y, (dy.float() @ w.float()) * dg) < 1e-2
    u, lw = rnd(M, 16, gen=g), rnd(16, N, s=0.1, gen=g)
    y2 = C().gemm_t(dy, w, False, True, EPI_LORA, lora_u=u, lora_w=lw)[0]
    assert relerr(y2, dy.float() @ w.float() + u.float() @ lw.float()) < 1e-2


@pytest.mark.parametrize("T,P,Q", [(65536, 2304, 768), (65536, 768, 3072), (65536, 3072, 768), (4096, 776, 136),
                                   (65536, 768, 50304), (65536, 2048, 640)])
def test_gemm8_tn_wgrad_splitk(T, P, Q):
    """dW[P, Q] += dy[T, P]^T x[T, Q] in fp32 (split-K slabs + deterministic reduce)."""
    g = torch.Generator(device="cuda").manual_seed(4)
    dy, x = rnd(T, P, gen=g), rnd(T, Q, gen=g)
    base = torch.randn(P, Q, device="cuda", generator=g)
    out = base.clone()
    C().gemm_t(dy, x, True, True, EPI_F32ACC, alpha=0.5, out=out)
    ref = base + 0.5 * (dy.float().t() @ x.float())
    assert relerr(out - base, ref - base) < 2e-3
    out2 = base.clone()
    C().gemm_t(dy, x, True, True, EPI_F32ACC, alpha=0.5, out=out2)
    assert torch.equal(out, out2), "split-K weight gradient must be deterministic"


def _gelu_and_grad(pf):
    t = torch.tanh(0.7978845608 * (pf + 0.044715 * pf ** 3))
    return 0.5 * pf * (1 + t), 0.5 * (1 + t) + 0.5 * pf * (1 - t ** 2) * 0.7978845608 * (1 + 3 * 0.044715 * pf ** 2)


def test_gemm8_gelu_mlp_epilogues():
    """fc forward: GELU(xW^T + b) and GELU'(xW^T + b) (aux) from one epilogue; mlp_proj data-grad:
    (dy W) * aux -- at the GPT-2 MLP shapes."""
    g = torch.Generator(device="cuda").manual_seed(5)
    M, K, N = 65536, 768, 3072
    x, w, b = rnd(M, K, gen=g), rnd(N, K, s=0.1, gen=g), rnd(N, s=0.5, gen=g)
    h, d = C().gemm_t(x, w, False, False, EPI_BIAS_GELU_D, bias=b)
    pre = x.float() @ w.float().t() + b.float()
    gl, dg = _gelu_and_grad(pre)
    assert relerr(h, gl) < 1e-2 and relerr(d, dg) < 1e-2
    dy, w2 = rnd(M, K, gen=g), rnd(K, N, s=0.05, gen=g)
    y = C().gemm_t(dy, w2, False, True, EPI_MUL_AUX, aux=d)[0]
    assert relerr(y, (dy.float() @ w2.float()) * d.float()) < 1e-2


def test_gemm8_lora_epilogue_n_tail():
    """NT + fused rank-16 LoRA update at Gemma-3's d_model 640 output width (3rd column tile half empty)."""
    g = torch.Generator(device="cuda").manual_seed(6)
    M, K, N = 65536, 1024, 640
    x, w = rnd(M, K, gen=g), rnd(N, K, s=0.05, gen=g)
    u, lw = rnd(M, 16, gen=g), rnd(16, N, s=0.1, gen=g)
    y = C().gemm_t(x, w, False, False, EPI_LORA, lora_u=u, lora_w=lw)[0]
    assert relerr(y, x.float() @ w.float().t() + u.float() @ lw.float()) < 1e-2
