"""LoRA weight-gradient kernels (lora.hip lora_wgrad: MFMA rank reduction for R % 8 == 0, R <= 32
without dropout; VALU kernel otherwise) against an fp32 PyTorch reference:
out[k, r] += scale * sum_m X[m, k] Y[m, r] -- dA = v^T x and dB = u^T dy of the LoRA backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("M,K,R", [(4096 + 17, 640, 8), (65536, 768, 8), (3000, 1024, 16), (5000, 2048, 24),
                                   (4096, 2304, 32), (1000, 136, 8), (2048, 704, 4), (777, 768, 12)])
def test_lora_wgrad_matches_fp32(M, K, R):
    from mobilefinetuner_amd._ext import native
    C = native()
    g = torch.Generator(device=DEV).manual_seed(M + K + R)
    # Y as a column slice of a wider row buffer (the augmented-K input u lives in columns K.. of xa)
    X = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    wide = torch.randn(M, R + 24, device=DEV, generator=g).bfloat16()
    Y = wide[:, 8:8 + R]
    out = torch.randn(R, K, device=DEV, generator=g)  # accumulated into: dA layout [r, K]
    ref = out + 0.5 * (X.float().t() @ Y.float()).t()
    C.lora_wgrad(X, Y, out, 1, K, 0.5, 0.0, 0, None)
    torch.cuda.synchronize()
    assert _rel(out, ref) < 2e-5, _rel(out, ref)


def test_lora_wgrad_multi_segments():
    from mobilefinetuner_amd._ext import native
    C = native()
    M, K = 65536, 640
    g = torch.Generator(device=DEV).manual_seed(3)
    X = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    Y = torch.randn(M, 24, device=DEV, generator=g).bfloat16()
    outs = [torch.zeros(8, K, device=DEV) for _ in range(3)]
    C.lora_wgrad_multi(X, Y, outs, 1.0)
    torch.cuda.synchronize()
    full = (X.float().t() @ Y.float()).t()
    for z in range(3):
        assert _rel(outs[z], full[8 * z:8 * z + 8]) < 2e-5
