"""lora_dy (one pass over dy for v = s dy B^T and dB += s u^T dy) vs an fp32 PyTorch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"{msg} max abs err {err:.3e} > {tol:.3e}"


@pytest.mark.parametrize("M,N", [(300, 768), (1000, 2304), (77, 264), (130, 520), (4096, 768)])
def test_lora_dy_matches_fp32(M, N):
    from mobilefinetuner_amd._ext import native
    C = native()
    torch.manual_seed(0)
    ld = N + 64
    dyb = torch.randn(M, ld, device=DEV).bfloat16()
    dy = dyb[:, 16:16 + N]                      # strided column slice (as q|k|v slices of dqkv)
    B = (torch.randn(8, N, device=DEV) * 0.1).bfloat16()
    ub = torch.randn(M, 24, device=DEV).bfloat16()
    u = ub[:, 8:16]                             # appended columns of the augmented input (row stride 24)
    dB = torch.randn(8, N, device=DEV)          # accumulation semantics (grad buffer)
    dB0 = dB.clone()
    vpart = torch.empty(((N + 255) // 256) * M * 8, device=DEV)
    v = torch.empty(M, 8, device=DEV, dtype=torch.bfloat16)
    C.lora_dy(dy, B, u, dB, vpart, v, 0.5)
    torch.cuda.synchronize()
    vr = 0.5 * dy.float() @ B.float().t()
    dBr = dB0 + 0.5 * u.float().t() @ dy.float()
    _close(v, vr, 0.02, 0.01, msg="v")
    _close(dB, dBr, 1e-3 * M ** 0.5, 1e-4, msg="dB")
