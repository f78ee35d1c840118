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


@pytest.mark.parametrize("M,N", [(300, 768), (1000, 2304), (77, 264), (130, 520), (4096, 768), (1000, 256), (77, 200)])
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


def test_lora_merge_kernel_matches_adapter_forward():
    """K10: Linear.merge_lora on GPU runs the lora_merge kernel; merged W x == adapter forward, and
    unmerge restores W (reference graph/test_lora_correctness.cpp:101-187)."""
    from mobilefinetuner_amd.models.layers import Linear
    torch.manual_seed(1)
    K, N = 256, 384
    lin = Linear(K, N, device=DEV)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(N, K) * 0.05)
        lin.bias.copy_(torch.randn(N) * 0.1)
    for c0, n in ((0, 128), (128, 256)):
        A, B = lin.add_lora(c0, n, 8, 2.0, torch.randn(8, K) * 0.05, name=f"m{c0}")
        with torch.no_grad():
            B.copy_(torch.randn_like(B) * 0.05)
        A.shadow, B.shadow = A.detach().bfloat16(), B.detach().bfloat16()  # what FlatParams provides
    x = torch.randn(64, K, device=DEV).bfloat16()
    with torch.no_grad():
        y_adapter = lin(x).float()
        w0 = lin.weight.detach().float().clone()
        lin.merge_lora(1.0)
        lin.lora_enabled = False
        y_merged = lin(x).float()
        ref = w0.clone()
        for sl in lin.lora_slices:
            ref[sl.col0:sl.col0 + sl.ncols] += 2.0 * sl.B.float().t() @ sl.A.float()
        _close(lin.weight, ref, 2e-3, 1e-2, msg="merged W")
        _close(y_merged, y_adapter, 0.03, 0.01, msg="merged forward")
        lin.merge_lora(-1.0)
        _close(lin.weight, w0, 2e-3, 1e-2, msg="unmerge")
