"""Run one gemm8 launch per layout at a fixed shape (for rocprofv3 --pmc counter passes)."""
import sys
import torch
sys.path.insert(0, ".")
from mobilefinetuner_amd._ext import native

C = native()
M, K, N = 65536, 3072, 768
x = torch.randn(M, K, device="cuda").bfloat16()
w_nt = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
w_nn = (torch.randn(K, N, device="cuda") * 0.05).bfloat16()
for _ in range(3):
    C.gemm_t(x, w_nt, False, False, 0)
    C.gemm_t(x, w_nn, False, True, 0)
torch.cuda.synchronize()
