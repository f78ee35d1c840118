"""gemm8 / gemm4 / hipBLASLt launches at 8192^3 NT (for rocprofv3 --pmc counter passes)."""
import sys
import torch
sys.path.insert(0, ".")
from mobilefinetuner_amd._ext import native

C = native()
M = N = K = 8192
x = ((torch.rand(M, K, device="cuda") * 2 - 1)).bfloat16()
w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
for _ in range(3):
    C.gemm_t(x, w, False, False, 0, impl=0)
    C.gemm_t(x, w, False, False, 0, impl=2)
    torch.mm(x, w.t())
torch.cuda.synchronize()
