"""Run gemm8 launches per layout at a fixed shape (for rocprofv3 --pmc counter passes).
usage: python scripts/diag/gemm_pmc_probe.py [nt,nn,tn]"""
import sys
import torch
sys.path.insert(0, ".")
from mobilefinetuner_amd._ext import native

C = native()
which = (sys.argv[1] if len(sys.argv) > 1 else "nt,nn").split(",")
M, K, N = 65536, 3072, 768
x = torch.randn(M, K, device="cuda").bfloat16()
w_nt = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
w_nn = (torch.randn(K, N, device="cuda") * 0.05).bfloat16()
dy = torch.randn(M, N, device="cuda").bfloat16()
dw = torch.zeros(N, K, device="cuda")
for _ in range(3):
    if "nt" in which:
        C.gemm_t(x, w_nt, False, False, 0)
    if "nn" in which:
        C.gemm_t(x, w_nn, False, True, 0)
    if "tn" in which:
        C.gemm_t(dy, x, True, True, 4, out=dw)   # dW[768, 3072] += dy^T x over 65536 tokens
torch.cuda.synchronize()
