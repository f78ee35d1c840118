"""gemm8 NT vs hipBLASLt (torch.mm) at the fc-forward shape (M 65536, K 768, N 3072), for
rocprofv3 --pmc counter passes.  usage: python scripts/diag/nt_pmc_probe.py"""
import sys
import torch
sys.path.insert(0, ".")
from mobilefinetuner_amd._ext import native

C = native()
M, K, N = 65536, 768, 3072
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
for _ in range(3):
    C.gemm_t(x, w, False, False, 0)
    torch.mm(x, w.t())
torch.cuda.synchronize()
