"""gemm4 / gemm8 / hipBLASLt launches (NT, no epilogue) at one shape, for rocprofv3 --pmc passes.
usage: python scripts/probes/gemm4_pmc_probe.py M N K"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mobilefinetuner_amd._ext import native  # noqa: E402

C = native()
M, N, K = (int(v) for v in sys.argv[1:4])
x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    C.gemm_t(x, w, False, False, 0, None, None, 1.0, y, None, None, 4)
    C.gemm_t(x, w, False, False, 0, None, None, 1.0, y, None, None, 0)
    torch.mm(x, w.t(), out=y)
torch.cuda.synchronize()
