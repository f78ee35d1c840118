"""lora_rowdot (u = s x A^T, the LoRA input projection) at the GPT-2 / Gemma-3 training shapes; run once
with MFT_ROWDOT_V1=1 (split-K-over-waves form) and once without (row-per-wave form) to A/B.

usage: PYTHONPATH=. [MFT_ROWDOT_V1=1] python scripts/bench_rowdot.py
"""
import os

import torch

from mobilefinetuner_amd._ext import native


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


C = native()
tag = "v1" if os.environ.get("MFT_ROWDOT_V1") == "1" else "w"
for name, M, K, ldx, R in [("gpt2 qkv-in", 131072, 768, 832, 8), ("gpt2 proj-in", 131072, 768, 832, 8),
                           ("gemma q|k|v-in", 65536, 640, 704, 24), ("gemma o-in", 65536, 1024, 1088, 8),
                           ("gemma down-in", 65536, 2048, 2112, 8)]:
    xb = torch.randn(M, ldx, device="cuda").bfloat16()
    x = xb[:, :K]
    A = (torch.randn(R, K, device="cuda") * 0.05).bfloat16()
    u = torch.empty(M, R, device="cuda", dtype=torch.bfloat16)
    t = min(timeit(lambda: C.lora_rowdot(x, A, u, 1.0, 0.0, 0, None)) for _ in range(3))
    print(f"rowdot[{tag}] {name:15s} M={M} K={K} R={R}: {t:7.1f} us  {M * K * 2 / t / 1e6:5.2f} TB/s", flush=True)
