"""gemm_s debug: error map of a small product (which rows / columns / K-tiles go wrong)."""
import torch
from mobilefinetuner_amd._ext import native
C = native()
for (M, N, K) in [(64, 64, 64), (64, 64, 128), (64, 64, 512), (64, 64, 1024), (128, 128, 512), (300, 264, 128)]:
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    C.gemm_t(x, w, False, False, 0, None, None, 1.0, y, None, None, 5)
    ref = x.float() @ w.float().t()
    d = (y.float() - ref).abs()
    bad = d > 0.05 * ref.abs().max()
    print(M, N, K, "max err", d.max().item(), "bad", bad.sum().item(), "rows", bad.any(1).nonzero().flatten()[:10].tolist(),
          "cols", bad.any(0).nonzero().flatten()[:10].tolist(), flush=True)
    # per K-tile contribution test: only K-tile t non-zero
    if K >= 128 and M == 64:
        for t in range(K // 64):
            xz = torch.zeros_like(x); xz[:, 64 * t:64 * t + 64] = x[:, 64 * t:64 * t + 64]
            C.gemm_t(xz, w, False, False, 0, None, None, 1.0, y, None, None, 5)
            r2 = xz.float() @ w.float().t()
            print("   only K-tile", t, "err", (y.float() - r2).abs().max().item(), "ref max", r2.abs().max().item(), flush=True)
