import torch
def timeit(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters
M = 32768
for N, K0 in [(2304, 768), (768, 768)]:
    for K in (K0, K0 + 8, K0 + 16, K0 + 32, K0 + 64):
        x = torch.randn(M, K, device="cuda").bfloat16(); w = torch.randn(N, K, device="cuda").bfloat16(); b = torch.randn(N, device="cuda").bfloat16()
        print(f"fwd N={N} K={K}: {timeit(lambda: torch.addmm(b, x, w.t())):.1f} us", flush=True)
    for Np in (K0, K0 + 8, K0 + 16, K0 + 64):
        dy = torch.randn(M, N, device="cuda").bfloat16(); w = torch.randn(N, Np, device="cuda").bfloat16()
        print(f"bwd dx N={N} -> {Np}: {timeit(lambda: torch.mm(dy, w)):.1f} us", flush=True)
