"""LM-head GEMM shapes (GPT-2: 8192 x 768 x 50304): torch.mm (hipBLASLt heuristic) vs the autotuned
hipBLASLt binding vs gemm8, forward logits and data-gradient."""
import torch

from mobilefinetuner_amd._ext import native


def timeit(fn, iters=10):
    for _ in range(3):
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
M, K, V = 8192, 768, 50304
h = (torch.rand(M, K, device="cuda") - 0.5).bfloat16()
w = ((torch.rand(V, K, device="cuda") - 0.5) * 0.1).bfloat16()
wt = w.t().contiguous()
dl = ((torch.rand(M, V, device="cuda") - 0.5) * 1e-3).bfloat16()
fl = 2.0 * M * K * V
for name, fn in [("fwd torch.mm", lambda: torch.mm(h, w.t())), ("fwd lt_linear", lambda: C.lt_linear(h, w, None)),
                 ("fwd gemm8", lambda: C.gemm(h, w, False, 0, None, None, 1.0, 8, None)),
                 ("dx torch.mm", lambda: torch.mm(dl, w)), ("dx lt_mm_dx", lambda: C.lt_mm_dx(dl, w)),
                 ("dx gemm8(NT, W^T copy)", lambda: C.gemm(dl, wt, False, 0, None, None, 1.0, 8, None))]:
    t = timeit(fn)
    print(f"{name:24s} {t:8.1f} us  {fl / t / 1e6:6.0f} TF", flush=True)
