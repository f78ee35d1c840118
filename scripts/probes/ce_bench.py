"""Time the fused LM-head CE pieces against plain gemm8 / hipBLASLt GEMMs of the same shapes.
usage: python scripts/probes/ce_bench.py [M K Vpad V]"""
import sys

import torch

from mobilefinetuner_amd._ext import native


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    M, K, Vpad, V = (int(x) for x in sys.argv[1:5]) if len(sys.argv) > 4 else (65536, 768, 50304, 50257)
    C = native()
    h = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    W = (torch.randn(Vpad, K, device="cuda") / K ** 0.5).bfloat16()
    labels = torch.randint(0, V, (M,), device="cuda")
    E = torch.empty(M, Vpad, device="cuda", dtype=torch.bfloat16)
    loss = torch.empty(M, device="cuda")
    dh = torch.empty_like(h)
    scale = torch.full((1,), 1.0 / M, device="cuda")
    t_fwd = timeit(lambda: C.lm_head_ce(h, W, labels, V, E, loss, scale, 1.0, None, False))
    t_nll = timeit(lambda: C.lm_head_ce(h, W, labels, V, None, loss, scale, 1.0, None, False))
    t_all = timeit(lambda: C.lm_head_ce(h, W, labels, V, E, loss, scale, 1.0, dh, False))
    t_mat = timeit(lambda: C.lm_head_ce(h, W, labels, V, E, loss, scale, 1.0, dh, True))
    t_g8_nt = timeit(lambda: C.gemm_t(h, W, False, False, 0, None, None, 1.0, E, None, None))
    t_g8_nn = timeit(lambda: C.gemm_t(E, W, False, True, 0, None, None, 1.0, dh, None, None))
    t_lt_nt = timeit(lambda: torch.mm(h, W.t(), out=E))
    t_xent = timeit(lambda: C.xent_fwd_bwd(E, labels, loss, V, scale, 1.0, True))
    fl = 2.0 * M * K * Vpad
    print(f"M={M} K={K} Vpad={Vpad}")
    print(f"fused fwd (CE_FWD + finalize)      {t_fwd:8.3f} ms  {fl / t_fwd / 1e9:7.1f} TF/s")
    print(f"fused fwd, no E stores (NLL only)  {t_nll:8.3f} ms  {fl / t_nll / 1e9:7.1f} TF/s")
    print(f"fused fwd + dgrad (CE_DGRAD)       {t_all:8.3f} ms  (dgrad ~ {t_all - t_fwd:.3f} ms, {fl / (t_all - t_fwd) / 1e9:.1f} TF/s)")
    print(f"fused fwd + materialize + NN       {t_mat:8.3f} ms")
    print(f"gemm8 NT plain                     {t_g8_nt:8.3f} ms  {fl / t_g8_nt / 1e9:7.1f} TF/s")
    print(f"gemm8 NN plain                     {t_g8_nn:8.3f} ms  {fl / t_g8_nn / 1e9:7.1f} TF/s")
    print(f"torch.mm NT (hipBLASLt)            {t_lt_nt:8.3f} ms  {fl / t_lt_nt / 1e9:7.1f} TF/s")
    print(f"xent_fwd_bwd                       {t_xent:8.3f} ms")
    print(f"old path (mm + xent + gemm8 NN)    {t_lt_nt + t_xent + t_g8_nn:8.3f} ms   new {t_all:.3f} ms")


if __name__ == "__main__":
    main()
