"""Micro-benchmark of the LoRA HIP kernels at the GPT-2 bench shapes (M = B*S = 8192 rows).

Prints one line per kernel/shape: average µs over `iters` launches and the effective HBM GB/s
(bytes of the streamed operand), so regressions show up without a whole-model profile.
usage: python scripts/bench_lora_kernels.py [--M 8192] [--iters 200]
"""
import argparse

import torch

from mobilefinetuner_amd._ext import native


def timeit(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--R", type=int, default=8)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--Ks", default="768,2304,3072")
    ap.add_argument("--ps", default="0.0,0.1")
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda")
    M, R = a.M, a.R
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    for K in [int(v) for v in a.Ks.split(",")]:
        X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        Wt = torch.randn(R, K, device=dev, dtype=torch.bfloat16)
        U = torch.empty(M, R, device=dev, dtype=torch.bfloat16)
        Y = torch.randn(M, R, device=dev, dtype=torch.bfloat16)
        out = torch.zeros(R, K, device=dev, dtype=torch.float32)
        gb = M * K * 2 / 1e9
        for p in [float(v) for v in a.ps.split(",")]:
            t = timeit(lambda: C.lora_rowdot(X, Wt, U, 1.0, p, 7, ctr), a.iters)
            print(f"rowdot  K={K:5d} R={R} p={p}: {t:7.1f} us  {gb / t * 1e6:7.0f} GB/s")
            t = timeit(lambda: C.lora_update(X, Y, Wt, X, 1.0, p, 7, ctr), a.iters)
            print(f"update  K={K:5d} R={R} p={p}: {t:7.1f} us  {2 * gb / t * 1e6:7.0f} GB/s")
            t = timeit(lambda: C.lora_wgrad(X, Y, out, 1, K, 1.0, p, 7, ctr), a.iters)
            print(f"wgrad   K={K:5d} R={R} p={p}: {t:7.1f} us  {gb / t * 1e6:7.0f} GB/s")
        ref = (Y.float().t() @ X.float())
        out.zero_()
        C.lora_wgrad(X, Y, out, 1, K, 1.0, 0.0, 0, None)
        err = (out - ref).abs().max().item() / ref.abs().max().item()
        print(f"wgrad   K={K:5d} rel err {err:.2e}")


if __name__ == "__main__":
    main()
