"""K sweep of the plain NT GEMM at fixed M x N: gemm8 (default / streaming form) vs hipBLASLt.

Fits t = a + b * (K / 64) per tile round (tiles / CUs): b = time per 64-deep K-tile of the main loop,
a = the per-tile cost outside it (prologue fill, epilogue, relaunch).  Separates main-loop efficiency
from the per-tile overhead that dominates at GPT-2's K = 768.

usage: PYTHONPATH=. python scripts/bench_gemm_ksweep.py [--M 65536] [--N 3072] [--iters 10] [--rounds 3]
"""
import argparse

import numpy as np
import torch

from mobilefinetuner_amd._ext import native


def timeit(fn, iters):
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
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--N", type=int, default=3072)
    ap.add_argument("--Ks", default="256,512,768,1536,3072,6144")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    C = native()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    M, N = a.M, a.N
    rounds_per = (M // 256) * ((N + 255) // 256) / cus
    Ks = [int(k) for k in a.Ks.split(",")]
    res = {"gemm8": [], "gemm8-stream": [], "hipBLASLt": []}
    for K in Ks:
        x = ((torch.rand(M, K, device="cuda") * 2 - 1)).bfloat16()
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
        t = {k: [] for k in res}
        for _ in range(a.rounds):
            for v, lab in ((0, "gemm8"), (1, "gemm8-stream")):
                C.gemm8_set_stream(v)
                t[lab].append(timeit(lambda: C.gemm_t(x, w, False, False, 0), a.iters))
            t["hipBLASLt"].append(timeit(lambda: torch.mm(x, w.t()), a.iters))
        C.gemm8_set_stream(0)
        fl = 2.0 * M * N * K
        line = f"M={M} N={N} K={K:5d} |"
        for k in res:
            us = min(t[k])
            res[k].append(us)
            line += f" {k} {us:8.1f} us {fl / us / 1e6:6.0f} TF |"
        print(line, flush=True)
        del x, w
        torch.cuda.empty_cache()
    kt = np.array(Ks) / 64.0
    for k, v in res.items():
        per_round = np.array(v) / rounds_per
        b, a0 = np.polyfit(kt, per_round, 1)
        # ideal per K-tile: 256x256x64 MACs at the 2.5 PF dense peak
        ideal = 2.0 * 256 * 256 * 64 / (2.5e15 / cus) * 1e6
        print(f"{k:13s}: per tile round a = {a0:6.2f} us + b = {b:5.3f} us per K-tile "
              f"(MFMA-bound ideal {ideal:5.3f} us at 2.5 PF -> main loop {ideal / b * 100:4.1f} %)", flush=True)


if __name__ == "__main__":
    main()
