"""gemm8 variant A/B on the NT shapes: variant 0 (the default: LATE order -- s_barrier then lgkmcnt(0), B
fragments first -- with B0 fragment reuse), 2 (early: lgkmcnt(0) then s_barrier, no reuse), 3 (LATE without the B0
reuse) vs hipBLASLt (torch.mm).  Each variant is checked against an fp32 reference first; interleaved rounds, min
over rounds.

usage: PYTHONPATH=. python scripts/bench_g8late.py [--iters 10] [--rounds 4] [--variants 2,3,0]
"""
import argparse

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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--variants", default="2,0")
    a = ap.parse_args()
    C = native()
    vs = [int(v) for v in a.variants.split(",")]
    labels = {0: "gemm8", 2: "g8-early", 3: "g8-nokeepb", 4: "g8-4ph"}
    shapes = [("gpt2 qkv fwd", 131072, 768, 2304), ("gpt2 proj fwd", 131072, 768, 768),
              ("gpt2 fc fwd", 131072, 768, 3072), ("gpt2 mproj fwd", 131072, 3072, 768),
              ("gpt2 lm_head", 32768, 768, 50304), ("xl qkv fwd", 8192, 1600, 4800), ("xl fc fwd", 8192, 1600, 6400),
              ("gemma gate|up", 131072, 640, 4096), ("8192^3", 8192, 8192, 8192)]
    for name, M, K, N in shapes:
        x = ((torch.rand(M, K, device="cuda") * 2 - 1)).bfloat16()
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
        ref = None
        if M * N <= 8192 * 8192:
            ref = x.float() @ w.float().t()
        for v in vs:
            C.gemm8_set_stream(v)
            y = C.gemm_t(x, w, False, False, 0)[0]
            if ref is not None:
                err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                assert err < 1e-2, (name, v, err)
        del ref
        fl = 2.0 * M * N * K
        res = {v: [] for v in vs}
        res["lt"] = []
        for _ in range(a.rounds):
            for v in vs:
                C.gemm8_set_stream(v)
                res[v].append(timeit(lambda: C.gemm_t(x, w, False, False, 0), a.iters))
            res["lt"].append(timeit(lambda: torch.mm(x, w.t()), a.iters))
        line = f"{name:14s} M={M:6d} K={K:5d} N={N:6d} |"
        for k, lab in [(v, labels[v]) for v in vs] + [("lt", "hipBLASLt")]:
            t = min(res[k])
            line += f" {lab} {t:8.1f} us {fl / t / 1e6:6.0f} TF |"
        print(line, flush=True)
        del x, w
        torch.cuda.empty_cache()
    C.gemm8_set_stream(0)


if __name__ == "__main__":
    main()
