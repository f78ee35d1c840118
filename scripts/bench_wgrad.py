"""Weight-gradient GEMMs (dW[N, K] += dy^T x, fp32 accumulate into the flat grad buffer) and the
plain NT forwards on the GPT-2 small / XL training shapes: the 4-wave TN kernel (gemm4_tn, split from
gemm4_tn_pick_ksplit) vs the 8-wave gemm8 (split from gemm8_pick_ksplit) vs torch.mm (bf16 out -- a
lower bound on an fp32-accumulate cost).  Each result is checked against an fp32 reference first.
Interleaved rounds, min over rounds.

usage: PYTHONPATH=. python scripts/bench_wgrad.py [--iters 10] [--rounds 3]
"""
import argparse

import torch

from mobilefinetuner_amd._ext import native

NONE, F32ACC = 0, 4


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
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    C = native()
    T, TX = 131072, 32768  # bench.py gpt2-full (1024 x 128) and gpt2-xl (256 x 128) tokens per step
    wg = [("gpt2 qkv", T, 2304, 768), ("gpt2 proj", T, 768, 768), ("gpt2 fc", T, 3072, 768),
          ("gpt2 mproj", T, 768, 3072), ("xl qkv", TX, 4800, 1600), ("xl proj", TX, 1600, 1600),
          ("xl fc", TX, 6400, 1600), ("xl mproj", TX, 1600, 6400)]
    for name, M, N, K in wg:
        dy = (torch.randn(M, N, device="cuda") * 0.1).bfloat16()
        x = torch.randn(M, K, device="cuda").bfloat16()
        ref = dy.float().t() @ x.float()
        err = {}
        for impl in (4, 0):
            buf = torch.zeros(N, K, device="cuda")
            C.gemm_t(dy, x, True, True, F32ACC, None, None, 1.0, buf, None, None, impl)
            err[impl] = ((buf - ref).abs().max() / ref.abs().max()).item()
            assert err[impl] < 1e-4, (name, impl, err[impl])
        fl = 2.0 * M * N * K
        g4, g8, lt = [], [], []
        for _ in range(a.rounds):
            g4.append(timeit(lambda: C.gemm_t(dy, x, True, True, F32ACC, None, None, 1.0, buf, None, None, 4), a.iters))
            g8.append(timeit(lambda: C.gemm_t(dy, x, True, True, F32ACC, None, None, 1.0, buf, None, None, 0), a.iters))
            lt.append(timeit(lambda: torch.mm(dy.t(), x), a.iters))
        print(f"wgrad {name:10s} tokens={M:6d} N={N:5d} K={K:5d} | gemm4_tn {min(g4):7.1f} us {fl / min(g4) / 1e6:5.0f} TF"
              f" | gemm8 {min(g8):7.1f} us {fl / min(g8) / 1e6:5.0f} TF | torch.mm(bf16 out) {min(lt):7.1f} us "
              f"{fl / min(lt) / 1e6:5.0f} TF | err {err[4]:.1e} / {err[0]:.1e}", flush=True)
        del dy, x, ref, buf
    nt = [("xl qkv fwd", 8192, 1600, 4800), ("xl proj fwd", 8192, 1600, 1600), ("xl fc fwd", 8192, 1600, 6400),
          ("xl mproj fwd", 8192, 6400, 1600)]
    for name, M, K, N in nt:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        y = C.gemm_t(x, w, False, False, NONE)[0]
        err = ((y.float() - x.float() @ w.float().t()).abs().max() / y.float().abs().max()).item()
        fl = 2.0 * M * N * K
        g8, lt = [], []
        for _ in range(a.rounds):
            g8.append(timeit(lambda: C.gemm_t(x, w, False, False, NONE), a.iters))
            lt.append(timeit(lambda: torch.mm(x, w.t()), a.iters))
        print(f"nt    {name:12s} M={M:6d} K={K:5d} N={N:5d} | gemm8 {min(g8):8.1f} us {fl / min(g8) / 1e6:6.0f} TF | "
              f"hipBLASLt {min(lt):8.1f} us {fl / min(lt) / 1e6:6.0f} TF | err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
