"""Weight-gradient GEMMs (dW[N, K] += dy^T x, fp32 accumulate into the flat grad buffer) and the
plain NT forwards on the GPT-2 small / XL training shapes: gemm8 (split-K from gemm8_pick_ksplit)
vs hipBLASLt (torch.mm, bf16 out -- a lower bound on its fp32-accumulate cost).  Each gemm8 result
is checked against an fp32 reference first.  Interleaved rounds, min over rounds.

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
    wg = [("gpt2 qkv", 65536, 2304, 768), ("gpt2 proj", 65536, 768, 768), ("gpt2 fc", 65536, 3072, 768),
          ("gpt2 mproj", 65536, 768, 3072), ("xl qkv", 8192, 4800, 1600), ("xl proj", 8192, 1600, 1600),
          ("xl fc", 8192, 6400, 1600), ("xl mproj", 8192, 1600, 6400)]
    for name, M, N, K in wg:
        dy = (torch.randn(M, N, device="cuda") * 0.1).bfloat16()
        x = torch.randn(M, K, device="cuda").bfloat16()
        ref = dy.float().t() @ x.float()
        buf = torch.zeros(N, K, device="cuda")
        C.gemm_t(dy, x, True, True, F32ACC, alpha=1.0, out=buf)
        err = ((buf - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-2, (name, err)
        fl = 2.0 * M * N * K
        g8, lt = [], []
        for _ in range(a.rounds):
            g8.append(timeit(lambda: C.gemm_t(dy, x, True, True, F32ACC, alpha=1.0, out=buf), a.iters))
            lt.append(timeit(lambda: torch.mm(dy.t(), x), a.iters))
        ks = C.gemm8_pick_ksplit(N, K, M) if hasattr(C, "gemm8_pick_ksplit") else -1
        print(f"wgrad {name:10s} tokens={M:6d} N={N:5d} K={K:5d} ks={ks:2d} | gemm8 {min(g8):8.1f} us "
              f"{fl / min(g8) / 1e6:6.0f} TF | hipBLASLt(bf16 out) {min(lt):8.1f} us {fl / min(lt) / 1e6:6.0f} TF "
              f"| err {err:.1e}", flush=True)
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
