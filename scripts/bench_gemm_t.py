"""gemm8 (every operand layout, csrc/kernels/gemm8.hip) vs hipBLASLt (torch.mm) on the GPT-2 / Gemma
training-step GEMM shapes at M = 65536 tokens.  Interleaved rounds in one process, random data
(CDNA HIP guide §5.4 rules 24/25); prints µs, TFLOP/s and max error vs an fp32 reference.

usage: PYTHONPATH=. python scripts/bench_gemm_t.py [--M 65536] [--iters 20] [--only NAME]
"""
import argparse

import torch

from mobilefinetuner_amd._ext import native

EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_DGELU, EPI_F32ACC = 0, 1, 2, 3, 4


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def rnd(*shape, s=1.0):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * s).bfloat16()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    C = native()
    M = a.M
    # (name, kind, K, N): kind nt = x[M,K] W[N,K]^T ; nn = dy[M,K] W[K,N] ; tn = dW[K?]: see below
    shapes = [
        ("qkv fwd (aug K)", "nt", 832, 2304), ("proj fwd (aug K)", "nt", 832, 768), ("fc fwd", "nt", 768, 3072),
        ("mlp_proj fwd", "nt", 3072, 768), ("lm_head fwd", "nt", 768, 50304),
        ("mlp_proj dx", "nn", 768, 3072), ("fc dx", "nn", 3072, 768), ("qkv dx", "nn", 2304, 768),
        ("proj dx", "nn", 768, 768), ("lm_head dx", "nn", 50304, 768),
        ("qkv dW", "tn", 2304, 768), ("proj dW", "tn", 768, 768), ("fc dW", "tn", 3072, 768),
        ("mlp_proj dW", "tn", 768, 3072),
        ("gemma qkv fwd", "nt", 640, 1536), ("gemma gate|up fwd", "nt", 640, 4096), ("gemma down fwd", "nt", 2048, 640),
        ("gemma lm_head fwd", "nt", 640, 262144), ("gemma lm_head dx", "nn", 262144, 640),
    ]
    for name, kind, K, N in shapes:
        if a.only and a.only not in name:
            continue
        Mr = M if "lm_head" not in name or "gemma" not in name else M // 8  # 262144-wide: one chunk
        if kind == "tn":
            # dW[P, Q] += dy[M, P]^T x[M, Q]: P = out features (K here), Q = in features (N)
            dy, x = rnd(Mr, K), rnd(Mr, N)
            out = torch.zeros(K, N, device="cuda")
            ref = dy.float().t() @ x.float()
            C.gemm_t(dy, x, True, True, EPI_F32ACC, out=out)
            err = ((out - ref).abs().max() / ref.abs().max()).item()
            fl = 2.0 * Mr * K * N
            t = timeit(lambda: C.gemm_t(dy, x, True, True, EPI_F32ACC, out=out), a.iters)
            tl = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32), a.iters)
        else:
            x = rnd(Mr, K)
            w = rnd(N, K, s=0.05) if kind == "nt" else rnd(K, N, s=0.05)
            ref = x.float() @ (w.float().t() if kind == "nt" else w.float())
            y = C.gemm_t(x, w, False, kind == "nn", EPI_NONE)[0]
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            del ref
            fl = 2.0 * Mr * K * N
            t = timeit(lambda: C.gemm_t(x, w, False, kind == "nn", EPI_NONE), a.iters)
            tl = timeit(lambda: torch.mm(x, w.t() if kind == "nt" else w), a.iters)
        print(f"{name:20s} {kind} M={Mr:6d} K={K:6d} N={N:6d} | gemm8 {t:8.1f} us {fl / t / 1e6:6.0f} TF err {err:.1e}"
              f" | hipBLASLt {tl:8.1f} us {fl / tl / 1e6:6.0f} TF | ratio {tl / t:.2f}", flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
