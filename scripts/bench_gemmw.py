"""gemmw (256x128x32, 4 waves, 2 workgroups / CU) vs gemm8 (256x256 8-phase) vs hipBLASLt (torch.mm)
on the NT training shapes, with every epilogue checked against an fp32 reference first.
Interleaved rounds in one process, random data (CDNA HIP guide §5.4 rules 24 / 25).

usage: PYTHONPATH=. python scripts/bench_gemmw.py [--M 131072] [--iters 10] [--rounds 3] [--only NAME]
"""
import argparse

import torch

from mobilefinetuner_amd._ext import native

NONE, BIAS, BIAS_GELU, DGELU, F32ACC, LORA, BIAS_GELU_D, MUL_AUX = 0, 1, 2, 3, 4, 5, 9, 10


def rnd(*shape, s=1.0):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * s).bfloat16()


def gelu(x):
    return 0.5 * x * (1 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))


def check(C):
    """every supported epilogue of gemmw on a mid-size problem (M not a multiple of 256, N tail)."""
    M, K, N = 1000, 832, 776
    x, w = rnd(M, K), rnd(N, K, s=0.05)
    b, aux = rnd(N, s=0.1), rnd(M, N)
    ref = x.float() @ w.float().t()
    worst = 0.0

    def err(got, want):
        return ((got.float() - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()

    for impl, stream in ((0, 0), (0, 1), (1, 0)):
        C.gemm8_set_stream(stream)
        y = C.gemm_t(x, w, False, False, NONE, impl=impl)[0]
        e = err(y, ref)
        y, pre = C.gemm_t(x, w, False, False, BIAS_GELU, bias=b, impl=impl)
        e = max(e, err(pre, ref + b.float()), err(y, gelu(ref + b.float())))
        y = C.gemm_t(x, w, False, False, MUL_AUX, aux=aux, impl=impl)[0]
        e = max(e, err(y, ref * aux.float()))
        u, lw = rnd(M, 8), rnd(8, N, s=0.1)
        y = C.gemm_t(x, w, False, False, LORA, alpha=0.5, lora_u=u, lora_w=lw, impl=impl)[0]
        e = max(e, err(y, 0.5 * ref + u.float() @ lw.float()))
        out = torch.randn(M, N, device="cuda")
        want = out + 2.0 * ref
        C.gemm_t(x, w, False, False, F32ACC, alpha=2.0, out=out, impl=impl)
        e = max(e, err(out, want))
        print(f"impl {impl} stream {stream}: max relative error over the epilogues {e:.2e}", flush=True)
        worst = max(worst, e)
    # the streaming form engages from 2 tiles per CU on: a 512-tile problem, NONE / BIAS / BIAS_GELU_D
    M, K, N = 65536 + 200, 768, 2048 - 8
    x, w, b = rnd(M, K), rnd(N, K, s=0.05), rnd(N, s=0.1)
    ref = x.float() @ w.float().t()
    for stream in (0, 1):
        C.gemm8_set_stream(stream)
        y = C.gemm_t(x, w, False, False, NONE)[0]
        e1 = err(y, ref)
        y = C.gemm_t(x, w, False, False, BIAS, bias=b)[0]
        e2 = err(y, ref + b.float())
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y = C.gemm_t(x, w, False, False, BIAS_GELU_D, bias=b, aux=aux)[0]
        z = ref + b.float()
        e3 = err(y, gelu(z))
        print(f"large NT, stream {stream}: errors none {e1:.2e} bias {e2:.2e} gelu {e3:.2e}", flush=True)
        worst = max(worst, e1, e2, e3)
    del ref
    assert worst < 2e-2, worst


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
    ap.add_argument("--M", type=int, default=131072)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    C = native()
    check(C)
    shapes = [("qkv fwd (aug K)", 832, 2304, NONE), ("proj fwd (aug K)", 832, 768, NONE),
              ("fc fwd +GELU", 768, 3072, BIAS_GELU_D), ("fc fwd", 768, 3072, NONE),
              ("mlp_proj fwd", 3072, 768, NONE), ("lm_head fwd", 768, 50304, NONE),
              ("gemma qkv fwd", 704, 1536, NONE), ("gemma gate|up fwd", 704, 4096, NONE),
              ("gemma down fwd", 2112, 640, NONE)]
    for name, K, N, epi in shapes:
        if a.only and a.only not in name:
            continue
        M = a.M if "lm_head" not in name else a.M // 4
        x, w, b = rnd(M, K), rnd(N, K, s=0.05), rnd(N, s=0.1)
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        kw = dict(bias=b, aux=aux) if epi == BIAS_GELU_D else {}
        fl = 2.0 * M * K * N
        res = {"gemm8": [], "gemm8s": [], "gemmw": [], "hipBLASLt": []}
        for _ in range(a.rounds):
            C.gemm8_set_stream(0)
            res["gemm8"].append(timeit(lambda: C.gemm_t(x, w, False, False, epi, impl=0, **kw), a.iters))
            C.gemm8_set_stream(1)
            res["gemm8s"].append(timeit(lambda: C.gemm_t(x, w, False, False, epi, impl=0, **kw), a.iters))
            res["gemmw"].append(timeit(lambda: C.gemm_t(x, w, False, False, epi, impl=1, **kw), a.iters))
            if epi == NONE:
                res["hipBLASLt"].append(timeit(lambda: torch.mm(x, w.t()), a.iters))
        line = f"{name:20s} M={M:6d} K={K:5d} N={N:6d} |"
        for k, v in res.items():
            if v:
                t = min(v)
                line += f" {k} {t:8.1f} us {fl / t / 1e6:6.0f} TF |"
        print(line, flush=True)
        del x, w, aux
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
