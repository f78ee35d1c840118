"""gemm4 (256x256x64, 4 waves, one per SIMD, AGPR accumulators) vs gemm8 (256x256 8-phase) vs hipBLASLt (torch.mm)
on the NT training shapes, with every epilogue checked against an fp32 reference first.
Interleaved rounds in one process, random data (CDNA HIP guide §5.4 rules 24 / 25).

usage: PYTHONPATH=. python scripts/bench_gemm4.py [--M 131072] [--iters 10] [--rounds 3] [--only NAME]
"""
import argparse
import os

import torch

from mobilefinetuner_amd._ext import native

NONE, BIAS, BIAS_GELU, DGELU, F32ACC, LORA, BIAS_GELU_D, MUL_AUX = 0, 1, 2, 3, 4, 5, 9, 10


def rnd(*shape, s=1.0):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * s).bfloat16()


def gelu(x):
    return 0.5 * x * (1 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))


def check(C):
    """every supported epilogue of gemm4 on a mid-size problem (M not a multiple of 256, N tail)."""
    M, K, N = 1000, 832, 776
    x, w = rnd(M, K), rnd(N, K, s=0.05)
    b, aux = rnd(N, s=0.1), rnd(M, N)
    ref = x.float() @ w.float().t()
    worst = 0.0

    def err(got, want):
        return ((got.float() - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()

    for impl, stream in ((0, 0), (2, 0), (2, 1)):
        os.environ["MFT_G4_A3"] = str(stream)  # (impl 2, 1) = gemm4 with the A3 ring
        C.gemm8_set_stream(0)
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
        print(f"impl {impl} A3 {stream}: max relative error over the epilogues {e:.2e}", flush=True)
        worst = max(worst, e)
    # many K-tiles, row and column tails: gemm4 vs gemm8 vs fp32
    M, K, N = 65536 + 200, 768, 2048 - 8
    x, w, b = rnd(M, K), rnd(N, K, s=0.05), rnd(N, s=0.1)
    ref = x.float() @ w.float().t()
    for impl, a3 in ((0, "0"), (2, "0"), (2, "1")):
        os.environ["MFT_G4_A3"] = a3
        y = C.gemm_t(x, w, False, False, NONE, impl=impl)[0]
        e1 = err(y, ref)
        y = C.gemm_t(x, w, False, False, BIAS, bias=b, impl=impl)[0]
        e2 = err(y, ref + b.float())
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y = C.gemm_t(x, w, False, False, BIAS_GELU_D, bias=b, aux=aux, impl=impl)[0]
        e3 = err(y, gelu(ref + b.float()))
        print(f"large NT, impl {impl} A3 {a3}: errors none {e1:.2e} bias {e2:.2e} gelu {e3:.2e}", flush=True)
        worst = max(worst, e1, e2, e3)
    del ref
    os.environ["MFT_G4_A3"] = "0"
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
              ("gemma down fwd", 2112, 640, NONE), ("square 8192", 8192, 8192, NONE)]
    for name, K, N, epi in shapes:
        if a.only and a.only not in name:
            continue
        M = a.M if "lm_head" not in name else a.M // 4
        if "square" in name:
            M = 8192
        x, w, b = rnd(M, K), rnd(N, K, s=0.05), rnd(N, s=0.1)
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        kw = dict(bias=b, aux=aux) if epi == BIAS_GELU_D else {}
        fl = 2.0 * M * K * N
        res = {"gemm8": [], "gemm4": [], "hipBLASLt": []}
        dbg = os.environ.get("MFT_G4_DBG") and epi == NONE
        if dbg:
            res.update({"g4-nomem": [], "g4-nobar": [], "g4-noglds": []})
        for _ in range(a.rounds):
            if dbg:
                for v, k in ((1, "g4-nomem"), (2, "g4-nobar"), (4, "g4-noglds")):
                    os.environ["MFT_G4_DBG_V"] = str(v)
                    res[k].append(timeit(lambda: C.gemm_t(x, w, False, False, epi, impl=2, **kw), a.iters))
                os.environ["MFT_G4_DBG_V"] = "0"
            res["gemm8"].append(timeit(lambda: C.gemm_t(x, w, False, False, epi, impl=0, **kw), a.iters))
            res["gemm4"].append(timeit(lambda: C.gemm_t(x, w, False, False, epi, impl=2, **kw), a.iters))
            os.environ["MFT_G4_A3"] = "1"
            res.setdefault("gemm4-A3", []).append(timeit(lambda: C.gemm_t(x, w, False, False, epi, impl=2, **kw), a.iters))
            os.environ["MFT_G4_A3"] = "0"
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
