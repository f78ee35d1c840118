"""gemm4 (hand-scheduled 4-wave GEMM, csrc/kernels/gemm4.hip) vs gemm8 vs hipBLASLt (torch.mm).

Random uniform [-1, 1) operands (guide §5.4 rule 25), every kernel checked against an fp32 reference
first, then interleaved timing rounds in one process (rule 24): per shape and kernel the median and the
min of `--rounds` rounds of `--iters` calls.
usage: python scripts/bench_gemm4.py [--rounds 5] [--iters 10] [--shapes all|train|sq]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mobilefinetuner_amd._ext import native

EPI_NONE, EPI_BIAS, EPI_DGELU, EPI_GELU_D, EPI_MUL_AUX, EPI_BIAS_ADD = 0, 1, 3, 9, 10, 11


def gelu_and_grad(x):
    t = torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3))
    return 0.5 * x * (1 + t), 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * x * x)


def check_epilogues(C, dev, shapes):
    """Fused epilogues of gemm4 (impl 4) against fp32 references: BIAS_GELU_D (two outputs), MUL_AUX, DGELU."""
    for name in shapes:
        M, N, K = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(1)
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.1).bfloat16()
        b = (torch.rand(N, device=dev, generator=g) - 0.5).bfloat16()
        aux = (torch.randn(M, N, device=dev, generator=g)).bfloat16()
        pre = torch.addmm(b.float(), x.float(), w.float().t())
        gl, gd = gelu_and_grad(pre)
        y, d = torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        C.gemm_t(x, w, False, False, EPI_GELU_D, b, d, 1.0, y, None, None, 4)
        mm = x.float() @ w.float().t()
        y2 = torch.empty_like(y)
        C.gemm_t(x, w, False, False, EPI_MUL_AUX, None, aux, 1.0, y2, None, None, 4)
        y3 = torch.empty_like(y)
        C.gemm_t(x, w, False, False, EPI_DGELU, None, aux, 1.0, y3, None, None, 4)
        y4 = aux.clone()  # residual added in place (aux aliases the output, as the engine's fused residual may)
        C.gemm_t(x, w, False, False, EPI_BIAS_ADD, b, y4, 1.0, y4, None, None, 4)
        torch.cuda.synchronize()
        r = lambda a, ref: ((a.float() - ref).abs().max() / ref.abs().max()).item()
        errs = (r(y, gl), r(d, gd), r(y2, mm * aux.float()), r(y3, mm * gelu_and_grad(aux.float())[1]),
                r(y4, mm + b.float() + aux.float()))
        print(f"{name:22s} epilogues gelu {errs[0]:.1e} gelu' {errs[1]:.1e} mul_aux {errs[2]:.1e} dgelu {errs[3]:.1e}"
              f" bias_add {errs[4]:.1e}", flush=True)
        assert max(errs) < 2e-2, (name, errs)
        del pre, gl, gd, mm
        fl = 2.0 * M * N * K
        line = f"{name:22s}"
        for tag, epi, bias, ax in (("gelu_d", EPI_GELU_D, b, d), ("mul_aux", EPI_MUL_AUX, None, aux)):
            for impl in (4, 0):
                f = lambda: C.gemm_t(x, w, False, False, epi, bias, ax, 1.0, y, None, None, impl)
                for _ in range(3):
                    f()
                ts = []
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        f()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 100)
                t = statistics.median(ts)
                line += f" | {tag} g{impl} {t:7.1f} us {fl / t / 1e6:5.0f} TF"
        print(line, flush=True)
        del x, w, aux, y, d, y2, y3, y4

SHAPES = {
    "8192^3": (8192, 8192, 8192),
    "4096^3": (4096, 4096, 4096),
    "gpt2 qkv fwd (aug K)": (131072, 2304, 832),
    "gpt2 proj fwd": (131072, 768, 768),
    "gpt2 fc fwd": (131072, 3072, 768),
    "gpt2 mproj fwd": (131072, 768, 3072),
    "gpt2 lm head": (32768, 50304, 768),
    "gemma gate|up fwd": (65536, 4096, 704),
    "gemma down fwd": (65536, 640, 2048),
    # the reference recipe: 4 x 128 tokens
    "b4 qkv fwd (aug K)": (512, 2304, 832),
    "b4 proj fwd": (512, 768, 768),
    "b4 fc fwd": (512, 3072, 768),
    "b4 mproj fwd": (512, 768, 3072),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default="all")
    ap.add_argument("--check_only", action="store_true")
    ap.add_argument("--no_check", action="store_true", help="diagnostic builds (MFT_G4_DIAG): wrong outputs")
    ap.add_argument("--only", default="", help="comma list of kernels to time (gemm4,gemm8,gemm_s,hipBLASLt)")
    ap.add_argument("--epi", action="store_true", help="check the fused epilogues (then exit)")
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda")
    names = list(SHAPES) if a.shapes == "all" else a.shapes.split(",")
    if a.epi:
        check_epilogues(C, dev, [n for n in names if SHAPES[n][0] * SHAPES[n][1] <= 2 ** 29])
        return
    for name in names:
        M, N, K = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(0)
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).bfloat16()
        b = (torch.rand(N, device=dev, generator=g) - 0.5).bfloat16()
        ref = torch.addmm(b.float(), x.float(), w.float().t()) if M * N <= 2 ** 31 and not a.no_check else None
        y4 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        y8 = torch.empty_like(y4)
        C.gemm_t(x, w, False, False, EPI_BIAS, b, None, 1.0, y4, None, None, 4)
        C.gemm_t(x, w, False, False, EPI_BIAS, b, None, 1.0, y8, None, None, 0)
        torch.cuda.synchronize()
        errs = ""
        if ref is not None:
            for tag, y in (("g4", y4), ("g8", y8)):
                e = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                errs += f" {tag} err {e:.1e}"
                assert e < 1e-2, (name, tag, e)
            del ref
        if a.check_only:
            print(f"{name:22s} M={M} N={N} K={K}{errs}", flush=True)
            continue
        fl = 2.0 * M * N * K
        fns = {
            "gemm4": lambda: C.gemm_t(x, w, False, False, EPI_BIAS, b, None, 1.0, y4, None, None, 4),
            "gemm8": lambda: C.gemm_t(x, w, False, False, EPI_BIAS, b, None, 1.0, y8, None, None, 0),
            "gemm_s": lambda: C.gemm_t(x, w, False, False, EPI_BIAS, b, None, 1.0, y8, None, None, 5),
            "hipBLASLt": lambda: torch.addmm(b, x, w.t(), out=y8),
        }
        if a.only:
            fns = {k: f for k, f in fns.items() if k in a.only.split(",")}
        times = {k: [] for k in fns}
        for f in fns.values():
            for _ in range(3):
                f()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for k, f in fns.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        line = f"{name:22s} M={M:6d} N={N:5d} K={K:5d}"
        for k, ts in times.items():
            med, mn = statistics.median(ts), min(ts)
            line += f" | {k} {med:8.1f} us {fl / med / 1e6:5.0f} TF (min {fl / mn / 1e6:5.0f})"
        print(line + errs, flush=True)
        del x, w, y4, y8


if __name__ == "__main__":
    main()
