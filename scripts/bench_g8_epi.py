"""gemm8 epilogue / first-round stagger A/B on the NT training shapes (round 4): variant 0 (register
epilogue, 16 rows x 64 B per store instruction) vs 5 (LDS-staged whole-row stores), each without and
with a first-round stagger (workgroup b < 256 sleeps (b >> 3) x S cycles, S ~ one tile round / 32), and
hipBLASLt.  Checked against fp32 first; interleaved rounds, min over rounds.

usage: PYTHONPATH=. python scripts/bench_g8_epi.py [--iters 10] [--rounds 4]
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
    a = ap.parse_args()
    C = native()
    shapes = [("gpt2 qkv fwd", 131072, 768, 2304), ("gpt2 proj fwd", 131072, 768, 768),
              ("gpt2 fc fwd", 131072, 768, 3072), ("gpt2 mproj fwd", 131072, 3072, 768),
              ("gpt2 lm_head", 32768, 768, 50304), ("gemma gate|up", 131072, 640, 4096), ("8192^3", 8192, 8192, 8192)]
    # fused epilogues at the fc shape: BIAS_GELU_D (h and GELU'(pre) out) and MUL_AUX (dpre = (dy W) * aux)
    M, K, N = 131072, 768, 3072
    x = ((torch.rand(M, K, device="cuda") * 2 - 1)).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
    b = (torch.rand(N, device="cuda") * 0.2 - 0.1).bfloat16()
    aux_in = (torch.rand(M, N, device="cuda") * 1.2 - 0.1).bfloat16()
    rnd = (K // 64) * 3000 + 15000
    cfgs = [(0, 0), (5, 0), (5, rnd // 32)]
    xs, ws_ = x[:4096], w  # numerics on a slice (rows / aux of the first 4096 rows)
    pre = xs.float() @ ws_.float().t() + b.float()
    for v, sg in cfgs:
        C.gemm8_set_stream(v)
        C.gemm8_set_stagger(sg)
        h, d = C.gemm_t(xs, ws_, False, False, 9, bias=b)
        xg = pre.clone().requires_grad_()
        torch.nn.functional.gelu(xg, approximate="tanh").sum().backward()
        eh = ((h.float() - torch.nn.functional.gelu(pre, approximate="tanh")).abs().max() / pre.abs().max()).item()
        ed = (d.float() - xg.grad).abs().max().item()
        y = C.gemm_t(xs, ws_, False, False, 10, aux=aux_in[:4096].contiguous())[0]
        ey = ((y.float() - (xs.float() @ ws_.float().t()) * aux_in[:4096].float()).abs().max() / pre.abs().max()).item()
        assert eh < 1e-2 and ed < 2e-2 and ey < 1e-2, (v, sg, eh, ed, ey)
    fl = 2.0 * M * N * K
    for epi, lab in [(9, "fc fwd +GELU_D"), (10, "fc dgrad *aux")]:
        res = {c: [] for c in cfgs}
        for _ in range(a.rounds):
            for c in cfgs:
                C.gemm8_set_stream(c[0])
                C.gemm8_set_stagger(c[1])
                if epi == 9:
                    res[c].append(timeit(lambda: C.gemm_t(x, w, False, False, 9, bias=b), a.iters))
                else:
                    res[c].append(timeit(lambda: C.gemm_t(x, w, False, False, 10, aux=aux_in), a.iters))
        line = f"{lab:14s} M={M:6d} K={K:5d} N={N:6d} |"
        for c in cfgs:
            t = min(res[c])
            line += f" v{c[0]}/s{c[1]} {t:7.1f} us {fl / t / 1e6:5.0f} TF |"
        print(line, flush=True)
    del x, w, aux_in
    torch.cuda.empty_cache()
    for name, M, K, N in shapes:
        x = ((torch.rand(M, K, device="cuda") * 2 - 1)).bfloat16()
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
        rnd = (K // 64) * 3000 + 15000  # ~ cycles per tile round
        cfgs = [(0, 0), (5, 0), (0, rnd // 32), (5, rnd // 32), (5, rnd // 64)]
        if M * N <= 8192 * 8192:
            ref = x.float() @ w.float().t()
            for v, sg in cfgs:
                C.gemm8_set_stream(v)
                C.gemm8_set_stagger(sg)
                y = C.gemm_t(x, w, False, False, 0)[0]
                err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                assert err < 1e-2, (name, v, sg, err)
            del ref
        fl = 2.0 * M * N * K
        res = {c: [] for c in cfgs}
        res["lt"] = []
        for _ in range(a.rounds):
            for c in cfgs:
                C.gemm8_set_stream(c[0])
                C.gemm8_set_stagger(c[1])
                res[c].append(timeit(lambda: C.gemm_t(x, w, False, False, 0), a.iters))
            res["lt"].append(timeit(lambda: torch.mm(x, w.t()), a.iters))
        line = f"{name:14s} M={M:6d} K={K:5d} N={N:6d} |"
        for c in cfgs + ["lt"]:
            t = min(res[c])
            lab = "hipBLASLt" if c == "lt" else f"v{c[0]}/s{c[1]}"
            line += f" {lab} {t:7.1f} us {fl / t / 1e6:5.0f} TF |"
        print(line, flush=True)
        del x, w
        torch.cuda.empty_cache()
    C.gemm8_set_stream(0)
    C.gemm8_set_stagger(0)


if __name__ == "__main__":
    main()
