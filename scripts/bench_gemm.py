"""Hand-written MFMA GEMM (csrc/kernels/gemm.hip) vs hipBLASLt (torch.mm) at the GPT-2 block shapes.

Prints per shape: our µs / TFLOP/s, hipBLASLt µs / TFLOP/s, and the max relative error of ours vs
an fp32 reference.  Timings are interleaved rounds in one process (guide §5.4 rule 24), random data.
usage: python scripts/bench_gemm.py [--M 32768] [--iters 20] [--bm 0,1,2,3]
"""
import argparse

import torch

from mobilefinetuner_amd._ext import native

EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_DGELU = 0, 1, 2, 3


def timeit(fn, iters):
    for _ in range(3):
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
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bm", default="0,2,8", help="tile configs (gemm.hip launch_e; 8 = gemm8.hip, NT only)")
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda")
    M = a.M
    # (name, K, N, nn)
    shapes = [("qkv fwd", 768, 2304, False), ("proj fwd", 768, 768, False), ("fc fwd", 768, 3072, False),
              ("mlp_proj fwd", 3072, 768, False), ("qkv dx", 2304, 768, True), ("proj dx", 768, 768, True),
              ("fc dx", 3072, 768, True), ("mlp_proj dx", 768, 3072, True)]
    for name, K, N, nn in shapes:
        x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        w = ((torch.rand(K, N, device=dev) * 2 - 1) * 0.05).bfloat16() if nn else \
            ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
        ref = (x.float() @ (w.float() if nn else w.float().t()))
        fl = 2.0 * M * N * K
        tl = timeit(lambda: torch.mm(x, w if nn else w.t()), a.iters)
        line = f"{name:13s} M={M} K={K:5d} N={N:5d}  hipBLASLt {tl:7.1f} us {fl / tl / 1e6:6.0f} TF"
        for bm in [int(v) for v in a.bm.split(",")]:
            if bm == 8 and nn:
                w_nt = w.t().contiguous()  # the model runs data-grad GEMMs through a transposed weight copy
                y = C.gemm(x, w_nt, False, EPI_NONE, None, None, 1.0, 8, None)[0]
                err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                t = timeit(lambda: C.gemm(x, w_nt, False, EPI_NONE, None, None, 1.0, 8, None), a.iters)
                line += f" | c8(NT) {t:7.1f} us {fl / t / 1e6:6.0f} TF err {err:.1e}"
                continue
            y = C.gemm(x, w, nn, EPI_NONE, None, None, 1.0, bm, None)[0]
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            t = timeit(lambda: C.gemm(x, w, nn, EPI_NONE, None, None, 1.0, bm, None), a.iters)
            line += f" | c{bm} {t:7.1f} us {fl / t / 1e6:6.0f} TF err {err:.1e}"
        print(line, flush=True)
    # epilogues at the fc shape
    K, N = 768, 3072
    x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
    b = (torch.rand(N, device=dev) - 0.5).bfloat16()
    pre_r = x.float() @ w.float().t() + b.float()
    h, pre = C.gemm(x, w, False, EPI_BIAS_GELU, b, None, 1.0, 0, None)
    h_r = torch.nn.functional.gelu(pre_r, approximate="tanh")
    print(f"bias+gelu: pre err {((pre.float() - pre_r).abs().max() / pre_r.abs().max()).item():.1e} "
          f"h err {((h.float() - h_r).abs().max() / h_r.abs().max()).item():.1e}")
    t = timeit(lambda: C.gemm(x, w, False, EPI_BIAS_GELU, b, pre, 1.0, 0, None), a.iters)
    tl = timeit(lambda: C.gelu_fwd(torch.addmm(b, x, w.t())), a.iters)
    print(f"fc+gelu fused {t:.1f} us vs hipBLASLt addmm + gelu kernel {tl:.1f} us")
    dy = (torch.rand(M, 768, device=dev) * 2 - 1).bfloat16()
    w2 = ((torch.rand(768, N, device=dev) * 2 - 1) * 0.05).bfloat16()  # mlp_proj weight [768, 3072]
    g = C.gemm(dy, w2, True, EPI_DGELU, None, pre, 1.0, 0, None)[0]
    pf = pre.float()
    t3 = torch.tanh(0.7978845608 * (pf + 0.044715 * pf ** 3))
    dg = 0.5 * (1 + t3) + 0.5 * pf * (1 - t3 ** 2) * 0.7978845608 * (1 + 3 * 0.044715 * pf ** 2)
    g_r = (dy.float() @ w2.float()) * dg
    print(f"dgelu err {((g.float() - g_r).abs().max() / g_r.abs().max()).item():.1e}")
    tl = timeit(lambda: C.gelu_bwd(pre, torch.mm(dy, w2)), a.iters)
    w2t = w2.t().contiguous()
    for cfg in (0, 8):
        t = timeit(lambda: C.gemm(dy, w2, True, EPI_DGELU, None, pre, 1.0, cfg, None), a.iters) if cfg != 8 else 0.0
        t2 = timeit(lambda: C.gemm(dy, w2t, False, EPI_DGELU, None, pre, 1.0, cfg, None), a.iters)
        t3 = timeit(lambda: C.gemm(x, w, False, EPI_BIAS_GELU, b, pre, 1.0, cfg, None), a.iters)
        print(f"cfg{cfg}: mlp_proj dx+dgelu fused NN {t:.1f} us, NT {t2:.1f} us | fc+gelu fused {t3:.1f} us; "
              f"hipBLASLt mm + gelu_bwd {tl:.1f} us")


if __name__ == "__main__":
    main()
