"""LM-head cross-entropy anatomy on one GPU: the fused CE forward (gemm8 CE_FWD epilogue: tile max /
sum-exp / label logit, optionally E = exp(logit - tile max) stored) and the CE dgrad, against plain gemm8
GEMMs of the same shapes (NONE epilogue, bf16 output stored) and hipBLASLt (torch.mm).  Splits the CE
forward's time into main loop + store vs softmax epilogue, and times the vocab-split dgrad of a short row
chunk.  Interleaved rounds, min over rounds.

usage: PYTHONPATH=. python scripts/bench_ce.py [--rounds 3] [--iters 5]
"""
import argparse
import os

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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    C = native()
    for name, M, K, V, Vp in [("gemma3 vocab", 16384, 640, 262144, 262144), ("gpt2 vocab", 32768, 768, 50257, 50304)]:
        g = torch.Generator(device="cuda").manual_seed(0)
        h = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        W = (torch.randn(Vp, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
        W[V:] = 0
        labels = torch.randint(0, V, (M,), device="cuda", generator=g)
        scale = torch.full((1,), 1.0 / M, device="cuda")
        loss = torch.empty(M, device="cuda")
        E = torch.empty(M, Vp, device="cuda", dtype=torch.bfloat16)
        dh = torch.empty_like(h)
        fl = 2.0 * M * Vp * K
        S = C.ce_dgrad_splits(M, K, Vp)
        cases = {
            "plain NT NONE (logits stored)": lambda: C.gemm_t(h, W, False, False, 0),
            "hipBLASLt NT (torch.mm)": lambda: torch.mm(h, W.t()),
            "CE fwd, no E (loss only)": lambda: C.lm_head_ce(h, W, labels, V, None, loss, scale, 1.0, None, False),
            "plain NN NONE (dgrad shape)": lambda: C.gemm_t(E, W, False, True, 0),
            f"CE fwd+E+dgrad (auto split {S})": lambda: C.lm_head_ce(h, W, labels, V, E, loss, scale, 1.0, dh, False),
        }

        def one_split():
            os.environ["MFT_CE_SPLIT"] = "1"
            C.lm_head_ce(h, W, labels, V, E, loss, scale, 1.0, dh, False)
            del os.environ["MFT_CE_SPLIT"]
        if S > 1:
            cases["CE fwd+E+dgrad (split 1)"] = one_split

        def lds_epi(fn):  # gemm8 LDS-staged epilogues (E leaves as whole tile rows): MFT_GEMM8_STREAM=5
            def run():
                C.gemm8_set_stream(5)
                fn()
                C.gemm8_set_stream(0)
            return run
        cases["CE fwd, no E, LDS epi"] = lds_epi(cases["CE fwd, no E (loss only)"])
        cases[f"CE fwd+E+dgrad, LDS epi"] = lds_epi(cases[f"CE fwd+E+dgrad (auto split {S})"])
        res = {k: [] for k in cases}
        for _ in range(a.rounds):
            for k, fn in cases.items():
                res[k].append(timeit(fn, a.iters))
        print(f"{name}: M={M} K={K} Vpad={Vp}  ({fl / 1e12:.2f} TFLOP per GEMM)", flush=True)
        for k in cases:
            t = min(res[k])
            nf = 2 if "+dgrad" in k else 1
            print(f"  {k:34s} {t:9.1f} us  {nf * fl / t / 1e6:6.0f} TF/s", flush=True)
        del h, W, E, dh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
