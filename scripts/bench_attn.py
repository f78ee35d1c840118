"""Micro-benchmark of the flash-attention kernels at a given shape (default: Gemma-3 270M bench
layer, B=256, S=256, 4 q-heads, 1 KV head, D=256, causal).  Prints per-call fwd / bwd times;
used under rocprofv3 for per-kernel counters."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--H", type=int, default=4)
    ap.add_argument("--Hkv", type=int, default=1)
    ap.add_argument("--D", type=int, default=256)
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from mobilefinetuner_amd._ext import native
    C = native()
    dev = "cuda"
    q = torch.randn(a.B, a.S, a.H, a.D, device=dev).bfloat16()
    k = torch.randn(a.B, a.S, a.Hkv, a.D, device=dev).bfloat16()
    v = torch.randn(a.B, a.S, a.Hkv, a.D, device=dev).bfloat16()
    scale = a.D ** -0.5
    o, lse, _ = C.attn_fwd(q, k, v, scale, True, a.window, None, 0)
    do = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    for name, fn in (("fwd", lambda: C.attn_fwd(q, k, v, scale, True, a.window, None, 0)),
                     ("bwd", lambda: C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, True, a.window, None))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        print(f"{name}: {(time.perf_counter() - t0) / a.iters * 1e6:.1f} us/call", flush=True)


if __name__ == "__main__":
    main()
