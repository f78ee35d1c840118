"""Gemma-3 D=256 attention timing at the bench shape (B=256, S=256, H=4, Hkv=1, causal): forward,
and forward+backward.  Variant selection by env (read once per process): MFT_ATTN_RPW=16|32, MFT_ATTN_FWD_RING=2|3|4,
MFT_ATTN_NW_FWD=4|8.

usage: MFT_ATTN_RPW=32 PYTHONPATH=. python scripts/bench_attn256.py [--window 0]
"""
import argparse
import os

import torch

from mobilefinetuner_amd._ext import native


def timeit(fn, iters=20):
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
    ap.add_argument("--window", type=int, default=0)
    a = ap.parse_args()
    C = native()
    B, S, H, Hkv, D = 256, 256, 4, 1, 256
    g = torch.Generator(device="cuda").manual_seed(3)
    q = torch.randn(B, S, H, D, device="cuda", generator=g).bfloat16()
    k = torch.randn(B, S, Hkv, D, device="cuda", generator=g).bfloat16()
    v = torch.randn(B, S, Hkv, D, device="cuda", generator=g).bfloat16()
    sc = D ** -0.5
    fwd = lambda: C.attn_fwd(q, k, v, sc, True, a.window, None, 0)  # noqa: E731
    o, lse, _ = fwd()
    go = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    bwd = lambda: C.attn_bwd(q, k, v, o, go, lse, dq, dk, dv, sc, True, a.window, None)  # noqa: E731
    tf = min(timeit(fwd) for _ in range(3))
    tb = min(timeit(bwd) for _ in range(3))
    fl = 4.0 * B * H * S * S * D / 2  # causal
    # fp32 reference of the forward (GQA heads expanded)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k.expand(B, S, H, D), v.expand(B, S, H, D)))
    ref = torch.nn.functional.scaled_dot_product_attention(qf, kf, vf, is_causal=True, scale=sc).transpose(1, 2)
    err = (o.float() - ref).abs().max().item()
    # backward vs fp32 autograd (relative to each gradient's max)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    orf = torch.nn.functional.scaled_dot_product_attention(
        qr.transpose(1, 2), kr.expand(B, S, H, D).transpose(1, 2), vr.expand(B, S, H, D).transpose(1, 2),
        is_causal=True, scale=sc).transpose(1, 2)
    orf.backward(go.float())
    bwd()
    gerr = max(((x.float() - y.grad).abs().max() / y.grad.abs().max()).item() for x, y in ((dq, qr), (dk, kr), (dv, vr)))
    tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("MFT_ATTN"))
    print(f"[{tag}] err {err:.1e} grad rel err {gerr:.1e} window={a.window}: fwd {tf:7.1f} us ({fl / tf / 1e6:5.0f} TF) "
          f"bwd {tb:7.1f} us ({2.5 * fl / tb / 1e6:5.0f} TF)  o[0,0,0,:4]={o[0, 0, 0, :4].float().tolist()}", flush=True)


if __name__ == "__main__":
    main()
