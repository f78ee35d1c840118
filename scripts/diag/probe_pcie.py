"""PCIe host<->device bandwidth probe: torch pinned tensors vs the native HostTier's pinned memory,
one direction at a time and both directions at once on two streams (full duplex)."""
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import mobilefinetuner_amd as mft  # noqa: F401
from mobilefinetuner_amd._ext import native

N = 1 << 28  # 1 GiB fp32
dev = torch.device("cuda")
d0 = torch.empty(N, device=dev)
d1 = torch.empty(N, device=dev)
hp0 = torch.empty(N, pin_memory=True)
hp1 = torch.empty(N, pin_memory=True)
tier = native().runtime.HostTier(0, "", 0)
tier.add("a", N * 4)
tier.add("b", N * 4)
ht0 = tier.host_tensor("a", torch.float32, [N])
ht1 = tier.host_tensor("b", torch.float32, [N])
print("pinned? torch", hp0.is_pinned(), "tier", ht0.is_pinned())
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def bench(name, fn, nbytes):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 3
    print(f"{name:40s} {nbytes / dt / 1e9:7.1f} GB/s")


for tag, h0, h1 in (("torch-pinned", hp0, hp1), ("hosttier", ht0, ht1)):
    bench(f"{tag} H2D", lambda: d0.copy_(h0, non_blocking=True), N * 4)
    bench(f"{tag} D2H", lambda: h0.copy_(d0, non_blocking=True), N * 4)

    def duplex():
        with torch.cuda.stream(s1):
            d0.copy_(h0, non_blocking=True)
        with torch.cuda.stream(s2):
            h1.copy_(d1, non_blocking=True)
    bench(f"{tag} H2D+D2H (2 streams, total)", duplex, 2 * N * 4)
