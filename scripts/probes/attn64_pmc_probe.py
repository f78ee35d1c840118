"""GPT-2 short attention (S 128, D 64, 12 heads, batch 1024, packed qkv) forward + backward, for rocprofv3 --pmc."""
import sys
import time
import torch
sys.path.insert(0, ".")
from mobilefinetuner_amd._ext import native

C = native()
B, S, H, D = 1024, 128, 12, 64
g = torch.Generator(device="cuda").manual_seed(3)
qkv = torch.randn(B, S, 3, H, D, device="cuda", generator=g).bfloat16()
q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
sc = D ** -0.5
o, lse, _ = C.attn_fwd(q, k, v, sc, True, 0, None, 0)
go = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
dq, dk, dv = dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2]
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
torch.cuda.synchronize()
t0 = time.time()
for _ in range(iters):
    o, lse, _ = C.attn_fwd(q, k, v, sc, True, 0, None, 0)
    C.attn_bwd(q, k, v, o, go, lse, dq, dk, dv, sc, True, 0, None)
torch.cuda.synchronize()
print(f"fwd+bwd {(time.time() - t0) / iters * 1e6:.1f} us per iteration")
