"""D=256 attention forward + backward at the Gemma-3 bench shape (for rocprofv3 --pmc passes)."""
import sys
import torch
sys.path.insert(0, ".")
from mobilefinetuner_amd._ext import native

C = native()
B, S, H, Hkv, D = 256, 256, 4, 1, 256
g = torch.Generator(device="cuda").manual_seed(3)
q = torch.randn(B, S, H, D, device="cuda", generator=g).bfloat16()
k = torch.randn(B, S, Hkv, D, device="cuda", generator=g).bfloat16()
v = torch.randn(B, S, Hkv, D, device="cuda", generator=g).bfloat16()
sc = D ** -0.5
for _ in range(3):
    o, lse, _ = C.attn_fwd(q, k, v, sc, True, 0, None, 0)
    go = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    C.attn_bwd(q, k, v, o, go, lse, dq, dk, dv, sc, True, 0, None)
torch.cuda.synchronize()
