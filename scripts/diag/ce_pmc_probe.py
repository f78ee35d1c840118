"""PMC probe of the fused LM-head CE at the Gemma-3 shape and the default 4 GiB E budget: one 8,192-row chunk
(262,144 vocab, d_model 640) -- CE forward (gemm8 CE_FWD), ce_finalize, vocab-split CE dgrad, ce_split_reduce --
three calls after a warm-up (run under rocprofv3 --pmc)."""
import torch

from mobilefinetuner_amd._ext import native

C = native()
M, K, V = 8192, 640, 262144
g = torch.Generator(device="cuda").manual_seed(0)
h = torch.randn(M, K, device="cuda", generator=g).bfloat16()
W = (torch.randn(V, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
labels = torch.randint(0, V, (M,), device="cuda", generator=g)
scale = torch.full((1,), 1.0 / M, device="cuda")
loss = torch.empty(M, device="cuda")
E = torch.empty(M, V, device="cuda", dtype=torch.bfloat16)
dh = torch.empty_like(h)
for _ in range(4):
    C.lm_head_ce(h, W, labels, V, E, loss, scale, 1.0, dh, False)
torch.cuda.synchronize()
print("ce probe ok", C.ce_dgrad_splits(M, K, V), float(loss.sum() * scale))
