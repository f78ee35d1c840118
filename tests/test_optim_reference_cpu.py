"""CPU numerics of the optimizer oracle (tests/oracle/reference.py::adam_step) -- the formulas the fused
AdamW kernel is checked against on the GPU (tests/test_kernels_gpu.py::test_adamw_amsgrad_matches_reference).

Without AMSGrad the reference's Adam is torch's Adam (coupled L2) / AdamW (decoupled decay); with
AMSGrad the reference keeps the max of the BIAS-CORRECTED v (optim/adam.cpp:75-80), which differs from
torch's max of the raw v while bc2 still changes -- checked here on a hand-computed two-step case."""
import math

import torch

from oracle.reference import adam_step


def _run(decoupled, amsgrad, steps=5):
    torch.manual_seed(0)
    p0 = torch.randn(257, dtype=torch.float64)
    grads = [torch.randn(257, dtype=torch.float64) * (3.0 if i == 1 else 0.3) for i in range(steps)]
    p, m, v, vh = p0.clone(), torch.zeros(257, dtype=torch.float64), torch.zeros(257, dtype=torch.float64), \
        torch.zeros(257, dtype=torch.float64)
    for i, g in enumerate(grads):
        adam_step(p, g, m, v, vh, i + 1, 1e-2, 0.9, 0.99, 1e-8, 0.05, decoupled, amsgrad)
    return p0, grads, p


def test_adam_oracle_equals_torch_without_amsgrad():
    for decoupled, cls in ((True, torch.optim.AdamW), (False, torch.optim.Adam)):
        p0, grads, p = _run(decoupled, False)
        ref = p0.clone().requires_grad_(True)
        opt = cls([ref], lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.05)
        for g in grads:
            ref.grad = g.clone()
            opt.step()
        assert torch.allclose(p, ref.detach(), rtol=1e-12, atol=1e-12), (decoupled, (p - ref.detach()).abs().max())


def test_adam_oracle_amsgrad_is_the_reference_rule():
    # two steps, one element, no decay: g1 = 1 then g2 = 0
    b1, b2, lr, eps = 0.9, 0.99, 0.1, 0.0
    p, m, v, vh = (torch.tensor([1.0], dtype=torch.float64) for _ in range(4))
    m.zero_(), v.zero_(), vh.zero_()
    adam_step(p, torch.tensor([1.0], dtype=torch.float64), m, v, vh, 1, lr, b1, b2, eps, 0.0, True, True)
    assert math.isclose(vh.item(), 1.0, rel_tol=1e-12)        # v1 / bc2(1) = 0.01 / 0.01
    adam_step(p, torch.tensor([0.0], dtype=torch.float64), m, v, vh, 2, lr, b1, b2, eps, 0.0, True, True)
    v2c = (0.99 * 0.01) / (1 - 0.99 ** 2)                    # 0.4975 < 1: the max stays 1
    assert math.isclose(vh.item(), max(1.0, v2c), rel_tol=1e-12)
    m2c = (0.9 * 0.1) / (1 - 0.9 ** 2)
    want = 1.0 - lr * 1.0 - lr * m2c / math.sqrt(1.0)        # step 1 moves by lr * 1 / 1
    assert math.isclose(p.item(), want, rel_tol=1e-12), (p.item(), want)
    # torch's rule would divide max(raw v) = 0.01 by bc2(2) = 0.0199 -> a different step
    torch_den = math.sqrt(max(0.01, 0.99 * 0.01) / (1 - 0.99 ** 2))
    assert abs(torch_den - 1.0) > 0.2
