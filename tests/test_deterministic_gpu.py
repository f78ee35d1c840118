"""Deterministic-reduction mode: with set_deterministic(True) every gradient is
bitwise reproducible run to run (LoRA dA / dB partials and the embedding-table gradient are summed
in a fixed order instead of fp32 atomics; split-K weight gradients use gemm8's ordered slab
reduction), and it agrees with the default (atomic) mode to fp32 rounding."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(model_name, full, det, B=8, S=128, seed=0):
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.ops import functional as Fx
    from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2, lora_parameters
    from mobilefinetuner_amd.utils.params import FlatParams

    Fx.set_deterministic(det)
    try:
        cfg = GPT2Config.preset(model_name)
        model = GPT2Model(cfg, device="cuda", seed=1234)
        if full:
            model.set_full_finetune()
            flat = FlatParams(model.named_parameters(), "cuda")
        else:
            inject_gpt2(model, LoraSpec(rank=8, alpha=16, targets=["AttnQKV", "AttnProj", "MlpFcIn", "MlpFcOut"]))
            with torch.no_grad():  # non-zero B so every adapter gradient is non-trivial
                g = torch.Generator().manual_seed(3)
                for m in model.modules():
                    for sl in getattr(m, "lora_slices", []):
                        sl.B.copy_(((torch.rand(sl.B.shape, generator=g) - 0.5) * 0.02).cuda())
            flat = FlatParams(lora_parameters(model), "cuda")
        gen = torch.Generator().manual_seed(seed)
        ids = torch.randint(0, cfg.vocab_size, (B, S + 1), generator=gen).cuda()
        out = []
        for _ in range(2):
            flat.zero_grad()
            loss = model(ids[:, :-1].contiguous(), ids[:, 1:].contiguous())
            loss.backward()
            torch.cuda.synchronize()
            out.append(flat.grad.clone())
        return out
    finally:
        Fx.set_deterministic(False)


@pytest.mark.parametrize("model_name,full", [("gpt2", False), ("gpt2-tiny", True)])
def test_deterministic_grads_bitwise(model_name, full):
    g1, g2 = _grads(model_name, full, det=True)
    assert torch.equal(g1, g2), (g1 - g2).abs().max().item()
    a1, _ = _grads(model_name, full, det=False)
    rel = ((a1 - g1).norm() / g1.norm()).item()
    assert rel < 1e-3, rel
    assert g1.abs().sum() > 0
