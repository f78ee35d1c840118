"""Measured bf16-GPU vs fp32-CPU errors of the tiny-model checks in tests/test_models_gpu.py (to size
their tolerances from data): GPT-2 tiny LoRA loss / grad rel-L2, Gemma-3 tiny logits rel-L2 / max and loss."""
import os
import sys
os.environ.setdefault("MFT_HOST_ORACLE", os.path.abspath("tests/oracle"))  # the fp32 host reference (as conftest)
import torch  # noqa: E402
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_models_gpu import _copy_weights, DEV  # noqa: E402
from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model  # noqa: E402
from mobilefinetuner_amd.models.gemma3 import Gemma3Config, Gemma3Model  # noqa: E402
from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2, lora_parameters  # noqa: E402
from mobilefinetuner_amd.utils.params import FlatParams  # noqa: E402

for seed in range(4):
    torch.manual_seed(seed)
    cfg = GPT2Config.preset("gpt2-tiny")
    cpu = GPT2Model(cfg, dtype=torch.float32, device="cpu", seed=3 + seed)
    gpu = GPT2Model(cfg, dtype=torch.bfloat16, device=DEV, init=False)
    _copy_weights(gpu, cpu)
    spec = LoraSpec(rank=8, alpha=16, targets=["AttnQKV", "AttnProj", "MlpFcIn", "MlpFcOut"])
    for m in (cpu, gpu):
        inject_gpt2(m, spec)
        with torch.no_grad():
            for mod in m.modules():
                for sl in getattr(mod, "lora_slices", []):
                    sl.B.copy_(torch.randn(sl.B.shape, generator=torch.Generator().manual_seed(sl.ncols)) * 0.05)
    fc = FlatParams(lora_parameters(cpu), "cpu", shadow=False)
    fg = FlatParams(lora_parameters(gpu), DEV)
    ids = torch.randint(0, cfg.vocab_size, (4, 65))
    lc = cpu(ids[:, :-1], ids[:, 1:])
    lg = gpu(ids[:, :-1].to(DEV), ids[:, 1:].to(DEV))
    lc.backward()
    lg.backward()
    gc, gg = fc.grad, fg.grad.cpu()
    print(f"gpt2-tiny seed {seed}: loss |d| {abs(lc.item() - lg.item()):.2e} (loss {lc.item():.3f}) "
          f"grad rel-L2 {((gc - gg).norm() / gc.norm()).item():.3e}", flush=True)
    cfg = Gemma3Config.preset("gemma3-tiny")
    cpu = Gemma3Model(cfg, dtype=torch.float32, device="cpu", seed=4 + seed)
    with torch.no_grad():
        for n, p in cpu.named_parameters():
            if p.dim() == 1:
                p.normal_(0, 0.1, generator=torch.Generator().manual_seed(len(n)))
    gpu = Gemma3Model(cfg, dtype=torch.bfloat16, device=DEV, init=False)
    _copy_weights(gpu, cpu)
    ids = torch.randint(0, cfg.vocab_size, (2, 48))
    with torch.no_grad():
        a = cpu.logits(ids)
        b = gpu.logits(ids.to(DEV)).float().cpu()
    lc = cpu(ids[:, :-1], ids[:, 1:]).item()
    lg = gpu(ids[:, :-1].to(DEV), ids[:, 1:].to(DEV)).item()
    print(f"gemma3-tiny seed {seed}: logits rel-L2 {((a - b).norm() / a.norm()).item():.3e} max|d|/max|a| "
          f"{((a - b).abs().max() / a.abs().max()).item():.3e}  loss |d| {abs(lc - lg):.2e}", flush=True)
