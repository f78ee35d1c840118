"""Probe which hipBLASLt epilogues have gfx950 bf16 solutions (prints a small table)."""
import torch

from mobilefinetuner_amd._ext import native

C = native()
EPI = {"DEFAULT": 1, "BIAS": 4, "GELU": 32, "GELU_BIAS": 36, "GELU_AUX": 160, "GELU_AUX_BIAS": 164,
       "DGELU": 192, "DGELU_BGRAD": 208, "BGRADB": 512}
R16BF, R32F = 14, 0
for (m, n, k) in [(3072, 32768, 768), (768, 32768, 3072), (128, 64, 64)]:
    for ta, tb in [(True, False), (False, False)]:
        for name, e in EPI.items():
            bias = "BIAS" in name and "BGRAD" not in name
            aux = "AUX" in name or "DGELU" in name
            for adt in ([-1, R16BF, R32F] if aux else [-1]):
                got = C.lt_solutions(m, n, k, ta, tb, e, bias, m if aux else 0, adt)
                print(f"m={m} n={n} k={k} ta={int(ta)} tb={int(tb)} {name:14s} auxdt={adt:3d}: {got}")
