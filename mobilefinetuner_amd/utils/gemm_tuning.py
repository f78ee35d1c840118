"""Offline-tuned library GEMMs: PyTorch TunableOp with a solution database shipped in the package.

The plain NT forward GEMMs that stay on the vendor library (``torch.mm`` / ``torch.addmm`` ->
hipBLASLt / rocBLAS, see the routing notes in ``ops/functional.py``) run with the solution that
TunableOp measured fastest on MI355X for each exact training shape, instead of hipBLASLt's
heuristic first pick.  Measured on the headline step (GPT-2 LoRA, M = 65536): qkv forward
(K = 832, N = 2304) 225 -> 173 us, LM-head forward (K = 768, N = 50304) 4.19 -> 3.83 ms.

The database (``mobilefinetuner_amd/tuning/tunableop_gfx950.csv``) is read-only at run time:
no tuning happens inside a benchmark or a training run unless ``MFT_GEMM_TUNE=1`` (which tunes
unseen shapes during the eager warm-up steps -- never under hipGraph capture -- and rewrites the
file on exit).  ``MFT_TUNED_GEMMS=0`` disables the lookup (hipBLASLt heuristics).  The file's
validator lines pin the ROCm / hipBLASLt / gfx build it was tuned on; TunableOp ignores it on a
mismatch.
"""
from __future__ import annotations

import os

DB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "tunableop_gfx950.csv")
_DONE = [False]


def enable_tuned_gemms(path: str | None = None) -> bool:
    """Turn on TunableOp lookups from the shipped database (idempotent).  Returns True if enabled."""
    if _DONE[0]:
        return True
    if os.environ.get("MFT_TUNED_GEMMS", "1") == "0":
        return False
    import torch
    if not torch.cuda.is_available():
        return False
    import torch.cuda.tunable as tn
    path = path or os.environ.get("MFT_GEMM_TUNE_DB", DB)
    tune = os.environ.get("MFT_GEMM_TUNE", "0") == "1"
    if not tune and not os.path.exists(path):
        return False
    tn.enable(True)
    tn.tuning_enable(tune)
    if tune:
        tn.set_max_tuning_duration(30)
    tn.set_filename(path, insert_device_ordinal=False)
    if os.path.exists(path):
        tn.read_file(path)
    _DONE[0] = True
    return True


class no_tuning:
    """Context: TunableOp lookups stay on but no new tuning happens inside (used around the
    262144-wide Gemma LM-head GEMM: one of hipBLASLt's candidate solutions faults on that shape
    while being tuned, so it keeps the library's heuristic pick)."""

    def __enter__(self):
        import torch.cuda.tunable as tn
        self.prev = _DONE[0] and tn.tuning_is_enabled()
        if self.prev:
            tn.tuning_enable(False)
        return self

    def __exit__(self, *exc):
        if self.prev:
            import torch.cuda.tunable as tn
            tn.tuning_enable(True)
        return False
