"""SafeTensors IO through the native C++ reader/writer (csrc/runtime/safetensors.cpp).

Reference: SafeTensorsReader / load_tensors_mapped (graph/safetensors_loader.h:26-92) — we keep
every stored dtype (no silent F16/BF16 -> F32 promotion) and read through mmap.
"""
from __future__ import annotations

import os

import torch

from .._ext import native


def _rt():
    return native().runtime


def load_file(path: str, device=None, keys=None) -> dict:
    f = _rt().SafeTensorsFile(os.fspath(path))
    out = {}
    for k in (keys if keys is not None else f.keys()):
        t = f.get(k)
        out[k] = t.to(device) if device is not None else t
    return out


def load_metadata(path: str) -> dict:
    return dict(_rt().SafeTensorsFile(os.fspath(path)).metadata())


def keys(path: str):
    return list(_rt().SafeTensorsFile(os.fspath(path)).keys())


def save_file(path: str, tensors: dict, metadata: dict | None = None, sort_keys: bool = True,
              align8: bool = True):
    """Write tensors (any device/dtype) + string metadata.  ``align8=False, sort_keys=True`` gives the
    reference LoraSaver byte layout; the default pads the header like HF safetensors."""
    items = [(k, v.detach().contiguous().cpu()) for k, v in tensors.items()]
    md = [(str(k), str(v)) for k, v in (metadata or {}).items()]
    _rt().save_safetensors(os.fspath(path), items, md, sort_keys, align8)


def load_model_dir(model_dir: str) -> dict:
    """Load every *.safetensors shard of an HF model directory into one CPU state dict."""
    import glob
    files = sorted(glob.glob(os.path.join(model_dir, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no .safetensors files in {model_dir}")
    sd = {}
    for f in files:
        sd.update(load_file(f))
    return sd
