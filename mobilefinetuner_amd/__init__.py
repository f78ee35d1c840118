"""mobilefinetuner_amd — an MI355X-native (gfx950) LLM fine-tuning framework.

Capabilities of jmha02/MobileFineTuner (GPT-2 / Gemma-3 LoRA and full fine-tuning, PEFT-style
safetensors LoRA checkpoints, WikiText-2 perplexity and MMLU evaluation, parameter sharding with a
host offload tier, energy-aware throttling), re-designed for AMD Instinct MI355X:
PyTorch-ROCm tensors + hand-written HIP/CDNA4 kernels (``csrc/kernels``) + RCCL over xGMI
(``parallel/``), with a native C++ runtime (``csrc/runtime``) for tokenization, IO, datasets and
host offload.
"""
__version__ = "0.1.0"


def __getattr__(name):
    # lazy: `python -m mobilefinetuner_amd._build --native` (the torch-free engine + CLIs) must not import
    # torch; native() loads torch before the extension that links it
    if name == "native":
        from ._ext import native
        return native
    raise AttributeError(f"module 'mobilefinetuner_amd' has no attribute {name!r}")
