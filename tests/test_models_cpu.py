"""Model-level parity on CPU: our GPT-2 / Gemma-3 graphs vs HF transformers on identical random
weights (the reference's PyTorch-golden tests, graph/test_gpt2_forward.cpp and
test_gemma_forward.cpp, used pretrained checkpoints we do not have: parity is pinned to HF
instead, on random-init weights + synthetic tokens)."""
import pytest
import torch

from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
from mobilefinetuner_amd.models import hf_io


def _hf_gpt2(cfg):
    from transformers import GPT2Config as HC, GPT2LMHeadModel
    hc = HC(vocab_size=cfg.vocab_size, n_positions=cfg.n_positions, n_embd=cfg.n_embd, n_layer=cfg.n_layer,
            n_head=cfg.n_head, resid_pdrop=0, embd_pdrop=0, attn_pdrop=0)
    torch.manual_seed(0)
    m = GPT2LMHeadModel(hc).eval()
    return m


def test_gpt2_forward_matches_hf():
    cfg = GPT2Config.preset("gpt2-tiny")
    hf = _hf_gpt2(cfg)
    ours = GPT2Model(cfg, dtype=torch.float32, device="cpu", init=False)
    hf_io.load_gpt2_state(ours, hf.transformer.state_dict())
    ids = torch.randint(0, cfg.vocab_size, (2, 33))
    with torch.no_grad():
        ref = hf(ids).logits
        got = ours.logits(ids)
    assert (got - ref).abs().max().item() < 1e-4
    lab = ids[:, 1:]
    with torch.no_grad():
        loss = ours(ids[:, :-1], lab)
        ref_loss = torch.nn.functional.cross_entropy(hf(ids[:, :-1]).logits.reshape(-1, cfg.vocab_size),
                                                     lab.reshape(-1))
    assert abs(loss.item() - ref_loss.item()) < 1e-4


def test_gpt2_export_roundtrip():
    cfg = GPT2Config.preset("gpt2-tiny")
    a = GPT2Model(cfg, dtype=torch.float32, device="cpu", seed=3)
    b = GPT2Model(cfg, dtype=torch.float32, device="cpu", init=False)
    hf_io.load_gpt2_state(b, hf_io.export_gpt2_state(a))
    for (n1, p1), (n2, p2) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(p1, p2), n1


def test_gpt2_lora_grads_reach_attention_cpu():
    """attention-side LoRA must receive a real gradient."""
    from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2, lora_parameters
    from mobilefinetuner_amd.utils.params import FlatParams
    cfg = GPT2Config.preset("gpt2-tiny")
    m = GPT2Model(cfg, dtype=torch.float32, device="cpu")
    inject_gpt2(m, LoraSpec(rank=4, alpha=8))
    flat = FlatParams(lora_parameters(m), "cpu", shadow=False)
    # make B non-zero so A also gets gradient
    for n, p in flat.named():
        if n.endswith("lora_B"):
            p.data.normal_(0, 0.1)
    ids = torch.randint(0, cfg.vocab_size, (2, 17))
    loss = m(ids[:, :-1], ids[:, 1:])
    loss.backward()
    for n, p in flat.named():
        assert p.grad is not None and p.grad.abs().sum() > 0, n
