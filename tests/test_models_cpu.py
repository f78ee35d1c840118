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


def _hf_gemma(cfg):
    from transformers import Gemma3ForCausalLM, Gemma3TextConfig
    hc = Gemma3TextConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                          intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_hidden_layers,
                          num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
                          head_dim=cfg.head_dim, sliding_window=cfg.sliding_window, layer_types=cfg.layer_types,
                          query_pre_attn_scalar=int(cfg.query_pre_attn_scalar),
                          max_position_embeddings=cfg.max_position_embeddings,
                          rope_parameters={"full_attention": {"rope_type": "default", "rope_theta": cfg.rope_theta},
                                           "sliding_attention": {"rope_type": "default",
                                                                 "rope_theta": cfg.rope_local_base_freq}},
                          attn_implementation="eager")
    torch.manual_seed(0)
    m = Gemma3ForCausalLM(hc).eval()
    with torch.no_grad():  # HF inits norms at zero; perturb so (1+w) is exercised
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(0, 0.1)
    return m


@pytest.mark.parametrize("S", [12, 40])
def test_gemma3_forward_matches_hf(S):
    from mobilefinetuner_amd.models.gemma3 import Gemma3Config, Gemma3Model
    cfg = Gemma3Config.preset("gemma3-tiny")
    hf = _hf_gemma(cfg)
    ours = Gemma3Model(cfg, dtype=torch.float32, device="cpu", init=False)
    hf_io.load_gemma_state(ours, hf.state_dict())
    ids = torch.randint(0, cfg.vocab_size, (2, S))
    with torch.no_grad():
        ref = hf(ids).logits
        got = ours.logits(ids)
    assert (got - ref).abs().max().item() < 2e-4, (got - ref).abs().max().item()


def test_gemma3_config_from_hf_dict():
    from mobilefinetuner_amd.models.gemma3 import Gemma3Config
    d = {"vocab_size": 262144, "hidden_size": 640, "intermediate_size": 2048, "num_hidden_layers": 18,
         "num_attention_heads": 4, "num_key_value_heads": 1, "head_dim": 256, "sliding_window": 512,
         "rope_theta": 1000000.0, "rope_local_base_freq": 10000.0, "query_pre_attn_scalar": 256,
         "max_position_embeddings": 32768}
    c = Gemma3Config.from_dict(d)
    assert c.layer_types[5] == "full_attention" and c.layer_types[0] == "sliding_attention"
    assert c.head_dim == 256 and c.num_key_value_heads == 1 and c.rope_local_base_freq == 10000.0
    assert Gemma3Config.preset("gemma3-270m").hidden_size == 640
