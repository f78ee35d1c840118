"""Cross-framework training alignment (the reference's pytorch_alignment/ harness):
N optimizer steps of OUR engine (model graph + LoRA injection + TrainStep with gradient accumulation,
global grad-norm clip and FusedAdamW) against a plain PyTorch baseline -- HF transformers with
hand-written LoRA adapters (PEFT is not installed here), ``torch.optim.AdamW`` and
``clip_grad_norm_`` -- on identical weights, adapters and token batches.  fp32 on CPU, so the loss
curves and the final adapters must agree to float rounding (the reference asked for "within 1-2 %",
pytorch_alignment/README.md:121-131)."""
import pytest
import torch

from mobilefinetuner_amd.models import hf_io
from mobilefinetuner_amd.optim.adamw import FusedAdamW
from mobilefinetuner_amd.peft import lora as L
from mobilefinetuner_amd.train.engine import TrainStep
from mobilefinetuner_amd.utils.params import FlatParams

LR, WD, CLIP, STEPS, ACCUM = 1e-2, 0.01, 1.0, 6, 2


class _LoraWrap(torch.nn.Module):
    """y = base(x) + s * (x A^T) B   (A [r, in], B [r, out]: the adapter layout of our LoRASlice)."""

    def __init__(self, base, A, B, s):
        super().__init__()
        self.base, self.s = base, s
        self.A = torch.nn.Parameter(A.detach().clone())
        self.B = torch.nn.Parameter(B.detach().clone())

    def forward(self, x):
        return self.base(x) + self.s * (x @ self.A.t()) @ self.B


def _batches(vocab, seed):
    """One fixed accumulation group replayed every step (as the reference's fixed-batch alignment
    runs): the loss must then fall step over step, not just match."""
    g = torch.Generator().manual_seed(seed)
    mb = []
    for _ in range(ACCUM):
        t = torch.randint(0, vocab, (2, 17), generator=g)
        mb.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
    return [mb] * STEPS


def _nonzero_b(added):
    """B = 0 at init gives A no step-1 gradient; start both sides from the same small random B."""
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for _, _, B in added:
            B.copy_(torch.randn(B.shape, generator=g) * 0.02)


def _run_ours(model, batches):
    flat = FlatParams(L.lora_parameters(model), "cpu", shadow=False)
    opt = FusedAdamW(flat, lr=LR, weight_decay=WD, max_grad_norm=CLIP)
    step = TrainStep(model, flat, opt, grad_accum=ACCUM)
    losses, grads1 = [], None
    for mb in batches:
        losses.append(float(step(mb).item()))
        if grads1 is None:  # step-1 gradients (pre-clip: the optimizer never rescales .grad in place)
            grads1 = {n: p.grad.detach().clone() for n, p in flat.named()}
    return losses, {n: p.detach().clone() for n, p in flat.named()}, grads1


def _run_torch(hf, wraps, batches, vocab):
    params = [p for w in wraps.values() for p in (w.A, w.B)]
    opt = torch.optim.AdamW(params, lr=LR, betas=(0.9, 0.999), eps=1e-8, weight_decay=WD)
    losses, grads1 = [], None
    for mb in batches:
        opt.zero_grad()
        tot = 0.0
        for ids, lab in mb:
            logits = hf(ids).logits[..., :vocab]
            loss = torch.nn.functional.cross_entropy(logits.reshape(-1, vocab).float(), lab.reshape(-1))
            (loss / ACCUM).backward()
            tot += float(loss.detach()) / ACCUM
        if grads1 is None:
            grads1 = {id(p): p.grad.detach().clone() for p in params}
        torch.nn.utils.clip_grad_norm_(params, CLIP)
        opt.step()
        losses.append(tot)
    return losses, grads1


def _compare(ours, ref, ours_params, wraps, g_ours, g_ref):
    # step-1 gradients of every adapter: the tight check (no optimizer in between)
    for name, w in wraps.items():
        for kind, p in (("lora_A", w.A), ("lora_B", w.B)):
            a, b = g_ours[f"{name}.{kind}"], g_ref[id(p)]
            assert torch.allclose(a, b, atol=1e-6 + 1e-4 * b.abs().max().item(), rtol=1e-4), (name, kind)
    assert len(ours) == len(ref)
    for a, b in zip(ours, ref):
        assert abs(a - b) <= 2e-5 * max(1.0, abs(b)), (ours, ref)
    assert ours[-1] < ours[0], "LoRA training did not reduce the loss"
    for name, w in wraps.items():
        for kind, p in (("lora_A", w.A), ("lora_B", w.B)):
            got = ours_params[f"{name}.{kind}"]
            assert torch.allclose(got, p.detach(), atol=0.05 * LR, rtol=1e-2), (name, kind, (got - p).abs().max())
    # (loose: Adam normalises each coordinate, so fp32 rounding in near-zero gradients can move a
    # weight by up to ~lr per step; the gradients above and the loss curve are the tight checks)
    # the adapters really moved (B starts at zero)
    assert any(ours_params[f"{n}.lora_B"].abs().max() > 0 for n in wraps)


def test_gpt2_lora_training_matches_torch_baseline():
    from transformers import GPT2Config as HC, GPT2LMHeadModel
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    cfg = GPT2Config.preset("gpt2-tiny")
    torch.manual_seed(0)
    hf = GPT2LMHeadModel(HC(vocab_size=cfg.vocab_size, n_positions=cfg.n_positions, n_embd=cfg.n_embd,
                            n_layer=cfg.n_layer, n_head=cfg.n_head, resid_pdrop=0, embd_pdrop=0, attn_pdrop=0))
    hf.train()
    ours = GPT2Model(cfg, dtype=torch.float32, device="cpu", init=False)
    hf_io.load_gpt2_state(ours, hf.transformer.state_dict())
    added = L.inject_gpt2(ours, L.LoraSpec(rank=4, alpha=8, targets=["AttnQKV", "AttnProj"]))
    _nonzero_b(added)
    for p in hf.parameters():
        p.requires_grad_(False)
    wraps = {}
    for name, A, B in added:  # layer.{i}.attn.qkv / layer.{i}.attn.proj  <->  HF c_attn / attn.c_proj
        i = int(name.split(".")[1])
        attn = hf.transformer.h[i].attn
        attr = "c_attn" if name.endswith("qkv") else "c_proj"
        w = _LoraWrap(getattr(attn, attr), A, B, 8 / 4)
        setattr(attn, attr, w)
        wraps[name] = w
    batches = _batches(cfg.vocab_size, 7)
    ref, g_ref = _run_torch(hf, wraps, batches, cfg.vocab_size)
    ours_losses, ours_params, g_ours = _run_ours(ours, batches)
    _compare(ours_losses, ref, ours_params, wraps, g_ours, g_ref)


@pytest.mark.parametrize("targets", ["full", "attention_only"])
def test_gemma3_lora_training_matches_torch_baseline(targets):
    from transformers import Gemma3ForCausalLM, Gemma3TextConfig
    from mobilefinetuner_amd.models.gemma3 import Gemma3Config, Gemma3Model
    cfg = Gemma3Config.preset("gemma3-tiny")
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
    hf = Gemma3ForCausalLM(hc)
    with torch.no_grad():  # HF zero-inits the (1 + w) norms: perturb them so the offset is exercised
        for n, p in hf.named_parameters():
            if "norm" in n:
                p.normal_(0, 0.1)
    hf.train()
    ours = Gemma3Model(cfg, dtype=torch.float32, device="cpu", init=False)
    hf_io.load_gemma_state(ours, hf.state_dict())
    added = L.inject_gemma(ours, L.LoraSpec(rank=4, alpha=8, targets=L.parse_gemma_targets(targets)))
    _nonzero_b(added)
    for p in hf.parameters():
        p.requires_grad_(False)
    hf_mod = {"attn.q": ("self_attn", "q_proj"), "attn.k": ("self_attn", "k_proj"), "attn.v": ("self_attn", "v_proj"),
              "attn.proj": ("self_attn", "o_proj"), "mlp.gate": ("mlp", "gate_proj"), "mlp.up": ("mlp", "up_proj"),
              "mlp.down": ("mlp", "down_proj")}
    wraps = {}
    for name, A, B in added:
        parts = name.split(".")
        i, key = int(parts[1]), ".".join(parts[2:])
        owner, attr = hf_mod[key]
        parent = getattr(hf.model.layers[i], owner)
        w = _LoraWrap(getattr(parent, attr), A, B, 8 / 4)
        setattr(parent, attr, w)
        wraps[name] = w
    batches = _batches(cfg.vocab_size, 11)
    ref, g_ref = _run_torch(hf, wraps, batches, cfg.vocab_size)
    ours_losses, ours_params, g_ours = _run_ours(ours, batches)
    _compare(ours_losses, ref, ours_params, wraps, g_ours, g_ref)
