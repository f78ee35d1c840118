"""Fused LM head + cross entropy (gemm8 CE epilogues, xent.hip lm_head_ce) vs plain PyTorch fp32
cross entropy on the same bf16 inputs: loss, dh and (materialised path) dW, at the GPT-2 (V = 50257,
padded 50304) and Gemma-3 (V = 262144) vocabularies, with ignored rows, ragged row counts and
pretrained-scale logits (|logit| ~ 100, where raw bf16 logits would be quantised to 0.5)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(h, W, labels, V):
    hf = h.float().requires_grad_(True)
    Wf = W.float().requires_grad_(True)
    logits = (hf @ Wf.t())[:, :V]
    loss = torch.nn.functional.cross_entropy(logits, labels, ignore_index=-100)
    loss.backward()
    return loss.detach(), hf.grad, Wf.grad


def _case(M, K, V, Vpad, logit_scale=1.0, ignore_frac=0.1, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    h = (torch.randn(M, K, device="cuda", generator=g) * logit_scale).bfloat16()
    W = (torch.randn(Vpad, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    W[V:] = 0
    labels = torch.randint(0, V, (M,), device="cuda", generator=g)
    labels[torch.rand(M, device="cuda", generator=g) < ignore_frac] = -100
    return h, W, labels


def _fused(h, W, labels, V, materialize):
    from mobilefinetuner_amd._ext import native
    C = native()
    M = h.shape[0]
    valid = (labels >= 0).sum().float()
    scale = (1.0 / valid.clamp(min=1.0)).reshape(1)
    loss_rows = torch.empty(M, device="cuda")
    E = torch.empty(M, W.shape[0], device="cuda", dtype=torch.bfloat16)
    dh = torch.empty_like(h)
    C.lm_head_ce(h, W, labels, V, E, loss_rows, scale, 1.0, dh, materialize)
    loss = loss_rows.sum() * scale
    return loss, dh, E


@pytest.mark.parametrize("M,K,V,Vpad,ls", [(8192, 768, 50257, 50304, 1.0), (1000, 768, 50257, 50304, 1.0),
                                           (8192, 640, 262144, 262144, 1.0), (4096, 768, 50257, 50304, 12.0)])
def test_lm_head_ce_matches_fp32(M, K, V, Vpad, ls):
    h, W, labels = _case(M, K, V, Vpad, ls)
    ref_loss, ref_dh, _ = _ref(h, W, labels, V)
    loss, dh, _ = _fused(h, W, labels, V, materialize=False)
    torch.cuda.synchronize()
    assert abs(loss.item() - ref_loss.item()) < 2e-3 * max(1.0, abs(ref_loss.item())), (loss.item(), ref_loss.item())
    err = (dh.float() - ref_dh).norm() / ref_dh.norm()
    assert err < 1e-2, err.item()
    # ignored rows get exactly zero gradient
    ign = labels < 0
    if ign.any():
        assert dh[ign].abs().max().item() == 0.0


def test_lm_head_ce_materialized_dlogits_and_dw():
    from mobilefinetuner_amd.ops.functional import _mm_wgrad_into  # noqa: F401  (routing used by the op)
    M, K, V, Vpad = 2048, 768, 50257, 50304
    h, W, labels = _case(M, K, V, Vpad, 1.0)
    ref_loss, ref_dh, ref_dW = _ref(h, W, labels, V)
    loss, dh, G = _fused(h, W, labels, V, materialize=True)
    dW = G.float().t() @ h.float()
    torch.cuda.synchronize()
    assert abs(loss.item() - ref_loss.item()) < 2e-3 * max(1.0, abs(ref_loss.item()))
    assert ((dh.float() - ref_dh).norm() / ref_dh.norm()).item() < 1e-2
    assert ((dW - ref_dW).norm() / ref_dW.norm()).item() < 1e-2
    assert G[:, V:].abs().max().item() == 0.0


def test_lm_head_ce_fused_and_materialized_dh_agree():
    M, K, V, Vpad = 4096, 768, 50257, 50304
    h, W, labels = _case(M, K, V, Vpad, 4.0, seed=3)
    l1, dh1, _ = _fused(h, W, labels, V, materialize=False)
    l2, dh2, _ = _fused(h, W, labels, V, materialize=True)
    torch.cuda.synchronize()
    assert l1.item() == l2.item()
    assert ((dh1.float() - dh2.float()).norm() / dh2.float().norm()).item() < 1e-2


def test_lm_head_token_nll_matches_fp32():
    from mobilefinetuner_amd.ops import functional as Fx
    M, K, V, Vpad = 3000, 768, 50257, 50304
    h, W, labels = _case(M, K, V, Vpad, 2.0, seed=5)
    ref = torch.nn.functional.cross_entropy((h.float() @ W.float().t())[:, :V], labels, ignore_index=-100,
                                            reduction="sum")
    nll, n = Fx.lm_head_token_nll(h, W, labels, V)
    torch.cuda.synchronize()
    assert n.item() == (labels >= 0).sum().item()
    assert abs(nll.item() - ref.item()) < 1e-4 * abs(ref.item()), (nll.item(), ref.item())


@pytest.mark.parametrize("M,K,V,Vpad,forced", [(8192, 640, 262144, 262144, "4"), (6000, 768, 50257, 50304, "9"),
                                                (512, 768, 50257, 50304, "22")])  # (the 4 x 128 chunk: 40 automatically)
def test_lm_head_ce_vocab_split_dgrad_matches_unsplit(M, K, V, Vpad, forced, monkeypatch):
    """The vocab-split CE dgrad (fp32 slabs per split, reduced in split order; chosen automatically when a
    row chunk's dh tiles cannot fill the CUs) against the single-pass dgrad (MFT_CE_SPLIT=1) and fp32."""
    from mobilefinetuner_amd._ext import native
    h, W, labels = _case(M, K, V, Vpad, 3.0, seed=7)
    auto = native().ce_dgrad_splits(M, K, Vpad)
    assert auto > 1, auto
    monkeypatch.setenv("MFT_CE_SPLIT", "1")
    l1, dh1, _ = _fused(h, W, labels, V, materialize=False)
    monkeypatch.setenv("MFT_CE_SPLIT", forced)
    l2, dh2, _ = _fused(h, W, labels, V, materialize=False)
    monkeypatch.delenv("MFT_CE_SPLIT")
    l3, dh3, _ = _fused(h, W, labels, V, materialize=False)
    _, ref_dh, _ = _ref(h, W, labels, V)
    torch.cuda.synchronize()
    assert l1.item() == l2.item() == l3.item()
    for dh in (dh1, dh2, dh3):
        assert ((dh.float() - ref_dh).norm() / ref_dh.norm()).item() < 1e-2
    assert ((dh2.float() - dh1.float()).norm() / dh1.float().norm()).item() < 1e-2
    assert dh2[labels < 0].abs().max().item() == 0.0


@pytest.mark.parametrize("M,K,V,Vpad", [(8192, 768, 50257, 50304), (1000, 768, 50257, 50304), (4096, 640, 262144, 262144),
                                        (777, 128, 70001, 70016)])
def test_lm_head_ce_gemm4_forward_matches_gemm8(M, K, V, Vpad, monkeypatch):
    """The CE forward on gemm4 (default where supported) against gemm8's CE epilogue (MFT_CE_G4=0): the same
    per-row losses (fp32 statistics of the same bf16 products), the same E operand up to bf16 rounding,
    and dh against fp32."""
    h, W, labels = _case(M, K, V, Vpad, 2.0, seed=11)
    l4, dh4, E4 = _fused(h, W, labels, V, materialize=False)
    monkeypatch.setenv("MFT_CE_G4", "0")
    l8, dh8, E8 = _fused(h, W, labels, V, materialize=False)
    monkeypatch.delenv("MFT_CE_G4")
    _, ref_dh, _ = _ref(h, W, labels, V)
    torch.cuda.synchronize()
    assert abs(l4.item() - l8.item()) < 1e-4 * max(1.0, abs(l8.item())), (l4.item(), l8.item())
    assert ((E4.float() - E8.float()).abs().max()).item() < 1e-2
    assert ((dh4.float() - ref_dh).norm() / ref_dh.norm()).item() < 1e-2
    assert dh4[labels < 0].abs().max().item() == 0.0
