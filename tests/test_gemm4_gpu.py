"""gemm4 (kernels/gemm4.hip: 4-wave hand-scheduled persistent MFMA GEMM, the product path for NT GEMMs)
against plain PyTorch fp32 on the same bf16 operands, for every epilogue it carries, on ragged shapes
(M, N not multiples of the 256 x 256 tile, the minimum K = 128, the augmented-K 832) -- the tails go
through the range-checked loads and stores."""
import pytest
import torch

pytestmark = pytest.mark.gpu

NONE, BIAS, DGELU, GELU_D, MUL_AUX, BIAS_ADD = 0, 1, 3, 9, 10, 11
# (the last two: gemm_s splits K over 4 workgroups per tile -- few tiles, long K; gemm_s runs 32-row tiles where
# the 64-row grid has < 128 tiles: (300, 264), (257, 8), (512, 768), (200, 136) -- and 64-row tiles on the rest)
SHAPES = [(300, 264, 128), (1000, 776, 832), (4096, 3072, 768), (257, 8, 192), (2048, 640, 2048), (512, 768, 3072),
          (200, 136, 2048)]


def _gelu(x):
    t = torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3))
    return 0.5 * x * (1 + t), 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * x * x)


def _ops(M, N, K, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.1).bfloat16()
    b = (torch.rand(N, device="cuda", generator=g) - 0.5).bfloat16()
    aux = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    return x, w, b, aux


def _rel(a, ref):
    return ((a.float() - ref).abs().max() / ref.abs().max().clamp(min=1e-6)).item()


@pytest.mark.parametrize("impl", [4, 5], ids=["gemm4", "gemm_s"])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm4_epilogues_match_fp32(M, N, K, impl):
    from mobilefinetuner_amd._ext import native
    C = native()
    x, w, b, aux = _ops(M, N, K)
    mm = x.float() @ w.float().t()
    pre = mm + b.float()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    C.gemm_t(x, w, False, False, NONE, None, None, 1.0, y, None, None, impl)
    assert _rel(y, mm) < 1e-2
    C.gemm_t(x, w, False, False, BIAS, b, None, 1.0, y, None, None, impl)
    assert _rel(y, pre) < 1e-2
    d = torch.empty_like(y)
    C.gemm_t(x, w, False, False, GELU_D, b, d, 1.0, y, None, None, impl)
    gl, gd = _gelu(pre)
    assert _rel(y, gl) < 2e-2 and _rel(d, gd) < 2e-2
    C.gemm_t(x, w, False, False, MUL_AUX, None, aux, 1.0, y, None, None, impl)
    assert _rel(y, mm * aux.float()) < 2e-2
    C.gemm_t(x, w, False, False, DGELU, None, aux, 1.0, y, None, None, impl)
    assert _rel(y, mm * _gelu(aux.float())[1]) < 2e-2
    r = aux.clone()  # fused residual, in place (aux aliases the output)
    C.gemm_t(x, w, False, False, BIAS_ADD, b, r, 1.0, r, None, None, impl)
    assert _rel(r, pre + aux.float()) < 2e-2
    torch.cuda.synchronize()


@pytest.mark.parametrize("impl", [4, 5], ids=["gemm4", "gemm_s"])
def test_gemm4_row_strided_output_and_alpha(impl):
    """Output written into a column slice of a wider buffer (row stride > N), alpha != 1: columns outside
    the slice stay untouched."""
    from mobilefinetuner_amd._ext import native
    C = native()
    M, N, K = 700, 512, 256
    x, w, b, _ = _ops(M, N, K, seed=3)
    buf = torch.full((M, N + 64), 7.0, device="cuda", dtype=torch.bfloat16)
    y = buf[:, :N]
    C.gemm_t(x, w, False, False, BIAS, b, None, 0.5, y, None, None, impl)
    torch.cuda.synchronize()
    assert _rel(y, 0.5 * (x.float() @ w.float().t()) + b.float()) < 1e-2
    assert (buf[:, N:] == 7.0).all()


@pytest.mark.parametrize("impl", [4, 5], ids=["gemm4", "gemm_s"])
def test_gemm4_is_deterministic(impl):
    from mobilefinetuner_amd._ext import native
    C = native()
    x, w, b, _ = _ops(3000, 2304, 768, seed=5)
    y1 = torch.empty(3000, 2304, device="cuda", dtype=torch.bfloat16)
    y2 = torch.empty_like(y1)
    C.gemm_t(x, w, False, False, BIAS, b, None, 1.0, y1, None, None, impl)
    C.gemm_t(x, w, False, False, BIAS, b, None, 1.0, y2, None, None, impl)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)


@pytest.mark.parametrize("impl", [4, 5], ids=["gemm4", "gemm_s"])
@pytest.mark.parametrize("M,N,K,K2", [(1000, 768, 2304, 64), (4096, 768, 768, 64), (300, 264, 128, 128), (512, 776, 64, 64),
                                      (512, 768, 2304, 64)])
def test_gemm4_second_k_segment(M, N, K, K2, impl):
    if impl == 4 and K < 128:
        pytest.skip("gemm4 needs K >= 128")
    """out = A B^T + A2 B2^T in one persistent pass (the LoRA data gradient dx = dy W + v A with v = s dy B
    zero-padded to 64 columns)."""
    from mobilefinetuner_amd._ext import native
    C = native()
    x, w, _, _ = _ops(M, N, K, seed=9)
    g = torch.Generator(device="cuda").manual_seed(4)
    a2 = torch.zeros(M, K2, device="cuda", dtype=torch.bfloat16)
    b2 = torch.zeros(N, K2, device="cuda", dtype=torch.bfloat16)
    a2[:, :8] = torch.randn(M, 8, device="cuda", generator=g).bfloat16()
    b2[:, :8] = (torch.randn(N, 8, device="cuda", generator=g) * 0.1).bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    C.gemm4_seg2(x, w, a2, b2, y, impl)
    ref = x.float() @ w.float().t() + a2.float() @ b2.float().t()
    torch.cuda.synchronize()
    assert _rel(y, ref) < 1e-2


def test_gemm_s_split_k_deterministic_and_rearmed():
    """gemm_s with K split across workgroups (last-arriving workgroup sums the partials in split order):
    bit-identical over repeated calls (the per-tile counters re-arm), and equal to the fp32 product."""
    from mobilefinetuner_amd._ext import native
    C = native()
    x, w, b, aux = _ops(256, 768, 3072, seed=7)  # 96 tiles of 32 x 64: S = 4 workgroups per tile
    ys = []
    for _ in range(6):
        y = torch.empty(256, 768, device="cuda", dtype=torch.bfloat16)
        C.gemm_t(x, w, False, False, MUL_AUX, None, aux, 1.0, y, None, None, 5)
        ys.append(y)
    torch.cuda.synchronize()
    assert all(torch.equal(ys[0], y) for y in ys[1:])
    assert _rel(ys[0], (x.float() @ w.float().t()) * aux.float()) < 2e-2


@pytest.mark.parametrize("M,I,K", [(4096, 2048, 704), (1000, 256, 640), (300, 384, 1152)])
def test_gemm4_geglu_epilogues_match_fp32(M, I, K):
    """The Gemma-3 GeGLU MLP in gemm4's epilogues against fp32 torch on the same bf16 operands:
    forward -- gu = x [Wg; Wu]^T and h = gelu(g) u (h into a wider, row-strided buffer whose tail stays
    untouched); backward -- dh = dy Wd (plus a LoRA-style second K segment) never stored, d gu = (dh u
    gelu'(g) | dh gelu(g)).  Ragged M, the 1B width (I 6912 is not tested: same code, I % 128)."""
    from mobilefinetuner_amd._ext import native
    C = native()
    g = torch.Generator(device="cuda").manual_seed(11)
    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(2 * I, K, device="cuda", generator=g) * 2 - 1) * 0.08).bfloat16()
    gu = torch.empty(M, 2 * I, device="cuda", dtype=torch.bfloat16)
    hbuf = torch.full((M, I + 64), 5.0, device="cuda", dtype=torch.bfloat16)
    C.gemm4_geglu(x, w, hbuf, gu, I, True)
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t()
    assert _rel(gu, ref) < 1e-2
    gq, uq = gu[:, :I].float(), gu[:, I:].float()  # h is formed from the stored (bf16) gu, like gated_fwd
    assert _rel(hbuf[:, :I], _gelu(gq)[0] * uq) < 2e-2
    assert (hbuf[:, I:] == 5.0).all()
    # backward (down projection H -> I data gradient), with and without the second K segment
    H = 640
    dy = (torch.rand(M, H, device="cuda", generator=g) * 2 - 1).bfloat16()
    wt = ((torch.rand(I, H, device="cuda", generator=g) * 2 - 1) * 0.08).bfloat16()
    a2 = torch.zeros(M, 64, device="cuda", dtype=torch.bfloat16)
    a2[:, :8] = (torch.rand(M, 8, device="cuda", generator=g) - 0.5).bfloat16()
    b2 = torch.zeros(I, 64, device="cuda", dtype=torch.bfloat16)
    b2[:, :8] = (torch.rand(I, 8, device="cuda", generator=g) - 0.5).bfloat16()
    for seg in (False, True):
        dgu = torch.empty(M, 2 * I, device="cuda", dtype=torch.bfloat16)
        if seg:
            C.gemm4_geglu(dy, wt, gu, dgu, I, False, a2, b2)
            dh = dy.float() @ wt.float().t() + a2.float() @ b2.float().t()
        else:
            C.gemm4_geglu(dy, wt, gu, dgu, I, False)
            dh = dy.float() @ wt.float().t()
        torch.cuda.synchronize()
        a, ag = _gelu(gq)
        assert _rel(dgu[:, :I], dh * uq * ag) < 2e-2, seg
        assert _rel(dgu[:, I:], dh * a) < 2e-2, seg


# gemm4 TN (gemm4_tn_kernel): the full fine-tune weight gradient C (fp32) += alpha A^T B over K tokens, both
# operands token-major.  Shapes: GPT-2 qkv / proj at a token split (fp32 slabs + ordered reduce), the
# minimum K = 128 (no split), ragged M / N (tiles past the edges read out of range), XL's 1600 columns,
# and row strides wider than the operands (column views).
TN_SHAPES = [(2304, 768, 8192, 0), (768, 768, 16384, 0), (256, 256, 128, 0), (1600, 1600, 4096, 0), (200, 72, 640, 0),
             (776, 264, 2048, 64), (50304, 768, 45056, 0)]  # (the last: the tied LM-head weight, a 4.5 GB operand)


@pytest.mark.parametrize("M,N,K,pad", TN_SHAPES)
def test_gemm4_tn_wgrad_matches_fp32(M, N, K, pad):
    from mobilefinetuner_amd._ext import native
    C = native()
    g = torch.Generator(device="cuda").manual_seed(1)
    a_full = (torch.rand(K, M + pad, device="cuda", generator=g) * 2 - 1).bfloat16()
    b_full = (torch.rand(K, N + pad, device="cuda", generator=g) * 2 - 1).bfloat16()
    a, b = a_full[:, :M], b_full[:, :N]
    c0 = torch.randn(M, N, device="cuda", generator=g)
    ref = c0.clone()
    for k in range(0, K, 8192):
        ref += 0.5 * (a[k:k + 8192].float().t() @ b[k:k + 8192].float())
    out = c0.clone()
    F32ACC = 4
    C.gemm_t(a, b, True, True, F32ACC, None, None, 0.5, out, None, None, 4)
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-4, _rel(out, ref)
    # and the 8-wave kernel it replaces agrees
    out8 = c0.clone()
    C.gemm_t(a, b, True, True, F32ACC, None, None, 0.5, out8, None, None, 0)
    assert _rel(out8, out) < 1e-4
