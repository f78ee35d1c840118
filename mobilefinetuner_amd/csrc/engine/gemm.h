// libmft engine: GEMM front-end -- every matrix product on a hand-written gfx950 kernel, no vendor GEMM
// library.  Replaces the reference's naive/cblas matmul (core/ops.cpp:486-802) and MatmulBackward
// (core/backward_functions.cpp:94-138).  Routing (static: identical on every rank and rerun;
// MFT_GEMM_MAP=1 prints it, profiles/r5_gemm_routing_map.txt):
//   * K-contiguous products -- NT forwards (+ bias, + fused residual), every fused NT epilogue (bias +
//     GELU / GELU', x aux, x GELU'(aux)), the LM-head CE forward, and data gradients through a
//     transposed weight: gemm4 (csrc/kernels/gemm4.hip, 4-wave hand-scheduled persistent kernel);
//   * token-major layouts -- split-K TN weight gradients, NN data gradients, the CE dgrad, the LoRA
//     epilogue: gemm8 (csrc/kernels/gemm8.hip, 8-phase pipeline, ds_read_b64_tr_b16);
//   * anything else (fp32, K % 64 != 0, unaligned strides): the generic fallback (kernels/gemm_simt.hip),
//     fp32 MFMA (v_mfma_f32_16x16x4_f32: exact fp32, the native --dtype fp32 mode runs on it).
#pragma once
#include "engine/tensor.h"

namespace mft {
namespace eng {

// y[M, N] = x[M, K] . W[N, K]^T (+ bias[N]); bf16; y row-major (may be a row-strided view)
void gemm_nt(const Tensor& x2, const Tensor& w, const Tensor& bias, Tensor& y, const Tensor& resid = Tensor());
// out[M, K] = dy[M, N] . W[N, K]   (data gradient; out may be a row-strided view)
void gemm_nn(const Tensor& dy2, const Tensor& w, Tensor& out, const Tensor& wt = Tensor());
// buf[N, K] (fp32) += alpha * dy[M, N]^T . x[M, K]
void gemm_wgrad(Tensor& buf, const Tensor& dy2, const Tensor& x2, float alpha = 1.f);
// gemm8 with one of the fused epilogues of csrc/kernels.h (GEMM_EPI_*): C = epi(alpha op(A) op(B));
// b_kn: B stored [K, N] (NN) instead of [N, K] (NT)
struct Gemm8Extra {
  const Tensor* bias = nullptr;
  Tensor* aux = nullptr;          // BIAS_GELU: pre-activation out; DGELU: pre-activation in
  const Tensor* lora_u = nullptr;  // LORA: C += lora_u[M, r] . lora_w[r, N]
  const Tensor* lora_w = nullptr;
  float alpha = 1.f;
};
void gemm8_call(const Tensor& a, const Tensor& b, bool b_kn, int epi, Tensor& c, const Gemm8Extra& ex = {});
// c[M, N] = a[M, K] b[N, K]^T + a2[M, K2] b2[N, K2]^T on gemm4 (second K segment, K2 % 64 == 0): the
// LoRA data gradient dx = dy W + v A with v zero-padded to 64 columns; lora_seg2_ok: the shape runs there
void gemm_nt_seg2(const Tensor& a, const Tensor& b, const Tensor& a2, const Tensor& b2, Tensor& c);
bool lora_seg2_ok(long M, long N, long K);
// Gemma-3 GeGLU MLP in the gemm4 epilogues (kernels.h GEMM_EPI_GEGLU_*), replacing the gated_fwd /
// gated_bwd passes.  geglu_fusable: gemm4 (not the short-token kernel) runs both the gate|up product
// (M x 2I x K) and the down data gradient (M x I x Kd), I % 128 == 0 (MFT_GEGLU_FUSE=0: off, A/B)
bool geglu_fusable(long M, long I, long K, long Kd);
// gu = x w^T [M, 2I] (w = [W_gate; W_up] rows) and h[:, :I] = gelu(g) u (h row stride >= I, its tail untouched)
void gemm_geglu_fwd(const Tensor& x2, const Tensor& w, Tensor& gu, Tensor& h);
// dh = dy wt^T (+ a2 b2^T: the LoRA data gradient's second K segment) feeds the epilogue only:
// dgu [M, 2I] = (dh u gelu'(g) | dh gelu(g)) from gu
void gemm_geglu_bwd(const Tensor& dy2, const Tensor& wt, const Tensor& gu, Tensor& dgu, const Tensor& a2 = Tensor(),
                    const Tensor& b2 = Tensor());
// generic (fp32 or bf16, any transposes) C = alpha op(A) op(B) + beta C (gemm4 / gemm8 / SIMT fallback)
void blas_gemm(const Tensor& a, bool ta, const Tensor& b, bool tb, Tensor& c, float alpha = 1.f, float beta = 0.f);
bool gemm8_all();
bool nt_gemm4();
bool deterministic();
void set_deterministic(bool on);
bool gemm4_on();                // MFT_GEMM4=0 -> gemm8 for every product (A/B)
bool short_tokens(long M, long N, long K, int epi);  // gemm_s takes this product

}  // namespace eng
}  // namespace mft
