// libmft engine: GEMM front-end -- routes every matrix product to the hand-written gfx950 MFMA
// kernels (csrc/kernels/gemm8.hip: 256x256x64 8-phase pipeline, NT / NN / TN, fused epilogues) or,
// for plain library-shaped products where it measured faster, to hipBLASLt called directly
// (autotuned plans, no torch).  Replaces the reference's naive/cblas matmul (core/ops.cpp:486-802)
// and MatmulBackward (core/backward_functions.cpp:94-138).  Routing (bench_gemm_t.py on MI355X):
//   * fused epilogues (bias+GELU, x GELU'(pre), rank-r LoRA update) and NN data-grads: gemm8;
//   * plain NT forwards y = x W^T + b: hipBLASLt (gemm8 0.74-0.93x there); MFT_GEMM8_ALL=1 -> gemm8;
//   * fp32 weight-grad accumulation: gemm8 split-K TN for <= 2304x768 outputs, hipBLASLt beyond.
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
// generic (fp32 or bf16, any transposes) C = alpha op(A) op(B) + beta C through hipBLASLt
void blas_gemm(const Tensor& a, bool ta, const Tensor& b, bool tb, Tensor& c, float alpha = 1.f, float beta = 0.f);
bool gemm8_all();
bool nt_gemm4();
bool deterministic();
void set_deterministic(bool on);
// hipBLASLt per-shape algorithm autotuning (timing the heuristic's candidates) on / off; multi-rank
// apps turn it off so every rank runs the same algorithms (an explicit MFT_LT_TUNE overrides)
void set_lt_autotune(bool on);

}  // namespace eng
}  // namespace mft
