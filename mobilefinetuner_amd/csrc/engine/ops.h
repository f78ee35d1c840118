// libmft engine: differentiable op catalog (functional API over eng::Tensor).
//
// The reference's core/ops.cpp (:167-2745) + core/backward_functions.cpp (35 BackwardFunction
// classes) re-designed for the GPU: every op runs one of the gfx950 kernels (engine/tensor_kernels.hip for
// the generic families, csrc/kernels/*.hip for the fused hot ops) on the current stream and records
// one autograd Node when an input needs a gradient.  Shapes broadcast NumPy-style for the binary
// ops (the reference's elementwise_binary_op); reshapes / transposes are zero-copy views
// (tensor.h) instead of the reference's copying transpose / permute (ops.cpp:804-961).
#pragma once
#include <vector>

#include "engine/tensor_kernels.h"
#include "engine/tensor.h"

namespace mft {
namespace eng {

k::Desc desc(const Tensor& t);
k::Desc desc_bcast(const Tensor& t, const Shape& over);
Shape broadcast_shape(const Shape& a, const Shape& b);
// reduce g (broadcast result) back to `shape` by summing the broadcast dims
Tensor sum_to(const Tensor& g, const Shape& shape);

// ---- elementwise (broadcasting), reference core/ops.cpp:282-484
Tensor add(const Tensor& a, const Tensor& b, float alpha = 1.f);
Tensor sub(const Tensor& a, const Tensor& b);
Tensor mul(const Tensor& a, const Tensor& b);
Tensor div(const Tensor& a, const Tensor& b);
Tensor maximum(const Tensor& a, const Tensor& b);
Tensor minimum(const Tensor& a, const Tensor& b);
Tensor add_scalar(const Tensor& a, float s);
Tensor mul_scalar(const Tensor& a, float s);
Tensor affine(const Tensor& a, float scale, float shift);  // scale * a + shift
// in-place accumulate (no autograd): a += alpha * b
void add_(Tensor& a, const Tensor& b, float alpha = 1.f);

// ---- unary math (:1033-2651) with backward
Tensor neg(const Tensor& x);
Tensor relu(const Tensor& x);
Tensor gelu(const Tensor& x, bool tanh_approx = true);
Tensor silu(const Tensor& x);
Tensor sigmoid(const Tensor& x);
Tensor tanh(const Tensor& x);
Tensor exp(const Tensor& x);
Tensor log(const Tensor& x);
Tensor sqrt(const Tensor& x);
Tensor rsqrt(const Tensor& x);
Tensor abs(const Tensor& x);
Tensor square(const Tensor& x);
Tensor pow(const Tensor& x, float p);
Tensor clamp(const Tensor& x, float lo, float hi);
Tensor sin(const Tensor& x);
Tensor cos(const Tensor& x);

// ---- comparisons (no grad; bool outputs)
Tensor eq(const Tensor& a, const Tensor& b);
Tensor ne(const Tensor& a, const Tensor& b);
Tensor gt(const Tensor& a, const Tensor& b);
Tensor lt(const Tensor& a, const Tensor& b);
Tensor ge(const Tensor& a, const Tensor& b);
Tensor le(const Tensor& a, const Tensor& b);

// ---- reductions (:1782-1939)
Tensor sum(const Tensor& x);                              // all elements -> [1]
Tensor sum(const Tensor& x, int dim, bool keepdim = false);
Tensor mean(const Tensor& x);
Tensor mean(const Tensor& x, int dim, bool keepdim = false);

// ---- softmax family (:1119-1230), last dim
Tensor softmax(const Tensor& x);
Tensor log_softmax(const Tensor& x);

// ---- losses (:1232-1714, core/lm_loss.cpp:106-210)
Tensor mse_loss(const Tensor& x, const Tensor& y);                 // mean
Tensor nll_loss(const Tensor& logp, const Tensor& target, int ignore_index = -100);  // mean over valid
Tensor cross_entropy(const Tensor& logits, const Tensor& target, int ignore_index = -100);
// HF-shifted LM loss over [B, S, V] logits (logits[:, :-1] vs labels[:, 1:]), reference lm_loss.cpp
Tensor lm_cross_entropy(const Tensor& logits, const Tensor& labels, int ignore_index = -100);

// ---- linear algebra (:486-1031)
// batched matmul with broadcasting of a 2-D right operand; bf16 or fp32
Tensor matmul(const Tensor& a, const Tensor& b);
// y = x W^T + b, W [out, in] (nn.Linear layout)
Tensor linear(const Tensor& x, const Tensor& w, const Tensor& b = Tensor());

// ---- misc
Tensor dropout(const Tensor& x, float p, uint64_t seed, bool training = true);
Tensor cat(const std::vector<Tensor>& ts, int dim);
Tensor where_mask(const Tensor& mask, const Tensor& a, float fill);  // mask ? a : fill (no grad on mask; finite fill)
Tensor embedding(const Tensor& ids, const Tensor& table);           // gather rows (scatter-add backward)

// ---- composite layers of the reference catalog, built from the ops above (the tape differentiates
// them); the training models run the fused kernels of nn.h instead.  Reference: layer_norm
// core/ops.cpp:1404-1458, rms_norm / rms_norm_affine :1489-1574, batch_norm, swiglu, causal mask /
// apply_mask and repeat_kv_heads :2072-2149, apply_rope :2151-2225.
Tensor layer_norm(const Tensor& x, const Tensor& w, const Tensor& b, float eps = 1e-5f);  // over the last dim
// x / rms(x) * (offset + w): offset 1 = Gemma's RMSNorm(1 + w), 0 = the affine variant
Tensor rms_norm(const Tensor& x, const Tensor& w, float eps = 1e-6f, float offset = 1.f);
// training-mode batch norm of x [N, C]: batch mean / biased variance per channel, then gamma, beta
Tensor batch_norm(const Tensor& x, const Tensor& gamma, const Tensor& beta, float eps = 1e-5f);
Tensor swiglu(const Tensor& gate, const Tensor& up);  // silu(gate) * up
Tensor geglu(const Tensor& gate, const Tensor& up);   // gelu_tanh(gate) * up
// [Sq, Sk] fp32 keep-mask (1 = attend): key j <= query i + (Sk - Sq), and within `window` (> 0)
Tensor causal_mask(int64_t Sq, int64_t Sk, int64_t window = 0);
// scores where mask == 0 -> -1e30 (finite, so a fully-masked row stays NaN-free; softmax weight 0)
Tensor apply_mask(const Tensor& scores, const Tensor& mask);
// GQA: [B, S, Hkv, D] -> [B, S, Hkv * n_rep, D] (q head h reads kv head h / n_rep)
Tensor repeat_kv(const Tensor& x, int n_rep);
// RoPE on x [.., S, H, D] with cos / sin [S, D / 2]: rotate-half pairs (d, d + D/2), or interleaved
// pairs (2d, 2d + 1) (the reference's layout)
Tensor apply_rope(const Tensor& x, const Tensor& cos_t, const Tensor& sin_t, bool interleaved = false);

}  // namespace eng
}  // namespace mft
