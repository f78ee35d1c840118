// libmft engine: the fused transformer ops the models are built from (autograd-aware).
//
// Each op wraps one or two of the gfx950 kernels of csrc/kernels/*.hip and records ONE node:
//   add_layer_norm   residual add + LayerNorm fwd/bwd (norm.hip)       reference ops.cpp:1404-1458
//   embed            token + position embedding gather / scatter-add    gpt2_model.cpp:346-381,500-528
//   attention_packed causal flash attention on the packed qkv GEMM output (attention.hip)
//                    reference memory_efficient_attention.cpp:40-185 (forward only there)
//   mlp_gelu         fc GEMM + bias + GELU epilogue, proj GEMM; backward dGELU fused (gemm8.hip)
//   lora_linear_aug  base GEMM over the augmented K dim [x | u] . [W | s B^T]^T (lora.hip + GEMM)
//                    reference LoRALinear nn/lora_linear.cpp:47-108
//   lm_head_ce       tied LM head + fused cross entropy fwd+bwd (gemm8 CE epilogues, xent.hip)
//                    reference lm_loss.cpp:19-210, gpt2_model.cpp:425-439
// Trainable parameters are fp32 masters (autograd leaves; their .grad is a view into the
// optimizer's flat fp32 buffer) with bf16 compute shadows; the kernels accumulate straight into
// those grad buffers.  A `Param` pairs the leaf with its compute view.
#pragma once
#include <cstdint>
#include <utility>
#include <vector>

#include "engine/tensor.h"

namespace mft {
namespace eng {

struct Param {
  Tensor leaf;  // autograd leaf: fp32 master (trainable) or the frozen compute weight itself
  Tensor c;     // compute view: bf16 shadow (trainable) or == leaf (frozen)
  Tensor wt;    // cached [in, out] transposed copy of a FROZEN 2-D weight (NT data-grad GEMMs)
  Tensor lora_acat;  // [sum r, in] the adapters' A stacked (one rowdot pass for several adapters), refreshed
                     // by the batched LoRA weight prep instead of a concatenation per step
  Tensor lora_at;  // [in, 64] A^T of the LoRA adapters on this frozen weight, zero-padded (gemm4 second K
                   // segment); allocated and zeroed once, the first r columns rewritten every backward
  bool streamed = false;  // a slot view of the weight-streaming tier: no cached copies of it
  bool trainable() const { return leaf.defined() && leaf.requires_grad(); }
  const Tensor& transposed();  // builds wt once (frozen weights only)
};

// s = x + delta (if delta defined), y = LayerNorm(s) (or RMSNorm(1+w) when rms); y allocated
// [M, out_cols] when out_cols > N (appended columns zeroed, for a LoRA consumer's augmented input).
// Returns {s, y} (s == x when no delta).
// lora_a [R, N] (bf16, defined only with out_cols >= N + R): the appended columns receive u = y A^T
// instead of zeros -- the LoRA consumer's input projection fused into the norm (lora_fused_a).
// resid_out (no delta): s is returned as an OUTPUT of the norm node (sharing x's storage), so the gradient
// the residual stream sends back through s is added by the norm backward kernel (its fused dresid input)
// instead of by a separate accumulation pass -- for an x that a GEMM epilogue already summed with the
// residual (gemm_nt resid).
std::pair<Tensor, Tensor> add_norm(const Tensor& x, const Tensor& delta, Param& w, Param* b, float eps, bool rms,
                                   float offset, int out_cols, const Tensor& lora_a = Tensor(), bool resid_out = false);
Tensor embed(const Tensor& ids, Param& wte, Param* wpe, float scale);
// qkv [B, S, 3, H, D] -> o [B, S, H*D] (or [B, S, out_cols] with zeroed tail when out_cols > H*D)
Tensor attention_packed(const Tensor& qkv, float scale, bool causal, int window, int out_cols);
// resid (optional, [..., N]): the returned tensor is resid + MLP(x), added in the projection GEMM's epilogue
Tensor mlp_gelu(const Tensor& x, Param& w1, Param& b1, Param& w2, Param& b2, const Tensor& resid = Tensor());
// Gemma-3 attention core on the packed q|k|v projection qkv [B, S, nq + 2 nkv, D]: per-head
// RMSNorm(offset + w) of q and k + RoPE (cos / sin [>= S, D/2] fp32 tables), then causal GQA flash
// attention (sliding window when window > 0).  O [B, S, nq*D] (or [B, S, out_cols], zeroed tail).
// One node owns the three slices: its backward writes ONE packed dqkv (dV by the attention
// backward, dQ / dK by the norm-RoPE backward kernels into their slices).
Tensor qknorm_rope_attention(const Tensor& qkv, int nq, int nkv, Param& wq, Param& wk, const Tensor& cos_t,
                             const Tensor& sin_t, float eps, float offset, bool interleaved, float scale, int window,
                             int out_cols);
// gated MLP activation on gu = [gate | up] [M, 2I]: act(gate) * up (act 0 GELU-tanh = GeGLU, 1 SiLU);
// [M, out_cols] with zeroed tail when out_cols > I (augmented-K input of a LoRA consumer)
Tensor gated_act(const Tensor& gu, int act, int out_cols);
// y = x W^T + b on bf16 [M, K] rows (trainable or frozen W).
// GeGLU MLP fusion (Gemma-3, gemm.h geglu_fusable):
//   geglu_h (gate|up projection): y = gu [M, 2I]; *geglu_h [M, >= I] also receives h = gelu(g) u from the
//     GEMM's epilogue (its columns past I are the caller's) -- no autograd edge of its own;
//   geglu_gu (down projection): x is that h buffer, the node's input is gu instead, and the backward's data
//     gradient GEMM writes d gu straight from its epilogue (the GeGLU backward; dh is never stored)
Tensor linear_p(const Tensor& x, Param& w, Param* b, Tensor* geglu_h = nullptr, const Tensor& geglu_gu = Tensor());

struct LoraAdapter {
  int col0 = 0, ncols = 0, rank = 8;
  Param A, B;  // A [r, in], B [r, ncols] (fp32 masters + bf16 shadows)
  float dropout = 0.f;
  uint32_t salt = 0;
};
// The LoRA layers' per-step weight prep (s B^T into each augmented-K weight, A^T into each padded
// second-segment operand) as ONE batched launch at the start of a model's forward: the first forwards
// run the copies one by one and register them; lora_prep_step_begin (at the start of a forward, outside
// graph capture for the first time) uploads the list and from then on launches it, and each layer skips
// the copy the batch already made (an entry whose tensors changed is simply redone by its layer).
void lora_prep_step_begin();
// the forward is over: a later LoRA layer call runs its own copies (no stale batch assumed)
void lora_prep_step_end();
// forget every registered entry (a model is destroyed); uploaded lists stay allocated for live graphs
void lora_prep_reset();
// width of the augmented input [x | u_1..u_n | 0]: in + sum(r), rounded to 64
int lora_aug_cols(int in_features, const std::vector<LoraAdapter>& ads);
// xa [M, Ka] holds x in its first K columns (zero tail); waug [N, Ka] = [W | s B^T.. | 0] (owned by
// the caller, W copied once); W frozen.
// u_ready: the producer already wrote u_1..u_n into xa's appended columns (add_norm with lora_a =
// lora_fused_a(ads)); the adapters' A must not change between that producer and this call.
// resid (optional, [..., N]): the returned tensor is resid + the LoRA linear, added in the GEMM's epilogue
// (needs a bias); its gradient is the output's
// geglu_h / geglu_gu: the GeGLU fusion of linear_p, on the augmented-K LoRA projection
Tensor lora_linear_aug(const Tensor& xa, int K, Param& w, Param* b, std::vector<LoraAdapter>& ads, float scale,
                       Tensor& waug, bool training, const Tensor& drop_ctr, bool u_ready = false,
                       const Tensor& resid = Tensor(), Tensor* geglu_h = nullptr, const Tensor& geglu_gu = Tensor());
// the [sum r_i, in] stack of the adapters' A (bf16 compute copies) when a producer can compute u for
// lora_linear_aug itself (no dropout in effect, sum r <= 32); undefined otherwise
Tensor lora_fused_a(const std::vector<LoraAdapter>& ads, bool training);
// plain (non-augmented) LoRA Linear: y = x W^T + b + s * (drop(x) A_i^T) B_i in column slices
Tensor lora_linear(const Tensor& x, Param& w, Param* b, std::vector<LoraAdapter>& ads, float scale, bool training,
                   const Tensor& drop_ctr);
// mean token NLL of logits = h W^T over the first V columns (labels -100 ignored); the W gradient
// (tied embedding in full fine-tuning) is produced during forward scaled by w_grad_scale
Tensor lm_head_ce(const Tensor& h, Param& w, const Tensor& labels, int V, int64_t chunk, float w_grad_scale,
                  bool sum_reduction = false);
// per-token NLL [M] fp32 (0 at ignored labels), no gradients (alignment dumps)
Tensor lm_head_token_nll(const Tensor& h, Param& w, const Tensor& labels, int V, int64_t chunk);
// (sum of NLL over valid rows, number of valid rows) without gradients -- evaluation
std::pair<Tensor, Tensor> lm_head_nll(const Tensor& h, Param& w, const Tensor& labels, int V, int64_t chunk);

// ------------------------------------------------------------------ reference-precision composite path
// --dtype: the models' compute precision.  BF16 (default) runs the fused kernels above; F32 runs the
// reference's own precision (it computes everything in fp32, core/ops.cpp:545-573) as a composite of the
// generic op catalog (ops.h: fp32 SIMT GEMMs, row softmax, elementwise / reduction kernels), every op
// differentiated by the tape.  Set before a model is built (its weights are allocated in that dtype).
void set_compute_dtype(DType d);
DType compute_dtype();
// materialized masked-softmax attention (the reference's standard path, graph/gpt2_model.cpp:679-711 and
// graph/gemma_model.cpp:481-508): q [B, Sq, H, D], k / v [B, Sk, Hkv, D] (GQA through repeat_kv) ->
// [B, Sq, H * D]; causal, window > 0 = sliding window.  --dtype fp32 and --attn_impl naive.
Tensor attention_ref(const Tensor& q, const Tensor& k, const Tensor& v, float scale, bool causal, int window);
// composite LoRA Linear on 2-D x (reference nn/lora_linear.cpp:47-108, + PEFT dropout on the adapter input):
// y = x W^T (+ b) + sum_i s drop(x) A_i^T B_i over output columns [col0_i, col0_i + ncols_i); drop_step
// seeds the dropout masks (one per step and adapter)
Tensor lora_linear_ref(const Tensor& x, Param& w, Param* b, std::vector<LoraAdapter>& ads, float s, bool training,
                       uint64_t drop_step);
// the tensor the composite path computes with: the autograd leaf of a trainable parameter (its fp32
// master -- the gradient lands in the flat grad buffer through the tape), else the compute view
inline const Tensor& cw(const Param& p) { return p.trainable() ? p.leaf : p.c; }
// x [M, n] -> [M, cols] with zero columns appended (differentiable); x itself when cols <= n
Tensor pad_cols(const Tensor& x, int64_t cols);
// number of labels != -100, fp32 [1] on the device
Tensor valid_count(const Tensor& labels);

}  // namespace eng
}  // namespace mft
