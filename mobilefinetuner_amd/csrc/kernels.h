// Host-side launcher API of the gfx950 kernels (raw device pointers + explicit stream).
// The torch bindings (csrc/bindings.cpp) are the only caller; nothing here allocates or
// synchronises, so every launcher is hipGraph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mft {
typedef uint16_t bf16_t;

// ---------------------------------------------------------------- norms (norm.hip)
int norm_bwd_partial_blocks(int M);
// out[i] (+)= sum_b part[b * N + i]  (deterministic partial-row reduction for weight grads)
void reduce_rows(const float* part, float* out, int nb, int N, int accumulate, hipStream_t st);
// ldy / lddy: row stride of the normalised output / of its gradient (0 = N).  A wider output row
// leaves room for appended columns (the LoRA augmented-K input [x | u], lora.hip).
// lora_a [lora_r, N] (row stride lda, bf16; lora_r <= 32 <= ldy - N): the appended columns receive
// u = y A^T (the LoRA consumer's input projection) instead of zeros.
void layernorm_fwd(const bf16_t* x, const bf16_t* resid_delta, bf16_t* resid_out, const float* w, const float* b,
                   bf16_t* y, float* mean, float* rstd, int M, int N, float eps, long ldy, hipStream_t st,
                   const bf16_t* lora_a = nullptr, long lda = 0, int lora_r = 0);
void rmsnorm_fwd(const bf16_t* x, const bf16_t* resid_delta, bf16_t* resid_out, const float* w, bf16_t* y, float* rstd,
                 int M, int N, float eps, float w_offset, long ldy, hipStream_t st, const bf16_t* lora_a = nullptr,
                 long lda = 0, int lora_r = 0);
void layernorm_bwd(const bf16_t* x, const bf16_t* dy, const float* w, const float* mean, const float* rstd,
                   const bf16_t* dresid, bf16_t* dx, float* dw, float* db, float* work, int M, int N, int accumulate,
                   long lddy, hipStream_t st);
void rmsnorm_bwd(const bf16_t* x, const bf16_t* dy, const float* w, const float* rstd, const bf16_t* dresid, bf16_t* dx,
                 float* dw, float* work, int M, int N, float w_offset, int accumulate, long lddy, hipStream_t st);

// ---------------------------------------------------------------- attention (attention.hip)
struct AttnArgs {
  const bf16_t *q, *k, *v;
  bf16_t* o;
  float* lse;
  long q_st[3], k_st[3], v_st[3], o_st[3];  // batch, seq, head strides (elements)
  int B, H, Hkv, Sq, Sk, D;
  float scale;
  int causal, window;
  const int* kv_lens;
  // zero o_pad columns (% 8) after the H heads of each output row (a widened output for an augmented-K
  // consumer; rows batch-contiguous): the short and DMA kernels write them, other paths by a zero_cols pass
  int o_pad;
};
struct AttnBwdArgs {
  const bf16_t *q, *k, *v, *o, *dout;
  const float* lse;
  float* delta;   // [B,H,Sq] workspace
  float* dq_acc;  // [B,Sq,H,D] fp32 workspace
  bf16_t *dq, *dk, *dv;
  bf16_t *dk_tmp, *dv_tmp;  // [B,Sk,H,D] workspaces (GQA only)
  long q_st[3], k_st[3], v_st[3], o_st[3], do_st[3], dq_st[3], dk_st[3], dv_st[3], tmp_st[3];
  int B, H, Hkv, Sq, Sk, D;
  float scale;
  int causal, window;
  const int* kv_lens;
};
void attn_fwd(const AttnArgs& a, hipStream_t s);
void attn_bwd(const AttnBwdArgs& a, hipStream_t s);
// true when the single-workgroup-per-(batch, head) kernels run (no delta / dq_acc workspaces)
bool attn_short_path(int D, int Sq, int Sk, int window);
// 0: short path; 1: long-sequence kernels with fp32 dQ atomics (needs delta + dq_acc, and the
// dk_tmp/dv_tmp workspaces under GQA); 2: split dK/dV + dQ kernels (needs delta only)
int attn_bwd_path(int D, int Sq, int Sk, int window);

// ---------------------------------------------------------------- GEMM (gemm8.hip)
enum GemmEpi { GEMM_EPI_NONE = 0, GEMM_EPI_BIAS = 1, GEMM_EPI_BIAS_GELU = 2, GEMM_EPI_DGELU = 3, GEMM_EPI_F32ACC = 4,
               GEMM_EPI_LORA = 5, GEMM_EPI_F32PART = 6 /* internal: split-K fp32 slab */,
               // fused LM-head cross entropy (gemm8 only, driven by lm_head_ce in xent.hip)
               GEMM_EPI_CE_FWD = 7, GEMM_EPI_CE_DGRAD = 8,
               // GELU MLP (gemm8 only): the forward stores GELU'(pre) -- not pre -- as aux (one
               // sigmoid serves GELU and its derivative), the backward multiplies by it
               GEMM_EPI_BIAS_GELU_D = 9, GEMM_EPI_MUL_AUX = 10,
               // residual-producing projection (gemm8 only): C = alpha A.B + bias + aux (aux = the
               // residual stream [M, N]), i.e. the transformer's residual add in the GEMM's epilogue
               GEMM_EPI_BIAS_ADD = 11,
               // Gemma-3 GeGLU MLP in the GEMM epilogues (gemm4 only; geglu_I = I, I % 128 == 0):
               // GEGLU_FWD -- C = gu = x [Wg; Wu]^T [M, 2I] and aux = h = gelu(g) u [M, I] (row stride
               // ldaux), the B rows of each 256-column tile are 128 gate rows + the matching 128 up rows;
               // GEGLU_BWD -- the accumulator is dh [M, I] (N = I); aux = gu [M, 2I] (read), C = dgu
               // [M, 2I] (ldc): dg = dh u gelu'(g), du = dh gelu(g)
               GEMM_EPI_GEGLU_FWD = 12, GEMM_EPI_GEGLU_BWD = 13 };
struct GemmArgs {
  const bf16_t* A;
  long lda;  // A [M, K] row-major
  const bf16_t* B;
  long ldb;  // NT: B [N, K]; NN: B [K, N]
  void* C;
  long ldc;  // bf16 [M, N] (fp32 for GEMM_EPI_F32ACC, accumulated)
  const bf16_t* bias;  // [N]
  bf16_t* aux;
  long ldaux;  // BIAS_GELU: pre-activation out; DGELU: pre-activation in
  int M, N, K;
  float alpha;
  // GEMM_EPI_LORA (gemm8 only): C += lora_u[M, lora_r] . lora_w[lora_r, N] (rank-r update fused
  // into the epilogue, e.g. dx = dy W + v A of a LoRA Linear's backward)
  const bf16_t* lora_u;
  long ld_lu;
  const bf16_t* lora_w;
  long ld_lw;
  int lora_r;
  // split-K (GEMM_EPI_F32ACC only): ksplit > 1 splits K into slabs ws[ksplit][M][N] (fp32) that
  // gemm_splitk_reduce adds into C in a fixed order (deterministic, no atomics)
  int ksplit;
  float* ws;
  // GEMM_EPI_CE_FWD (NT, C = h W^T never stored as logits): per 256-column vocab tile and row the
  // epilogue writes (tile max, tile sum-exp) to ce_stats [M][ceil(N/256)] (float pairs), the label
  // logit to ce_lbl [M], and -- when C is set -- E = exp(logit - tile max) (bf16; columns >= ce_V
  // are 0).  GEMM_EPI_CE_DGRAD (NN, dh = softmax(logits) W - onehot W from E): the accumulator is
  // rescaled by ce_ratio at every vocab-tile start ([T][Mpad] in the tile-row order of
  // lm_head_ce), the epilogue applies ce_fin [M] and subtracts ce_wlab [M] x W[label].
  const int64_t* ce_labels;
  float* ce_stats;
  float* ce_lbl;
  const float* ce_ratio;
  const float* ce_fin;
  const float* ce_wlab;
  int ce_V;
  // gemm8: 1 = compute the (A*, B1) quadrants of an N-tail tile anyway (set by gemm8x from
  // MFT_GEMM8_NTAIL=0 for A/B runs; the CE dgrad never skips them)
  int ntail_full;
  // gemm8: > 0 delays the first-round workgroups (blockIdx < 256) by (blockIdx >> 3) x stagger
  // cycles, spreading every XCD's CUs over a tile round so their prologue fills and epilogue
  // stores do not all hit HBM at once (MFT_G8_STAGGER, A/B)
  int stagger;
  // gemm4 second K segment (NONE epilogue): C = A B^T + A2 B2^T, A2 [M, K2], B2 [N, K2] (row strides
  // lda2 / ldb2, K2 % 64 == 0; 0 = none)
  const bf16_t* A2;
  long lda2;
  const bf16_t* B2;
  long ldb2;
  int K2;
  // gemm4 epilogue operand (aux) loads: 0 = non-temporal (default), 1 = default cache policy (A/B)
  int aux_pol;
  // GEGLU_FWD / GEGLU_BWD: the MLP width I (gate | up halves of gu)
  int geglu_I;
  // gemm_s split-K hand-off: 1 = agent-scope release / acquire fences around the arrival counter
  // (MFT_STRICT_HANDOFF=1); 0 = the sc1-store / sc1-load form alone (see gemm_s.hip)
  int handoff_fence;
};
// 256x256 8-phase pipelined GEMM (gemm8.hip); same epilogues.  a_t: A stored [K, M]; b_t: B stored
// [K, N] (NN data-grad); both: TN weight-grad (use GEMM_EPI_F32ACC with gemm8_pick_ksplit / ws)
void gemm8(const GemmArgs& g, int epi, hipStream_t st);  // NT
void gemm8x(const GemmArgs& g, int epi, bool a_t, bool b_t, hipStream_t st);
// 256x256x64 4-wave GEMM with a hand-scheduled K-tile body (gemm4.hip); NT layout
void gemm4x(const GemmArgs& g, int epi, bool a_t, bool b_t, hipStream_t st);
bool gemm4_supported(int M, int N, int K, bool a_t, bool b_t);
// TN weight gradient on the 4-wave kernel: C fp32 [M, N] (ldc) += alpha A^T B, A [K, M] (lda), B [K, N]
// (ldb), K = tokens; ksplit > 1 (gemm4_tn_pick_ksplit) needs ws = ksplit x M x N floats
bool gemm4_tn_supported(int M, int N, int K, long lda, long ldb);
int gemm4_tn_pick_ksplit(int M, int N, int K);
void gemm4_tn(const GemmArgs& g, hipStream_t st);
// persistent gemm4 grids leave n CUs free (for a long-running kernel on a side stream; 0 = every CU)
void gemm4_reserve_cus(int n);
// short-token NT GEMM (gemm_s.hip): 64 x 64 tiles, K split over the 4 waves; NONE / BIAS / BIAS_GELU_D /
// MUL_AUX / DGELU / BIAS_ADD and the second K segment (K2, NONE only).  gemm_s_preferred: the shape's
// gemm4 tiles would fill less than half the CUs
bool gemm_s_supported(int M, int N, int K, int epi);
bool gemm_s_preferred(int M, int N, int K);
void gemm_s(const GemmArgs& g, int epi, hipStream_t st);
bool gemm8_supported(int M, int N, int K, bool a_t, bool b_t);
int gemm8_pick_ksplit(int M, int N, int K);
// NT NONE / BIAS / BIAS_GELU_D: the persistent streaming form with the deferred epilogue (opt-in,
// MFT_GEMM8_STREAM=1); A/B switch for benchmarks
void gemm8_set_stream(int on);
void gemm8_set_stagger(int cycles);  // first-round stagger (cycles per XCD slot), A/B
// generic fallback (gemm_simt.hip, fp32 MFMA v_mfma_f32_16x16x4_f32): D = alpha op(A) op(B) (+ bias[N]) + beta Cin; fp32 or bf16
// operands (x_f32 flags), fp32 accumulation; ta: A stored [K, M]; tb: B stored [N, K]
struct SimtGemmArgs {
  const void* A;
  long lda;
  int a_f32, ta;
  const void* B;
  long ldb;
  int b_f32, tb;
  void* D;
  long ldd;
  int d_f32;
  const void* Cin;
  long ldcin;
  int cin_f32;
  const bf16_t* bias;
  int M, N, K;
  float alpha, beta;
};
void gemm_simt(const SimtGemmArgs& a, hipStream_t st);
void gemm_splitk_reduce(const float* ws, int ksplit, int M, int N, float* C, long ldc, float alpha, int accumulate,
                        hipStream_t st);

// ---------------------------------------------------------------- activations (act.hip)
void gelu_fwd(const bf16_t* x, bf16_t* y, long n, hipStream_t st);
void gelu_bwd(const bf16_t* x, const bf16_t* dy, bf16_t* dx, long n, hipStream_t st);
// gu: [M, 2I] (gate | up); y: [M, I]; act 0 = gelu_tanh (GeGLU), 1 = silu (SwiGLU)
void gated_fwd(const bf16_t* gu, bf16_t* y, long M, int I, long ldy, int act, hipStream_t st, int zpad = 0);  // zpad: zero cols after I
void gated_bwd(const bf16_t* gu, const bf16_t* dy, long ldd, bf16_t* dgu, long M, int I, int act, hipStream_t st);

// ---------------------------------------------------------------- embedding (embed.hip)
// out[m] = wte[ids[m]] * scale (+ wpe[pos0 + m % S])
void embed_fwd(const int64_t* ids, const bf16_t* wte, const bf16_t* wpe, bf16_t* out, long M, int C, int S, int pos0,
               float scale, hipStream_t st);
// dwte[ids[m]] += dout[m]*scale (fp32 atomics); dwpe[p] += sum over batch.  det_vocab > 0: the
// deterministic form (fixed summation order per table row, no float atomics; V = det_vocab rows)
void embed_bwd(const int64_t* ids, const bf16_t* dout, float* dwte, float* dwpe, long M, int C, int S, int pos0,
               float scale, hipStream_t st, long det_vocab = 0);

// ---------------------------------------------------------------- cross entropy (xent.hip)
// logits [M, ld] bf16 (first V columns valid); labels [M] (-100 = ignore).  Writes per-row loss
// (0 for ignored rows) and overwrites logits[:, :V] with dlogits = (softmax - onehot) * (*scale)
// (columns >= V set to 0).  scale may be null (=> 1.0); extra multiplies it.
void xent_fwd_bwd(bf16_t* logits, const int64_t* labels, float* loss, long M, int V, long ld, const float* scale,
                  float extra, int write_grad, hipStream_t st);
// Fused LM head + cross entropy over a chunk of rows: logits = h W^T are never written to HBM.
//   1. gemm8 NT with the CE_FWD epilogue: E = exp(logit - tile max) (bf16) + per-tile (max, sum-exp)
//      + label logit from the fp32 accumulators;
//   2. ce_finalize: row lse, loss, per-tile rescale factors;
//   3. (grad) gemm8 NN with the CE_DGRAD main loop: dh = (softmax - onehot) W * scale from E with
//      the per-(row, tile) softmax factor applied as an accumulator rescale at each vocab-tile
//      boundary (no elementwise pass over the [M, V] operand), or -- when the W gradient is needed
//      too (materialize) -- E is turned into dlogits in place and multiplied by a plain NN GEMM
//      (the caller then forms dW = dlogits^T h from it).
struct CeArgs {
  const bf16_t* h; long ldh;   // [M, K]
  const bf16_t* W; long ldw;   // [Vpad, K]
  const int64_t* labels;       // [M] (-100 / out of range = ignored)
  int M, K, Vpad, V;
  bf16_t* E; long lde;         // [M, Vpad] workspace (null: loss only)
  float* loss;                 // [M] per-row NLL (0 for ignored rows)
  float* lse;                  // [M] (optional)
  const float* scale;          // device scalar weight of a valid row (e.g. 1 / n_valid), null = 1
  float extra;
  bf16_t* dh; long lddh;       // [M, K] out (null: no gradient)
  int materialize;             // E := dlogits (for a W gradient by the caller)
  float* ws;                   // lm_head_ce_ws_floats(M, Vpad, K) floats
  const bf16_t* Wt; long ldwt; // optional W^T [K, Vpad] (materialize): dh = dlogits W as gemm4's NT product
};
long lm_head_ce_ws_floats(int M, int Vpad, int K);
// vocab splits of the CE dgrad for an M-row chunk (1 = one pass straight into dh)
int ce_dgrad_splits(int M, int K, int Vpad);
void lm_head_ce(const CeArgs& a, hipStream_t st);
// log-softmax gather: out[m, c] = logits[m, idx[c]] - lse(logits[m])  (MMLU scoring)
void logsoftmax_gather(const bf16_t* logits, const int64_t* idx, float* out, long M, int V, long ld, int nidx,
                       hipStream_t st);

// ---------------------------------------------------------------- optimizer (optim.hip)
// sum of squares of n fp32 values -> partial[nblk]; then out[0] = sum(partial)
int sumsq_blocks(long n);
void sumsq(const float* x, long n, float* partial, float* out, int accumulate, hipStream_t st);
// Fused AdamW over flat fp32 buffers.  clip: grads scaled by min(1, max_norm/(sqrt(*sumsq)+1e-6))
// if sumsq != null.  lr read from device (*lr_ptr) so a captured graph can replay with new LRs.
// If shadow != null also writes the bf16 copy of the updated params (shadow[i] at shadow_idx map).
struct AdamWArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  long n;
  const float* lr_ptr;
  float beta1, beta2, eps, weight_decay;
  const float* step_ptr;  // device count of applied steps (this update uses t = *step_ptr + 1)
  const float* sumsq;     // device grad-norm^2 (or null)
  float max_norm;
  int l2_coupled;         // reference-compat: g += wd*p instead of decoupled decay
  bf16_t* shadow;         // optional bf16 copy
  const int* nonfinite;   // optional device flag: skip the step when set
  int moments_bf16;       // m / v are bf16 (stochastically rounded; host-offloaded optimizer state)
  long sr_offset;         // global element index of p[0] (chunked / sharded launches): keys the SR hash
  float* vmax;            // AMSGrad: running max of v (fp32 moments only; null = plain Adam(W))
  const int* enable;      // optional device gate: the update runs only when *enable != 0 (a delayed
                          // optimizer's "gradients pending" flag)
  int max_grid;           // > 0: at most this many workgroups (an update that runs beside compute
                          // kernels, latency-bound on PCIe, keeps to a few CUs); 0 = fill the chip
};
void adamw_step(const AdamWArgs& a, hipStream_t st);
// after every adamw_step launch of one update: *step += 1 unless the update was skipped (or gated
// off by *enable == 0); clear_enable: then *enable = 0 (the pending update is consumed)
void adamw_commit(float* step, const int* nonfinite, const float* sumsq, hipStream_t st, int* flag_out = nullptr,
                  int* enable = nullptr, int clear_enable = 0);
// flag[0] = any(!isfinite(x))  (accumulates with OR)
void nonfinite_check(const float* x, long n, int* flag, hipStream_t st);

// ---------------------------------------------------------------- LoRA (lora.hip)
// Layouts: A [R, K] (PEFT lora_A.weight), B [R, N].
// LoRA-input dropout: mask(m, k) = hash(*ctr, salt, m*K + k) >= p, kept values scaled 1/(1-p).
struct LoraDrop {
  const int64_t* ctr;  // device step counter (may be null)
  uint32_t salt;       // per-adapter constant
  float p;             // 0 disables
};
// U[m, r] = s * sum_k X[m, k] * Wt[r, k]          (u = x A^T with Wt = A; v = s dy B^T with Wt = B)
// every LoRA layer's per-step weight prep in ONE launch (engine/nn.cpp LoraPrep): dst[r][c] = scale * src at
// (r * srs + c * scs) for each entry (s B^T into the augmented-K weight, A^T into the padded second-segment
// operand); entries live in device memory, one workgroup per entry
struct LoraPrepEntry {
  bf16_t* dst;
  long dld;
  const bf16_t* src;
  long srs, scs;
  int rows, cols;
  float scale;
};
void lora_prep_batched(const LoraPrepEntry* dev_entries, int n, hipStream_t st);
void lora_rowdot(const bf16_t* X, long ldx, const bf16_t* Wt, long ldw, bf16_t* U, long ldu, long M, int K, int R, float s,
                 LoraDrop drop, hipStream_t st);
// Y[m, n] = base[m, n] + s * sum_r U[m, r] * W[r, n]   (Y may alias base; y += s u B, dx += v A)
void lora_update(const bf16_t* base, long ldb, const bf16_t* U, long ldu, const bf16_t* W, long ldw, bf16_t* Y, long ldy,
                 long M, int N, int R, float s, LoraDrop drop, hipStream_t st);
// out[k*osk + r*osr] += scale * sum_m X[m, k] * Y[m, r]   (fp32 atomics into the grad buffer)
// Segmented form (outs != null, outs->n = R / 8): ranks 8z..8z+7 accumulate into outs->p[z] (rank
// index restarting at 0) -- dA of several rank-8 adapters that share one input, one pass over X.
struct WgradOuts {
  float* p[8];
  int n;
};
// det_ws != null: deterministic mode -- per-row-chunk partials (lora_wgrad_ws_floats(M, K, R) floats)
// summed in a fixed order instead of fp32 atomics
void lora_wgrad(const bf16_t* X, long ldx, const bf16_t* Y, long ldy, float* out, long osk, long osr, long M, int K, int R,
                float scale, LoraDrop drop, hipStream_t st, const WgradOuts* outs = nullptr, float* det_ws = nullptr);
long lora_wgrad_ws_floats(long M, int K, int R);
// rank 8, one pass over dy [M, N]:  dB[r*ldd + n] += s * sum_m u[m, r] dy[m, n]  (fp32 atomics) and
// v[m*ldv + r] = s * sum_n dy[m, n] B[r, n]  (bf16); vpart = fp32 scratch of cdiv(N, 256) * M * 8
void lora_dy(const bf16_t* dy, long ldy, const bf16_t* B, long ldb, const bf16_t* u, long ldu, float* dB, long ldd,
             float* vpart, bf16_t* v, long ldv, long M, int N, float s, hipStream_t st, float* det_ws = nullptr, int vzero = 0);
long lora_dy_ws_floats(long M, int N);  // deterministic-mode workspace of lora_dy (det_ws)
// lora_dy over up to 4 rank-8 adapters on column ranges of ONE dy (q | k | v of a fused projection): one
// launch + one finish.  col0 % 256 == 0, ranges ascending and disjoint in 256-column strips; vz: zero columns
// 8 .. 8 + vz - 1 of that adapter's v (% 8).  vpart: fp32 scratch of (strips of the whole range) * M * 8
struct LoraDyAdapter {
  const bf16_t* B;
  long ldb;
  const bf16_t* u;
  long ldu;
  float* dB;
  long ldd;
  bf16_t* v;
  long ldv;
  int col0, N, vz;
};
bool lora_dy_multi_ok(const LoraDyAdapter* ads, int n);
long lora_dy_multi_vpart_floats(const LoraDyAdapter* ads, int n, long M);
void lora_dy_multi(const bf16_t* dy, long ldy, const LoraDyAdapter* ads, int n, float* vpart, long M, float s,
                   hipStream_t st);
// workgroups of the lora_dy / lora_xty (MFMA) grids for an [M, N] operand: <= 512, one resident round
long lora_dy_grid_blocks(long M, int N);
// W[k*wsk + n*wsn] += s * sum_r A[r, k] * B[r, n]   (A [R,K], B [R,N] fp32)
void lora_merge(void* W, int w_is_bf16, long wsk, long wsn, const float* A, const float* B, int K, int N, int R, float s,
                hipStream_t st);

// ---------------------------------------------------------------- RoPE (rope.hip)
// x strided [B,S,H,D] (st = batch, seq, head strides), in place.  cos/sin tables [S_max, D/2].
void rope_apply(bf16_t* x, const long* st, int B, int S, int H, int D, const float* cos_t, const float* sin_t, int pos0,
                int interleaved, int inverse, hipStream_t stream);
// y[row, :] = rope(rmsnorm(x[row]) * (w + off)), y contiguous [B*S*H, D]; rstd [B*S*H]
void qknorm_rope_fwd(const bf16_t* x, const long* st, bf16_t* y, float* rstd, const float* w, int B, int S, int H, int D,
                     const float* cos_t, const float* sin_t, int pos0, float eps, float off, int interleaved,
                     hipStream_t stream);
int qknorm_rope_bwd_blocks(long rows);
void qknorm_rope_bwd(const bf16_t* x, const long* st, const bf16_t* dy, const float* rstd, const float* w, bf16_t* dx,
                     const long* dst, float* dw, float* work, int B, int S, int H, int D, const float* cos_t,
                     const float* sin_t, int pos0, float off, int interleaved, int accumulate, hipStream_t stream);

// ---------------------------------------------------------------- misc (misc.hip)
void cast_f32_bf16(const float* x, bf16_t* y, long n, hipStream_t st);
void cast_bf16_f32(const bf16_t* x, float* y, long n, hipStream_t st);
void scale_bf16(const bf16_t* x, bf16_t* y, long n, const float* scale_dev, float scale, hipStream_t st);
void add_bf16(const bf16_t* a, const bf16_t* b, bf16_t* y, long n, hipStream_t st);
// bias gradients: part[b][n] = column sums of row block b (then reduce_rows into the fp32 grad)
int colsum_partial_blocks(long M);
void colsum_partial(const bf16_t* x, long ld, long M, int N, float* part, hipStream_t st);
// p[row, c0 : c0 + ncols] = 0 for every row (c0, ncols, ld multiples of 8)
void zero_cols(bf16_t* p, long ld, long M, int c0, int ncols, hipStream_t st);
}  // namespace mft
