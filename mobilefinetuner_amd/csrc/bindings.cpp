// Torch bindings of the gfx950 kernels (module mobilefinetuner_amd._C).
// Every op validates dtype/device/layout, allocates outputs/workspaces through PyTorch's
// stream-ordered caching allocator (so the ops are hipGraph-capturable) and launches on the
// current HIP stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "kernels.h"

namespace py = pybind11;
using torch::Tensor;
using mft::bf16_t;

namespace {

inline hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

// deterministic-reduction mode: the LoRA weight-gradient and embedding-gradient
// kernels sum per-block partials in a fixed order instead of fp32 atomics (workspaces from torch's
// caching allocator, so the mode is hipGraph-capturable).  MFT_DETERMINISTIC=1 or set_deterministic().
bool g_det = [] {
  const char* e = getenv("MFT_DETERMINISTIC");
  return e && e[0] == '1';
}();
void set_deterministic(bool on) { g_det = on; }
bool get_deterministic() { return g_det; }
Tensor det_ws(const Tensor& like, long n) { return torch::empty({n}, like.options().dtype(torch::kFloat32)); }

#define CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == torch::kBFloat16, #t " must be bf16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == torch::kFloat32, #t " must be fp32")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")

inline bf16_t* bp(const Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
inline float* fp(const Tensor& t) { return t.data_ptr<float>(); }
template <typename T>
inline T* optp(const c10::optional<Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// ------------------------------------------------------------------ norms
// out_cols > N: y is allocated [M, out_cols] and only its first N columns are written (room for
// appended LoRA columns); the caller owns the rest.
Tensor alloc_wide(const Tensor& x, int M, int N, int64_t out_cols) {
  if (out_cols <= N) return torch::empty_like(x);
  TORCH_CHECK(out_cols % 8 == 0, "out_cols must be a multiple of 8");
  return torch::empty({M, out_cols}, x.options());
}

std::vector<Tensor> layernorm_fwd(Tensor x, c10::optional<Tensor> delta, Tensor w, Tensor b, double eps,
                                  int64_t out_cols) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(w); CHECK_F32(b);
  const int N = x.size(-1);
  TORCH_CHECK(N % 8 == 0 && N <= 4096, "layernorm: width must be a multiple of 8 and <= 4096");
  const int M = x.numel() / N;
  c10::DeviceGuard g(x.device());
  auto y = alloc_wide(x, M, N, out_cols);
  auto mean = torch::empty({M}, x.options().dtype(torch::kFloat32));
  auto rstd = torch::empty({M}, x.options().dtype(torch::kFloat32));
  Tensor s;
  if (delta.has_value()) {
    CHECK_CONTIG((*delta));
    s = torch::empty_like(x);
  }
  mft::layernorm_fwd(bp(x), delta ? bp(*delta) : nullptr, s.defined() ? bp(s) : nullptr, fp(w), fp(b), bp(y), fp(mean),
                     fp(rstd), M, N, (float)eps, y.size(-1), stream());
  return {y, s.defined() ? s : Tensor(), mean, rstd};
}

// dy may be a wide [M, >= N] row-strided gradient (see out_cols); only its first N columns are read
Tensor layernorm_bwd(Tensor x, Tensor dy, Tensor w, Tensor mean, Tensor rstd, c10::optional<Tensor> dresid,
                     c10::optional<Tensor> dw, c10::optional<Tensor> db) {
  CHECK_CONTIG(x);
  const int N = x.size(-1), M = x.numel() / N;
  TORCH_CHECK(dy.stride(-1) == 1 && dy.size(-1) >= N && dy.numel() / dy.size(-1) == M && dy.stride(0) % 8 == 0,
              "layernorm_bwd: dy must be [M, >= N] with unit column stride");
  c10::DeviceGuard g(x.device());
  auto dx = torch::empty_like(x);
  Tensor work;
  float* dwp = optp<float>(dw);
  if (dwp) work = torch::empty({2L * mft::norm_bwd_partial_blocks(M) * N}, x.options().dtype(torch::kFloat32));
  mft::layernorm_bwd(bp(x), bp(dy), fp(w), fp(mean), fp(rstd), dresid ? bp(*dresid) : nullptr, bp(dx), dwp,
                     optp<float>(db), dwp ? fp(work) : nullptr, M, N, 1, dy.dim() == 2 ? dy.stride(0) : N, stream());
  return dx;
}

std::vector<Tensor> rmsnorm_fwd(Tensor x, c10::optional<Tensor> delta, Tensor w, double eps, double offset,
                                int64_t out_cols) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(w);
  const int N = x.size(-1);
  TORCH_CHECK(N % 8 == 0 && N <= 4096, "rmsnorm: width must be a multiple of 8 and <= 4096");
  const int M = x.numel() / N;
  c10::DeviceGuard g(x.device());
  auto y = alloc_wide(x, M, N, out_cols);
  auto rstd = torch::empty({M}, x.options().dtype(torch::kFloat32));
  Tensor s;
  if (delta.has_value()) s = torch::empty_like(x);
  mft::rmsnorm_fwd(bp(x), delta ? bp(*delta) : nullptr, s.defined() ? bp(s) : nullptr, fp(w), bp(y), fp(rstd), M, N,
                   (float)eps, (float)offset, y.size(-1), stream());
  return {y, s.defined() ? s : Tensor(), rstd};
}

Tensor rmsnorm_bwd(Tensor x, Tensor dy, Tensor w, Tensor rstd, c10::optional<Tensor> dresid, double offset,
                   c10::optional<Tensor> dw) {
  CHECK_CONTIG(x);
  const int N = x.size(-1), M = x.numel() / N;
  TORCH_CHECK(dy.stride(-1) == 1 && dy.size(-1) >= N && dy.numel() / dy.size(-1) == M && dy.stride(0) % 8 == 0,
              "rmsnorm_bwd: dy must be [M, >= N] with unit column stride");
  c10::DeviceGuard g(x.device());
  auto dx = torch::empty_like(x);
  Tensor work;
  float* dwp = optp<float>(dw);
  if (dwp) work = torch::empty({2L * mft::norm_bwd_partial_blocks(M) * N}, x.options().dtype(torch::kFloat32));
  mft::rmsnorm_bwd(bp(x), bp(dy), fp(w), fp(rstd), dresid ? bp(*dresid) : nullptr, bp(dx), dwp,
                   dwp ? fp(work) : nullptr, M, N, (float)offset, 1, dy.dim() == 2 ? dy.stride(0) : N, stream());
  return dx;
}

// ------------------------------------------------------------------ attention
void fill_st(long* st, const Tensor& t) {  // [B, S, H, D] strides
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, "attention tensors must be [B,S,H,D] with contiguous D");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0,
              "attention strides must be multiples of 8 elements (16-B vector access)");
  st[0] = t.stride(0); st[1] = t.stride(1); st[2] = t.stride(2);
}

// out_cols > H*D: the output is allocated [B, Sq, out_cols] with O in the first H*D columns (room
// for the appended LoRA columns of the consumer); the kernel writes it through its row strides.
std::vector<Tensor> attn_fwd(Tensor q, Tensor k, Tensor v, double scale, bool causal, int64_t window,
                             c10::optional<Tensor> kv_lens, int64_t out_cols) {
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v);
  const int B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3);
  const int Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(H % Hkv == 0, "H must be a multiple of Hkv");
  TORCH_CHECK(D == 64 || D == 128 || D == 256, "head dim must be 64, 128 or 256");
  c10::DeviceGuard g(q.device());
  Tensor o_full, o;
  if (out_cols > (int64_t)H * D) {
    TORCH_CHECK(out_cols % 8 == 0, "attn_fwd: out_cols must be a multiple of 8");
    o_full = torch::empty({B, Sq, out_cols}, q.options());
    o = o_full.narrow(2, 0, (int64_t)H * D).view({B, Sq, H, D});
  } else {
    o = torch::empty({B, Sq, H, D}, q.options());
    o_full = o;
  }
  auto lse = torch::empty({B, H, Sq}, q.options().dtype(torch::kFloat32));
  mft::AttnArgs a{};
  a.q = bp(q); a.k = bp(k); a.v = bp(v); a.o = bp(o); a.lse = fp(lse);
  fill_st(a.q_st, q); fill_st(a.k_st, k); fill_st(a.v_st, v); fill_st(a.o_st, o);
  a.B = B; a.H = H; a.Hkv = Hkv; a.Sq = Sq; a.Sk = Sk; a.D = D;
  a.scale = (float)scale; a.causal = causal; a.window = (int)window;
  a.kv_lens = kv_lens ? kv_lens->data_ptr<int>() : nullptr;
  mft::attn_fwd(a, stream());
  if (o_full.dim() == 3)  // widened output: the appended columns start out zero (consumer contract)
    mft::zero_cols(bp(o_full), out_cols, (long)B * Sq, H * D, (int)(out_cols - (int64_t)H * D), stream());
  return {o_full, lse, o};
}

void attn_bwd(Tensor q, Tensor k, Tensor v, Tensor o, Tensor dout, Tensor lse, Tensor dq, Tensor dk, Tensor dv,
              double scale, bool causal, int64_t window, c10::optional<Tensor> kv_lens) {
  const int B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3);
  const int Sk = k.size(1), Hkv = k.size(2);
  c10::DeviceGuard g(q.device());
  const int path = mft::attn_bwd_path(D, Sq, Sk, (int)window);
  const bool short_path = path == 0;
  Tensor delta, dq_acc;
  if (!short_path) delta = torch::empty({B, H, Sq}, q.options().dtype(torch::kFloat32));
  if (path == 1) dq_acc = torch::empty({B, Sq, H, D}, q.options().dtype(torch::kFloat32));
  Tensor dk_tmp, dv_tmp;
  mft::AttnBwdArgs a{};
  if (H != Hkv && path != 2) {
    dk_tmp = torch::empty({B, Sk, H, D}, q.options());
    dv_tmp = torch::empty({B, Sk, H, D}, q.options());
    a.dk_tmp = bp(dk_tmp); a.dv_tmp = bp(dv_tmp);
    fill_st(a.tmp_st, dk_tmp);
  }
  a.q = bp(q); a.k = bp(k); a.v = bp(v); a.o = bp(o); a.dout = bp(dout); a.lse = fp(lse);
  a.delta = short_path ? nullptr : fp(delta);
  a.dq_acc = path == 1 ? fp(dq_acc) : nullptr;
  a.dq = bp(dq); a.dk = bp(dk); a.dv = bp(dv);
  fill_st(a.q_st, q); fill_st(a.k_st, k); fill_st(a.v_st, v); fill_st(a.o_st, o); fill_st(a.do_st, dout);
  fill_st(a.dq_st, dq); fill_st(a.dk_st, dk); fill_st(a.dv_st, dv);
  a.B = B; a.H = H; a.Hkv = Hkv; a.Sq = Sq; a.Sk = Sk; a.D = D;
  a.scale = (float)scale; a.causal = causal; a.window = (int)window;
  a.kv_lens = kv_lens ? kv_lens->data_ptr<int>() : nullptr;
  mft::attn_bwd(a, stream());
}

// ------------------------------------------------------------------ activations
Tensor gelu_fwd(Tensor x) {
  CHECK_BF16(x); CHECK_CONTIG(x);
  auto y = torch::empty_like(x);
  mft::gelu_fwd(bp(x), bp(y), x.numel(), stream());
  return y;
}
Tensor gelu_bwd(Tensor x, Tensor dy) {
  CHECK_CONTIG(x); CHECK_CONTIG(dy);
  auto dx = torch::empty_like(x);
  mft::gelu_bwd(bp(x), bp(dy), bp(dx), x.numel(), stream());
  return dx;
}
// out_cols > I: y is [M, out_cols] with the activation in the first I columns and the rest zeroed
// (augmented-K input of the LoRA down projection); gated_bwd then reads that wide dy row-strided.
Tensor gated_fwd(Tensor gu, int64_t act, int64_t out_cols) {
  CHECK_CUDA(gu); CHECK_BF16(gu); CHECK_CONTIG(gu);
  const int I = gu.size(-1) / 2;
  TORCH_CHECK(I % 8 == 0, "gated: intermediate size must be a multiple of 8");
  const long M = gu.numel() / (2 * I);
  if (out_cols > I) {
    TORCH_CHECK(out_cols % 8 == 0, "gated: out_cols must be a multiple of 8");
    auto y = torch::empty({M, out_cols}, gu.options());
    mft::gated_fwd(bp(gu), bp(y), M, I, out_cols, (int)act, stream());
    mft::zero_cols(bp(y), out_cols, M, I, (int)(out_cols - I), stream());
    return y;
  }
  auto sizes = gu.sizes().vec();
  sizes.back() = I;
  auto y = torch::empty(sizes, gu.options());
  mft::gated_fwd(bp(gu), bp(y), M, I, I, (int)act, stream());
  return y;
}
Tensor gated_bwd(Tensor gu, Tensor dy, int64_t act) {
  CHECK_CONTIG(gu); CHECK_BF16(gu); CHECK_BF16(dy);
  const int I = gu.size(-1) / 2;
  const long M = gu.numel() / (2 * I);
  TORCH_CHECK(dy.stride(-1) == 1 && dy.size(-1) >= I && dy.numel() / dy.size(-1) == M, "gated_bwd: dy shape");
  const long ldd = dy.dim() >= 2 ? dy.stride(-2) : I;
  TORCH_CHECK(dy.dim() <= 2 || dy.is_contiguous(), "gated_bwd: dy must be 2-D row-strided or contiguous");
  TORCH_CHECK(ldd % 8 == 0 && ldd >= I, "gated_bwd: dy row stride");
  auto dgu = torch::empty_like(gu);
  mft::gated_bwd(bp(gu), bp(dy), ldd, bp(dgu), M, I, (int)act, stream());
  return dgu;
}

// ------------------------------------------------------------------ embedding
Tensor embed_fwd(Tensor ids, Tensor wte, c10::optional<Tensor> wpe, int64_t S, int64_t pos0, double scale) {
  CHECK_CUDA(ids); TORCH_CHECK(ids.scalar_type() == torch::kInt64, "ids must be int64"); CHECK_CONTIG(ids);
  CHECK_BF16(wte); CHECK_CONTIG(wte);
  const long M = ids.numel();
  const int C = wte.size(1);
  TORCH_CHECK(C % 8 == 0, "embedding width must be a multiple of 8");
  auto out = torch::empty({M, C}, wte.options());
  mft::embed_fwd(ids.data_ptr<int64_t>(), bp(wte), wpe ? bp(*wpe) : nullptr, bp(out), M, C, (int)S, (int)pos0,
                 (float)scale, stream());
  return out;
}
void embed_bwd(Tensor ids, Tensor dout, c10::optional<Tensor> dwte, c10::optional<Tensor> dwpe, int64_t S, int64_t pos0,
               double scale) {
  CHECK_CONTIG(dout);
  const long M = ids.numel();
  const int C = dout.size(-1);
  const long det_vocab = (g_det && dwte.has_value() && dwte->defined()) ? dwte->numel() / C : 0;
  mft::embed_bwd(ids.data_ptr<int64_t>(), bp(dout), optp<float>(dwte), optp<float>(dwpe), M, C, (int)S, (int)pos0,
                 (float)scale, stream(), det_vocab);
}

// ------------------------------------------------------------------ cross entropy
void xent_fwd_bwd(Tensor logits, Tensor labels, Tensor loss, int64_t V, c10::optional<Tensor> scale, double extra,
                  bool write_grad) {
  CHECK_BF16(logits); TORCH_CHECK(logits.stride(1) == 1, "logits rows must be contiguous");
  TORCH_CHECK(logits.stride(0) % 8 == 0, "logits row stride must be a multiple of 8");
  TORCH_CHECK(labels.scalar_type() == torch::kInt64 && labels.is_contiguous(), "labels must be contiguous int64");
  CHECK_F32(loss);
  mft::xent_fwd_bwd(bp(logits), labels.data_ptr<int64_t>(), fp(loss), logits.size(0), (int)V, logits.stride(0),
                    optp<float>(scale), (float)extra, write_grad, stream());
}
// Fused LM head + cross entropy over one chunk of rows (xent.hip lm_head_ce): logits = h W^T never
// reach HBM.  E ([M, Vpad] bf16 workspace) receives exp(logit - tile max), or dlogits when
// materialize (the caller then forms dW = E^T h); loss [M] fp32 per-row NLL; dh [M, K] bf16.
void lm_head_ce(Tensor h, Tensor W, Tensor labels, int64_t V, c10::optional<Tensor> E, Tensor loss,
                c10::optional<Tensor> scale, double extra, c10::optional<Tensor> dh, bool materialize) {
  CHECK_CUDA(h); CHECK_BF16(h); CHECK_BF16(W); CHECK_F32(loss);
  TORCH_CHECK(h.dim() == 2 && W.dim() == 2 && h.stride(1) == 1 && W.stride(1) == 1 && h.size(1) == W.size(1),
              "lm_head_ce: h [M, K], W [Vpad, K] row-contiguous");
  TORCH_CHECK(labels.scalar_type() == torch::kInt64 && labels.is_contiguous() && labels.numel() == h.size(0),
              "lm_head_ce: labels [M] contiguous int64");
  const int M = h.size(0), K = h.size(1), Vpad = W.size(0);
  TORCH_CHECK(K % 64 == 0 && Vpad % 64 == 0 && V > 0 && V <= Vpad, "lm_head_ce: K, Vpad multiples of 64, V <= Vpad");
  TORCH_CHECK(h.stride(0) % 8 == 0 && W.stride(0) % 8 == 0, "lm_head_ce: leading dimensions must be multiples of 8");
  TORCH_CHECK(loss.numel() == M && loss.is_contiguous(), "lm_head_ce: loss [M]");
  if (E.has_value()) {
    CHECK_BF16((*E));
    TORCH_CHECK(E->size(0) == M && E->size(1) == Vpad && E->stride(1) == 1 && E->stride(0) % 8 == 0, "lm_head_ce: E [M, Vpad]");
  }
  if (dh.has_value()) {
    CHECK_BF16((*dh));
    TORCH_CHECK(E.has_value(), "lm_head_ce: the gradient needs E");
    TORCH_CHECK(dh->size(0) == M && dh->size(1) == K && dh->stride(1) == 1 && dh->stride(0) % 8 == 0, "lm_head_ce: dh [M, K]");
  }
  c10::DeviceGuard g(h.device());
  auto ws = torch::empty({mft::lm_head_ce_ws_floats(M, Vpad, dh.has_value() ? K : 0)}, h.options().dtype(torch::kFloat32));
  mft::CeArgs a{};
  a.h = bp(h); a.ldh = h.stride(0);
  a.W = bp(W); a.ldw = W.stride(0);
  a.labels = labels.data_ptr<int64_t>();
  a.M = M; a.K = K; a.Vpad = Vpad; a.V = (int)V;
  a.E = E.has_value() ? bp(*E) : nullptr; a.lde = E.has_value() ? E->stride(0) : 0;
  a.loss = fp(loss);
  a.scale = optp<float>(scale); a.extra = (float)extra;
  a.dh = dh.has_value() ? bp(*dh) : nullptr; a.lddh = dh.has_value() ? dh->stride(0) : 0;
  a.materialize = materialize;
  a.ws = fp(ws);
  Tensor wt;  // the engine's form: with E := dlogits, dh = dlogits W on gemm4 through W^T
  if (materialize && dh.has_value()) {
    wt = W.t().contiguous();
    a.Wt = bp(wt); a.ldwt = wt.stride(0);
  }
  mft::lm_head_ce(a, stream());
}
Tensor logsoftmax_gather(Tensor logits, Tensor idx, int64_t V) {
  CHECK_BF16(logits); TORCH_CHECK(logits.stride(1) == 1, "logits rows must be contiguous");
  auto out = torch::empty({logits.size(0), idx.numel()}, logits.options().dtype(torch::kFloat32));
  mft::logsoftmax_gather(bp(logits), idx.data_ptr<int64_t>(), fp(out), logits.size(0), (int)V, logits.stride(0),
                         idx.numel(), stream());
  return out;
}

// ------------------------------------------------------------------ optimizer
void sumsq(Tensor x, Tensor out, bool accumulate) {
  CHECK_F32(x); CHECK_CONTIG(x);
  auto part = torch::empty({mft::sumsq_blocks(x.numel())}, x.options());
  mft::sumsq(fp(x), x.numel(), fp(part), fp(out), accumulate, stream());
}
void nonfinite_check(Tensor x, Tensor flag) {
  CHECK_F32(x); CHECK_CONTIG(x);
  mft::nonfinite_check(fp(x), x.numel(), flag.data_ptr<int>(), stream());
}
void adamw_step(Tensor p, Tensor g, Tensor m, Tensor v, Tensor lr, Tensor step, c10::optional<Tensor> sumsq_t,
                double beta1, double beta2, double eps, double wd, double max_norm, bool l2_coupled,
                c10::optional<Tensor> shadow, c10::optional<Tensor> nonfinite, int64_t sr_offset,
                c10::optional<Tensor> vmax) {
  CHECK_F32(p); CHECK_F32(g);
  CHECK_CONTIG(p); CHECK_CONTIG(g); CHECK_CONTIG(m); CHECK_CONTIG(v);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adamw: size mismatch");
  const bool mb = m.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(m.scalar_type() == v.scalar_type() && (mb || m.scalar_type() == torch::kFloat32),
              "adamw: moments must both be fp32 or both bf16");
  mft::AdamWArgs a{};
  a.p = fp(p); a.g = fp(g); a.n = p.numel();
  a.m = reinterpret_cast<float*>(m.data_ptr()); a.v = reinterpret_cast<float*>(v.data_ptr());
  a.moments_bf16 = mb;
  a.lr_ptr = fp(lr); a.step_ptr = fp(step); a.sumsq = optp<float>(sumsq_t);
  a.beta1 = beta1; a.beta2 = beta2; a.eps = eps; a.weight_decay = wd; a.max_norm = max_norm; a.l2_coupled = l2_coupled;
  a.shadow = optp<bf16_t>(shadow);
  if (a.shadow) TORCH_CHECK(shadow->numel() == p.numel() && shadow->is_contiguous(), "shadow must match params");
  a.nonfinite = optp<int>(nonfinite);
  a.sr_offset = sr_offset;
  a.vmax = optp<float>(vmax);
  if (a.vmax) TORCH_CHECK(vmax->numel() == p.numel() && vmax->is_contiguous() && !mb, "vmax: fp32 [n], fp32 moments");
  mft::adamw_step(a, stream());
}
void adamw_commit(Tensor step, c10::optional<Tensor> nonfinite, c10::optional<Tensor> sumsq_t) {
  CHECK_F32(step);
  mft::adamw_commit(fp(step), optp<int>(nonfinite), optp<float>(sumsq_t), stream());
}

// ------------------------------------------------------------------ LoRA
// U = s * X Wt^T   (X [.., K] rows contiguous, Wt [R, K] contiguous rows)
mft::LoraDrop mkdrop(double p, int64_t salt, c10::optional<Tensor> ctr) {
  mft::LoraDrop d{};
  d.p = (float)p;
  d.salt = (uint32_t)salt;
  d.ctr = (ctr.has_value() && ctr->defined()) ? ctr->data_ptr<int64_t>() : nullptr;
  return d;
}
void lora_rowdot(Tensor X, Tensor Wt, Tensor U, double s, double drop_p, int64_t salt, c10::optional<Tensor> ctr) {
  CHECK_BF16(X); CHECK_BF16(Wt); CHECK_BF16(U);
  TORCH_CHECK(X.stride(-1) == 1 && U.stride(-1) == 1 && Wt.stride(-1) == 1, "rows must be contiguous");
  const int K = X.size(-1), R = Wt.size(0);
  TORCH_CHECK(Wt.size(1) == K && U.size(-1) == R, "lora_rowdot: shape mismatch");
  TORCH_CHECK(K % 8 == 0, "lora_rowdot: in-features must be a multiple of 8");
  TORCH_CHECK(X.stride(-2) % 8 == 0 && Wt.stride(0) % 8 == 0, "lora_rowdot: row strides must be multiples of 8");
  const long M = X.numel() / K;
  mft::lora_rowdot(bp(X), X.stride(-2), bp(Wt), Wt.stride(0), bp(U), U.stride(-2), M, K, R, (float)s,
                   mkdrop(drop_p, salt, ctr), stream());
}
// Y = base + s * U W   (W [R, N]); Y may alias base
void lora_update(Tensor base, Tensor U, Tensor W, Tensor Y, double s, double drop_p, int64_t salt,
                 c10::optional<Tensor> ctr) {
  CHECK_BF16(base); CHECK_BF16(Y); CHECK_BF16(U); CHECK_BF16(W);
  const int N = Y.size(-1), R = U.size(-1);
  TORCH_CHECK(W.size(0) == R && W.size(1) == N && W.stride(1) == 1, "lora_update: W must be [R, N]");
  TORCH_CHECK(N % 8 == 0 && W.stride(0) % 8 == 0 && base.stride(-2) % 8 == 0 && Y.stride(-2) % 8 == 0,
              "lora_update: widths/strides must be multiples of 8");
  const long M = Y.numel() / N;
  mft::lora_update(bp(base), base.stride(-2), bp(U), U.stride(-2), bp(W), W.stride(0), bp(Y), Y.stride(-2), M, N, R,
                   (float)s, mkdrop(drop_p, salt, ctr), stream());
}
void lora_wgrad(Tensor X, Tensor Y, Tensor out, int64_t osk, int64_t osr, double scale, double drop_p, int64_t salt,
                c10::optional<Tensor> ctr) {
  CHECK_BF16(X); CHECK_BF16(Y); CHECK_F32(out);
  TORCH_CHECK(X.stride(-1) == 1 && X.stride(-2) % 8 == 0, "lora_wgrad: X rows must be contiguous, stride % 8 == 0");
  const int K = X.size(-1), R = Y.size(-1);
  TORCH_CHECK(K % 8 == 0, "lora_wgrad: K must be a multiple of 8");
  const long M = X.numel() / K;
  mft::lora_wgrad(bp(X), X.stride(-2), bp(Y), Y.stride(-2), fp(out), osk, osr, M, K, R, (float)scale,
                  mkdrop(drop_p, salt, ctr), stream(), nullptr, g_det ? det_ws(X, mft::lora_wgrad_ws_floats(M, K, R)).data_ptr<float>() : nullptr);
}
// dA_z += scale * X^T Y[:, 8z:8z+8] for every rank-8 adapter z sharing the input X (one pass over X);
// outs[z] are contiguous fp32 [8, K] grad buffers
void lora_wgrad_multi(Tensor X, Tensor Y, std::vector<Tensor> outs, double scale) {
  CHECK_BF16(X); CHECK_BF16(Y);
  TORCH_CHECK(X.stride(-1) == 1 && X.stride(-2) % 8 == 0, "lora_wgrad_multi: X rows must be contiguous, stride % 8 == 0");
  const int K = X.size(-1), R = Y.size(-1);
  TORCH_CHECK(K % 8 == 0 && Y.stride(-1) == 1, "lora_wgrad_multi: K % 8, Y rows contiguous");
  TORCH_CHECK(!outs.empty() && outs.size() <= 8 && R == 8 * (int)outs.size(), "lora_wgrad_multi: R must be 8 per output");
  mft::WgradOuts o{};
  o.n = (int)outs.size();
  for (size_t i = 0; i < outs.size(); ++i) {
    CHECK_F32(outs[i]);
    TORCH_CHECK(outs[i].is_contiguous() && outs[i].numel() == 8L * K, "lora_wgrad_multi: outputs must be contiguous [8, K]");
    o.p[i] = fp(outs[i]);
  }
  const long M = X.numel() / K;
  mft::lora_wgrad(bp(X), X.stride(-2), bp(Y), Y.stride(-2), nullptr, 1, K, M, K, R, (float)scale, mft::LoraDrop{nullptr, 0, 0.f},
                  stream(), &o, g_det ? det_ws(X, mft::lora_wgrad_ws_floats(M, K, R)).data_ptr<float>() : nullptr);
}
// rank 8: v = s dy B^T (bf16 [M, 8]) and dB += s u^T dy (fp32 [8, N] grad buffer) in one pass over dy
void lora_dy(Tensor dy, Tensor B, Tensor u, Tensor dB, Tensor vpart, Tensor v, double s) {
  CHECK_BF16(dy); CHECK_BF16(B); CHECK_BF16(u); CHECK_BF16(v); CHECK_F32(dB); CHECK_F32(vpart);
  TORCH_CHECK(dy.dim() == 2 && dy.stride(1) == 1, "lora_dy: dy must be a row-contiguous 2-D view");
  const long M = dy.size(0);
  const int N = dy.size(1);
  TORCH_CHECK(B.dim() == 2 && B.size(0) == 8 && B.size(1) == N && B.stride(1) == 1, "lora_dy: B must be [8, N]");
  TORCH_CHECK(u.dim() == 2 && u.size(0) == M && u.size(1) == 8 && u.stride(1) == 1, "lora_dy: u must be [M, 8]");
  TORCH_CHECK(v.dim() == 2 && v.size(0) == M && v.size(1) == 8 && v.stride(1) == 1, "lora_dy: v must be [M, 8]");
  TORCH_CHECK(dB.is_contiguous() && dB.numel() == 8L * N, "lora_dy: dB must be a contiguous [8, N] buffer");
  TORCH_CHECK(vpart.is_contiguous() && vpart.numel() >= (long)((N + 255) / 256) * M * 8, "lora_dy: vpart too small");
  TORCH_CHECK(N % 8 == 0 && dy.stride(0) % 8 == 0 && B.stride(0) % 8 == 0 && u.stride(0) % 8 == 0 &&
              reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(B.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(u.data_ptr()) % 16 == 0,
              "lora_dy: alignment (N and row strides % 8, 16-B aligned rows)");
  mft::lora_dy(bp(dy), dy.stride(0), bp(B), B.stride(0), bp(u), u.stride(0), fp(dB), N, fp(vpart), bp(v), v.stride(0),
               M, N, (float)s, stream(), g_det ? det_ws(dy, mft::lora_dy_ws_floats(M, N)).data_ptr<float>() : nullptr);
}
void lora_merge(Tensor W, int64_t wsk, int64_t wsn, Tensor A, Tensor B, double s) {
  CHECK_F32(A); CHECK_F32(B); CHECK_CONTIG(A); CHECK_CONTIG(B);
  const int R = A.size(0), K = A.size(1), N = B.size(1);
  const bool isbf = W.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(isbf || W.scalar_type() == torch::kFloat32, "merge target must be bf16 or fp32");
  mft::lora_merge(W.data_ptr(), isbf, wsk, wsn, fp(A), fp(B), K, N, R, (float)s, stream());
}

// ------------------------------------------------------------------ RoPE
void rope_apply(Tensor x, Tensor cos_t, Tensor sin_t, int64_t pos0, bool interleaved, bool inverse) {
  long st[3];
  fill_st(st, x);
  mft::rope_apply(bp(x), st, x.size(0), x.size(1), x.size(2), x.size(3), fp(cos_t), fp(sin_t), (int)pos0, interleaved,
                  inverse, stream());
}
std::vector<Tensor> qknorm_rope_fwd(Tensor x, Tensor w, Tensor cos_t, Tensor sin_t, int64_t pos0, double eps,
                                    double offset, bool interleaved) {
  long st[3];
  fill_st(st, x);
  const int B = x.size(0), S = x.size(1), H = x.size(2), D = x.size(3);
  auto y = torch::empty({B, S, H, D}, x.options());
  auto rstd = torch::empty({(long)B * S * H}, x.options().dtype(torch::kFloat32));
  mft::qknorm_rope_fwd(bp(x), st, bp(y), fp(rstd), fp(w), B, S, H, D, fp(cos_t), fp(sin_t), (int)pos0, (float)eps,
                       (float)offset, interleaved, stream());
  return {y, rstd};
}
void qknorm_rope_bwd(Tensor x, Tensor dy, Tensor rstd, Tensor w, Tensor dx, c10::optional<Tensor> dw, Tensor cos_t,
                     Tensor sin_t, int64_t pos0, double offset, bool interleaved) {
  long st[3], dst[3];
  fill_st(st, x);
  fill_st(dst, dx);
  CHECK_CONTIG(dy);
  const int B = x.size(0), S = x.size(1), H = x.size(2), D = x.size(3);
  Tensor work;
  float* dwp = optp<float>(dw);
  if (dwp) work = torch::empty({(long)mft::qknorm_rope_bwd_blocks((long)B * S * H) * D}, x.options().dtype(torch::kFloat32));
  mft::qknorm_rope_bwd(bp(x), st, bp(dy), fp(rstd), fp(w), bp(dx), dst, dwp, dwp ? fp(work) : nullptr, B, S, H, D,
                       fp(cos_t), fp(sin_t), (int)pos0, (float)offset, interleaved, 1, stream());
}

// ------------------------------------------------------------------ misc
void cast_f32_bf16(Tensor x, Tensor y) {
  CHECK_F32(x); CHECK_BF16(y); CHECK_CONTIG(x); CHECK_CONTIG(y);
  TORCH_CHECK(x.numel() == y.numel(), "cast: size mismatch");
  mft::cast_f32_bf16(fp(x), bp(y), x.numel(), stream());
}
void cast_bf16_f32(Tensor x, Tensor y) {
  CHECK_BF16(x); CHECK_F32(y); CHECK_CONTIG(x); CHECK_CONTIG(y);
  TORCH_CHECK(x.numel() == y.numel(), "cast: size mismatch");
  mft::cast_bf16_f32(bp(x), fp(y), x.numel(), stream());
}
Tensor scale_bf16(Tensor x, c10::optional<Tensor> sdev, double s) {
  CHECK_BF16(x); CHECK_CONTIG(x);
  auto y = torch::empty_like(x);
  mft::scale_bf16(bp(x), bp(y), x.numel(), optp<float>(sdev), (float)s, stream());
  return y;
}
Tensor add_bf16(Tensor a, Tensor b) {
  CHECK_BF16(a); CHECK_CONTIG(a); CHECK_CONTIG(b);
  auto y = torch::empty_like(a);
  mft::add_bf16(bp(a), bp(b), bp(y), a.numel(), stream());
  return y;
}


// ------------------------------------------------------------------ GEMM (gemm8.hip)
// C = epi(alpha * A op(B)); A [M,K]; B [N,K] (b_nn = false) or [K,N] (b_nn = true).  `bm` is kept
// for the call signature (the round-1 tile configurations are gone): every call runs gemm8.
// Returns {C, aux}: aux is the pre-activation written by GEMM_EPI_BIAS_GELU.
std::vector<Tensor> gemm_op(Tensor A, Tensor B, bool b_nn, int64_t epi, c10::optional<Tensor> bias,
                            c10::optional<Tensor> aux, double alpha, int64_t bm, c10::optional<Tensor> out,
                            c10::optional<Tensor> lora_u, c10::optional<Tensor> lora_w) {
  CHECK_CUDA(A); CHECK_BF16(A); CHECK_BF16(B);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1, "gemm: row-contiguous 2-D operands");
  const int M = A.size(0), K = A.size(1);
  const int N = b_nn ? B.size(1) : B.size(0);
  TORCH_CHECK((b_nn ? B.size(0) : B.size(1)) == K, "gemm: inner dimensions differ");
  TORCH_CHECK(mft::gemm8_supported(M, N, K, false, b_nn), "gemm: needs K % 64 == 0 and N % 8 == 0");
  TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0, "gemm: leading dimensions must be multiples of 8");
  c10::DeviceGuard g(A.device());
  Tensor C;
  if (out.has_value()) {
    C = *out;
    TORCH_CHECK(C.size(0) == M && C.size(1) == N && C.stride(1) == 1, "gemm: out shape");
    TORCH_CHECK(C.scalar_type() == (epi == mft::GEMM_EPI_F32ACC ? torch::kFloat32 : torch::kBFloat16), "gemm: out dtype");
  } else {
    TORCH_CHECK(epi != mft::GEMM_EPI_F32ACC, "gemm: fp32 accumulate needs out=");
    C = torch::empty({M, N}, A.options());
  }
  Tensor X;
  if (epi == mft::GEMM_EPI_BIAS_GELU) {
    X = aux.has_value() ? *aux : torch::empty({M, N}, A.options());
  } else if (epi == mft::GEMM_EPI_DGELU) {
    TORCH_CHECK(aux.has_value(), "gemm: dGELU needs aux (pre-activation)");
    X = *aux;
  }
  if (X.defined()) TORCH_CHECK(X.size(0) == M && X.size(1) == N && X.stride(1) == 1 && X.stride(0) % 8 == 0, "gemm: aux shape");
  if (epi == mft::GEMM_EPI_BIAS || epi == mft::GEMM_EPI_BIAS_GELU) {
    TORCH_CHECK(bias.has_value() && bias->numel() == N && bias->scalar_type() == torch::kBFloat16, "gemm: bf16 bias [N]");
  }
  mft::GemmArgs a{};
  a.A = bp(A); a.lda = A.stride(0);
  a.B = bp(B); a.ldb = B.stride(0);
  a.C = C.data_ptr(); a.ldc = C.stride(0);
  a.bias = bias.has_value() ? bp(*bias) : nullptr;
  a.aux = X.defined() ? bp(X) : nullptr; a.ldaux = X.defined() ? X.stride(0) : 0;
  a.M = M; a.N = N; a.K = K; a.alpha = (float)alpha;
  if (epi == mft::GEMM_EPI_LORA) {
    TORCH_CHECK(lora_u.has_value() && lora_w.has_value(), "gemm: LoRA epilogue needs u and w");
    CHECK_BF16((*lora_u)); CHECK_BF16((*lora_w));
    TORCH_CHECK(lora_u->size(0) == M && lora_w->size(1) == N && lora_u->size(1) == lora_w->size(0) &&
                lora_u->stride(1) == 1 && lora_w->stride(1) == 1, "gemm: LoRA u [M, r], w [r, N]");
    a.lora_u = bp(*lora_u); a.ld_lu = lora_u->stride(0);
    a.lora_w = bp(*lora_w); a.ld_lw = lora_w->stride(0);
    a.lora_r = lora_u->size(1);
  }
  (void)bm;
  mft::gemm8x(a, (int)epi, false, b_nn, stream());
  return {C, X};
}

// General 8-phase GEMM, every operand layout (gemm8.hip):
//   A: a_t ? [K, M] : [M, K];  B: b_t ? [K, N] : [N, K];  C [M, N] (bf16, or fp32 += for F32ACC)
// F32ACC with a_t && b_t is the TN weight gradient: split over K into fp32 slabs + deterministic
// reduce when the output has few 256x256 tiles.
// out[M, N] = A[M, K] B[N, K]^T + A2[M, K2] B2[N, K2]^T on gemm4 (second K segment; the LoRA data-gradient
// form of engine/nn.cpp)
void gemm4_seg2(Tensor A, Tensor B, Tensor A2, Tensor B2, Tensor out, int64_t impl) {
  CHECK_CUDA(A); CHECK_BF16(A); CHECK_BF16(B); CHECK_BF16(A2); CHECK_BF16(B2); CHECK_BF16(out);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A2.dim() == 2 && B2.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1 &&
              A2.stride(1) == 1 && B2.stride(1) == 1 && out.stride(1) == 1, "gemm4_seg2: row-contiguous 2-D operands");
  const int M = A.size(0), K = A.size(1), N = B.size(0), K2 = A2.size(1);
  TORCH_CHECK(B.size(1) == K && A2.size(0) == M && B2.size(0) == N && B2.size(1) == K2 && out.size(0) == M &&
              out.size(1) == N, "gemm4_seg2: shapes");
  TORCH_CHECK((impl == 5 ? mft::gemm_s_supported(M, N, K, 0) : mft::gemm4_supported(M, N, K, false, false)) &&
              K2 % 64 == 0 && K2 > 0, "gemm4_seg2: K, K2 % 64, N % 8");
  c10::DeviceGuard g(A.device());
  mft::GemmArgs a{};
  a.A = bp(A); a.lda = A.stride(0);
  a.B = bp(B); a.ldb = B.stride(0);
  a.C = out.data_ptr(); a.ldc = out.stride(0);
  a.A2 = bp(A2); a.lda2 = A2.stride(0);
  a.B2 = bp(B2); a.ldb2 = B2.stride(0);
  a.M = M; a.N = N; a.K = K; a.K2 = K2; a.alpha = 1.f;
  if (impl == 5) mft::gemm_s(a, mft::GEMM_EPI_NONE, stream());
  else mft::gemm4x(a, mft::GEMM_EPI_NONE, false, false, stream());
}

// The Gemma-3 GeGLU epilogues of gemm4 (kernels.h GEMM_EPI_GEGLU_*).  fwd: out = gu = A B^T [M, 2I] (B = [Wg; Wu]),
// aux [M, >= I] <- h = gelu(g) u.  bwd: the accumulator dh = A B^T (+ A2 B2^T) [M, I] (B [I, K]) is never stored:
// out [M, 2I] <- d gu from dh and aux = gu [M, 2I].
void gemm4_geglu(Tensor A, Tensor B, Tensor aux, Tensor out, int64_t I, bool fwd, c10::optional<Tensor> A2,
                 c10::optional<Tensor> B2) {
  CHECK_CUDA(A); CHECK_BF16(A); CHECK_BF16(B); CHECK_BF16(aux); CHECK_BF16(out);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1 && aux.stride(1) == 1 && out.stride(1) == 1,
              "gemm4_geglu: row-contiguous 2-D operands");
  const int M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K && out.size(0) == M && out.size(1) == 2 * I && aux.size(0) == M &&
                  (fwd ? N == 2 * I && aux.size(1) >= I : N == I && aux.size(1) == 2 * I) &&
                  mft::gemm4_supported(M, N, K, false, false) && I % 128 == 0,
              "gemm4_geglu: shapes");
  c10::DeviceGuard g(A.device());
  mft::GemmArgs a{};
  a.A = bp(A); a.lda = A.stride(0);
  a.B = bp(B); a.ldb = B.stride(0);
  a.C = out.data_ptr(); a.ldc = out.stride(0);
  a.aux = bp(aux); a.ldaux = aux.stride(0);
  a.M = M; a.N = N; a.K = K; a.alpha = 1.f; a.geglu_I = (int)I;
  if (A2.has_value()) {
    TORCH_CHECK(!fwd && B2.has_value() && A2->size(0) == M && B2->size(0) == N && A2->size(1) == B2->size(1) &&
                    A2->size(1) % 64 == 0, "gemm4_geglu: second K segment");
    a.A2 = bp(*A2); a.lda2 = A2->stride(0);
    a.B2 = bp(*B2); a.ldb2 = B2->stride(0);
    a.K2 = A2->size(1);
  }
  mft::gemm4x(a, fwd ? mft::GEMM_EPI_GEGLU_FWD : mft::GEMM_EPI_GEGLU_BWD, false, false, stream());
}

std::vector<Tensor> gemm_t(Tensor A, Tensor B, bool a_t, bool b_t, int64_t epi, c10::optional<Tensor> bias,
                           c10::optional<Tensor> aux, double alpha, c10::optional<Tensor> out,
                           c10::optional<Tensor> lora_u, c10::optional<Tensor> lora_w, int64_t impl) {
  CHECK_CUDA(A); CHECK_BF16(A); CHECK_BF16(B);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1, "gemm_t: row-contiguous 2-D operands");
  const int M = a_t ? A.size(1) : A.size(0), K = a_t ? A.size(0) : A.size(1);
  const int N = b_t ? B.size(1) : B.size(0);
  TORCH_CHECK((b_t ? B.size(0) : B.size(1)) == K, "gemm_t: inner dimensions differ");
  TORCH_CHECK(mft::gemm8_supported(M, N, K, a_t, b_t), "gemm_t: needs K % 64 == 0, N % 8 == 0 (and M % 8 for a_t)");
  TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0, "gemm_t: leading dimensions must be multiples of 8");
  c10::DeviceGuard g(A.device());
  const bool f32 = epi == mft::GEMM_EPI_F32ACC;
  Tensor C;
  if (out.has_value()) {
    C = *out;
    TORCH_CHECK(C.size(0) == M && C.size(1) == N && C.stride(1) == 1 && C.stride(0) % 8 == 0, "gemm_t: out shape");
    TORCH_CHECK(C.scalar_type() == (f32 ? torch::kFloat32 : torch::kBFloat16), "gemm_t: out dtype");
  } else {
    TORCH_CHECK(!f32, "gemm_t: fp32 accumulate needs out=");
    C = torch::empty({M, N}, A.options());
  }
  Tensor X;
  if (epi == mft::GEMM_EPI_BIAS_GELU || epi == mft::GEMM_EPI_BIAS_GELU_D) {
    X = aux.has_value() ? *aux : torch::empty({M, N}, A.options());
  } else if (epi == mft::GEMM_EPI_DGELU || epi == mft::GEMM_EPI_MUL_AUX || epi == mft::GEMM_EPI_BIAS_ADD) {
    TORCH_CHECK(aux.has_value(), "gemm_t: dGELU / MUL_AUX / BIAS_ADD need aux");
    X = *aux;
  }
  if (X.defined()) TORCH_CHECK(X.size(0) == M && X.size(1) == N && X.stride(1) == 1 && X.stride(0) % 8 == 0, "gemm_t: aux shape");
  if (epi == mft::GEMM_EPI_BIAS || epi == mft::GEMM_EPI_BIAS_GELU || epi == mft::GEMM_EPI_BIAS_GELU_D ||
      epi == mft::GEMM_EPI_BIAS_ADD)
    TORCH_CHECK(bias.has_value() && bias->numel() == N && bias->scalar_type() == torch::kBFloat16, "gemm_t: bf16 bias [N]");
  mft::GemmArgs a{};
  a.A = bp(A); a.lda = A.stride(0);
  a.B = bp(B); a.ldb = B.stride(0);
  a.C = C.data_ptr(); a.ldc = C.stride(0);
  a.bias = bias.has_value() ? bp(*bias) : nullptr;
  a.aux = X.defined() ? bp(X) : nullptr; a.ldaux = X.defined() ? X.stride(0) : 0;
  a.M = M; a.N = N; a.K = K; a.alpha = (float)alpha;
  Tensor ws;
  const bool tn4 = impl == 4 && a_t && b_t;  // the 4-wave TN weight-gradient kernel (gemm4_tn)
  if (f32) {
    a.ksplit = tn4 ? mft::gemm4_tn_pick_ksplit(M, N, K) : mft::gemm8_pick_ksplit(M, N, K);
    if (a.ksplit > 1) {
      ws = torch::empty({(long)a.ksplit * M * N}, A.options().dtype(torch::kFloat32));
      a.ws = fp(ws);
    }
  }
  if (epi == mft::GEMM_EPI_LORA) {
    TORCH_CHECK(lora_u.has_value() && lora_w.has_value(), "gemm_t: LoRA epilogue needs u and w");
    CHECK_BF16((*lora_u)); CHECK_BF16((*lora_w));
    TORCH_CHECK(lora_u->size(0) == M && lora_w->size(1) == N && lora_u->size(1) == lora_w->size(0) &&
                lora_u->stride(1) == 1 && lora_w->stride(1) == 1, "gemm_t: LoRA u [M, r], w [r, N]");
    a.lora_u = bp(*lora_u); a.ld_lu = lora_u->stride(0);
    a.lora_w = bp(*lora_w); a.ld_lw = lora_w->stride(0);
    a.lora_r = lora_u->size(1);
  }
  TORCH_CHECK(impl == 0 || impl == 4 || impl == 5,
              "gemm_t: impl 0 (gemm8), 4 (gemm4, hand-scheduled 4-wave kernel) or 5 (gemm_s, short-token kernel)");
  if (impl == 5) {
    TORCH_CHECK(!a_t && !b_t && mft::gemm_s_supported(M, N, K, (int)epi), "gemm_t: shape / epilogue not supported by gemm_s");
    mft::gemm_s(a, (int)epi, stream());
  } else if (tn4) {
    TORCH_CHECK(f32 && mft::gemm4_tn_supported(M, N, K, a.lda, a.ldb), "gemm_t: gemm4 TN needs the F32ACC epilogue and a supported shape");
    mft::gemm4_tn(a, stream());
  } else if (impl == 4) {
    TORCH_CHECK(mft::gemm4_supported(M, N, K, a_t, b_t), "gemm_t: shape / layout not supported by gemm4");
    mft::gemm4x(a, (int)epi, a_t, b_t, stream());
  } else {
    mft::gemm8x(a, (int)epi, a_t, b_t, stream());
  }
  return {C, X};
}

// out[N] (fp32) (+)= column sums of x[M, N] (bf16, row stride ld): bias gradients accumulated
// straight into the flat fp32 grad buffer (deterministic two-stage reduction, no fp32 copy of x).
void colsum_acc(Tensor x, Tensor out, bool accumulate) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_F32(out);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && x.size(1) % 8 == 0 && out.numel() == x.size(1),
              "colsum_acc: x [M, N] row-contiguous (N, ld multiples of 8), out [N]");
  c10::DeviceGuard g(x.device());
  const long M = x.size(0);
  const int N = x.size(1);
  const int nb = mft::colsum_partial_blocks(M);
  auto part = torch::empty({(long)nb * N}, out.options());
  mft::colsum_partial(bp(x), x.stride(0), M, N, fp(part), stream());
  mft::reduce_rows(fp(part), fp(out), nb, N, accumulate ? 1 : 0, stream());
}

// Zero columns [c0, ncols) of a row-strided 2-D bf16 tensor (one small kernel, graph-capturable).
// Deliberately outside autograd: the padding columns of augmented LoRA inputs are read by no
// autograd-visible op (an in-place torch op there would trip the view/version checks).
void zero_cols(Tensor t, int64_t c0) {
  CHECK_CUDA(t); CHECK_BF16(t);
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.stride(0) % 8 == 0 && c0 % 8 == 0 && t.size(1) % 8 == 0,
              "zero_cols: 2-D row-contiguous bf16 tensor, 8-aligned columns");
  c10::DeviceGuard g(t.device());
  mft::zero_cols(bp(t), t.stride(0), t.size(0), (int)c0, (int)(t.size(1) - c0), stream());
}
}  // namespace

void register_runtime(py::module_& m);  // csrc/runtime_bindings.cpp

PYBIND11_MODULE(_C, m) {
  m.doc() = "mobilefinetuner_amd native kernels (gfx950 HIP) and C++ runtime";
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("gated_fwd", &gated_fwd);
  m.def("gated_bwd", &gated_bwd);
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd);
  m.def("xent_fwd_bwd", &xent_fwd_bwd);
  m.def("lm_head_ce", &lm_head_ce);
  m.def("ce_dgrad_splits", &mft::ce_dgrad_splits, "vocab splits of the LM-head CE dgrad for an M-row chunk");
  m.def("lora_dy_grid_blocks", &mft::lora_dy_grid_blocks, "workgroups of the lora_dy / lora_xty grids");
  m.def("logsoftmax_gather", &logsoftmax_gather);
  m.def("sumsq", &sumsq);
  m.def("nonfinite_check", &nonfinite_check);
  m.def("adamw_step", &adamw_step, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("lr"),
        py::arg("step"), py::arg("sumsq"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"), py::arg("wd"),
        py::arg("max_norm"), py::arg("l2_coupled"), py::arg("shadow"), py::arg("nonfinite"),
        py::arg("sr_offset") = 0, py::arg("vmax") = py::none());
  m.def("adamw_commit", &adamw_commit);
  m.def("lora_rowdot", &lora_rowdot);
  m.def("lora_update", &lora_update);
  m.def("lora_wgrad", &lora_wgrad);
  m.def("lora_wgrad_multi", &lora_wgrad_multi);
  m.def("lora_merge", &lora_merge);
  m.def("lora_dy", &lora_dy);
  m.def("gemm4_seg2", &gemm4_seg2, "out = A B^T + A2 B2^T on gemm4 (impl 4) or gemm_s (impl 5): second K segment",
        py::arg("A"), py::arg("B"), py::arg("A2"), py::arg("B2"), py::arg("out"), py::arg("impl") = 4);
  m.def("gemm4_geglu", &gemm4_geglu, "the GeGLU MLP epilogues of gemm4 (gate|up -> gu + h; down dgrad -> d gu)",
        py::arg("A"), py::arg("B"), py::arg("aux"), py::arg("out"), py::arg("I"), py::arg("fwd"),
        py::arg("A2") = py::none(), py::arg("B2") = py::none());
  m.def("gemm_t", &gemm_t, py::arg("A"), py::arg("B"), py::arg("a_t"), py::arg("b_t"), py::arg("epi"),
        py::arg("bias") = py::none(), py::arg("aux") = py::none(), py::arg("alpha") = 1.0, py::arg("out") = py::none(),
        py::arg("lora_u") = py::none(), py::arg("lora_w") = py::none(), py::arg("impl") = 0);
  m.def("gemm8_set_stream", [](int64_t on) { mft::gemm8_set_stream((int)on); });
  m.def("gemm8_set_stagger", [](int64_t c) { mft::gemm8_set_stagger((int)c); });
  m.def("gemm", &gemm_op, py::arg("A"), py::arg("B"), py::arg("b_nn"), py::arg("epi"), py::arg("bias"), py::arg("aux"),
        py::arg("alpha"), py::arg("cfg"), py::arg("out"), py::arg("lora_u") = py::none(), py::arg("lora_w") = py::none());
  m.def("zero_cols", &zero_cols);
  m.def("set_deterministic", &set_deterministic);
  m.def("get_deterministic", &get_deterministic);
  m.def("colsum_acc", &colsum_acc);
  m.def("rope_apply", &rope_apply);
  m.def("qknorm_rope_fwd", &qknorm_rope_fwd);
  m.def("qknorm_rope_bwd", &qknorm_rope_bwd);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("cast_bf16_f32", &cast_bf16_f32);
  m.def("scale_bf16", &scale_bf16);
  m.def("add_bf16", &add_bf16);
  register_runtime(m);
}
