// libmft engine: fused transformer ops (see nn.h).
#include "engine/nn.h"

#include <cstring>
#include <unordered_map>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "engine/autograd.h"
#include "engine/gemm.h"
#include "engine/lm.h"
#include "engine/ops.h"
#include "kernels.h"

namespace mft {
namespace eng {

namespace {
hipStream_t S() { return current_stream(); }
inline ::mft::bf16_t* bp(const Tensor& t) { return (::mft::bf16_t*)t.data_ptr(); }
inline float* fp(const Tensor& t) { return (float*)t.data_ptr(); }
inline float* fp_or_null(const Tensor& t) { return t.defined() ? (float*)t.data_ptr() : nullptr; }

Tensor f32_of(Param& p) {  // norm weights are fp32 compute
  return p.c.dtype() == DType::F32 ? p.c : p.c.to(DType::F32);
}
// fp32 grad buffer of a trainable param (allocated on first use), or undefined
// deterministic-mode workspace (fixed-order partial sums instead of fp32 atomics), else undefined
Tensor det_ws(long n) { return deterministic() ? empty({(int64_t)n}, DType::F32) : Tensor(); }
float* dptr(const Tensor& t) { return t.defined() ? (float*)t.data_ptr() : nullptr; }
Tensor gbuf(Param* p) {
  if (!p || !p->trainable()) return Tensor();
  return grad_buffer(p->leaf);
}
}  // namespace

const Tensor& Param::transposed() {
  MFT_CHECK(!streamed, "Param::transposed: a streamed weight has no resident transposed copy");
  if (!wt.defined()) {
    NoGradGuard ng;
    wt = c.t().contiguous();
  }
  return wt;
}

// ------------------------------------------------------------------ model helpers (lm.h)
int64_t default_ce_chunk(int vocab_padded) {
  if (const char* env = std::getenv("MFT_CE_CHUNK")) return std::atoll(env);
  // 4 GiB: with the vocab-split dgrad a short row chunk still fills the CUs, so bounding the E buffer
  // costs ~1.6 % on Gemma-3 at 256 x 256 (542 vs 551 K tok/s) for 81.5 instead of 139 GB peak HBM
  // (profiles/r4b_ce_budget_ab.txt; round 3 paid 17 % for the same bound)
  const char* gbs = std::getenv("MFT_CE_BUDGET_GB");
  const double gb = gbs ? std::atof(gbs) : 4.0;
  const int64_t rows = (int64_t)(gb * (1ull << 30) / (2.0 * vocab_padded));
  return std::max<int64_t>(64, std::min<int64_t>(65536, rows / 64 * 64));
}

uint32_t adapter_salt(const std::string& name) {
  uint32_t h = 2166136261u;
  for (char c : name) h = (h ^ (uint8_t)c) * 16777619u;
  return h;
}

LoraAdapter make_adapter(int col0, int n, int r, const Tensor& A_init, float dropout, const std::string& name) {
  LoraAdapter a;
  a.col0 = col0;
  a.ncols = n;
  a.rank = r;
  a.dropout = dropout;
  a.salt = adapter_salt(name);
  NoGradGuard ng;
  Tensor A = A_init.to(DType::F32).contiguous().clone();
  A.requires_grad_(true);
  Tensor B = zeros({r, n}, DType::F32);
  B.requires_grad_(true);
  a.A.leaf = A;
  a.B.leaf = B;
  // (--dtype fp32: the adapters compute on their fp32 masters; FlatParams keeps them that way)
  const bool f32 = compute_dtype() == DType::F32;
  a.A.c = f32 ? A : A.to(DType::BF16);
  a.B.c = f32 ? B : B.to(DType::BF16);
  return a;
}

// ------------------------------------------------------------------ reference-precision composite path
namespace {
DType g_compute_dtype = DType::BF16;
}
void set_compute_dtype(DType d) {
  MFT_CHECK(d == DType::BF16 || d == DType::F32, "compute dtype: bf16 or fp32");
  g_compute_dtype = d;
}
DType compute_dtype() { return g_compute_dtype; }

Tensor pad_cols(const Tensor& x, int64_t cols) {
  MFT_CHECK(x.dim() == 2, "pad_cols: 2-D input");
  if (cols <= x.size(1)) return x;
  Tensor z = zeros({x.size(0), cols - x.size(1)}, x.dtype(), x.device());
  return cat({x, z}, 1);
}

Tensor valid_count(const Tensor& labels) {
  NoGradGuard ng;
  Tensor c = zeros({1}, DType::F32, labels.device());
  Tensor lc = labels.contiguous();
  k::count_valid(lc.data<int64_t>(), (long)lc.numel(), -100, c.data<float>(), current_stream());
  return c;
}

Tensor attention_ref(const Tensor& q, const Tensor& k, const Tensor& v, float scale, bool causal, int window) {
  MFT_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4 && k.size(2) == v.size(2) && q.size(2) % k.size(2) == 0,
            "attention_ref: q [B, Sq, H, D], k / v [B, Sk, Hkv, D]");
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3), Sk = k.size(1), rep = H / k.size(2);
  Tensor kk = repeat_kv(k, (int)rep), vv = repeat_kv(v, (int)rep);
  Tensor sc = mul_scalar(matmul(q.transpose(1, 2), kk.transpose(1, 2).transpose(2, 3)), scale);  // [B, H, Sq, Sk]
  if (causal || window > 0) sc = apply_mask(sc, causal_mask(Sq, Sk, window).to(q.device()));
  Tensor o = matmul(softmax(sc), vv.transpose(1, 2));  // [B, H, Sq, D]
  return o.transpose(1, 2).reshape({B, Sq, H * D});
}

Tensor lora_linear_ref(const Tensor& x, Param& w, Param* b, std::vector<LoraAdapter>& ads, float s, bool training,
                       uint64_t drop_step) {
  MFT_CHECK(x.dim() == 2, "lora_linear_ref: 2-D input");
  Tensor y = linear(x, cw(w), b ? cw(*b) : Tensor());
  const int64_t M = x.size(0), N = y.size(1);
  for (auto& a : ads) {
    const uint64_t seed = (drop_step + 1) * 0x9E3779B97F4A7C15ull ^ ((uint64_t)a.salt << 17);
    Tensor xin = training && a.dropout > 0.f ? dropout(x, a.dropout, seed, true) : x;
    Tensor d = mul_scalar(matmul(matmul(xin, cw(a.A).t()), cw(a.B)), s);  // [M, ncols]
    if (a.col0 == 0 && a.ncols == N) {
      y = add(y, d);
    } else {
      std::vector<Tensor> parts;
      if (a.col0 > 0) parts.push_back(zeros({M, (int64_t)a.col0}, d.dtype(), d.device()));
      parts.push_back(d);
      if (a.col0 + a.ncols < N) parts.push_back(zeros({M, N - a.col0 - a.ncols}, d.dtype(), d.device()));
      y = add(y, cat(parts, 1));
    }
  }
  return y;
}

// ------------------------------------------------------------------ norms
namespace {
struct NormNode : Node {
  Tensor xs, w32, mean, rstd;
  Param* w = nullptr;
  Param* b = nullptr;
  bool rms = false, has_delta = false, has_sout = false;  // has_sout: s is an output (delta or resid_out)
  float offset = 0.f;
  int N = 0;
  std::vector<Tensor> apply(std::vector<Tensor>& g) override {
    // outputs: {s, y}; inputs: {x, delta, w.leaf, b.leaf}
    Tensor ds = has_sout ? g[0] : Tensor();
    Tensor dy = g[1];
    const long M = xs.numel() / N;
    if (!dy.defined()) dy = zeros({M, (int64_t)N}, DType::BF16, xs.device());
    Tensor dy2 = dy.reshape({M, dy.size(-1)});
    if (dy2.stride(1) != 1 || dy2.stride(0) % 8) dy2 = dy2.contiguous();
    Tensor ds2 = ds.defined() ? ds.reshape({M, (int64_t)N}).contiguous() : Tensor();
    Tensor dx = empty(xs.shape(), DType::BF16, xs.device());
    Tensor dw = gbuf(w), db = rms ? Tensor() : gbuf(b);
    Tensor work;
    if (dw.defined()) work = empty({2L * ::mft::norm_bwd_partial_blocks((int)M) * N}, DType::F32, xs.device());
    if (rms) {
      ::mft::rmsnorm_bwd(bp(xs), bp(dy2), fp(w32), fp(rstd), ds2.defined() ? bp(ds2) : nullptr, bp(dx),
                         fp_or_null(dw), fp_or_null(work), (int)M, N, offset, 1, dy2.stride(0), S());
    } else {
      ::mft::layernorm_bwd(bp(xs), bp(dy2), fp(w32), fp(mean), fp(rstd), ds2.defined() ? bp(ds2) : nullptr, bp(dx),
                           fp_or_null(dw), fp_or_null(db), fp_or_null(work), (int)M, N, 1, dy2.stride(0), S());
    }
    return {dx, has_delta ? dx : Tensor(), Tensor(), Tensor()};
  }
};
}  // namespace

std::pair<Tensor, Tensor> add_norm(const Tensor& x, const Tensor& delta, Param& w, Param* b, float eps, bool rms,
                                   float offset, int out_cols, const Tensor& lora_a, bool resid_out) {
  const int N = (int)x.size(-1);
  MFT_CHECK(x.dtype() == DType::BF16 && N % 8 == 0 && N <= 4096, "norm: bf16 rows, width % 8, <= 4096");
  const long M = x.numel() / N;
  Tensor x2 = x.detach().reshape({M, (int64_t)N}).contiguous();
  Tensor d2 = delta.defined() ? delta.detach().reshape({M, (int64_t)N}).contiguous() : Tensor();
  Tensor w32 = f32_of(w);
  Tensor b32 = (!rms && b) ? f32_of(*b) : Tensor();
  const int oc = out_cols > N ? out_cols : N;
  MFT_CHECK(oc % 8 == 0, "norm: out_cols % 8");
  Tensor y = empty({M, (int64_t)oc}, DType::BF16, x.device());
  Tensor mean = rms ? Tensor() : empty({M}, DType::F32, x.device());
  Tensor rstd = empty({M}, DType::F32, x.device());
  Tensor s = d2.defined() ? empty({M, (int64_t)N}, DType::BF16, x.device()) : Tensor();
  const int lr = lora_a.defined() ? (int)lora_a.size(0) : 0;
  if (lr) {
    MFT_CHECK(lora_a.dtype() == DType::BF16 && lora_a.dim() == 2 && lora_a.size(1) == N && lora_a.stride(1) == 1 &&
                  lora_a.stride(0) % 8 == 0 && lr <= 32 && oc >= N + lr,
              "add_norm: fused LoRA A [R <= 32, N] bf16 with R appended columns");
  }
  const ::mft::bf16_t* la = lr ? bp(lora_a) : nullptr;
  const long lda = lr ? lora_a.stride(0) : 0;
  if (rms) {
    ::mft::rmsnorm_fwd(bp(x2), d2.defined() ? bp(d2) : nullptr, s.defined() ? bp(s) : nullptr, fp(w32), bp(y),
                       fp(rstd), (int)M, N, eps, offset, oc, S(), la, lda, lr);
  } else {
    ::mft::layernorm_fwd(bp(x2), d2.defined() ? bp(d2) : nullptr, s.defined() ? bp(s) : nullptr, fp(w32), fp(b32),
                         bp(y), fp(mean), fp(rstd), (int)M, N, eps, oc, S(), la, lda, lr);
  }
  Shape ys = x.shape();
  ys.back() = oc;
  y = y.detach().view(ys);
  const bool pass = resid_out && !d2.defined();  // s = x, but as this node's output
  Tensor sv = s.defined() ? s.view(x.shape()) : pass ? x2.view(x.shape()) : x;
  auto n = std::make_shared<NormNode>();
  n->name = rms ? "RMSNormBackward" : "LayerNormBackward";
  n->xs = s.defined() ? s : x2;
  n->w32 = w32;
  n->mean = mean;
  n->rstd = rstd;
  n->w = &w;
  n->b = b;
  n->rms = rms;
  n->has_delta = d2.defined();
  n->has_sout = d2.defined() || pass;
  n->offset = offset;
  n->N = N;
  Tensor s_out = n->has_sout ? sv : Tensor();
  // (grads of trainable w / b land in their flat buffers inside apply())
  connect(n, {x, delta, w.leaf, b ? b->leaf : Tensor()}, {s_out, y});
  return {n->has_sout ? s_out : x, y};
}

// ------------------------------------------------------------------ embedding
Tensor embed(const Tensor& ids, Param& wte, Param* wpe, float scale) {
  MFT_CHECK(ids.dim() == 2 && ids.dtype() == DType::I64, "embed: ids [B, S] int64");
  const long M = ids.numel();
  const int S_ = (int)ids.size(1);
  const int C = (int)wte.c.size(1);
  Tensor idc = ids.contiguous();
  Tensor out = empty({M, (int64_t)C}, DType::BF16, ids.device());
  ::mft::embed_fwd(idc.data<int64_t>(), bp(wte.c), wpe ? bp(wpe->c) : nullptr, bp(out), M, C, S_, 0, scale, S());
  if (wte.trainable() || (wpe && wpe->trainable())) {
    Param* pw = &wte;
    auto n = lambda_node("EmbeddingBackward", [idc, pw, wpe, M, C, S_, scale](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor(), Tensor()};
      Tensor d = g[0].contiguous();
      Tensor bte = gbuf(pw), bpe = gbuf(wpe);
      ::mft::embed_bwd(idc.data<int64_t>(), bp(d), fp_or_null(bte), fp_or_null(bpe), M, C, S_, 0, scale, S(),
                       (deterministic() && bte.defined()) ? bte.numel() / C : 0);
      return std::vector<Tensor>{Tensor(), Tensor()};
    });
    connect(n, {wte.leaf, wpe ? wpe->leaf : Tensor()}, {out});
  }
  return out;
}

// ------------------------------------------------------------------ attention
namespace {
void fill_st(long* st, const Tensor& t) {
  MFT_CHECK(t.dim() == 4 && t.stride(3) == 1 && t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0,
            "attention: [B, S, H, D] views with unit D stride and 8-aligned strides");
  st[0] = t.stride(0);
  st[1] = t.stride(1);
  st[2] = t.stride(2);
}
}  // namespace

Tensor attention_packed(const Tensor& qkv, float scale, bool causal, int window, int out_cols) {
  MFT_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.dtype() == DType::BF16, "attention: qkv [B, S, 3, H, D] bf16");
  const int B = (int)qkv.size(0), Sq = (int)qkv.size(1), H = (int)qkv.size(3), D = (int)qkv.size(4);
  MFT_CHECK(D == 64 || D == 128 || D == 256, "attention: head dim 64 / 128 / 256");
  Tensor qd = qkv.detach();
  Tensor q = qd.select(2, 0), k = qd.select(2, 1), v = qd.select(2, 2);
  const int HD = H * D;
  const int oc = out_cols > HD ? out_cols : HD;
  Tensor o_full = empty({B, Sq, (int64_t)oc}, DType::BF16, qkv.device());
  Tensor o = o_full.slice(2, 0, HD).view({B, Sq, H, D});
  Tensor lse = empty({B, H, Sq}, DType::F32, qkv.device());
  ::mft::AttnArgs a{};
  a.q = bp(q);
  a.k = bp(k);
  a.v = bp(v);
  a.o = bp(o);
  a.lse = fp(lse);
  fill_st(a.q_st, q);
  fill_st(a.k_st, k);
  fill_st(a.v_st, v);
  fill_st(a.o_st, o);
  a.B = B;
  a.H = H;
  a.Hkv = H;
  a.Sq = Sq;
  a.Sk = Sq;
  a.D = D;
  a.scale = scale;
  a.causal = causal;
  a.window = window;
  a.o_pad = oc - HD;  // the widened output's zero columns (written by the attention kernel where it can)
  ::mft::attn_fwd(a, S());
  if (needs_grad(qkv)) {
    auto n = lambda_node("FlashAttentionBackward", [qd, o, lse, scale, causal, window, B, Sq, H, D,
                                                     HD](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor()};
      Tensor dqkv = empty(qd.shape(), DType::BF16, qd.device());
      Tensor dout = g[0].slice(2, 0, HD).view({B, Sq, H, D});
      if (dout.stride(3) != 1 || dout.stride(1) % 8) dout = dout.contiguous();
      const int path = ::mft::attn_bwd_path(D, Sq, Sq, window);
      Tensor delta, dq_acc;
      if (path != 0) delta = empty({B, H, Sq}, DType::F32, qd.device());
      if (path == 1) dq_acc = empty({B, Sq, H, D}, DType::F32, qd.device());
      ::mft::AttnBwdArgs b{};
      Tensor q = qd.select(2, 0), k = qd.select(2, 1), v = qd.select(2, 2);
      Tensor dq = dqkv.select(2, 0), dk = dqkv.select(2, 1), dv = dqkv.select(2, 2);
      b.q = bp(q);
      b.k = bp(k);
      b.v = bp(v);
      b.o = bp(o);
      b.dout = bp(dout);
      b.lse = fp(lse);
      b.delta = path != 0 ? fp(delta) : nullptr;
      b.dq_acc = path == 1 ? fp(dq_acc) : nullptr;
      b.dq = bp(dq);
      b.dk = bp(dk);
      b.dv = bp(dv);
      fill_st(b.q_st, q);
      fill_st(b.k_st, k);
      fill_st(b.v_st, v);
      fill_st(b.o_st, o);
      fill_st(b.do_st, dout);
      fill_st(b.dq_st, dq);
      fill_st(b.dk_st, dk);
      fill_st(b.dv_st, dv);
      b.B = B;
      b.H = H;
      b.Hkv = H;
      b.Sq = Sq;
      b.Sk = Sq;
      b.D = D;
      b.scale = scale;
      b.causal = causal;
      b.window = window;
      ::mft::attn_bwd(b, S());
      return std::vector<Tensor>{dqkv};
    });
    connect(n, {qkv}, {o_full});
  }
  return o_full;
}

// ------------------------------------------------------------------ Gemma-3 attention core
Tensor qknorm_rope_attention(const Tensor& qkv, int nq, int nkv, Param& wq, Param& wk, const Tensor& cos_t,
                             const Tensor& sin_t, float eps, float offset, bool interleaved, float scale, int window,
                             int out_cols) {
  MFT_CHECK(qkv.dim() == 4 && qkv.dtype() == DType::BF16 && qkv.size(2) == nq + 2 * nkv,
            "qknorm_rope_attention: qkv [B, S, nq + 2 nkv, D] bf16");
  MFT_CHECK(nkv > 0 && nq % nkv == 0, "qknorm_rope_attention: nq must be a multiple of nkv");
  const int B = (int)qkv.size(0), Sq = (int)qkv.size(1), D = (int)qkv.size(3);
  MFT_CHECK(D == 64 || D == 128 || D == 256, "qknorm_rope_attention: head dim 64 / 128 / 256");
  MFT_CHECK(cos_t.size(0) >= Sq && cos_t.size(1) == D / 2, "qknorm_rope_attention: RoPE tables too short");
  Tensor qd = qkv.detach();
  Tensor xq = qd.slice(2, 0, nq), xk = qd.slice(2, nq, nq + nkv), v = qd.slice(2, nq + nkv, nq + 2 * nkv);
  Tensor wq32 = f32_of(wq), wk32 = f32_of(wk);
  // normalised + rotated q / k (contiguous [B, S, h, D]) and their per-(row, head) rstd
  Tensor q = empty({B, Sq, nq, D}, DType::BF16, qkv.device()), k = empty({B, Sq, nkv, D}, DType::BF16, qkv.device());
  Tensor rq = empty({(int64_t)B * Sq * nq}, DType::F32, qkv.device());
  Tensor rk = empty({(int64_t)B * Sq * nkv}, DType::F32, qkv.device());
  long st[3];
  fill_st(st, xq);
  ::mft::qknorm_rope_fwd(bp(xq), st, bp(q), fp(rq), fp(wq32), B, Sq, nq, D, fp(cos_t), fp(sin_t), 0, eps, offset,
                         interleaved, S());
  fill_st(st, xk);
  ::mft::qknorm_rope_fwd(bp(xk), st, bp(k), fp(rk), fp(wk32), B, Sq, nkv, D, fp(cos_t), fp(sin_t), 0, eps, offset,
                         interleaved, S());
  const int HD = nq * D;
  const int oc = out_cols > HD ? out_cols : HD;
  Tensor o_full = empty({B, Sq, (int64_t)oc}, DType::BF16, qkv.device());
  Tensor o = o_full.slice(2, 0, HD).view({B, Sq, nq, D});
  Tensor lse = empty({B, nq, Sq}, DType::F32, qkv.device());
  ::mft::AttnArgs a{};
  a.q = bp(q);
  a.k = bp(k);
  a.v = bp(v);
  a.o = bp(o);
  a.lse = fp(lse);
  fill_st(a.q_st, q);
  fill_st(a.k_st, k);
  fill_st(a.v_st, v);
  fill_st(a.o_st, o);
  a.B = B;
  a.H = nq;
  a.Hkv = nkv;
  a.Sq = Sq;
  a.Sk = Sq;
  a.D = D;
  a.scale = scale;
  a.causal = 1;
  a.window = window;
  a.o_pad = oc - HD;  // the widened output's zero columns (written by the attention kernel where it can)
  ::mft::attn_fwd(a, S());
  if (any_needs_grad({qkv, wq.leaf, wk.leaf})) {
    Param *pq = &wq, *pk = &wk;
    auto n = lambda_node("QKNormRoPEAttentionBackward", [qd, q, k, o, lse, rq, rk, wq32, wk32, cos_t, sin_t, pq, pk,
                                                         nq, nkv, B, Sq, D, HD, scale, window, offset,
                                                         interleaved](std::vector<Tensor>& g) {
      std::vector<Tensor> out(3);
      if (!g[0].defined()) return out;
      Tensor dqkv = empty(qd.shape(), DType::BF16, qd.device());
      Tensor dout = g[0].slice(2, 0, HD).view({B, Sq, nq, D});
      if (dout.stride(3) != 1 || dout.stride(1) % 8) dout = dout.contiguous();
      const int path = ::mft::attn_bwd_path(D, Sq, Sq, window);
      Tensor delta, dq_acc, dk_tmp, dv_tmp;
      if (path != 0) delta = empty({B, nq, Sq}, DType::F32, qd.device());
      if (path == 1) dq_acc = empty({B, Sq, nq, D}, DType::F32, qd.device());
      // dQ / dK of the rotated normalised q / k (the norm-RoPE backward reads them), dV in place
      Tensor dq = empty({B, Sq, nq, D}, DType::BF16, qd.device()), dk = empty({B, Sq, nkv, D}, DType::BF16, qd.device());
      Tensor v = qd.slice(2, nq + nkv, nq + 2 * nkv), dv = dqkv.slice(2, nq + nkv, nq + 2 * nkv);
      ::mft::AttnBwdArgs b{};
      if (nq != nkv && path != 2) {
        dk_tmp = empty({B, Sq, nq, D}, DType::BF16, qd.device());
        dv_tmp = empty({B, Sq, nq, D}, DType::BF16, qd.device());
        b.dk_tmp = bp(dk_tmp);
        b.dv_tmp = bp(dv_tmp);
        fill_st(b.tmp_st, dk_tmp);
      }
      b.q = bp(q);
      b.k = bp(k);
      b.v = bp(v);
      b.o = bp(o);
      b.dout = bp(dout);
      b.lse = fp(lse);
      b.delta = path != 0 ? fp(delta) : nullptr;
      b.dq_acc = path == 1 ? fp(dq_acc) : nullptr;
      b.dq = bp(dq);
      b.dk = bp(dk);
      b.dv = bp(dv);
      fill_st(b.q_st, q);
      fill_st(b.k_st, k);
      fill_st(b.v_st, v);
      fill_st(b.o_st, o);
      fill_st(b.do_st, dout);
      fill_st(b.dq_st, dq);
      fill_st(b.dk_st, dk);
      fill_st(b.dv_st, dv);
      b.B = B;
      b.H = nq;
      b.Hkv = nkv;
      b.Sq = Sq;
      b.Sk = Sq;
      b.D = D;
      b.scale = scale;
      b.causal = 1;
      b.window = window;
      ::mft::attn_bwd(b, S());
      // q / k norm-RoPE backward straight into their dqkv slices (+ norm-weight grads if trainable)
      auto nr_bwd = [&](int h0, int nh, const Tensor& dy, const Tensor& r, const Tensor& w32, Param* pw) {
        Tensor x = qd.slice(2, h0, h0 + nh), dx = dqkv.slice(2, h0, h0 + nh);
        Tensor dw = gbuf(pw), work;
        if (dw.defined()) work = empty({(int64_t)::mft::qknorm_rope_bwd_blocks((long)B * Sq * nh) * D}, DType::F32, qd.device());
        long xs[3], ds[3];
        fill_st(xs, x);
        fill_st(ds, dx);
        ::mft::qknorm_rope_bwd(bp(x), xs, bp(dy), fp(r), fp(w32), bp(dx), ds, fp_or_null(dw), fp_or_null(work), B, Sq,
                               nh, D, fp(cos_t), fp(sin_t), 0, offset, interleaved, 1, S());
      };
      nr_bwd(0, nq, dq, rq, wq32, pq);
      nr_bwd(nq, nkv, dk, rk, wk32, pk);
      out[0] = dqkv;
      return out;
    });
    connect(n, {qkv, wq.leaf, wk.leaf}, {o_full});
  }
  return o_full;
}

// ------------------------------------------------------------------ gated MLP activation
Tensor gated_act(const Tensor& gu, int act, int out_cols) {
  const int64_t I2 = gu.size(-1), I = I2 / 2;
  MFT_CHECK(gu.dtype() == DType::BF16 && I2 % 16 == 0, "gated_act: bf16 [M, 2I], I % 8 == 0");
  Tensor g2 = gu.detach().reshape({-1, I2}).contiguous();
  const int64_t M = g2.size(0);
  const int64_t oc = out_cols > I ? out_cols : I;
  MFT_CHECK(oc % 8 == 0, "gated_act: out_cols % 8");
  Tensor y = empty({M, oc}, DType::BF16, gu.device());
  ::mft::gated_fwd(bp(g2), bp(y), M, (int)I, oc, act, S(), (int)(oc - I));  // (zeroes the widened columns too)
  if (needs_grad(gu)) {
    Shape gshape = gu.shape();
    auto n = lambda_node("GatedActBackward", [g2, gshape, M, I, act](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor()};
      Tensor dy = g[0];
      if (dy.stride(1) != 1 || dy.stride(0) % 8) dy = dy.contiguous();
      Tensor dgu = empty({M, 2 * I}, DType::BF16, dy.device());
      ::mft::gated_bwd(bp(g2), bp(dy), dy.stride(0), bp(dgu), M, (int)I, act, S());
      return std::vector<Tensor>{dgu.view(gshape)};
    });
    connect(n, {gu}, {y});
  }
  return y;
}

// ------------------------------------------------------------------ linear / MLP
static void bias_grad(Param* b, const Tensor& dy2) {
  if (!b || !b->trainable()) return;
  Tensor buf = grad_buffer(b->leaf);
  const long M = dy2.size(0);
  const int N = (int)dy2.size(1);
  const int nb = ::mft::colsum_partial_blocks(M);
  Tensor part = empty({(int64_t)nb * N}, DType::F32, dy2.device());
  ::mft::colsum_partial(bp(dy2), dy2.stride(0), M, N, fp(part), S());
  ::mft::reduce_rows(fp(part), fp(buf), nb, N, 1, S());
}

// the GeGLU backward outside a fused epilogue: d gu from dh (any producer) and gu
static Tensor geglu_bwd_unfused(const Tensor& dh, const Tensor& gu2) {
  Tensor dy = dh;
  if (dy.stride(1) != 1 || dy.stride(0) % 8) dy = dy.contiguous();
  const int64_t M = gu2.size(0), I = gu2.size(1) / 2;
  Tensor dgu = empty({M, 2 * I}, DType::BF16, dh.device());
  ::mft::gated_bwd(bp(gu2), bp(dy), dy.stride(0), bp(dgu), M, (int)I, 0, S());
  return dgu;
}

Tensor linear_p(const Tensor& x, Param& w, Param* b, Tensor* geglu_h, const Tensor& geglu_gu) {
  const int64_t K = x.size(-1), N = w.c.size(0);
  Tensor x2 = x.detach().reshape({-1, K});
  if (x2.stride(1) != 1 || x2.stride(0) % 8) x2 = x2.contiguous();
  Shape ys = x.shape();
  ys.back() = N;
  Tensor y = empty({x2.size(0), N}, DType::BF16, x.device());
  if (geglu_h) {
    MFT_CHECK(!b, "linear_p: the GeGLU epilogue takes no bias");
    gemm_geglu_fwd(x2, w.c, y, *geglu_h);
  } else {
    gemm_nt(x2, w.c, b ? b->c : Tensor(), y);
  }
  const bool gg = geglu_gu.defined();
  const Tensor xin = gg ? geglu_gu : x;  // the GeGLU-fused down projection's input edge is gu
  if (any_needs_grad({xin, w.leaf, b ? b->leaf : Tensor()})) {
    Param* pw = &w;
    const Tensor gu2 = gg ? geglu_gu.detach().reshape({-1, geglu_gu.size(-1)}) : Tensor();
    const Shape gshape = gg ? geglu_gu.shape() : Shape{};
    auto n = lambda_node("LinearBackward", [x2, pw, b, K, N, gu2, gshape, gg](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor(), Tensor(), Tensor()};
      Tensor dy2 = g[0].reshape({-1, N});
      if (dy2.stride(1) != 1 || dy2.stride(0) % 8) dy2 = dy2.contiguous();
      Tensor dx;
      const Tensor wt = !pw->trainable() && !pw->streamed ? pw->transposed() : Tensor();
      if (gg && wt.defined() && geglu_fusable(dy2.size(0), gu2.size(1) / 2, N, N)) {
        dx = empty({dy2.size(0), gu2.size(1)}, DType::BF16, dy2.device());
        gemm_geglu_bwd(dy2, wt.slice(0, 0, gu2.size(1) / 2), gu2, dx);
      } else {
        dx = empty({dy2.size(0), K}, DType::BF16, dy2.device());
        gemm_nn(dy2, pw->c, dx, wt);
        if (gg) dx = geglu_bwd_unfused(dx.slice(1, 0, gu2.size(1) / 2), gu2);
      }
      if (pw->trainable()) {
        Tensor buf = grad_buffer(pw->leaf).view({N, K});
        gemm_wgrad(buf, dy2, x2);
      }
      bias_grad(b, dy2);
      return std::vector<Tensor>{gg ? dx.view(gshape) : dx, Tensor(), Tensor()};
    });
    connect(n, {xin, w.leaf, b ? b->leaf : Tensor()}, {y});
  }
  return y.view(ys);
}

Tensor mlp_gelu(const Tensor& x, Param& w1, Param& b1, Param& w2, Param& b2, const Tensor& resid) {
  const int64_t K = x.size(-1), I = w1.c.size(0), N = w2.c.size(0);
  Tensor x2 = x.detach().reshape({-1, K}).contiguous();
  const int64_t M = x2.size(0);
  Tensor h = empty({M, I}, DType::BF16, x.device()), pre = empty({M, I}, DType::BF16, x.device());
  Gemm8Extra ex;
  ex.bias = &b1.c;
  ex.aux = &pre;
  gemm8_call(x2, w1.c, false, ::mft::GEMM_EPI_BIAS_GELU_D, h, ex);  // aux = GELU'(pre)
  Tensor y = empty({M, N}, DType::BF16, x.device());
  // resid: y = resid + MLP(x) straight from the projection's epilogue (the block's residual add)
  const Tensor r2 = resid.defined() ? resid.detach().reshape({M, N}).contiguous() : Tensor();
  gemm_nt(h, w2.c, b2.c, y, r2);
  Shape ys = x.shape();
  ys.back() = N;
  if (any_needs_grad({x, w1.leaf, b1.leaf, w2.leaf, b2.leaf, resid})) {
    Param *p1 = &w1, *q1 = &b1, *p2 = &w2, *q2 = &b2;
    auto n = lambda_node("MLPGeluBackward", [x2, h, pre, p1, q1, p2, q2, M, K, I, N](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>(5);
      Tensor dy2 = g[0].reshape({M, N}).contiguous();
      Tensor dpre = empty({M, I}, DType::BF16, dy2.device());
      Gemm8Extra e2;
      Tensor aux = pre;
      e2.aux = &aux;
      if (!p2->trainable() && !p2->streamed) gemm8_call(dy2, p2->transposed(), false, ::mft::GEMM_EPI_MUL_AUX, dpre, e2);
      else if (gemm4_on()) {
        // trainable / streamed W2: a transposed copy (|W2| bytes) puts the product on gemm4's NT path
        Tensor w2t;
        {
          NoGradGuard ng;
          w2t = p2->c.t().contiguous();
        }
        gemm8_call(dy2, w2t, false, ::mft::GEMM_EPI_MUL_AUX, dpre, e2);
      } else gemm8_call(dy2, p2->c, true, ::mft::GEMM_EPI_MUL_AUX, dpre, e2);
      Tensor dx = empty({M, K}, DType::BF16, dy2.device());
      gemm_nn(dpre, p1->c, dx, !p1->trainable() && !p1->streamed ? p1->transposed() : Tensor());
      if (p2->trainable()) {
        Tensor b2v = grad_buffer(p2->leaf).view({N, I});
        gemm_wgrad(b2v, dy2, h);
      }
      if (p1->trainable()) {
        Tensor b1v = grad_buffer(p1->leaf).view({I, K});
        gemm_wgrad(b1v, dpre, x2);
      }
      bias_grad(q2, dy2);
      bias_grad(q1, dpre);
      // the fused residual's gradient is the output's (an identity branch)
      return std::vector<Tensor>{dx, Tensor(), Tensor(), Tensor(), Tensor(), g[0]};
    });
    connect(n, {x, w1.leaf, b1.leaf, w2.leaf, b2.leaf, resid}, {y});
  }
  return y.view(ys);
}

// ------------------------------------------------------------------ LoRA weight prep (batched)
namespace {
struct LoraPrep {
  struct Item {
    Tensor dst, src;  // (held: the batch may still write a dst its layer has dropped -- harmless)
    ::mft::LoraPrepEntry e;
    bool uploaded = false;  // the device list holds exactly this entry
  };
  std::vector<Item> items;
  std::unordered_map<const void*, size_t> by_dst;
  ::mft::LoraPrepEntry* dev = nullptr;
  int ndev = 0;
  bool dirty = false;   // items changed since the upload
  bool active = false;  // the batch ran at the start of this forward
  // A captured training graph keeps the device list (and every dst / src it names) it was recorded
  // with: a list replaced later -- e.g. an eager eval forward that registers new entries -- is retired
  // here, never freed, so a later replay of that graph still reads live memory.
  std::vector<::mft::LoraPrepEntry*> retired_dev;
  std::vector<Item> retired_items;
};
LoraPrep& lprep() {
  static LoraPrep p;
  return p;
}
bool prep_off() {
  static const bool off = std::getenv("MFT_LORA_PREP_BATCH") && std::getenv("MFT_LORA_PREP_BATCH")[0] == '0';
  return off;
}

// dst = scale * src (2-D bf16 views, dst row-major): skipped when this forward's batch already wrote it
void prep_copy(const Tensor& dst, const Tensor& src, float scale) {
  auto& P = lprep();
  ::mft::LoraPrepEntry e{(::mft::bf16_t*)dst.data_ptr(), (long)dst.stride(0), (const ::mft::bf16_t*)src.data_ptr(),
                         (long)src.stride(0), (long)src.stride(1), (int)dst.size(0), (int)dst.size(1), scale};
  auto it = P.by_dst.find(e.dst);
  const bool same = it != P.by_dst.end() && [&] {
    const auto& o = P.items[it->second].e;
    return o.src == e.src && o.srs == e.srs && o.scs == e.scs && o.rows == e.rows && o.cols == e.cols &&
           o.dld == e.dld && o.scale == e.scale;
  }();
  if (P.active && same && P.items[it->second].uploaded) return;  // done by the batch
  k::unary(desc(dst), desc(src), k::U_AFFINE, scale, 0.f, S());
  if (prep_off() || dst.dtype() != DType::BF16 || src.dtype() != DType::BF16 || dst.stride(1) != 1) return;
  if (it == P.by_dst.end()) {
    P.by_dst.emplace(e.dst, P.items.size());
    P.items.push_back({dst, src, e, false});
    P.dirty = true;
  } else if (!same) {  // (the batch may still write the old entry first: this copy, later in the stream, wins)
    if (P.items[it->second].uploaded) P.retired_items.push_back(P.items[it->second]);  // a graph may name it
    P.items[it->second] = {dst, src, e, false};
    P.dirty = true;
  }
}
}  // namespace

void lora_prep_step_end() { lprep().active = false; }

void lora_prep_reset() {
  // the model that registered the entries is going away: forget them (its tensors are released with
  // the items) but keep the uploaded list's memory -- a graph of that model may not be destroyed yet
  auto& P = lprep();
  if (P.dev) P.retired_dev.push_back(P.dev);
  P.dev = nullptr;
  P.ndev = 0;
  P.items.clear();
  P.by_dst.clear();
  P.retired_items.clear();
  P.dirty = false;
  P.active = false;
}

void lora_prep_step_begin() {
  auto& P = lprep();
  P.active = false;
  if (prep_off() || P.items.empty()) return;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_OK(hipStreamIsCapturing(S(), &cap));
  // (re)upload -- only outside a capture; inside one the uploaded list still runs and the layers whose
  // entries changed since make their own copies.  The previous list is retired, not freed: a captured
  // graph's lora_prep node still reads it on every replay.
  if (P.dirty && cap == hipStreamCaptureStatusNone) {
    std::vector<::mft::LoraPrepEntry> es;
    for (auto& it : P.items) es.push_back(it.e);
    if (P.dev) P.retired_dev.push_back(P.dev);
    P.dev = nullptr;
    HIP_OK(hipMalloc(&P.dev, es.size() * sizeof(::mft::LoraPrepEntry)));
    HIP_OK(hipMemcpy(P.dev, es.data(), es.size() * sizeof(::mft::LoraPrepEntry), hipMemcpyHostToDevice));
    P.ndev = (int)es.size();
    P.dirty = false;
    for (auto& it : P.items) it.uploaded = true;
  }
  if (P.ndev == 0) return;
  ::mft::lora_prep_batched(P.dev, P.ndev, S());
  P.active = true;
}

// ------------------------------------------------------------------ LoRA (augmented K)
int lora_aug_cols(int in_features, const std::vector<LoraAdapter>& ads) {
  int r = 0;
  for (auto& a : ads) r += a.rank;
  return (in_features + r + 63) / 64 * 64;
}

Tensor lora_fused_a(const std::vector<LoraAdapter>& ads, bool training) {
  // The norm-fused u = y A^T (norm_fwd_kernel LR > 0: one wave per row, every rank reduced across the
  // wave and A re-read per row) measured 2-8x the plain norm's time -- Gemma-3 +5.4 ms, GPT-2 +0.9 ms
  // per step against norm + lora_rowdot (profiles/r4b_norm_lora_regression.txt): opt-in only
  // (MFT_NORM_LORA=1), the MFMA rowdot pass is the default.
  static const bool on = std::getenv("MFT_NORM_LORA") && std::getenv("MFT_NORM_LORA")[0] == '1';
  if (!on || ads.empty()) return Tensor();
  int rt = 0;
  for (auto& a : ads) {
    if (a.dropout > 0.f && training) return Tensor();
    if (a.A.c.dtype() != DType::BF16 || a.A.c.stride(1) != 1) return Tensor();
    rt += a.rank;
  }
  if (rt > 32) return Tensor();
  if (ads.size() == 1) return ads[0].A.c;
  NoGradGuard ng;
  std::vector<Tensor> as;
  for (auto& a : ads) as.push_back(a.A.c);
  return cat(as, 0);
}

Tensor lora_linear_aug(const Tensor& xa, int K, Param& w, Param* b, std::vector<LoraAdapter>& ads, float s,
                       Tensor& waug, bool training, const Tensor& drop_ctr, bool u_ready, const Tensor& resid,
                       Tensor* geglu_h, const Tensor& geglu_gu) {
  MFT_CHECK(!w.trainable(), "lora_linear_aug: the base weight must be frozen");
  const int64_t Ka = xa.size(-1), N = w.c.size(0);
  Tensor xa2 = xa.detach().reshape({-1, Ka});
  MFT_CHECK(xa2.stride(1) == 1, "lora_linear_aug: input rows must be contiguous");
  const int64_t M = xa2.size(0);
  Tensor x2 = xa2.slice(1, 0, K);
  if (!waug.defined() || waug.size(1) != Ka) {
    NoGradGuard ng;
    waug = zeros({N, Ka}, DType::BF16, xa.device());
    Tensor wl = waug.slice(1, 0, K);
    wl.copy_(w.c);
  }
  bool nodrop = true;
  for (auto& a : ads) nodrop = nodrop && (a.dropout <= 0.f || !training);
  int off = K;
  Tensor acat;  // [sum r_i, K]: built once per step, reused by the backward's fused dx epilogue
  MFT_CHECK(!u_ready || nodrop, "lora_linear_aug: u precomputed by the producer needs dropout off");
  if (u_ready) {
    // u_1..u_n already in the appended columns (the norm that produced xa computed them)
  } else if (nodrop && ads.size() > 1) {  // one pass over x for every u_i (adjacent appended columns)
    int rsum = 0;
    for (auto& a : ads) rsum += a.rank;
    Tensor& ac = w.lora_acat;  // persistent stack of the A's, refreshed by the batched weight prep
    if (!ac.defined() || ac.size(0) != rsum || ac.size(1) != K) ac = empty({(int64_t)rsum, K}, DType::BF16, xa.device());
    int o = 0;
    for (auto& a : ads) {
      prep_copy(ac.slice(0, o, o + a.rank), a.A.c, 1.f);
      o += a.rank;
    }
    acat = ac;
    const int R = (int)acat.size(0);
    ::mft::lora_rowdot(bp(x2), x2.stride(0), bp(acat), acat.stride(0), bp(xa2) + K, xa2.stride(0), M, K, R, 1.f,
                       ::mft::LoraDrop{nullptr, 0, 0.f}, S());
  }
  for (auto& a : ads) {
    const int R = a.rank;
    if (!u_ready && !(nodrop && ads.size() > 1)) {
      ::mft::LoraDrop d{drop_ctr.defined() ? drop_ctr.data<int64_t>() : nullptr, a.salt, training ? a.dropout : 0.f};
      ::mft::lora_rowdot(bp(x2), x2.stride(0), bp(a.A.c), a.A.c.stride(0), bp(xa2) + off, xa2.stride(0), M, K, R, 1.f,
                         d, S());
    }
    // s B_i^T into the slice's rows of the augmented weight
    Tensor dst = waug.slice(0, a.col0, a.col0 + a.ncols).slice(1, off, off + R);
    prep_copy(dst, a.B.c.t(), s);
    off += R;
  }
  Tensor y = empty({M, N}, DType::BF16, xa.device());
  // resid: y = resid + LoRA-linear(x) straight from the GEMM's epilogue (the block's residual add)
  const Tensor r2 = resid.defined() ? resid.detach().reshape({M, N}).contiguous() : Tensor();
  if (geglu_h) {  // y = gu, and h = gelu(g) u from the same epilogue
    MFT_CHECK(!b && !resid.defined(), "lora_linear_aug: the GeGLU epilogue takes no bias / residual");
    gemm_geglu_fwd(xa2, waug, y, *geglu_h);
  } else {
    gemm_nt(xa2, waug, b ? b->c : Tensor(), y, r2);
  }
  Shape ys = xa.shape();
  ys.back() = N;
  const bool gg = geglu_gu.defined();  // (the GeGLU-fused down projection: its input edge is gu)
  std::vector<Tensor> ins{gg ? geglu_gu : xa};
  for (auto& a : ads) {
    ins.push_back(a.A.leaf);
    ins.push_back(a.B.leaf);
  }
  const bool has_resid = resid.defined();
  if (has_resid) ins.push_back(resid);  // last input: gradient = the output's (identity branch)
  if (any_needs_grad(ins)) {
    Param* pw = &w;
    std::vector<LoraAdapter>* pads = &ads;
    Tensor wa = waug;
    Shape xshape = gg ? geglu_gu.shape() : xa.shape();
    const Tensor gu2 = gg ? geglu_gu.detach().reshape({-1, geglu_gu.size(-1)}) : Tensor();
    auto n = lambda_node("LoRALinearBackward", [xa2, xshape, K, Ka, M, N, pw, pads, s, wa, training, drop_ctr, acat_f = acat,
                                                 nin = ins.size(), has_resid, gu2, gg](std::vector<Tensor>& g) {
      std::vector<Tensor> out(nin);
      if (!g[0].defined()) return out;
      if (has_resid) out[nin - 1] = g[0];
      auto& ads = *pads;
      Tensor dy2 = g[0].reshape({M, N});
      if (dy2.stride(1) != 1 || dy2.stride(0) % 8) dy2 = dy2.contiguous();
      Tensor x2 = xa2.slice(1, 0, K);
      int rt = 0;
      bool nodrop = true;
      for (auto& a : ads) {
        rt += a.rank;
        nodrop = nodrop && (a.dropout <= 0.f || !training);
      }
      const bool fused = nodrop && rt > 0 && rt <= 32 && rt % 8 == 0 && N % 64 == 0 && K % 8 == 0;
      Tensor dxa = empty({M, gg ? gu2.size(1) : Ka}, DType::BF16, dy2.device());
      Tensor dx = gg ? Tensor() : dxa.slice(1, 0, K);
      // GeGLU-fused down projection: the seg2 GEMM's epilogue writes d gu into dxa; other data-gradient
      // paths compute dh first, then the unfused GeGLU backward
      const bool geglu_epi = gg && geglu_fusable(M, K, N, N);
      // gemm4 form of the fused data gradient: v (= s dy B) in the first rt of 64 columns, the rest zero, read
      // as a second K segment against A^T (dx = dy W + v A in one pass, gemm_nt_seg2)
      const bool seg2 = (fused && gemm4_on() && Ka % 8 == 0 && lora_seg2_ok(M, K, N)) || (geglu_epi && fused);
      if (gg && !(geglu_epi && seg2)) dx = empty({M, (int64_t)K}, DType::BF16, dy2.device());
      Tensor vall = empty({M, seg2 ? (int64_t)64 : (int64_t)std::max(rt, 8)}, DType::BF16, dy2.device());
      bool v_padded = false;  // lora_dy zeroes the padding itself (one adapter of rank 8)
      int o = 0;
      std::vector<bool> db_done(ads.size(), false);
      // several rank-8 adapters on 256-aligned column ranges of this dy (Gemma-3's q | k | v, gate | up): one
      // lora_dy launch over all of them and one finish (MFT_LORA_DY_MULTI=0: per adapter, A/B)
      static const bool multi_off = std::getenv("MFT_LORA_DY_MULTI") && std::getenv("MFT_LORA_DY_MULTI")[0] == '0';
      if (!multi_off && ads.size() > 1 && ads.size() <= 4 && !deterministic()) {
        std::vector<::mft::LoraDyAdapter> la;
        int oo = 0;
        for (size_t i = 0; i < ads.size(); ++i) {
          auto& a = ads[i];
          if (a.rank != 8 || !a.B.trainable() || (K + oo) % 8) break;
          ::mft::LoraDyAdapter e{};
          e.B = (const ::mft::bf16_t*)a.B.c.data_ptr();
          e.ldb = a.B.c.stride(0);
          e.u = (const ::mft::bf16_t*)bp(xa2) + K + oo;
          e.ldu = xa2.stride(0);
          e.dB = fp(grad_buffer(a.B.leaf));
          e.ldd = a.ncols;
          e.v = (::mft::bf16_t*)bp(vall) + oo;
          e.ldv = vall.stride(0);
          e.col0 = a.col0;
          e.N = a.ncols;
          e.vz = seg2 && i + 1 == ads.size() && oo + 8 == rt ? 64 - rt : 0;
          la.push_back(e);
          oo += a.rank;
        }
        if (la.size() == ads.size() && ::mft::lora_dy_multi_ok(la.data(), (int)la.size()) && dy2.stride(0) % 8 == 0) {
          Tensor vpart = empty({::mft::lora_dy_multi_vpart_floats(la.data(), (int)la.size(), M)}, DType::F32, dy2.device());
          ::mft::lora_dy_multi(bp(dy2), dy2.stride(0), la.data(), (int)la.size(), fp(vpart), M, s, S());
          std::fill(db_done.begin(), db_done.end(), true);
          v_padded = la.back().vz > 0;
          o = rt;
        }
      }
      for (size_t i = 0; i < ads.size() && o < rt; ++i) {
        auto& a = ads[i];
        Tensor v = vall.slice(1, o, o + a.rank);
        Tensor dys = dy2.slice(1, a.col0, a.col0 + a.ncols);
        Tensor dB = a.B.trainable() ? grad_buffer(a.B.leaf) : Tensor();
        if (dB.defined() && a.rank == 8 && a.ncols % 8 == 0 && a.col0 % 8 == 0 && (K + o) % 8 == 0) {
          Tensor vpart = empty({(int64_t)((a.ncols + 255) / 256) * M * 8}, DType::F32, dy2.device());
          Tensor dw = det_ws(::mft::lora_dy_ws_floats(M, a.ncols));
          // the last adapter's finish also zeroes the padding right after its 8 columns (o + 8 == rt)
          const int vz = seg2 && i + 1 == ads.size() && o + 8 == rt ? 64 - rt : 0;
          ::mft::lora_dy(bp(dys), dys.stride(0), bp(a.B.c), a.B.c.stride(0), bp(xa2) + K + o, xa2.stride(0), fp(dB),
                         a.ncols, fp(vpart), bp(v), v.stride(0), M, a.ncols, s, S(), dptr(dw), vz);
          db_done[i] = true;
          v_padded = vz > 0;
        } else {
          ::mft::lora_rowdot(bp(dys), dys.stride(0), bp(a.B.c), a.B.c.stride(0), bp(v), v.stride(0), M, a.ncols,
                             a.rank, s, ::mft::LoraDrop{nullptr, 0, 0.f}, S());
        }
        o += a.rank;
      }
      Tensor acat = acat_f;
      if (!acat.defined()) {
        std::vector<Tensor> as;
        for (auto& a : ads) as.push_back(a.A.c);
        acat = as.size() == 1 ? as[0] : cat(as, 0);
      }
      if (seg2) {
        if (!v_padded) ::mft::zero_cols(bp(vall), 64, M, rt, 64 - rt, S());
        Tensor& at = pw->lora_at;  // A^T, zero-padded to 64 columns (persistent: the padding stays zero)
        if (!at.defined() || at.size(0) != K) at = zeros({K, 64}, DType::BF16, dy2.device());
        int oc = 0;  // per adapter (stable sources: a concatenated A is a new tensor every step)
        for (auto& a : ads) {
          prep_copy(at.slice(1, oc, oc + a.rank), a.A.c.t(), 1.f);
          oc += a.rank;
        }
        if (geglu_epi) gemm_geglu_bwd(dy2, pw->transposed(), gu2, dxa, vall, at);
        else gemm_nt_seg2(dy2, pw->transposed(), vall, at, dx);
      } else if (fused) {
        Gemm8Extra ex;
        Tensor vu = vall.slice(1, 0, rt);
        ex.lora_u = &vu;
        ex.lora_w = &acat;
        gemm8_call(dy2, pw->transposed(), false, ::mft::GEMM_EPI_LORA, dx, ex);
      } else {
        gemm_nn(dy2, wa.slice(1, 0, K), dx);
        o = 0;
        for (auto& a : ads) {
          Tensor v = vall.slice(1, o, o + a.rank);
          ::mft::LoraDrop d{drop_ctr.defined() ? drop_ctr.data<int64_t>() : nullptr, a.salt,
                            training ? a.dropout : 0.f};
          ::mft::lora_update(bp(dx), dx.stride(0), bp(v), v.stride(0), bp(a.A.c), a.A.c.stride(0), bp(dx),
                             dx.stride(0), M, (int)K, a.rank, 1.f, d, S());
          o += a.rank;
        }
      }
      // dA (one pass over x for several rank-8 adapters) and the remaining dB
      bool da_done = false;
      if (nodrop && ads.size() > 1 && ads.size() <= 8) {
        bool all8 = true;
        for (auto& a : ads) all8 = all8 && a.rank == 8 && a.A.trainable();
        if (all8) {
          ::mft::WgradOuts wo{};
          wo.n = (int)ads.size();
          for (size_t i = 0; i < ads.size(); ++i) wo.p[i] = fp(grad_buffer(ads[i].A.leaf));
          Tensor dw = det_ws(::mft::lora_wgrad_ws_floats(M, K, rt));
          ::mft::lora_wgrad(bp(x2), x2.stride(0), bp(vall), vall.stride(0), nullptr, 1, K, M, K, rt, 1.f,
                            ::mft::LoraDrop{nullptr, 0, 0.f}, S(), &wo, dptr(dw));
          da_done = true;
        }
      }
      o = 0;
      int off = K;
      for (size_t i = 0; i < ads.size(); ++i) {
        auto& a = ads[i];
        Tensor v = vall.slice(1, o, o + a.rank);
        if (!da_done && a.A.trainable()) {
          ::mft::LoraDrop d{drop_ctr.defined() ? drop_ctr.data<int64_t>() : nullptr, a.salt,
                            training ? a.dropout : 0.f};
          Tensor dw = det_ws(::mft::lora_wgrad_ws_floats(M, K, a.rank));
          ::mft::lora_wgrad(bp(x2), x2.stride(0), bp(v), v.stride(0), fp(grad_buffer(a.A.leaf)), 1, K, M, K, a.rank,
                            1.f, d, S(), nullptr, dptr(dw));
        }
        if (a.B.trainable() && !db_done[i]) {
          Tensor dys = dy2.slice(1, a.col0, a.col0 + a.ncols);
          Tensor dw = det_ws(::mft::lora_wgrad_ws_floats(M, a.ncols, a.rank));
          ::mft::lora_wgrad(bp(dys), dys.stride(0), bp(xa2) + off, xa2.stride(0), fp(grad_buffer(a.B.leaf)), 1,
                            a.ncols, M, a.ncols, a.rank, s, ::mft::LoraDrop{nullptr, 0, 0.f}, S(), nullptr, dptr(dw));
        }
        o += a.rank;
        off += a.rank;
      }
      if (gg && !(geglu_epi && seg2)) dxa = geglu_bwd_unfused(dx, gu2);
      out[0] = dxa.view(xshape);
      return out;
    });
    connect(n, ins, {y});
  }
  return y.view(ys);
}

Tensor lora_linear(const Tensor& x, Param& w, Param* b, std::vector<LoraAdapter>& ads, float s, bool training,
                   const Tensor& drop_ctr) {
  MFT_CHECK(!w.trainable(), "lora_linear: the base weight must be frozen");
  const int64_t K = x.size(-1), N = w.c.size(0);
  Tensor x2 = x.detach().reshape({-1, K});
  if (x2.stride(1) != 1 || x2.stride(0) % 8) x2 = x2.contiguous();
  const int64_t M = x2.size(0);
  Tensor y = empty({M, N}, DType::BF16, x.device());
  gemm_nt(x2, w.c, b ? b->c : Tensor(), y);
  std::vector<Tensor> us;
  for (auto& a : ads) {
    Tensor u = empty({M, (int64_t)a.rank}, DType::BF16, x.device());
    ::mft::LoraDrop d{drop_ctr.defined() ? drop_ctr.data<int64_t>() : nullptr, a.salt, training ? a.dropout : 0.f};
    ::mft::lora_rowdot(bp(x2), x2.stride(0), bp(a.A.c), a.A.c.stride(0), bp(u), u.stride(0), M, (int)K, a.rank, 1.f, d,
                       S());
    Tensor ys = y.slice(1, a.col0, a.col0 + a.ncols);
    ::mft::lora_update(bp(ys), ys.stride(0), bp(u), u.stride(0), bp(a.B.c), a.B.c.stride(0), bp(ys), ys.stride(0), M,
                       a.ncols, a.rank, s, ::mft::LoraDrop{nullptr, 0, 0.f}, S());
    us.push_back(u);
  }
  Shape ys = x.shape();
  ys.back() = N;
  std::vector<Tensor> ins{x};
  for (auto& a : ads) {
    ins.push_back(a.A.leaf);
    ins.push_back(a.B.leaf);
  }
  if (any_needs_grad(ins)) {
    Param* pw = &w;
    std::vector<LoraAdapter>* pads = &ads;
    Shape xshape = x.shape();
    auto n = lambda_node("LoRALinearBackward", [x2, xshape, us, K, M, N, pw, pads, s, training, drop_ctr,
                                                 nin = ins.size()](std::vector<Tensor>& g) {
      std::vector<Tensor> out(nin);
      if (!g[0].defined()) return out;
      Tensor dy2 = g[0].reshape({M, N});
      if (dy2.stride(1) != 1 || dy2.stride(0) % 8) dy2 = dy2.contiguous();
      Tensor dx = empty({M, K}, DType::BF16, dy2.device());
      gemm_nn(dy2, pw->c, dx, !pw->streamed ? pw->transposed() : Tensor());
      for (size_t i = 0; i < pads->size(); ++i) {
        auto& a = (*pads)[i];
        ::mft::LoraDrop d{drop_ctr.defined() ? drop_ctr.data<int64_t>() : nullptr, a.salt, training ? a.dropout : 0.f};
        Tensor dys = dy2.slice(1, a.col0, a.col0 + a.ncols);
        Tensor v = empty({M, (int64_t)a.rank}, DType::BF16, dy2.device());
        ::mft::lora_rowdot(bp(dys), dys.stride(0), bp(a.B.c), a.B.c.stride(0), bp(v), v.stride(0), M, a.ncols, a.rank,
                           s, ::mft::LoraDrop{nullptr, 0, 0.f}, S());
        ::mft::lora_update(bp(dx), dx.stride(0), bp(v), v.stride(0), bp(a.A.c), a.A.c.stride(0), bp(dx), dx.stride(0),
                           M, (int)K, a.rank, 1.f, d, S());
        if (a.A.trainable()) {
          Tensor dw = det_ws(::mft::lora_wgrad_ws_floats(M, (int)K, a.rank));
          ::mft::lora_wgrad(bp(x2), x2.stride(0), bp(v), v.stride(0), fp(grad_buffer(a.A.leaf)), 1, K, M, (int)K,
                            a.rank, 1.f, d, S(), nullptr, dptr(dw));
        }
        if (a.B.trainable()) {
          Tensor dw = det_ws(::mft::lora_wgrad_ws_floats(M, a.ncols, a.rank));
          ::mft::lora_wgrad(bp(dys), dys.stride(0), bp(us[i]), us[i].stride(0), fp(grad_buffer(a.B.leaf)), 1, a.ncols,
                            M, a.ncols, a.rank, s, ::mft::LoraDrop{nullptr, 0, 0.f}, S(), nullptr, dptr(dw));
        }
      }
      out[0] = dx.view(xshape);
      return out;
    });
    connect(n, ins, {y});
  }
  return y.view(ys);
}

// ------------------------------------------------------------------ LM head + cross entropy
namespace {
Tensor inv_valid(const Tensor& labels) {
  NoGradGuard ng;
  Tensor cnt = empty({1}, DType::F32, labels.device());
  k::count_valid(labels.data<int64_t>(), labels.numel(), -100, fp(cnt), S());
  Tensor one = ones({1}, DType::F32, labels.device());
  return div(one, maximum(cnt, one));
}
}  // namespace

Tensor lm_head_ce(const Tensor& h, Param& w, const Tensor& labels, int V, int64_t chunk, float w_grad_scale,
                  bool sum_reduction) {
  const int64_t M = h.size(0), C = h.size(1), Vp = w.c.size(0);
  Tensor hc = h.detach().contiguous();
  Tensor lab = labels.reshape({-1}).contiguous();
  // mean: the loss and every gradient scaled by 1 / valid tokens; sum: unscaled
  Tensor scale = sum_reduction ? ones({1}, DType::F32, h.device()) : inv_valid(lab);
  Tensor loss_rows = empty({M}, DType::F32, h.device());
  const bool need_h = needs_grad(h);
  const bool need_w = w.trainable() && grad_enabled();
  const bool need = need_h || need_w;
  Tensor dh = need ? empty({M, C}, DType::BF16, h.device()) : Tensor();
  Tensor wbuf = need_w ? grad_buffer(w.leaf).view({Vp, C}) : Tensor();
  // the trainable (tied) head: dh = dlogits W on gemm4 through W^T, one transposed copy per call (|W|
  // bytes, against the 4 x 32768 x Vp dlogits the chunks' products read)
  Tensor wt;
  if (need_h && need_w) {
    NoGradGuard ng;
    wt = w.c.t().contiguous();
  }
  if (chunk <= 0) chunk = M;
  for (int64_t i = 0; i < M; i += chunk) {
    const int64_t r = std::min(chunk, M - i);
    Tensor hi = hc.slice(0, i, i + r);
    // fused forward (softmax statistics from the fp32 logits tile, E = exp(logit - tile max)) +
    // per-tile-rescaled NN dgrad; E becomes dlogits in place only when W itself trains
    Tensor E = need ? empty({r, Vp}, DType::BF16, h.device()) : Tensor();
    Tensor ws = empty({::mft::lm_head_ce_ws_floats((int)r, (int)Vp, (int)C)}, DType::F32, h.device());
    ::mft::CeArgs a{};
    a.h = bp(hi); a.ldh = C;
    a.W = bp(w.c); a.ldw = C;
    a.labels = lab.data<int64_t>() + i;
    a.M = (int)r; a.K = (int)C; a.Vpad = (int)Vp; a.V = V;
    a.E = need ? bp(E) : nullptr; a.lde = Vp;
    a.loss = fp(loss_rows) + i;
    a.scale = fp(scale); a.extra = 1.f;
    a.dh = need ? bp(dh) + i * C : nullptr; a.lddh = C;
    a.materialize = need_w ? 1 : 0;
    a.ws = fp(ws);
    if (wt.defined()) a.Wt = bp(wt), a.ldwt = wt.stride(0);
    ::mft::lm_head_ce(a, S());
    if (need_w) gemm_wgrad(wbuf, E, hi, w_grad_scale);
  }
  Tensor loss = mul(sum(loss_rows), scale);
  if (need) {
    auto n = lambda_node("LMHeadCEBackward", [dh, M](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor(), Tensor()};
      Tensor gs = g[0].to(DType::F32).contiguous();
      Tensor out = empty(dh.shape(), DType::BF16, dh.device());
      ::mft::scale_bf16(bp(dh), bp(out), dh.numel(), fp(gs), 1.f, S());
      return std::vector<Tensor>{out, Tensor()};
    });
    connect(n, {h, w.leaf}, {loss});
  }
  return loss;
}

Tensor lm_head_token_nll(const Tensor& h, Param& w, const Tensor& labels, int V, int64_t chunk) {
  NoGradGuard ng;
  const int64_t M = h.size(0), Vp = w.c.size(0);
  Tensor hc = h.detach().contiguous();
  Tensor lab = labels.reshape({-1}).contiguous();
  Tensor loss_rows = empty({M}, DType::F32, h.device());
  if (chunk <= 0) chunk = M;
  for (int64_t i = 0; i < M; i += chunk) {
    const int64_t r = std::min(chunk, M - i);
    Tensor ws = empty({::mft::lm_head_ce_ws_floats((int)r, (int)Vp, 0)}, DType::F32, h.device());
    ::mft::CeArgs a{};  // loss only: no logits are stored
    a.h = bp(hc) + i * hc.size(1); a.ldh = hc.size(1);
    a.W = bp(w.c); a.ldw = w.c.size(1);
    a.labels = lab.data<int64_t>() + i;
    a.M = (int)r; a.K = (int)hc.size(1); a.Vpad = (int)Vp; a.V = V;
    a.loss = fp(loss_rows) + i;
    a.extra = 1.f;
    a.ws = fp(ws);
    ::mft::lm_head_ce(a, S());
  }
  return loss_rows;
}

std::pair<Tensor, Tensor> lm_head_nll(const Tensor& h, Param& w, const Tensor& labels, int V, int64_t chunk) {
  NoGradGuard ng;
  Tensor loss_rows = lm_head_token_nll(h, w, labels, V, chunk);
  Tensor lab = labels.reshape({-1}).contiguous();
  Tensor cnt = empty({1}, DType::F32, h.device());
  k::count_valid(lab.data<int64_t>(), lab.numel(), -100, fp(cnt), S());
  return {sum(loss_rows), cnt};
}

}  // namespace eng
}  // namespace mft
