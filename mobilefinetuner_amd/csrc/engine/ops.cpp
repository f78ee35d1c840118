// libmft engine: generic differentiable ops (see ops.h).  Backward formulas follow the
// reference's BackwardFunction catalog (core/backward_functions.cpp: Add/Sub/Mul/Div :66-221,
// unary :140-266, Softmax :297-340, LogSoftmax :665-676, Sum :833-885, MSE :396-411, NLL :951-968,
// Matmul :94-138, Linear :342-394), computed by the generic kernels of engine/tensor_kernels.hip.
#include "engine/ops.h"

#include <algorithm>
#include <cmath>

#include "engine/autograd.h"
#include "engine/gemm.h"
#include "kernels.h"

namespace mft {
namespace eng {

namespace {
hipStream_t S() { return current_stream(); }

DType float_result(const Tensor& a, const Tensor& b) {
  if (a.dtype() == DType::F32 || b.dtype() == DType::F32) return DType::F32;
  if (a.dtype() == DType::BF16 || b.dtype() == DType::BF16) return DType::BF16;
  if (a.dtype() == DType::F16 || b.dtype() == DType::F16) return DType::F16;
  return DType::F32;
}
DType float_of(const Tensor& a) {
  return (a.dtype() == DType::F32 || a.dtype() == DType::BF16 || a.dtype() == DType::F16) ? a.dtype() : DType::F32;
}
}  // namespace

Shape broadcast_shape(const Shape& a, const Shape& b) {
  const size_t n = std::max(a.size(), b.size());
  Shape o(n);
  for (size_t i = 0; i < n; ++i) {
    const int64_t x = i < n - a.size() ? 1 : a[i - (n - a.size())];
    const int64_t y = i < n - b.size() ? 1 : b[i - (n - b.size())];
    MFT_CHECK(x == y || x == 1 || y == 1, "broadcast: ", shape_str(a), " vs ", shape_str(b));
    o[i] = x == 1 ? y : x;
  }
  return o;
}

Tensor sum_to(const Tensor& g, const Shape& shape) {
  if (g.shape() == shape) return g;
  NoGradGuard ng;
  Tensor cur = g;
  // sum away extra leading dims, then size-1 broadcast dims
  while (cur.dim() > (int)shape.size()) cur = sum(cur, 0, false);
  for (int d = 0; d < (int)shape.size(); ++d)
    if (shape[d] == 1 && cur.size(d) != 1) cur = sum(cur, d, true);
  return cur.reshape(shape);
}

// ------------------------------------------------------------------ binary
static Tensor binary_raw(const Tensor& a, const Tensor& b, int op, float alpha, DType out) {
  Shape s = broadcast_shape(a.shape(), b.shape());
  Tensor o = empty(s, out, a.device());
  k::binary(desc(o), desc_bcast(a, s), desc_bcast(b, s), op, alpha, S());
  return o;
}

Tensor add(const Tensor& a, const Tensor& b, float alpha) {
  Tensor o;
  {
    NoGradGuard ng;
    o = binary_raw(a, b, k::B_ADD, alpha, float_result(a, b));
  }
  Shape sa = a.shape(), sb = b.shape();
  DType da = a.dtype(), db = b.dtype();
  auto n = lambda_node("AddBackward", [sa, sb, da, db, alpha](std::vector<Tensor>& g) {
    if (!g[0].defined()) return std::vector<Tensor>{Tensor(), Tensor()};
    return std::vector<Tensor>{sum_to(g[0], sa).to(da), mul_scalar(sum_to(g[0], sb), alpha).to(db)};
  });
  connect(n, {a, b}, {o});
  return o;
}

Tensor sub(const Tensor& a, const Tensor& b) { return add(a, b, -1.f); }

Tensor mul(const Tensor& a, const Tensor& b) {
  Tensor o;
  {
    NoGradGuard ng;
    o = binary_raw(a, b, k::B_MUL, 1.f, float_result(a, b));
  }
  if (any_needs_grad({a, b})) {
    Tensor ad = a.detach(), bd = b.detach();
    auto n = lambda_node("MulBackward", [ad, bd](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor(), Tensor()};
      return std::vector<Tensor>{sum_to(mul(g[0], bd), ad.shape()).to(ad.dtype()),
                                 sum_to(mul(g[0], ad), bd.shape()).to(bd.dtype())};
    });
    connect(n, {a, b}, {o});
  }
  return o;
}

Tensor div(const Tensor& a, const Tensor& b) {
  Tensor o;
  {
    NoGradGuard ng;
    o = binary_raw(a, b, k::B_DIV, 1.f, float_result(a, b));
  }
  if (any_needs_grad({a, b})) {
    Tensor ad = a.detach(), bd = b.detach(), od = o.detach();
    auto n = lambda_node("DivBackward", [ad, bd, od](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor(), Tensor()};
      Tensor ga = div(g[0], bd);
      Tensor gb = neg(mul(ga, od));  // -g a / b^2 = -(g / b) * (a / b)
      return std::vector<Tensor>{sum_to(ga, ad.shape()).to(ad.dtype()), sum_to(gb, bd.shape()).to(bd.dtype())};
    });
    connect(n, {a, b}, {o});
  }
  return o;
}

static Tensor minmax(const Tensor& a, const Tensor& b, int op) {
  Tensor o;
  {
    NoGradGuard ng;
    o = binary_raw(a, b, op, 1.f, float_result(a, b));
  }
  if (any_needs_grad({a, b})) {
    Tensor ad = a.detach(), bd = b.detach(), od = o.detach();
    auto n = lambda_node(op == k::B_MAX ? "MaximumBackward" : "MinimumBackward", [ad, bd, od](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor(), Tensor()};
      Tensor ma = eq(ad, od), mb = ne(ad, od);  // ties -> a
      return std::vector<Tensor>{sum_to(mul(g[0], ma), ad.shape()).to(ad.dtype()),
                                 sum_to(mul(g[0], mb), bd.shape()).to(bd.dtype())};
    });
    connect(n, {a, b}, {o});
  }
  return o;
}
Tensor maximum(const Tensor& a, const Tensor& b) { return minmax(a, b, k::B_MAX); }
Tensor minimum(const Tensor& a, const Tensor& b) { return minmax(a, b, k::B_MIN); }

void add_(Tensor& a, const Tensor& b, float alpha) {
  NoGradGuard ng;
  k::axpy(desc(a), desc_bcast(b, a.shape()), alpha, 1, S());
}

// ------------------------------------------------------------------ unary
static Tensor unary_op(const Tensor& x, int op, float pa, float pb, const char* name) {
  Tensor o;
  {
    NoGradGuard ng;
    o = empty(x.shape(), float_of(x), x.device());
    k::unary(desc(o), desc(x), op, pa, pb, S());
  }
  if (needs_grad(x)) {
    Tensor xd = x.detach();
    auto n = lambda_node(name, [xd, op, pa, pb](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor()};
      Tensor dx = empty(xd.shape(), xd.dtype(), xd.device());
      k::unary_bwd(desc(dx), desc_bcast(g[0], xd.shape()), desc(xd), op, pa, pb, S());
      return std::vector<Tensor>{dx};
    });
    connect(n, {x}, {o});
  }
  return o;
}

Tensor neg(const Tensor& x) { return unary_op(x, k::U_NEG, 0, 0, "NegBackward"); }
Tensor relu(const Tensor& x) { return unary_op(x, k::U_RELU, 0, 0, "ReluBackward"); }
Tensor gelu(const Tensor& x, bool t) { return unary_op(x, t ? k::U_GELU_TANH : k::U_GELU_ERF, 0, 0, "GeluBackward"); }
Tensor silu(const Tensor& x) { return unary_op(x, k::U_SILU, 0, 0, "SiLUBackward"); }
Tensor sigmoid(const Tensor& x) { return unary_op(x, k::U_SIGMOID, 0, 0, "SigmoidBackward"); }
Tensor tanh(const Tensor& x) { return unary_op(x, k::U_TANH, 0, 0, "TanhBackward"); }
Tensor exp(const Tensor& x) { return unary_op(x, k::U_EXP, 0, 0, "ExpBackward"); }
Tensor log(const Tensor& x) { return unary_op(x, k::U_LOG, 0, 0, "LogBackward"); }
Tensor sqrt(const Tensor& x) { return unary_op(x, k::U_SQRT, 0, 0, "SqrtBackward"); }
Tensor rsqrt(const Tensor& x) { return unary_op(x, k::U_RSQRT, 0, 0, "RsqrtBackward"); }
Tensor abs(const Tensor& x) { return unary_op(x, k::U_ABS, 0, 0, "AbsBackward"); }
Tensor square(const Tensor& x) { return unary_op(x, k::U_SQUARE, 0, 0, "SquareBackward"); }
Tensor pow(const Tensor& x, float p) { return unary_op(x, k::U_POW, p, 0, "PowBackward"); }
Tensor clamp(const Tensor& x, float lo, float hi) { return unary_op(x, k::U_CLAMP, lo, hi, "ClampBackward"); }
Tensor sin(const Tensor& x) { return unary_op(x, k::U_SIN, 0, 0, "SinBackward"); }
Tensor cos(const Tensor& x) { return unary_op(x, k::U_COS, 0, 0, "CosBackward"); }
Tensor affine(const Tensor& x, float a, float b) { return unary_op(x, k::U_AFFINE, a, b, "ScaleBackward"); }
Tensor mul_scalar(const Tensor& x, float s) { return affine(x, s, 0.f); }
Tensor add_scalar(const Tensor& x, float s) { return affine(x, 1.f, s); }

// ------------------------------------------------------------------ comparisons
static Tensor cmp(const Tensor& a, const Tensor& b, int op) {
  NoGradGuard ng;
  return binary_raw(a, b, op, 1.f, DType::BOOL);
}
Tensor eq(const Tensor& a, const Tensor& b) { return cmp(a, b, k::B_EQ); }
Tensor ne(const Tensor& a, const Tensor& b) { return cmp(a, b, k::B_NE); }
Tensor gt(const Tensor& a, const Tensor& b) { return cmp(a, b, k::B_GT); }
Tensor lt(const Tensor& a, const Tensor& b) { return cmp(a, b, k::B_LT); }
Tensor ge(const Tensor& a, const Tensor& b) { return cmp(a, b, k::B_GE); }
Tensor le(const Tensor& a, const Tensor& b) { return cmp(a, b, k::B_LE); }

// ------------------------------------------------------------------ reductions
Tensor sum(const Tensor& x, int dim, bool keepdim) {
  const int nd = x.dim();
  if (dim < 0) dim += nd;
  MFT_CHECK(dim >= 0 && dim < nd, "sum: dim");
  Tensor o;
  Shape oshape = x.shape();
  {
    NoGradGuard ng;
    // move `dim` last, make contiguous rows, reduce rows
    std::vector<int> perm;
    for (int i = 0; i < nd; ++i)
      if (i != dim) perm.push_back(i);
    perm.push_back(dim);
    Tensor xc = x.permute(perm).contiguous();
    const int64_t n = x.size(dim), rows = x.numel() / std::max<int64_t>(n, 1);
    oshape[dim] = 1;
    o = empty(oshape, float_of(x), x.device());
    k::sum_rows(xc.data_ptr(), (int)xc.dtype(), o.data_ptr(), (int)o.dtype(), rows, (int)n, 1.f, S());
    if (!keepdim) o = o.squeeze(dim);
  }
  if (needs_grad(x)) {
    Shape xs = x.shape(), ks = oshape;
    DType dt = x.dtype();
    auto n = lambda_node("SumBackward", [xs, ks, dt](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor()};
      Tensor gi = empty(xs, dt, g[0].device());
      gi.copy_(g[0].reshape(ks));
      return std::vector<Tensor>{gi};
    });
    connect(n, {x}, {o});
  }
  return o;
}

Tensor sum(const Tensor& x) {
  Tensor o;
  {
    NoGradGuard ng;
    Tensor xc = x.contiguous();
    o = empty({1}, DType::F32, x.device());
    // two-stage: rows of 4096 (one wave each), then the row sums -- a single wave only for n <= 4096
    // (one wave over Gemma's 65,536 per-token losses was a 0.5 ms dependent-load chain per step)
    const int64_t n = x.numel();
    if (n <= 4096) {
      k::sum_rows(xc.data_ptr(), (int)xc.dtype(), o.data_ptr(), (int)DType::F32, 1, (int)n, 1.f, S());
    } else {
      const int64_t w = 4096, rows = n / w, rem = n - rows * w;
      Tensor part = empty({rows + 1}, DType::F32, x.device());
      part.zero_();
      k::sum_rows(xc.data_ptr(), (int)xc.dtype(), part.data_ptr(), (int)DType::F32, rows, (int)w, 1.f, S());
      if (rem) {
        Tensor tail = xc.view({n}).slice(0, rows * w, n);
        k::sum_rows(tail.data_ptr(), (int)xc.dtype(), part.data<float>() + rows, (int)DType::F32, 1, (int)rem, 1.f,
                    S());
      }
      k::sum_rows(part.data_ptr(), (int)DType::F32, o.data_ptr(), (int)DType::F32, 1, (int)(rows + 1), 1.f, S());
    }
    if (float_of(x) != DType::F32) o = o.to(float_of(x));
  }
  if (needs_grad(x)) {
    Shape xs = x.shape();
    DType dt = x.dtype();
    auto n = lambda_node("SumAllBackward", [xs, dt](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor()};
      Tensor gi = empty(xs, dt, g[0].device());
      gi.copy_(g[0].reshape({}));
      return std::vector<Tensor>{gi};
    });
    connect(n, {x}, {o});
  }
  return o;
}

Tensor mean(const Tensor& x) { return mul_scalar(sum(x), 1.f / (float)std::max<int64_t>(1, x.numel())); }
Tensor mean(const Tensor& x, int dim, bool keepdim) {
  const int64_t n = x.size(dim);
  return mul_scalar(sum(x, dim, keepdim), 1.f / (float)std::max<int64_t>(1, n));
}

// ------------------------------------------------------------------ softmax
static Tensor softmax_impl(const Tensor& x, bool logm) {
  Tensor o;
  const int64_t n = x.size(-1), rows = x.numel() / std::max<int64_t>(n, 1);
  {
    NoGradGuard ng;
    Tensor xc = x.contiguous();
    o = empty(x.shape(), float_of(x), x.device());
    k::softmax_rows(xc.data_ptr(), (int)xc.dtype(), o.data_ptr(), (int)o.dtype(), rows, (int)n, n, n, logm, S());
  }
  if (needs_grad(x)) {
    Tensor od = o.detach();
    auto nd = lambda_node(logm ? "LogSoftmaxBackward" : "SoftmaxBackward", [od, rows, n, logm](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor()};
      Tensor gc = g[0].to(od.dtype()).contiguous();
      Tensor dx = empty(od.shape(), od.dtype(), od.device());
      k::softmax_rows_bwd(od.data_ptr(), gc.data_ptr(), dx.data_ptr(), (int)od.dtype(), rows, (int)n, logm, S());
      return std::vector<Tensor>{dx};
    });
    connect(nd, {x}, {o});
  }
  return o;
}
Tensor softmax(const Tensor& x) { return softmax_impl(x, false); }
Tensor log_softmax(const Tensor& x) { return softmax_impl(x, true); }

// ------------------------------------------------------------------ losses
Tensor mse_loss(const Tensor& x, const Tensor& y) { return mean(square(sub(x, y))); }

Tensor nll_loss(const Tensor& logp, const Tensor& target, int ignore) {
  MFT_CHECK(logp.dim() == 2 && target.numel() == logp.size(0) && target.dtype() == DType::I64,
            "nll_loss: logp [N, C], target int64 [N]");
  const int64_t N = logp.size(0), C = logp.size(1);
  Tensor lc = logp.contiguous();
  Tensor tc = target.contiguous();
  Tensor rows, cnt, scale, loss;
  {
    NoGradGuard ng;
    rows = empty({N}, DType::F32, logp.device());
    k::nll_rows(lc.data_ptr(), (int)lc.dtype(), tc.data<int64_t>(), rows.data<float>(), N, (int)C, C, ignore, S());
    cnt = empty({1}, DType::F32, logp.device());
    k::count_valid(tc.data<int64_t>(), N, ignore, cnt.data<float>(), S());
    scale = div(ones({1}, DType::F32, logp.device()), maximum(cnt, ones({1}, DType::F32, logp.device())));
    loss = mul(sum(rows), scale);
  }
  if (needs_grad(logp)) {
    Tensor sd = scale, td = tc, ld = lc.detach();
    auto n = lambda_node("NLLLossBackward", [sd, td, ld, N, C, ignore](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor()};
      Tensor s = mul(sd, g[0].to(DType::F32));
      Tensor d = empty(ld.shape(), ld.dtype(), ld.device());
      k::nll_rows_bwd(d.data_ptr(), (int)d.dtype(), td.data<int64_t>(), N, (int)C, C, ignore, s.data<float>(), S());
      return std::vector<Tensor>{d};
    });
    connect(n, {logp}, {loss});
  }
  return loss;
}

Tensor cross_entropy(const Tensor& logits, const Tensor& target, int ignore) {
  return nll_loss(log_softmax(logits.dim() == 2 ? logits : logits.reshape({-1, logits.size(-1)})),
                  target.reshape({-1}), ignore);
}

Tensor lm_cross_entropy(const Tensor& logits, const Tensor& labels, int ignore) {
  MFT_CHECK(logits.dim() == 3 && labels.dim() == 2, "lm_cross_entropy: logits [B, S, V], labels [B, S]");
  const int64_t S_ = logits.size(1);
  Tensor lg = logits.slice(1, 0, S_ - 1);
  Tensor lb = labels.slice(1, 1, S_).contiguous();
  return cross_entropy(lg.reshape({-1, logits.size(2)}), lb.reshape({-1}), ignore);
}

// ------------------------------------------------------------------ matmul / linear
Tensor matmul(const Tensor& a, const Tensor& b) {
  MFT_CHECK(a.dim() >= 2 && b.dim() >= 2, "matmul: operands need >= 2 dims");
  MFT_CHECK(a.size(-1) == b.size(-2), "matmul: ", a.str(), " x ", b.str());
  Tensor o;
  const int64_t M = a.size(-2), K = a.size(-1), N = b.size(-1);
  {
    NoGradGuard ng;
    if (b.dim() == 2) {  // 2-D weight shared over the batch (MatmulBackward :104-127): one GEMM
      Tensor a2 = a.reshape({-1, K}).contiguous(), b2 = b.contiguous();
      Shape os = a.shape();
      os.back() = N;
      o = empty(os, a.dtype(), a.device());
      Tensor o2 = o.view({-1, N});
      blas_gemm(a2, false, b2, false, o2);
    } else {
      MFT_CHECK(a.dim() == b.dim(), "matmul: batched operands need equal rank");
      Tensor a3 = a.reshape({-1, M, K}).contiguous(), b3 = b.reshape({-1, K, N}).contiguous();
      const int64_t B = a3.size(0);
      MFT_CHECK(b3.size(0) == B, "matmul: batch mismatch");
      Shape os = a.shape();
      os.back() = N;
      o = empty(os, a.dtype(), a.device());
      Tensor o3 = o.view({B, M, N});
      for (int64_t i = 0; i < B; ++i) {
        Tensor oi = o3.select(0, i);
        blas_gemm(a3.select(0, i), false, b3.select(0, i), false, oi);
      }
    }
  }
  if (any_needs_grad({a, b})) {
    Tensor ad = a.detach(), bd = b.detach();
    auto n = lambda_node("MatmulBackward", [ad, bd](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor(), Tensor()};
      Tensor ga = matmul(g[0], bd.transpose(-1, -2).contiguous());
      Tensor gb;
      if (bd.dim() == 2) {
        Tensor a2 = ad.reshape({-1, ad.size(-1)}).contiguous();
        Tensor g2 = g[0].reshape({-1, g[0].size(-1)}).contiguous();
        gb = empty(bd.shape(), bd.dtype(), bd.device());
        blas_gemm(a2, true, g2, false, gb);
      } else {
        gb = matmul(ad.transpose(-1, -2).contiguous(), g[0]);
      }
      return std::vector<Tensor>{ga, gb};
    });
    connect(n, {a, b}, {o});
  }
  return o;
}

Tensor linear(const Tensor& x, const Tensor& w, const Tensor& b) {
  const int64_t K = x.size(-1), N = w.size(0);
  MFT_CHECK(w.size(1) == K, "linear: ", x.str(), " x ", w.str());
  Tensor o;
  Tensor x2 = x.detach().reshape({-1, K}).contiguous();
  {
    NoGradGuard ng;
    Shape os = x.shape();
    os.back() = N;
    o = empty(os, x.dtype(), x.device());
    Tensor o2 = o.view({-1, N});
    if (x.dtype() == DType::BF16 && w.dtype() == DType::BF16 && (!b.defined() || b.dtype() == DType::BF16)) {
      gemm_nt(x2, w, b, o2);
    } else {
      blas_gemm(x2, false, w.contiguous(), true, o2);
      if (b.defined()) add_(o2, b);
    }
  }
  if (any_needs_grad({x, w, b})) {
    Tensor wd = w.detach();
    const bool need_w = needs_grad(w), need_b = b.defined() && needs_grad(b);
    Shape xs = x.shape();
    Shape bs = b.defined() ? b.shape() : Shape{};
    auto n = lambda_node("LinearBackward", [x2, wd, need_w, need_b, xs, bs, K, N](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor(), Tensor(), Tensor()};
      Tensor g2 = g[0].reshape({-1, N}).contiguous();
      Tensor gx = empty(xs, x2.dtype(), x2.device());
      Tensor gx2 = gx.view({-1, K});
      if (g2.dtype() == DType::BF16 && wd.dtype() == DType::BF16) gemm_nn(g2, wd, gx2);
      else blas_gemm(g2.to(wd.dtype()), false, wd, false, gx2);
      Tensor gw, gb;
      if (need_w) {
        gw = zeros(wd.shape(), DType::F32, wd.device());
        if (g2.dtype() == DType::BF16 && x2.dtype() == DType::BF16) gemm_wgrad(gw, g2, x2);
        else blas_gemm(g2.to(DType::F32), true, x2.to(DType::F32), false, gw);
      }
      if (need_b) gb = sum(g2.to(DType::F32), 0, false).reshape(bs);
      return std::vector<Tensor>{gx, gw, gb};
    });
    connect(n, {x, w, b}, {o});
  }
  return o;
}

// ------------------------------------------------------------------ misc
Tensor dropout(const Tensor& x, float p, uint64_t seed, bool training) {
  if (!training || p <= 0.f) return x;
  Tensor xc = x.contiguous();
  Tensor o, mask;
  {
    NoGradGuard ng;
    o = empty(x.shape(), x.dtype(), x.device());
    mask = empty(x.shape(), DType::U8, x.device());
    k::dropout(xc.data_ptr(), o.data_ptr(), mask.data<uint8_t>(), (int)x.dtype(), x.numel(), seed, p, S());
  }
  if (needs_grad(x)) {
    auto n = lambda_node("DropoutBackward", [mask, p](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor()};
      Tensor gc = g[0].contiguous();
      Tensor dx = empty(gc.shape(), gc.dtype(), gc.device());
      k::dropout_bwd(gc.data_ptr(), mask.data<uint8_t>(), dx.data_ptr(), (int)gc.dtype(), gc.numel(), p, S());
      return std::vector<Tensor>{dx};
    });
    connect(n, {x}, {o});
  }
  return o;
}

Tensor cat(const std::vector<Tensor>& ts, int dim) {
  MFT_CHECK(!ts.empty(), "cat: empty list");
  const int nd = ts[0].dim();
  if (dim < 0) dim += nd;
  Shape os = ts[0].shape();
  os[dim] = 0;
  for (auto& t : ts) os[dim] += t.size(dim);
  Tensor o;
  std::vector<int64_t> offs;
  {
    NoGradGuard ng;
    o = empty(os, ts[0].dtype(), ts[0].device());
    int64_t off = 0;
    for (auto& t : ts) {
      offs.push_back(off);
      Tensor dst = o.slice(dim, off, off + t.size(dim));
      dst.copy_(t);
      off += t.size(dim);
    }
  }
  if (any_needs_grad(ts)) {
    std::vector<int64_t> lens;
    for (auto& t : ts) lens.push_back(t.size(dim));
    auto n = lambda_node("CatBackward", [offs, lens, dim](std::vector<Tensor>& g) {
      std::vector<Tensor> r;
      for (size_t i = 0; i < offs.size(); ++i)
        r.push_back(g[0].defined() ? g[0].slice(dim, offs[i], offs[i] + lens[i]).contiguous() : Tensor());
      return r;
    });
    connect(n, ts, {o});
  }
  return o;
}

Tensor where_mask(const Tensor& mask, const Tensor& a, float fill) {
  // mask * a + (1 - mask) * fill: `fill` must be finite (inf * 0 would be NaN); use -1e30 for -inf
  MFT_CHECK(std::isfinite(fill), "where_mask: fill must be finite (use e.g. -1e30 instead of -inf)");
  Tensor m = mask.to(float_of(a));
  Tensor keep = mul(a, m);
  NoGradGuard ng;
  Tensor inv = affine(m, -fill, fill);
  Tensor r;
  {
    r = keep;
  }
  add_(r, inv);
  return r;
}

// ------------------------------------------------------------------ composite catalog layers
Tensor layer_norm(const Tensor& x, const Tensor& w, const Tensor& b, float eps) {
  Tensor xc = sub(x, mean(x, -1, true));
  Tensor y = mul(mul(xc, rsqrt(add_scalar(mean(square(xc), -1, true), eps))), w);
  return b.defined() ? add(y, b) : y;
}

Tensor rms_norm(const Tensor& x, const Tensor& w, float eps, float offset) {
  Tensor y = mul(x, rsqrt(add_scalar(mean(square(x), -1, true), eps)));
  return mul(y, offset != 0.f ? add_scalar(w, offset) : w);
}

Tensor batch_norm(const Tensor& x, const Tensor& gamma, const Tensor& beta, float eps) {
  MFT_CHECK(x.dim() == 2, "batch_norm: x must be [N, C]");
  Tensor xc = sub(x, mean(x, 0, true));
  Tensor y = mul(mul(xc, rsqrt(add_scalar(mean(square(xc), 0, true), eps))), gamma);
  return beta.defined() ? add(y, beta) : y;
}

Tensor swiglu(const Tensor& gate, const Tensor& up) { return mul(silu(gate), up); }
Tensor geglu(const Tensor& gate, const Tensor& up) { return mul(gelu(gate, true), up); }

Tensor causal_mask(int64_t Sq, int64_t Sk, int64_t window) {
  std::vector<float> m((size_t)(Sq * Sk));
  const int64_t coff = Sk - Sq;
  for (int64_t i = 0; i < Sq; ++i)
    for (int64_t j = 0; j < Sk; ++j)
      m[(size_t)(i * Sk + j)] = (j <= i + coff && (window <= 0 || i + coff - j < window)) ? 1.f : 0.f;
  return from_vector(m, {Sq, Sk}, DType::F32);
}

Tensor apply_mask(const Tensor& scores, const Tensor& mask) { return where_mask(mask, scores, -1e30f); }

Tensor repeat_kv(const Tensor& x, int n_rep) {
  MFT_CHECK(x.dim() == 4 && n_rep >= 1, "repeat_kv: x must be [B, S, Hkv, D]");
  if (n_rep == 1) return x;
  Tensor u = x.unsqueeze(3);  // [B, S, Hkv, 1, D]
  std::vector<Tensor> parts((size_t)n_rep, u);
  return cat(parts, 3).reshape({x.size(0), x.size(1), x.size(2) * n_rep, x.size(3)});
}

Tensor apply_rope(const Tensor& x, const Tensor& cos_t, const Tensor& sin_t, bool interleaved) {
  MFT_CHECK(x.dim() >= 3, "apply_rope: x must be [.., S, H, D]");
  const int nd = x.dim();
  const int64_t S = x.size(nd - 3), D = x.size(nd - 1), h = D / 2;
  MFT_CHECK(D % 2 == 0 && cos_t.numel() == S * h && sin_t.numel() == S * h, "apply_rope: cos / sin must be [S, D/2]");
  if (!interleaved) {
    Tensor c = cos_t.reshape({S, 1, h}), s = sin_t.reshape({S, 1, h});
    Tensor x1 = x.slice(nd - 1, 0, h), x2 = x.slice(nd - 1, h, D);
    return cat({sub(mul(x1, c), mul(x2, s)), add(mul(x2, c), mul(x1, s))}, nd - 1);
  }
  Shape ps = x.shape();
  ps.back() = h;
  ps.push_back(2);
  Tensor xp = x.reshape(ps);  // [.., S, H, D/2, 2]
  Tensor c = cos_t.reshape({S, 1, h, 1}), s = sin_t.reshape({S, 1, h, 1});
  Tensor x1 = xp.slice(nd, 0, 1), x2 = xp.slice(nd, 1, 2);
  return cat({sub(mul(x1, c), mul(x2, s)), add(mul(x2, c), mul(x1, s))}, nd).reshape(x.shape());
}

Tensor embedding(const Tensor& ids, const Tensor& table) {
  MFT_CHECK(ids.dtype() == DType::I64 && table.dim() == 2 && table.stride(1) == 1 && table.stride(0) == table.size(1),
            "embedding: int64 ids, contiguous [V, C] table");
  const int64_t n = ids.numel(), C = table.size(1), V = table.size(0);
  Tensor idc = ids.contiguous();
  Tensor o;
  {
    NoGradGuard ng;
    o = empty({n, C}, table.dtype(), table.device());
    // one gather launch (rows by id); the ids are range-checked on the host first -- the kernel skips
    // an out-of-range id, the check makes it an error instead of a silent zero-free row
    Tensor hi = idc.to(Device::cpu());
    for (int64_t i = 0; i < n; ++i)
      MFT_CHECK(hi.data<int64_t>()[i] >= 0 && hi.data<int64_t>()[i] < V, "embedding: id ", hi.data<int64_t>()[i],
                " outside [0, ", V, ")");
    k::gather_rows(o.data_ptr(), (int)o.dtype(), table.data_ptr(), (int)table.dtype(), idc.data<int64_t>(), n, (int)C,
                   V, S());
  }
  Shape os = ids.shape();
  os.push_back(C);
  o = o.view(os);
  if (needs_grad(table)) {
    Shape ts = table.shape();
    auto nd = lambda_node("EmbeddingBackward", [ts, idc, n, C, V](std::vector<Tensor>& g) {
      if (!g[0].defined()) return std::vector<Tensor>{Tensor()};
      Tensor gt = zeros(ts, DType::F32, g[0].device());
      Tensor g2 = g[0].reshape({n, C}).contiguous();
      k::scatter_add_rows(gt.data<float>(), g2.data_ptr(), (int)g2.dtype(), idc.data<int64_t>(), n, (int)C, V, S());
      return std::vector<Tensor>{gt};
    });
    connect(nd, {table}, {o});
  }
  return o;
}

}  // namespace eng
}  // namespace mft
