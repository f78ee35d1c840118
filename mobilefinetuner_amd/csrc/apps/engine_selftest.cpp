// libmft engine self-test (GPU): every generic op of the engine's catalog and its backward against a
// host fp64 oracle written here (the oracle lives with the test, not in the op layer), plus the
// allocator and autograd-tape semantics.  Prints one line per check and "ALL OK" at the end.
// Run by tests/test_engine_gpu.py.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "engine/allocator.h"
#include "engine/autograd.h"
#include "engine/gemm.h"
#include "engine/nn.h"
#include "engine/ops.h"
#include "engine/tensor.h"

using namespace mft::eng;

namespace {
int g_fail = 0;
std::mt19937 rng(123);

std::vector<double> rnd(size_t n, double lo = -1, double hi = 1) {
  std::uniform_real_distribution<double> d(lo, hi);
  std::vector<double> v(n);
  for (auto& x : v) x = d(rng);
  return v;
}
Tensor dev(const std::vector<double>& v, Shape s, DType dt = DType::F32) {
  std::vector<float> f(v.begin(), v.end());
  Tensor h = from_blob(f.data(), s, DType::F32, Device::cpu());
  Tensor d = empty(s, dt);
  d.copy_(h);
  synchronize();
  return d;
}
std::vector<double> host(const Tensor& t) {
  auto f = t.to_vector_f32();
  return std::vector<double>(f.begin(), f.end());
}
void check(const std::string& name, const std::vector<double>& got, const std::vector<double>& ref, double tol) {
  double err = 0, mx = 1e-12;
  bool size_ok = got.size() == ref.size();
  for (size_t i = 0; size_ok && i < ref.size(); ++i) {
    err = std::max(err, std::fabs(got[i] - ref[i]));
    mx = std::max(mx, std::fabs(ref[i]));
  }
  const bool ok = size_ok && err / mx <= tol && std::isfinite(err);
  std::printf("%-44s %s  rel_err=%.2e (n=%zu)\n", name.c_str(), ok ? "ok  " : "FAIL", err / mx, ref.size());
  if (!ok) ++g_fail;
}
void expect(const std::string& name, bool ok) {
  std::printf("%-44s %s\n", name.c_str(), ok ? "ok" : "FAIL");
  if (!ok) ++g_fail;
}

// numeric gradient of scalar f(x) by central differences (fp32 device ops, fp64 accumulate)
std::vector<double> numgrad(const std::function<double(const std::vector<double>&)>& f, std::vector<double> x,
                            double h = 1e-2) {
  std::vector<double> g(x.size());
  for (size_t i = 0; i < x.size(); ++i) {
    const double x0 = x[i];
    x[i] = x0 + h;
    const double fp = f(x);
    x[i] = x0 - h;
    const double fm = f(x);
    x[i] = x0;
    g[i] = (fp - fm) / (2 * h);
  }
  return g;
}
// tape gradient of sum(f(x) * c) with respect to x vs central differences of the same device ops
void gradcheck(const std::string& name, const std::vector<double>& x0, Shape shape,
               const std::function<Tensor(const Tensor&)>& f, double tol = 3e-3) {
  Tensor tx = dev(x0, shape);
  tx.requires_grad_(true);
  Tensor y = f(tx);
  Tensor tc = dev(rnd((size_t)y.numel()), y.shape());
  sum(mul(y, tc)).backward();
  auto fn = [&](const std::vector<double>& xv) {
    NoGradGuard ng;
    return host(sum(mul(f(dev(xv, shape)), tc)))[0];
  };
  check(name, host(tx.grad()), numgrad(fn, x0), tol);
}
}  // namespace

int main() {
  HIP_OK(hipSetDevice(0));
  hipStream_t s;
  HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  set_current_stream(s);

  // ---------------------------------------------------------------- elementwise + broadcast
  {
    auto a = rnd(4 * 1 * 8), b = rnd(3 * 8);
    Tensor ta = dev(a, {4, 1, 8}), tb = dev(b, {3, 8});
    std::vector<double> radd(4 * 3 * 8), rmul(4 * 3 * 8), rdiv(4 * 3 * 8);
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 8; ++k) {
          const double x = a[i * 8 + k], y = b[j * 8 + k];
          radd[(i * 3 + j) * 8 + k] = x + 0.5 * y;
          rmul[(i * 3 + j) * 8 + k] = x * y;
          rdiv[(i * 3 + j) * 8 + k] = x / (y + 2.0);
        }
    check("add broadcast [4,1,8]+[3,8]", host(add(ta, tb, 0.5f)), radd, 1e-6);
    check("mul broadcast", host(mul(ta, tb)), rmul, 1e-6);
    check("div broadcast", host(div(ta, add_scalar(tb, 2.f))), rdiv, 1e-6);
    Tensor tbf = dev(a, {4, 1, 8}, DType::BF16);
    check("bf16 storage add", host(add(tbf, tb)), [&] {
      std::vector<double> r(4 * 3 * 8);
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 3; ++j)
          for (int k = 0; k < 8; ++k) r[(i * 3 + j) * 8 + k] = bf16_to_f32(f32_to_bf16((float)a[i * 8 + k])) + b[j * 8 + k];
      return r;
    }(), 1e-2);
  }
  // ---------------------------------------------------------------- unary
  {
    auto x = rnd(1000, -3, 3);
    Tensor t = dev(x, {10, 100});
    auto map = [&](double (*f)(double)) {
      std::vector<double> r(x.size());
      for (size_t i = 0; i < x.size(); ++i) r[i] = f(x[i]);
      return r;
    };
    check("relu", host(relu(t)), map([](double v) { return v > 0 ? v : 0.0; }), 1e-6);
    check("gelu(tanh)", host(gelu(t)), map([](double v) {
            return 0.5 * v * (1 + std::tanh(0.7978845608028654 * (v + 0.044715 * v * v * v)));
          }), 1e-4);
    check("silu", host(silu(t)), map([](double v) { return v / (1 + std::exp(-v)); }), 1e-4);
    check("sigmoid", host(sigmoid(t)), map([](double v) { return 1 / (1 + std::exp(-v)); }), 1e-4);
    check("tanh", host(mft::eng::tanh(t)), map([](double v) { return std::tanh(v); }), 1e-5);
    check("exp", host(mft::eng::exp(t)), map([](double v) { return std::exp(v); }), 1e-4);
    check("abs", host(mft::eng::abs(t)), map([](double v) { return std::fabs(v); }), 1e-6);
    check("clamp", host(clamp(t, -1.f, 0.5f)), map([](double v) { return std::min(std::max(v, -1.0), 0.5); }), 1e-6);
    check("pow 3", host(mft::eng::pow(t, 3.f)), map([](double v) { return v * v * v; }), 1e-4);
  }
  // ---------------------------------------------------------------- softmax / reductions
  {
    const int R = 37, N = 301;
    auto x = rnd(R * N, -4, 4);
    Tensor t = dev(x, {R, N});
    std::vector<double> sm(R * N), lsm(R * N), rs(R), cs(N, 0.0);
    double tot = 0;
    for (int r = 0; r < R; ++r) {
      double m = -1e30, z = 0;
      for (int j = 0; j < N; ++j) m = std::max(m, x[r * N + j]);
      for (int j = 0; j < N; ++j) z += std::exp(x[r * N + j] - m);
      rs[r] = 0;
      for (int j = 0; j < N; ++j) {
        sm[r * N + j] = std::exp(x[r * N + j] - m) / z;
        lsm[r * N + j] = x[r * N + j] - m - std::log(z);
        rs[r] += x[r * N + j];
        cs[j] += x[r * N + j];
        tot += x[r * N + j];
      }
    }
    check("softmax rows", host(softmax(t)), sm, 1e-5);
    check("log_softmax rows", host(log_softmax(t)), lsm, 1e-5);
    check("sum(dim=1)", host(sum(t, 1)), rs, 1e-5);
    check("sum(dim=0)", host(sum(t, 0)), cs, 1e-5);
    check("sum(all)", host(sum(t)), {tot}, 1e-5);
    auto big = rnd(300000);
    double bt = 0;
    for (double v : big) bt += v;
    check("sum(all) two-stage 300k", host(sum(dev(big, {300000}))), {bt}, 1e-4);
  }
  // ---------------------------------------------------------------- matmul / linear
  {
    const int B = 3, M = 17, K = 40, N = 24;
    auto a = rnd(B * M * K), b = rnd(K * N), b3 = rnd(B * K * N);
    std::vector<double> r(B * M * N, 0.0), r3(B * M * N, 0.0);
    for (int i = 0; i < B; ++i)
      for (int m = 0; m < M; ++m)
        for (int n = 0; n < N; ++n)
          for (int k = 0; k < K; ++k) {
            r[(i * M + m) * N + n] += a[(i * M + m) * K + k] * b[k * N + n];
            r3[(i * M + m) * N + n] += a[(i * M + m) * K + k] * b3[(i * K + k) * N + n];
          }
    check("matmul fp32 [3,17,40]x[40,24]", host(matmul(dev(a, {B, M, K}), dev(b, {K, N}))), r, 1e-5);
    check("matmul fp32 batched", host(matmul(dev(a, {B, M, K}), dev(b3, {B, K, N}))), r3, 1e-5);
    {  // several 64 x 64 tiles and 19 K stages of the fp32-MFMA generic GEMM, ragged on every side
      const int M2 = 130, K2 = 300, N2 = 77;
      auto a2 = rnd(M2 * K2), b2 = rnd(K2 * N2);
      std::vector<double> r2(M2 * N2, 0.0);
      for (int m = 0; m < M2; ++m)
        for (int n = 0; n < N2; ++n)
          for (int k = 0; k < K2; ++k) r2[m * N2 + n] += a2[m * K2 + k] * b2[k * N2 + n];
      check("matmul fp32 [130,300]x[300,77] (f32 MFMA)", host(matmul(dev(a2, {M2, K2}), dev(b2, {K2, N2}))), r2, 1e-5);
    }
    // bf16 linear on the GEMM front (hipBLASLt / gemm8): x [256, 128] W [192, 128]
    const int LM = 256, LK = 128, LN = 192;
    auto x = rnd(LM * LK), w = rnd(LN * LK, -0.1, 0.1), bias = rnd(LN, -0.5, 0.5);
    Tensor tx = dev(x, {LM, LK}, DType::BF16), tw = dev(w, {LN, LK}, DType::BF16), tb = dev(bias, {LN}, DType::BF16);
    auto xb = host(tx), wb = host(tw), bb = host(tb);
    std::vector<double> y(LM * LN);
    for (int m = 0; m < LM; ++m)
      for (int n = 0; n < LN; ++n) {
        double acc = bb[n];
        for (int k = 0; k < LK; ++k) acc += xb[m * LK + k] * wb[n * LK + k];
        y[m * LN + n] = acc;
      }
    check("linear bf16 (GEMM front)", host(linear(tx, tw, tb)), y, 1e-2);
    Tensor y8 = empty({LM, LN}, DType::BF16);
    Gemm8Extra ex;
    ex.bias = &tb;
    gemm8_call(tx, tw, false, 1 /* GEMM_EPI_BIAS */, y8, ex);
    check("gemm8 NT + bias epilogue", host(y8), y, 1e-2);
  }
  // ---------------------------------------------------------------- autograd
  {
    // d/dx sum(softmax(x * w) * c): analytic (tape) vs numeric
    const int R = 3, N = 7;
    auto x = rnd(R * N), w = rnd(N), c = rnd(R * N);
    Tensor tw = dev(w, {N}), tc = dev(c, {R, N});
    auto f = [&](const std::vector<double>& xv) {
      NoGradGuard ng;
      return host(sum(mul(softmax(mul(dev(xv, {R, N}), tw)), tc)))[0];
    };
    Tensor tx = dev(x, {R, N});
    tx.requires_grad_(true);
    Tensor loss = sum(mul(softmax(mul(tx, tw)), tc));
    loss.backward();
    check("autograd softmax*mul chain vs numeric", host(tx.grad()), numgrad(f, x), 2e-3);
    // accumulation: a second backward adds (reference overwrote, autograd_engine.cpp:243)
    auto g1 = host(tx.grad());
    Tensor loss2 = sum(mul(softmax(mul(tx, tw)), tc));
    loss2.backward();
    auto g2 = host(tx.grad());
    std::vector<double> twice(g1.size());
    for (size_t i = 0; i < g1.size(); ++i) twice[i] = 2 * g1[i];
    check("grad accumulates across backward calls", g2, twice, 1e-5);
    // hooks fire once per backward when the leaf's grad is final (used twice in the graph)
    Tensor p = dev(rnd(5), {5});
    p.requires_grad_(true);
    int fired = 0;
    add_ready_hook(p, [&](TensorImpl*) { ++fired; });
    Tensor l3 = add(sum(mul(p, p)), sum(exp(p)));
    l3.backward();
    expect("grad-ready hook fires once per backward", fired == 1);
    // no-grad mode records nothing
    {
      NoGradGuard ng;
      Tensor q = mul(p, p);
      expect("NoGradGuard: no graph recorded", !q.requires_grad());
    }
    // view backward: slice + transpose + reshape
    auto xv = rnd(4 * 6);
    Tensor tv = dev(xv, {4, 6});
    tv.requires_grad_(true);
    Tensor l4 = sum(square(tv.slice(1, 1, 4).t().reshape({-1})));
    l4.backward();
    std::vector<double> gv(24, 0.0);
    for (int i = 0; i < 4; ++i)
      for (int j = 1; j < 4; ++j) gv[i * 6 + j] = 2 * xv[i * 6 + j];
    check("view/slice/transpose backward", host(tv.grad()), gv, 1e-5);
    // transposed 2-D views copied into row-major tensors (the LDS-tiled transpose path of k::copy): a
    // column slice of a wider matrix, ragged 64-tiles, fp32 and bf16
    for (DType dt : {DType::F32, DType::BF16}) {
      const int Rr = 131, Cc = 70, ld = 77;
      auto xs = rnd((size_t)Rr * ld);
      Tensor src = dev(xs, {Rr, ld}, dt);
      Tensor tr = src.slice(1, 0, Cc).t().contiguous();  // [Cc, Rr]
      std::vector<double> want((size_t)Cc * Rr);
      const std::vector<double> hs = host(src);
      for (int i = 0; i < Cc; ++i)
        for (int j = 0; j < Rr; ++j) want[(size_t)i * Rr + j] = hs[(size_t)j * ld + i];
      check(dt == DType::F32 ? "transposed copy fp32" : "transposed copy bf16", host(tr), want, 0.0);
    }
    // cross entropy with ignore_index vs host
    const int Nr = 9, C = 13;
    auto lg = rnd(Nr * C, -2, 2);
    std::vector<int64_t> tg = {0, 3, -100, 12, 5, 5, -100, 1, 7};
    Tensor tl = dev(lg, {Nr, C});
    tl.requires_grad_(true);
    Tensor tt = from_vector(tg, {Nr}, DType::I64);
    Tensor ce = cross_entropy(tl, tt);
    ce.backward();
    double ref = 0;
    int valid = 0;
    std::vector<double> gref(Nr * C, 0.0);
    for (int r = 0; r < Nr; ++r) {
      if (tg[r] < 0) continue;
      ++valid;
    }
    for (int r = 0; r < Nr; ++r) {
      if (tg[r] < 0) continue;
      double m = -1e30, z = 0;
      for (int j = 0; j < C; ++j) m = std::max(m, lg[r * C + j]);
      for (int j = 0; j < C; ++j) z += std::exp(lg[r * C + j] - m);
      ref += -(lg[r * C + tg[r]] - m - std::log(z));
      for (int j = 0; j < C; ++j) gref[r * C + j] = (std::exp(lg[r * C + j] - m) / z - (j == tg[r])) / valid;
    }
    check("cross_entropy (ignore -100) loss", host(ce), {ref / valid}, 1e-5);
    check("cross_entropy backward", host(tl.grad()), gref, 1e-4);
    // linear backward (fp32 path) vs host
    auto lx = rnd(6 * 5), lw = rnd(4 * 5), lb = rnd(4);
    Tensor x2 = dev(lx, {6, 5}), w2 = dev(lw, {4, 5}), b2 = dev(lb, {4});
    x2.requires_grad_(true);
    w2.requires_grad_(true);
    b2.requires_grad_(true);
    sum(linear(x2, w2, b2)).backward();
    std::vector<double> gx(30, 0.0), gw(20, 0.0), gb(4, 6.0);
    for (int m = 0; m < 6; ++m)
      for (int n = 0; n < 4; ++n)
        for (int k = 0; k < 5; ++k) {
          gx[m * 5 + k] += lw[n * 5 + k];
          gw[n * 5 + k] += lx[m * 5 + k];
        }
    check("linear backward dx", host(x2.grad()), gx, 1e-5);
    check("linear backward dW", host(w2.grad()), gw, 1e-5);
    check("linear backward db", host(b2.grad()), gb, 1e-5);
  }
  // ---------------------------------------------------------------- composite catalog layers
  {
    const int R = 5, C = 16;
    auto x = rnd(R * C, -2, 2), w = rnd(C), b = rnd(C);
    Tensor tw = dev(w, {C}), tb = dev(b, {C});
    std::vector<double> ln(R * C), rms(R * C);
    for (int r = 0; r < R; ++r) {
      double mu = 0, ss = 0, ms = 0;
      for (int j = 0; j < C; ++j) mu += x[r * C + j] / C;
      for (int j = 0; j < C; ++j) ss += (x[r * C + j] - mu) * (x[r * C + j] - mu) / C;
      for (int j = 0; j < C; ++j) ms += x[r * C + j] * x[r * C + j] / C;
      for (int j = 0; j < C; ++j) {
        ln[r * C + j] = (x[r * C + j] - mu) / std::sqrt(ss + 1e-5) * w[j] + b[j];
        rms[r * C + j] = x[r * C + j] / std::sqrt(ms + 1e-6) * (1.0 + w[j]);
      }
    }
    check("layer_norm (composite)", host(layer_norm(dev(x, {R, C}), tw, tb)), ln, 1e-5);
    check("rms_norm(1 + w) (composite)", host(rms_norm(dev(x, {R, C}), tw)), rms, 1e-5);
    gradcheck("layer_norm backward vs numeric", x, {R, C}, [&](const Tensor& t) { return layer_norm(t, tw, tb); });
    gradcheck("rms_norm backward vs numeric", x, {R, C}, [&](const Tensor& t) { return rms_norm(t, tw); });
    const int N = 8, F = 6;
    auto bx = rnd(N * F, -2, 2), gm = rnd(F), bt = rnd(F);
    Tensor tg = dev(gm, {F}), tbt = dev(bt, {F});
    std::vector<double> bn(N * F);
    for (int j = 0; j < F; ++j) {
      double mu = 0, var = 0;
      for (int i = 0; i < N; ++i) mu += bx[i * F + j] / N;
      for (int i = 0; i < N; ++i) var += (bx[i * F + j] - mu) * (bx[i * F + j] - mu) / N;
      for (int i = 0; i < N; ++i) bn[i * F + j] = (bx[i * F + j] - mu) / std::sqrt(var + 1e-5) * gm[j] + bt[j];
    }
    check("batch_norm (training stats)", host(batch_norm(dev(bx, {N, F}), tg, tbt)), bn, 1e-5);
    gradcheck("batch_norm backward vs numeric", bx, {N, F}, [&](const Tensor& t) { return batch_norm(t, tg, tbt); });
    auto gt = rnd(64, -3, 3), up = rnd(64);
    Tensor tu = dev(up, {4, 16});
    std::vector<double> sw(64), gg(64);
    for (int i = 0; i < 64; ++i) {
      const double v = gt[i];
      sw[i] = v / (1 + std::exp(-v)) * up[i];
      gg[i] = 0.5 * v * (1 + std::tanh(0.7978845608028654 * (v + 0.044715 * v * v * v))) * up[i];
    }
    check("swiglu", host(swiglu(dev(gt, {4, 16}), tu)), sw, 1e-4);
    check("geglu", host(geglu(dev(gt, {4, 16}), tu)), gg, 1e-4);
    gradcheck("swiglu backward (gate) vs numeric", gt, {4, 16}, [&](const Tensor& t) { return swiglu(t, tu); });
    // masked softmax: causal + sliding window 3, Sq = 5 queries over Sk = 7 keys (2 cached)
    const int Sq = 5, Sk = 7, Wn = 3;
    auto sc = rnd(Sq * Sk, -2, 2);
    std::vector<double> msm(Sq * Sk, 0.0);
    for (int i = 0; i < Sq; ++i) {
      double m = -1e30, z = 0;
      auto ok = [&](int j) { return j <= i + (Sk - Sq) && i + (Sk - Sq) - j < Wn; };
      for (int j = 0; j < Sk; ++j)
        if (ok(j)) m = std::max(m, sc[i * Sk + j]);
      for (int j = 0; j < Sk; ++j)
        if (ok(j)) z += std::exp(sc[i * Sk + j] - m);
      for (int j = 0; j < Sk; ++j) msm[i * Sk + j] = ok(j) ? std::exp(sc[i * Sk + j] - m) / z : 0.0;
    }
    check("causal_mask(window) + apply_mask + softmax",
          host(softmax(apply_mask(dev(sc, {Sq, Sk}), causal_mask(Sq, Sk, Wn)))), msm, 1e-5);
    // GQA repeat: [2, 3, 2, 4] -> [2, 3, 6, 4]
    auto kv = rnd(2 * 3 * 2 * 4);
    std::vector<double> rk(2 * 3 * 6 * 4);
    for (int b = 0; b < 2; ++b)
      for (int t = 0; t < 3; ++t)
        for (int hq = 0; hq < 6; ++hq)
          for (int d = 0; d < 4; ++d) rk[((b * 3 + t) * 6 + hq) * 4 + d] = kv[((b * 3 + t) * 2 + hq / 3) * 4 + d];
    check("repeat_kv (GQA 3:1)", host(repeat_kv(dev(kv, {2, 3, 2, 4}), 3)), rk, 1e-6);
    gradcheck("repeat_kv backward vs numeric", kv, {2, 3, 2, 4}, [&](const Tensor& t) { return repeat_kv(t, 3); });
    // RoPE on [B = 2, S = 3, H = 2, D = 8], both pair layouts
    const int RB = 2, RS = 3, RH = 2, RD = 8, hh = RD / 2;
    auto rx = rnd(RB * RS * RH * RD);
    std::vector<double> cs(RS * hh), sn(RS * hh);
    for (int t = 0; t < RS; ++t)
      for (int i = 0; i < hh; ++i) {
        const double ang = t * std::pow(10000.0, -2.0 * i / RD);
        cs[t * hh + i] = std::cos(ang);
        sn[t * hh + i] = std::sin(ang);
      }
    Tensor tcs = dev(cs, {RS, hh}), tsn = dev(sn, {RS, hh});
    std::vector<double> rh(rx.size()), ri(rx.size());
    for (int b = 0; b < RB; ++b)
      for (int t = 0; t < RS; ++t)
        for (int hd = 0; hd < RH; ++hd) {
          const int o = ((b * RS + t) * RH + hd) * RD;
          for (int i = 0; i < hh; ++i) {
            const double c = cs[t * hh + i], sv = sn[t * hh + i];
            rh[o + i] = rx[o + i] * c - rx[o + i + hh] * sv;
            rh[o + i + hh] = rx[o + i + hh] * c + rx[o + i] * sv;
            ri[o + 2 * i] = rx[o + 2 * i] * c - rx[o + 2 * i + 1] * sv;
            ri[o + 2 * i + 1] = rx[o + 2 * i + 1] * c + rx[o + 2 * i] * sv;
          }
        }
    check("apply_rope rotate-half", host(apply_rope(dev(rx, {RB, RS, RH, RD}), tcs, tsn, false)), rh, 1e-5);
    check("apply_rope interleaved", host(apply_rope(dev(rx, {RB, RS, RH, RD}), tcs, tsn, true)), ri, 1e-5);
    gradcheck("apply_rope backward vs numeric", rx, {RB, RS, RH, RD},
              [&](const Tensor& t) { return apply_rope(t, tcs, tsn, true); });
  }
  // ---------------------------------------------------------------- allocator
  {
    auto& al = CachingAllocator::get(Device::current_hip_device());
    synchronize();
    const auto s0 = al.stats();
    { Tensor big = empty({64 << 20}, DType::F32); }
    const auto s1 = al.stats();
    { Tensor again = empty({64 << 20}, DType::F32); }
    const auto s2 = al.stats();
    expect("allocator: freed block is reused (no new hipMalloc)", s2.n_hip_malloc == s1.n_hip_malloc);
    expect("allocator: allocated bytes return to baseline", s2.allocated == s0.allocated);
    expect("allocator: peak tracks the 256 MB tensor", s2.peak_allocated >= s0.allocated + (256u << 20));
    std::vector<Tensor> smalls;
    for (int i = 0; i < 100; ++i) smalls.push_back(empty({100 + i}, DType::F32));
    smalls.clear();
    expect("allocator: small blocks coalesce back", al.stats().allocated == s0.allocated);
  }
  synchronize();
  {  // fused LoRA input projection in the norm (nn.h add_norm with lora_a): the appended columns hold
     // u = y A^T of the stored bf16 row, the rest of the tail is zero; LayerNorm and RMSNorm(1 + w)
    NoGradGuard ng;
    for (int rms = 0; rms < 2; ++rms)
      for (int R : {8, 24}) {
        const int M = 37, N = 96, OC = 128;
        Tensor x = dev(rnd((size_t)M * N), {M, N}, DType::BF16);
        Param w, b;
        w.c = w.leaf = dev(rnd(N, 0.5, 1.5), {N});
        b.c = b.leaf = dev(rnd(N), {N});
        Tensor A = dev(rnd((size_t)R * N, -0.2, 0.2), {R, N}, DType::BF16);
        Tensor y = add_norm(x, Tensor(), w, rms ? nullptr : &b, 1e-5f, rms == 1, rms ? 1.f : 0.f, OC, A).second;
        const std::vector<double> yv = host(y), av = host(A);
        std::vector<double> got, ref;
        for (int m = 0; m < M; ++m)
          for (int c = N; c < OC; ++c) {
            double u = 0.0;
            if (c < N + R)
              for (int k = 0; k < N; ++k) u += yv[(size_t)m * OC + k] * av[(size_t)(c - N) * N + k];
            ref.push_back(u);
            got.push_back(yv[(size_t)m * OC + c]);
          }
        check(std::string(rms ? "rms" : "layer") + "_norm + fused LoRA u (R=" + std::to_string(R) + ")", got, ref, 1e-2);
      }
  }
  std::printf(g_fail ? "FAILED: %d check(s)\n" : "ALL OK\n", g_fail);
  return g_fail ? 1 : 0;
}
