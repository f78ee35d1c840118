// libmft engine: GEMM routing (see gemm.h).  Every product of the engine runs on a hand-written kernel:
// gemm4 (kernels/gemm4.hip, the 4-wave hand-scheduled persistent NT GEMM) for every K-contiguous
// product and fused epilogue it carries, gemm4_tn (the same 4-wave design with token-major K-tiles) for
// the split-K weight gradients, gemm8 (kernels/gemm8.hip) for the other token-major layouts (NN data
// gradients of trainable weights without a transposed copy, the LM-head CE dgrad, the LoRA epilogue),
// and the fp32-MFMA generic fallback (kernels/gemm_simt.hip) for operands neither takes
// (fp32, K % 64 != 0, unaligned strides).  No vendor GEMM library is linked.
#include "engine/gemm.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <unordered_map>

#include "engine/allocator.h"
#include "engine/autograd.h"
#include "kernels.h"

namespace mft {
namespace eng {

namespace {

bool g_det = std::getenv("MFT_DETERMINISTIC") && std::getenv("MFT_DETERMINISTIC")[0] == '1';

// MFT_GEMM_MAP=1: one line per GEMM shape and kernel the first time it is routed (two ranks' maps must
// be identical)
bool gemm_map() {
  static const bool v = std::getenv("MFT_GEMM_MAP") && std::getenv("MFT_GEMM_MAP")[0] == '1';
  return v;
}
void map_line(const char* op, long M, long N, long K, const char* backend) {
  if (!gemm_map()) return;
  static std::mutex mu;
  static std::unordered_map<std::string, bool> seen;
  char b[160];
  snprintf(b, sizeof(b), "[gemm-map] %s M=%ld N=%ld K=%ld -> %s", op, M, N, K, backend);
  std::lock_guard<std::mutex> g(mu);
  if (seen.emplace(b, true).second) std::fprintf(stderr, "%s\n", b);
}

const char* epi_name(int epi) {
  switch (epi) {
    case ::mft::GEMM_EPI_NONE: return "epi none";
    case ::mft::GEMM_EPI_BIAS: return "epi bias";
    case ::mft::GEMM_EPI_BIAS_GELU_D: return "epi bias+gelu (+gelu')";
    case ::mft::GEMM_EPI_MUL_AUX: return "epi x aux";
    case ::mft::GEMM_EPI_DGELU: return "epi x gelu'(aux)";
    case ::mft::GEMM_EPI_LORA: return "epi lora";
    case ::mft::GEMM_EPI_BIAS_ADD: return "epi bias+resid";
    default: return "epi other";
  }
}

int cur_dev() {
  int d = 0;
  HIP_OK(hipGetDevice(&d));
  return d;
}

bool rowmajor2(const Tensor& t) { return t.dim() == 2 && t.stride(1) == 1; }

::mft::GemmArgs args_for(const Tensor& a, const Tensor& b, Tensor& c) {
  ::mft::GemmArgs g{};
  g.A = (const ::mft::bf16_t*)a.data_ptr();
  g.lda = a.stride(0);
  g.B = (const ::mft::bf16_t*)b.data_ptr();
  g.ldb = b.stride(0);
  g.C = c.data_ptr();
  g.ldc = c.stride(0);
  g.alpha = 1.f;
  return g;
}

bool f32_or_bf16(const Tensor& t) { return t.dtype() == DType::F32 || t.dtype() == DType::BF16; }

// D = alpha op(A) op(B) (+ bias) + beta Cin on the SIMT fallback (row-major 2-D; ta: a stored [K, M], tb:
// b stored [N, K])
void simt(const Tensor& a, bool ta, const Tensor& b, bool tb, Tensor& d, float alpha, const Tensor& bias,
          const Tensor& cin, float beta, const char* op) {
  MFT_CHECK(f32_or_bf16(a) && f32_or_bf16(b) && f32_or_bf16(d) && (!cin.defined() || f32_or_bf16(cin)) &&
                (!bias.defined() || bias.dtype() == DType::BF16),
            "gemm (SIMT fallback): fp32 / bf16 operands, bf16 bias");
  ::mft::SimtGemmArgs s{};
  s.A = a.data_ptr(), s.lda = a.stride(0), s.a_f32 = a.dtype() == DType::F32, s.ta = ta;
  s.B = b.data_ptr(), s.ldb = b.stride(0), s.b_f32 = b.dtype() == DType::F32, s.tb = tb;
  s.D = d.data_ptr(), s.ldd = d.stride(0), s.d_f32 = d.dtype() == DType::F32;
  if (cin.defined()) s.Cin = cin.data_ptr(), s.ldcin = cin.stride(0), s.cin_f32 = cin.dtype() == DType::F32;
  s.bias = bias.defined() ? (const ::mft::bf16_t*)bias.data_ptr() : nullptr;
  s.M = (int)d.size(0), s.N = (int)d.size(1), s.K = (int)(ta ? a.size(0) : a.size(1));
  s.alpha = alpha, s.beta = beta;
  map_line(op, s.M, s.N, s.K, "simt");
  ::mft::gemm_simt(s, current_stream());
}

}  // namespace

// MFT_GEMM4=0 keeps every GEMM off gemm4 (A/B against gemm8)
bool gemm4_on() {
  static const bool v = !(std::getenv("MFT_GEMM4") && std::getenv("MFT_GEMM4")[0] == '0');
  return v;
}

bool gemm4_route(int epi, bool b_kn, long M, long N, long K, long lda, long ldb) {
  if (!gemm4_on() || b_kn || !::mft::gemm4_supported((int)M, (int)N, (int)K, false, false)) return false;
  if (lda % 8 || ldb % 8) return false;
  // every epilogue gemm4 carries is faster there than on gemm8 (profiles/r5_gemm4_nt_stores.txt)
  return epi == ::mft::GEMM_EPI_MUL_AUX || epi == ::mft::GEMM_EPI_DGELU || epi == ::mft::GEMM_EPI_BIAS_GELU_D ||
         epi == ::mft::GEMM_EPI_NONE || epi == ::mft::GEMM_EPI_BIAS || epi == ::mft::GEMM_EPI_BIAS_ADD;
}

bool nt_gemm4() { return gemm4_on(); }

// MFT_GEMM_S=0 keeps short-token products on gemm4 / gemm8 (A/B)
bool short_tokens(long M, long N, long K, int epi) {
  static const bool off = std::getenv("MFT_GEMM_S") && std::getenv("MFT_GEMM_S")[0] == '0';
  return !off && gemm4_on() && ::mft::gemm_s_preferred((int)M, (int)N, (int)K) &&
         ::mft::gemm_s_supported((int)M, (int)N, (int)K, epi);
}

bool gemm8_all() { return !gemm4_on(); }
bool deterministic() { return g_det; }
void set_deterministic(bool on) { g_det = on; }

void gemm8_call(const Tensor& a, const Tensor& b, bool b_kn, int epi, Tensor& c, const Gemm8Extra& ex) {
  MFT_CHECK(a.dtype() == DType::BF16 && b.dtype() == DType::BF16 && rowmajor2(a) && rowmajor2(b) && rowmajor2(c),
            "gemm8: bf16 row-major 2-D operands (", a.str(), ", ", b.str(), ", ", c.str(), ")");
  const int M = (int)a.size(0), K = (int)a.size(1);
  const int N = (int)(b_kn ? b.size(1) : b.size(0));
  MFT_CHECK((b_kn ? b.size(0) : b.size(1)) == K && c.size(0) == M && c.size(1) == N, "gemm8: shape mismatch ",
            a.str(), " x ", b.str(), " -> ", c.str());
  MFT_CHECK(::mft::gemm8_supported(M, N, K, false, b_kn), "gemm8: unsupported shape M=", M, " N=", N, " K=", K);
  MFT_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && c.stride(0) % 8 == 0, "gemm8: 16-B aligned rows");
  ::mft::GemmArgs g = args_for(a, b, c);
  g.M = M;
  g.N = N;
  g.K = K;
  g.alpha = ex.alpha;
  if (ex.bias) {
    MFT_CHECK(ex.bias->dtype() == DType::BF16 && ex.bias->numel() == N, "gemm8: bias bf16 [N]");
    g.bias = (const ::mft::bf16_t*)ex.bias->data_ptr();
  }
  if (ex.aux) {
    MFT_CHECK(rowmajor2(*ex.aux) && ex.aux->size(0) == M && ex.aux->size(1) == N, "gemm8: aux [M, N]");
    g.aux = (::mft::bf16_t*)ex.aux->data_ptr();
    g.ldaux = ex.aux->stride(0);
  }
  if (ex.lora_u) {
    g.lora_u = (const ::mft::bf16_t*)ex.lora_u->data_ptr();
    g.ld_lu = ex.lora_u->stride(0);
    g.lora_w = (const ::mft::bf16_t*)ex.lora_w->data_ptr();
    g.ld_lw = ex.lora_w->stride(0);
    g.lora_r = (int)ex.lora_u->size(1);
  }
  // short token counts: the 64 x 64 split-K-over-waves kernel (kernels/gemm_s.hip)
  if (!b_kn && short_tokens(M, N, K, epi) && g.ldc % 8 == 0) {
    map_line(epi_name(epi), M, N, K, "gemm_s");
    ::mft::gemm_s(g, epi, current_stream());
    return;
  }
  // gemm4 (the 4-wave hand-scheduled persistent kernel, kernels/gemm4.hip) where it beats gemm8:
  // the MUL_AUX / dGELU data gradient (+11 % at the GPT-2 MLP shape, profiles/r5_gemm4_epilogues.txt)
  if (gemm4_route(epi, b_kn, M, N, K, g.lda, g.ldb)) {
    map_line(epi_name(epi), M, N, K, "gemm4");
    ::mft::gemm4x(g, epi, false, false, current_stream());
    return;
  }
  map_line(epi_name(epi), M, N, K, b_kn ? "gemm8 NN" : "gemm8");
  ::mft::gemm8x(g, epi, false, b_kn, current_stream());
}


bool lora_seg2_ok(long M, long N, long K) {
  static const bool off = std::getenv("MFT_LORA_SEG2") && std::getenv("MFT_LORA_SEG2")[0] == '0';  // A/B: gemm8 LORA
  return !off && gemm4_on() &&
         (::mft::gemm4_supported((int)M, (int)N, (int)K, false, false) || short_tokens(M, N, K, ::mft::GEMM_EPI_NONE));
}

void gemm_nt_seg2(const Tensor& a, const Tensor& b, const Tensor& a2, const Tensor& b2, Tensor& c) {
  MFT_CHECK(rowmajor2(a) && rowmajor2(b) && rowmajor2(a2) && rowmajor2(b2) && rowmajor2(c) && a.dtype() == DType::BF16 &&
                b.dtype() == DType::BF16 && a2.dtype() == DType::BF16 && b2.dtype() == DType::BF16,
            "gemm_nt_seg2: bf16 row-major operands");
  const long M = a.size(0), K = a.size(1), N = b.size(0), K2 = a2.size(1);
  MFT_CHECK(b.size(1) == K && a2.size(0) == M && b2.size(0) == N && b2.size(1) == K2 && c.size(0) == M && c.size(1) == N &&
                K2 % 64 == 0 && a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && a2.stride(0) % 8 == 0 &&
                b2.stride(0) % 8 == 0 && c.stride(0) % 8 == 0 && lora_seg2_ok(M, N, K),
            "gemm_nt_seg2: shapes / strides ", a.str(), " ", b.str(), " ", a2.str(), " ", b2.str(), " -> ", c.str());
  ::mft::GemmArgs g = args_for(a, b, c);
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.A2 = (const ::mft::bf16_t*)a2.data_ptr();
  g.lda2 = a2.stride(0);
  g.B2 = (const ::mft::bf16_t*)b2.data_ptr();
  g.ldb2 = b2.stride(0);
  g.K2 = (int)K2;
  if (short_tokens(M, N, K, ::mft::GEMM_EPI_NONE)) {
    map_line("nt + second K segment (LoRA dgrad)", M, N, K, "gemm_s");
    ::mft::gemm_s(g, ::mft::GEMM_EPI_NONE, current_stream());
    return;
  }
  map_line("nt + second K segment (LoRA dgrad)", M, N, K, "gemm4");
  ::mft::gemm4x(g, ::mft::GEMM_EPI_NONE, false, false, current_stream());
}

bool geglu_fusable(long M, long I, long K, long Kd) {
  static const bool off = std::getenv("MFT_GEGLU_FUSE") && std::getenv("MFT_GEGLU_FUSE")[0] == '0';
  return !off && gemm4_on() && I % 128 == 0 && K % 64 == 0 && Kd % 64 == 0 &&
         ::mft::gemm4_supported((int)M, (int)(2 * I), (int)K, false, false) &&
         ::mft::gemm4_supported((int)M, (int)I, (int)Kd, false, false) && !short_tokens(M, 2 * I, K, ::mft::GEMM_EPI_NONE) &&
         !short_tokens(M, I, Kd, ::mft::GEMM_EPI_NONE);
}

void gemm_geglu_fwd(const Tensor& x2, const Tensor& w, Tensor& gu, Tensor& h) {
  const long M = x2.size(0), K = x2.size(1), I2 = w.size(0), I = I2 / 2;
  MFT_CHECK(rowmajor2(x2) && rowmajor2(w) && rowmajor2(gu) && rowmajor2(h) && x2.dtype() == DType::BF16 &&
                w.dtype() == DType::BF16 && gu.dtype() == DType::BF16 && h.dtype() == DType::BF16 && w.size(1) == K &&
                gu.size(0) == M && gu.size(1) == I2 && h.size(0) == M && h.size(1) >= I && geglu_fusable(M, I, K, K) &&
                x2.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && gu.stride(0) % 8 == 0 && h.stride(0) % 8 == 0,
            "gemm_geglu_fwd: shapes / strides ", x2.str(), " ", w.str(), " -> ", gu.str(), " + ", h.str());
  ::mft::GemmArgs g = args_for(x2, w, gu);
  g.M = (int)M, g.N = (int)I2, g.K = (int)K;
  g.aux = (::mft::bf16_t*)h.data_ptr();
  g.ldaux = h.stride(0);
  g.geglu_I = (int)I;
  map_line("gate|up + GeGLU (h) epilogue", M, I2, K, "gemm4");
  ::mft::gemm4x(g, ::mft::GEMM_EPI_GEGLU_FWD, false, false, current_stream());
}

void gemm_geglu_bwd(const Tensor& dy2, const Tensor& wt, const Tensor& gu, Tensor& dgu, const Tensor& a2, const Tensor& b2) {
  const long M = dy2.size(0), K = dy2.size(1), I = wt.size(0);
  MFT_CHECK(rowmajor2(dy2) && rowmajor2(wt) && rowmajor2(gu) && rowmajor2(dgu) && dy2.dtype() == DType::BF16 &&
                wt.dtype() == DType::BF16 && wt.size(1) == K && gu.size(0) == M && gu.size(1) == 2 * I &&
                dgu.size(0) == M && dgu.size(1) == 2 * I && dy2.stride(0) % 8 == 0 && wt.stride(0) % 8 == 0 &&
                gu.stride(0) % 8 == 0 && dgu.stride(0) % 8 == 0,
            "gemm_geglu_bwd: shapes / strides ", dy2.str(), " ", wt.str(), " ", gu.str(), " -> ", dgu.str());
  ::mft::GemmArgs g = args_for(dy2, wt, dgu);
  g.M = (int)M, g.N = (int)I, g.K = (int)K;
  g.aux = (::mft::bf16_t*)gu.data_ptr();
  g.ldaux = gu.stride(0);
  g.geglu_I = (int)I;
  if (a2.defined()) {
    MFT_CHECK(rowmajor2(a2) && rowmajor2(b2) && a2.size(0) == M && b2.size(0) == I && a2.size(1) == b2.size(1) &&
                  a2.size(1) % 64 == 0 && a2.stride(0) % 8 == 0 && b2.stride(0) % 8 == 0,
              "gemm_geglu_bwd: second K segment ", a2.str(), " ", b2.str());
    g.A2 = (const ::mft::bf16_t*)a2.data_ptr();
    g.lda2 = a2.stride(0);
    g.B2 = (const ::mft::bf16_t*)b2.data_ptr();
    g.ldb2 = b2.stride(0);
    g.K2 = (int)a2.size(1);
  }
  map_line(a2.defined() ? "down dgrad + LoRA segment + GeGLU backward epilogue" : "down dgrad + GeGLU backward epilogue", M,
           I, K, "gemm4");
  ::mft::gemm4x(g, ::mft::GEMM_EPI_GEGLU_BWD, false, false, current_stream());
}

void gemm_nt(const Tensor& x2, const Tensor& w, const Tensor& bias, Tensor& y, const Tensor& resid) {
  MFT_CHECK(rowmajor2(x2) && rowmajor2(w) && rowmajor2(y) && x2.dtype() == DType::BF16 && w.dtype() == DType::BF16,
            "gemm_nt: bf16 row-major");
  const long M = x2.size(0), K = x2.size(1), N = w.size(0);
  MFT_CHECK(w.size(1) == K && y.size(0) == M && y.size(1) == N, "gemm_nt: shapes ", x2.str(), " ", w.str(), " ",
            y.str());
  // resid: the residual stream [M, N] added in the epilogue (y = x W^T + b + resid) -- the residual add
  // never makes its own pass
  MFT_CHECK(!resid.defined() || (rowmajor2(resid) && resid.dtype() == DType::BF16 && resid.size(0) == M &&
                                 resid.size(1) == N && resid.stride(0) == y.stride(0) && bias.defined()),
            "gemm_nt: the fused residual must match y (bf16 [M, N], same row stride) and come with a bias");
  const int epi = resid.defined() ? ::mft::GEMM_EPI_BIAS_ADD : bias.defined() ? ::mft::GEMM_EPI_BIAS : ::mft::GEMM_EPI_NONE;
  const bool aligned = x2.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && y.stride(0) % 8 == 0;
  if (aligned && N % 8 == 0 && K % 64 == 0 && (gemm4_route(epi, false, M, N, K, x2.stride(0), w.stride(0)) ||
                                               ::mft::gemm8_supported((int)M, (int)N, (int)K, false, false))) {
    Gemm8Extra ex;  // (gemm8_call sends it to gemm4 where that runs)
    ex.bias = bias.defined() ? &bias : nullptr;
    Tensor r = resid;
    if (resid.defined()) ex.aux = &r;
    gemm8_call(x2, w, false, epi, y, ex);
    return;
  }
  simt(x2, false, w, true, y, 1.f, bias, resid, resid.defined() ? 1.f : 0.f, "nt");
}

void gemm_nn(const Tensor& dy2, const Tensor& w, Tensor& out, const Tensor& wt_in) {
  const long N = w.size(0), M = dy2.size(0), K = w.size(1);
  MFT_CHECK(rowmajor2(dy2) && rowmajor2(w) && rowmajor2(out) && dy2.size(1) == N && out.size(0) == M &&
                out.size(1) == K,
            "gemm_nn: shapes ", dy2.str(), " ", w.str(), " ", out.str());
  const bool aligned = dy2.stride(0) % 8 == 0 && out.stride(0) % 8 == 0;
  // gemm4 reads K-contiguous operands only: the data gradient dx = dy W is the NT product dy (W^T)^T with
  // the frozen weight's resident transposed copy (Param::transposed), or -- a trainable weight -- a
  // transposed copy made here (|W| bytes, ~1 % of the GEMM's own traffic at the benchmark shapes)
  const bool g4 = ::mft::gemm4_supported((int)M, (int)K, (int)N, false, false);
  const bool gs = short_tokens(M, K, N, ::mft::GEMM_EPI_NONE);
  if (gemm4_on() && aligned && (g4 || gs) && K % 8 == 0 && dy2.dtype() == DType::BF16 && w.dtype() == DType::BF16) {
    Tensor wt = wt_in;
    if (!wt.defined() || !rowmajor2(wt) || wt.stride(0) % 8) {
      NoGradGuard ng;
      wt = w.t().contiguous();
    }
    ::mft::GemmArgs g = args_for(dy2, wt, out);
    g.M = (int)M;
    g.N = (int)K;
    g.K = (int)N;
    map_line(wt_in.defined() ? "nn (resident W^T)" : "nn (W^T copy)", M, K, N, gs ? "gemm_s" : "gemm4");
    if (gs) ::mft::gemm_s(g, ::mft::GEMM_EPI_NONE, current_stream());
    else ::mft::gemm4x(g, ::mft::GEMM_EPI_NONE, false, false, current_stream());
    return;
  }
  if (aligned && w.stride(0) % 8 == 0 && N % 64 == 0 && K % 8 == 0 && dy2.dtype() == DType::BF16 &&
      w.dtype() == DType::BF16 && ::mft::gemm8_supported((int)M, (int)K, (int)N, false, true)) {
    gemm8_call(dy2, w, true, ::mft::GEMM_EPI_NONE, out);
    return;
  }
  simt(dy2, false, w, false, out, 1.f, Tensor(), Tensor(), 0.f, "nn");
}

void gemm_wgrad(Tensor& buf, const Tensor& dy2, const Tensor& x2, float alpha) {
  MFT_CHECK(buf.dtype() == DType::F32 && buf.is_contiguous(), "gemm_wgrad: fp32 contiguous grad buffer");
  const long M = dy2.size(0), N = dy2.size(1), K = x2.size(1);
  MFT_CHECK(x2.size(0) == M && buf.numel() == N * K, "gemm_wgrad: shapes");
  // the 4-wave TN kernel (gemm4_tn: AGPR accumulators, transposed LDS reads, token split into fp32 slabs);
  // MFT_WGRAD=gemm8 keeps the 8-wave kernel below (A/B)
  static const bool wg8 = getenv("MFT_WGRAD") && std::string(getenv("MFT_WGRAD")) == "gemm8";
  if (!wg8 && M % 64 == 0 && dy2.dtype() == DType::BF16 && x2.dtype() == DType::BF16 &&
      reinterpret_cast<uintptr_t>(dy2.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(x2.data_ptr()) % 16 == 0 &&
      ::mft::gemm4_tn_supported((int)N, (int)K, (int)M, dy2.stride(0), x2.stride(0))) {
    ::mft::GemmArgs g{};
    g.A = (const ::mft::bf16_t*)dy2.data_ptr();
    g.lda = dy2.stride(0);
    g.B = (const ::mft::bf16_t*)x2.data_ptr();
    g.ldb = x2.stride(0);
    g.C = buf.data_ptr();
    g.ldc = K;
    g.M = (int)N;
    g.N = (int)K;
    g.K = (int)M;
    g.alpha = alpha;
    g.ksplit = ::mft::gemm4_tn_pick_ksplit((int)N, (int)K, (int)M);
    map_line("wgrad", N, K, M, g.ksplit > 1 ? "gemm4_tn split-K" : "gemm4_tn");
    void* ws = nullptr;
    auto& al = CachingAllocator::get(cur_dev());
    if (g.ksplit > 1) {
      ws = al.allocate((size_t)g.ksplit * N * K * 4, current_stream());
      g.ws = (float*)ws;
    }
    ::mft::gemm4_tn(g, current_stream());
    if (ws) al.release(ws);
    return;
  }
  // gemm8 TN (both operands token-major, read with ds_read_b64_tr_b16) with the F32ACC epilogue straight
  // into the flat grad, split-K over the tokens when the output alone does not fill the CUs
  if (M % 64 == 0 && N % 8 == 0 && K % 8 == 0 && dy2.stride(0) % 8 == 0 && x2.stride(0) % 8 == 0 &&
      dy2.dtype() == DType::BF16 && x2.dtype() == DType::BF16 &&
      ::mft::gemm8_supported((int)N, (int)K, (int)M, true, true)) {
    ::mft::GemmArgs g{};
    g.A = (const ::mft::bf16_t*)dy2.data_ptr();
    g.lda = dy2.stride(0);
    g.B = (const ::mft::bf16_t*)x2.data_ptr();
    g.ldb = x2.stride(0);
    g.C = buf.data_ptr();
    g.ldc = K;
    g.M = (int)N;
    g.N = (int)K;
    g.K = (int)M;
    g.alpha = alpha;
    g.ksplit = ::mft::gemm8_pick_ksplit((int)N, (int)K, (int)M);
    map_line("wgrad", N, K, M, g.ksplit > 1 ? "gemm8 split-K" : "gemm8");
    void* ws = nullptr;
    auto& al = CachingAllocator::get(cur_dev());
    if (g.ksplit > 1) {
      ws = al.allocate((size_t)g.ksplit * N * K * 4, current_stream());
      g.ws = (float*)ws;
    }
    ::mft::gemm8x(g, ::mft::GEMM_EPI_F32ACC, true, true, current_stream());
    if (ws) al.release(ws);
    return;
  }
  // a token count that is not a multiple of 64 (odd batch x seq): zero-padded copies of both token-major
  // operands to the next multiple (the padding rows add 0 to every sum) -- two copies of the operands
  // instead of the SIMT kernel, orders of magnitude slower on a full fine-tune
  if (M % 64 && N % 8 == 0 && K % 8 == 0 && dy2.dtype() == DType::BF16 && x2.dtype() == DType::BF16 &&
      ::mft::gemm8_supported((int)N, (int)K, (int)((M + 63) / 64 * 64), true, true)) {
    NoGradGuard ng;
    const long Mp = (M + 63) / 64 * 64;
    Tensor dyp = zeros({Mp, N}, DType::BF16, dy2.device()), xp = zeros({Mp, K}, DType::BF16, x2.device());
    dyp.slice(0, 0, M).copy_(dy2);
    xp.slice(0, 0, M).copy_(x2);
    map_line("wgrad (tokens padded to 64)", N, K, M, "gemm4_tn / gemm8");
    gemm_wgrad(buf, dyp, xp, alpha);
    return;
  }
  // buf [N, K] += alpha dy^T x
  if (dy2.dtype() == DType::BF16 && x2.dtype() == DType::BF16) {
    static bool warned = false;
    if (!warned) {
      warned = true;
      std::fprintf(stderr, "[gemm] weight gradient M=%ld N=%ld K=%ld on the SIMT fallback (unaligned operands)\n", M, N, K);
    }
  }
  Tensor b2 = buf.view({N, K});
  simt(dy2, true, x2, false, b2, alpha, Tensor(), b2, 1.f, "wgrad");
}

void blas_gemm(const Tensor& a, bool ta, const Tensor& b, bool tb, Tensor& c, float alpha, float beta) {
  MFT_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1,
            "blas_gemm: row-major 2-D operands");
  MFT_CHECK(a.dtype() == b.dtype(), "blas_gemm: operand dtypes differ");
  const long M = ta ? a.size(1) : a.size(0), K = ta ? a.size(0) : a.size(1);
  const long N = tb ? b.size(0) : b.size(1);
  MFT_CHECK((tb ? b.size(1) : b.size(0)) == K && c.size(0) == M && c.size(1) == N, "blas_gemm: shapes");
  // bf16 in / bf16 out without accumulation: the MFMA kernels (gemm8 takes every layout)
  if (a.dtype() == DType::BF16 && c.dtype() == DType::BF16 && beta == 0.f && alpha == 1.f && K % 64 == 0 &&
      N % 8 == 0 && a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && c.stride(0) % 8 == 0 &&
      (!ta || M % 8 == 0) && ::mft::gemm8_supported((int)M, (int)N, (int)K, ta, !tb)) {
    if (!ta && tb) {  // NT: gemm4 where it runs
      Tensor cc = c;
      gemm8_call(a, b, false, ::mft::GEMM_EPI_NONE, cc);
      return;
    }
    ::mft::GemmArgs g = args_for(a, b, c);
    g.M = (int)M;
    g.N = (int)N;
    g.K = (int)K;
    map_line(ta ? (tb ? "matmul TT" : "matmul TN") : "matmul NN", M, N, K, "gemm8");
    ::mft::gemm8x(g, ::mft::GEMM_EPI_NONE, ta, !tb, current_stream());
    return;
  }
  simt(a, ta, b, tb, c, alpha, Tensor(), c, beta, "matmul");
}

}  // namespace eng
}  // namespace mft
