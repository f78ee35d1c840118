// libmft engine: GEMM routing + a torch-free hipBLASLt plan cache (see gemm.h).
#include "engine/gemm.h"

#include <hipblaslt/hipblaslt.h>

#include <functional>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>

#include "engine/allocator.h"
#include "kernels.h"

namespace mft {
namespace eng {

namespace {

#define LT_OK(expr)                                                                     \
  do {                                                                                  \
    hipblasStatus_t s_ = (expr);                                                        \
    MFT_CHECK(s_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt error ", (int)s_, " in " #expr); \
  } while (0)

constexpr size_t kWorkspace = 32u << 20;
bool g_det = std::getenv("MFT_DETERMINISTIC") && std::getenv("MFT_DETERMINISTIC")[0] == '1';
// hipBLASLt algorithm choice: time the heuristic's candidates on the real operands (one process), or
// take its first pick (MFT_LT_TUNE=0; and by default under a multi-rank communicator, so every rank
// -- and every rerun -- runs the same algorithm: set_lt_autotune(false) from the app's comm setup)
int g_lt_tune = [] {
  const char* e = std::getenv("MFT_LT_TUNE");
  return e ? (e[0] == '0' ? 0 : 1) : -1;  // -1: not forced
}();
bool g_lt_tune_on = g_lt_tune != 0;
// MFT_GEMM_MAP=1: one line per GEMM shape the first time it is routed (backend, hipBLASLt algorithm
// index) -- two ranks' maps must be identical
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

hipblasLtHandle_t lt_handle() {
  static std::mutex mu;
  static std::unordered_map<int, hipblasLtHandle_t> hs;
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  auto it = hs.find(dev);
  if (it != hs.end()) return it->second;
  hipblasLtHandle_t h;
  LT_OK(hipblasLtCreate(&h));
  hs[dev] = h;
  return h;
}

hipDataType lt_type(DType d) {
  switch (d) {
    case DType::F32: return HIP_R_32F;
    case DType::BF16: return HIP_R_16BF;
    case DType::F16: return HIP_R_16F;
    default: MFT_CHECK(false, "hipBLASLt: unsupported dtype ", dtype_name(d));
  }
  return HIP_R_32F;
}

// column-major problem D (m x n, ld ldd) = alpha op(A) op(B) + beta D
struct Problem {
  int dev = 0, ta = 0, tb = 0, epi = HIPBLASLT_EPILOGUE_DEFAULT, has_bias = 0;
  long m = 0, n = 0, k = 0, lda = 0, ldb = 0, ldd = 0;
  DType ab = DType::BF16, d = DType::BF16;
  std::string key() const {
    char b[256];
    snprintf(b, sizeof(b), "%d|%d|%d|%d|%d|%ld|%ld|%ld|%ld|%ld|%ld|%d|%d", dev, ta, tb, epi, has_bias, m, n, k, lda, ldb,
             ldd, (int)ab, (int)d);
    return b;
  }
};

struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
};

Plan& plan_for(const Problem& p, const void* A, const void* B) {
  static std::mutex mu;
  static std::unordered_map<std::string, Plan> plans;
  std::lock_guard<std::mutex> g(mu);
  const std::string key = p.key();
  auto it = plans.find(key);
  if (it != plans.end()) return it->second;
  hipblasLtHandle_t h = lt_handle();
  Plan pl;
  LT_OK(hipblasLtMatmulDescCreate(&pl.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t ta = p.ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = p.tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  LT_OK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_OK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  hipblasLtEpilogue_t epi = (hipblasLtEpilogue_t)p.epi;
  LT_OK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (p.has_bias) {
    hipDataType bt = lt_type(p.d);
    LT_OK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  LT_OK(hipblasLtMatrixLayoutCreate(&pl.a, lt_type(p.ab), p.ta ? p.k : p.m, p.ta ? p.m : p.k, p.lda));
  LT_OK(hipblasLtMatrixLayoutCreate(&pl.b, lt_type(p.ab), p.tb ? p.n : p.k, p.tb ? p.k : p.n, p.ldb));
  LT_OK(hipblasLtMatrixLayoutCreate(&pl.d, lt_type(p.d), p.m, p.n, p.ldd));
  hipblasLtMatmulPreference_t pref;
  LT_OK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t ws = kWorkspace;
  LT_OK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
  constexpr int kCand = 16;
  hipblasLtMatmulHeuristicResult_t res[kCand];
  int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, pl.op, pl.a, pl.b, pl.d, pl.d, pref, kCand, res, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  MFT_CHECK(st == HIPBLAS_STATUS_SUCCESS && got > 0, "hipBLASLt: no algorithm for m=", p.m, " n=", p.n, " k=", p.k);
  int best = 0;
  // autotune on the real operands (skipped under graph capture / MFT_LT_TUNE=0): time every
  // candidate into a scratch output
  hipStream_t s = current_stream();
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (s) (void)hipStreamIsCapturing(s, &cap);
  // (deterministic mode and multi-rank runs keep the heuristic's first pick: a timing-based choice
  // can differ between processes, and different algorithms sum in different orders)
  if (got > 1 && A && B && cap == hipStreamCaptureStatusNone && g_lt_tune_on && !g_det) {
    auto& al = CachingAllocator::get(p.dev);
    size_t wmax = 1;
    for (int i = 0; i < got; ++i) wmax = std::max(wmax, (size_t)res[i].workspaceSize);
    void* scratch = al.allocate((size_t)p.ldd * p.n * dtype_size(p.d), s);
    void* wsb = al.allocate(wmax, s);
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    const float alpha = 1.f, beta = 0.f;
    float best_ms = 1e30f;
    for (int i = 0; i < got; ++i) {
      bool ok = true;
      for (int r = 0; r < 2 && ok; ++r)
        ok = hipblasLtMatmul(h, pl.op, &alpha, A, pl.a, B, pl.b, &beta, scratch, pl.d, scratch, pl.d, &res[i].algo, wsb,
                             res[i].workspaceSize, s) == HIPBLAS_STATUS_SUCCESS;
      if (!ok) continue;
      HIP_OK(hipEventRecord(e0, s));
      for (int r = 0; r < 5; ++r)
        (void)hipblasLtMatmul(h, pl.op, &alpha, A, pl.a, B, pl.b, &beta, scratch, pl.d, scratch, pl.d, &res[i].algo,
                              wsb, res[i].workspaceSize, s);
      HIP_OK(hipEventRecord(e1, s));
      HIP_OK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best_ms) {
        best_ms = ms;
        best = i;
      }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    al.release(scratch);
    al.release(wsb);
  }
  pl.algo = res[best].algo;
  pl.ws = res[best].workspaceSize;
  if (gemm_map())
    std::fprintf(stderr, "[gemm-map] hipBLASLt m=%ld n=%ld k=%ld ta=%d tb=%d epi=%d -> algorithm %d of %d (%s)\n", p.m, p.n,
                 p.k, p.ta, p.tb, p.epi, best, got, (g_lt_tune_on && !g_det) ? "timed" : "heuristic first");
  return plans.emplace(key, pl).first->second;
}

// D = alpha op(A) op(B) (+ bias) + beta C, C = D unless given (same layout)
void lt_run(const Problem& p, const void* A, const void* B, void* D, const void* bias, float alpha, float beta,
            const void* C = nullptr) {
  Plan& pl = plan_for(p, A, B);
  if (bias) LT_OK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  void* ws = nullptr;
  auto& al = CachingAllocator::get(p.dev);
  if (pl.ws) ws = al.allocate(pl.ws, current_stream());
  LT_OK(hipblasLtMatmul(lt_handle(), pl.op, &alpha, A, pl.a, B, pl.b, &beta, C ? C : D, pl.d, D, pl.d, &pl.algo, ws,
                        pl.ws, current_stream()));
  if (ws) al.release(ws);  // stream-ordered reuse
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

}  // namespace

// MFT_GEMM4=0 keeps every GEMM off gemm4 (A/B)
bool gemm4_route(int epi, bool b_kn, long M, long N, long K, long lda, long ldb) {
  static const int mode = [] {
    const char* e = std::getenv("MFT_GEMM4");
    return !e ? 1 : e[0] == '0' ? 0 : 1;
  }();
  if (mode == 0 || b_kn || deterministic() || !::mft::gemm4_supported((int)M, (int)N, (int)K, false, false)) return false;
  if (lda % 8 || ldb % 8) return false;
  // every epilogue gemm4 carries is faster there than on gemm8 (profiles/r5_gemm4_nt_stores.txt)
  return epi == ::mft::GEMM_EPI_MUL_AUX || epi == ::mft::GEMM_EPI_DGELU || epi == ::mft::GEMM_EPI_BIAS_GELU_D ||
         epi == ::mft::GEMM_EPI_NONE || epi == ::mft::GEMM_EPI_BIAS || epi == ::mft::GEMM_EPI_BIAS_ADD;
}

// plain NT forwards (bias / fused residual) and the W^T data gradients on gemm4: MFT_NT=gemm4 (default)
bool nt_gemm4() {
  static const bool v = [] {
    const char* e = std::getenv("MFT_NT");
    const char* g = std::getenv("MFT_GEMM4");
    if (g && g[0] == '0') return false;
    return !e || std::string(e) == "gemm4";
  }();
  return v;
}

bool gemm8_all() {
  static int v = -1;
  if (v < 0) v = (std::getenv("MFT_GEMM8_ALL") && std::getenv("MFT_GEMM8_ALL")[0] == '1') ? 1 : 0;
  return v == 1;
}
bool deterministic() { return g_det; }
void set_lt_autotune(bool on) {
  if (g_lt_tune < 0) g_lt_tune_on = on;  // an explicit MFT_LT_TUNE wins
}
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


void gemm_nt(const Tensor& x2, const Tensor& w, const Tensor& bias, Tensor& y, const Tensor& resid) {
  MFT_CHECK(rowmajor2(x2) && rowmajor2(w) && rowmajor2(y) && x2.dtype() == DType::BF16 && w.dtype() == DType::BF16,
            "gemm_nt: bf16 row-major");
  const long M = x2.size(0), K = x2.size(1), N = w.size(0);
  MFT_CHECK(w.size(1) == K && y.size(0) == M && y.size(1) == N, "gemm_nt: shapes ", x2.str(), " ", w.str(), " ",
            y.str());
  // resid: the residual stream [M, N] added in the epilogue (y = x W^T + b + resid): hipBLASLt's beta = 1
  // with C = resid, gemm8's BIAS_ADD epilogue -- the residual add never makes its own pass
  MFT_CHECK(!resid.defined() || (rowmajor2(resid) && resid.dtype() == DType::BF16 && resid.size(0) == M &&
                                 resid.size(1) == N && resid.stride(0) == y.stride(0) && bias.defined()),
            "gemm_nt: the fused residual must match y (bf16 [M, N], same row stride) and come with a bias");
  auto run_g8 = [&]() {
    Gemm8Extra ex;
    ex.bias = bias.defined() ? &bias : nullptr;
    Tensor r = resid;
    if (resid.defined()) ex.aux = &r;
    gemm8_call(x2, w, false,
               resid.defined() ? ::mft::GEMM_EPI_BIAS_ADD
                               : bias.defined() ? ::mft::GEMM_EPI_BIAS : ::mft::GEMM_EPI_NONE,
               y, ex);
  };
  auto run_lt = [&]() {
    // col-major view: y^T [N, M] = W [N, K] . x^T  -> op(A) = T on W (stored K x N col-major)
    Problem p;
    p.dev = cur_dev();
    p.ta = 1;
    p.tb = 0;
    p.has_bias = bias.defined();
    p.epi = bias.defined() ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT;
    p.m = N;
    p.n = M;
    p.k = K;
    p.lda = w.stride(0);
    p.ldb = x2.stride(0);
    p.ldd = y.stride(0);
    lt_run(p, w.data_ptr(), x2.data_ptr(), y.data_ptr(), bias.defined() ? bias.data_ptr() : nullptr, 1.f,
           resid.defined() ? 1.f : 0.f, resid.defined() ? resid.data_ptr() : nullptr);
  };
  const bool g8_ok = K % 64 == 0 && N % 8 == 0 && x2.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 &&
                     y.stride(0) % 8 == 0 && ::mft::gemm8_supported((int)M, (int)N, (int)K, false, false);
  if (!g8_ok) return run_lt();
  if (nt_gemm4() && !deterministic() && ::mft::gemm4_supported((int)M, (int)N, (int)K, false, false)) {
    ::mft::GemmArgs g = args_for(x2, w, y);
    g.M = (int)M;
    g.N = (int)N;
    g.K = (int)K;
    if (bias.defined()) g.bias = (const ::mft::bf16_t*)bias.data_ptr();
    if (resid.defined()) {
      g.aux = (::mft::bf16_t*)resid.data_ptr();
      g.ldaux = resid.stride(0);
    }
    map_line(resid.defined() ? "nt+resid" : "nt", M, N, K, "gemm4");
    ::mft::gemm4x(g, resid.defined() ? ::mft::GEMM_EPI_BIAS_ADD : bias.defined() ? ::mft::GEMM_EPI_BIAS : ::mft::GEMM_EPI_NONE,
                  false, false, current_stream());
    return;
  }
  // Static routing (no timing, identical on every rank and rerun): a PLAIN GEMM (no fused epilogue
  // beyond the bias) is a library GEMM -> hipBLASLt; every fused-epilogue GEMM (GELU, dGELU, LoRA,
  // LM-head cross entropy, split-K weight gradients) is the hand-written gemm8.  MFT_NT=gemm8|lt or
  // MFT_GEMM8_ALL=1 (every GEMM of the step hand-written) override it; deterministic mode keeps gemm8
  // (one fixed reduction order whatever the operands' addresses and the library's heuristic pick).
  static const char* env = std::getenv("MFT_NT");
  static const int forced = !env ? -1 : std::string(env) == "gemm8" ? 1 : std::string(env) == "lt" ? 0 : -1;
  // A residual-producing projection is a standard GEMM with a C input (D = A.B + bias + C, beta = 1), which
  // hipBLASLt runs natively: 1.611-1.614 M tok/s vs 1.597-1.598 M with gemm8's BIAS_ADD epilogue on the
  // headline (3 interleaved rounds, profiles/r4b_resid_routing_ab.txt).  MFT_RESID_G8=1 forces gemm8.
  static const bool resid_g8 = std::getenv("MFT_RESID_G8") && std::getenv("MFT_RESID_G8")[0] == '1';
  const bool g8 = forced >= 0 ? forced == 1 : (deterministic() || gemm8_all() || (resid.defined() && resid_g8));
  map_line(resid.defined() ? "nt+resid" : "nt", M, N, K, g8 ? "gemm8" : "hipBLASLt");
  return g8 ? run_g8() : run_lt();
}

void gemm_nn(const Tensor& dy2, const Tensor& w, Tensor& out, const Tensor& wt) {
  const long N = w.size(0), M = dy2.size(0), K = w.size(1);
  // a resident transposed copy of a frozen weight (Param::transposed) turns the data gradient into an
  // NT GEMM for gemm4 (the hand-scheduled kernel reads K-contiguous operands only)
  if (wt.defined() && nt_gemm4() && !deterministic() && rowmajor2(wt) && wt.size(0) == K && wt.size(1) == N &&
      dy2.stride(0) % 8 == 0 && wt.stride(0) % 8 == 0 && out.stride(0) % 8 == 0 &&
      ::mft::gemm4_supported((int)M, (int)K, (int)N, false, false)) {
    ::mft::GemmArgs g = args_for(dy2, wt, out);
    g.M = (int)M;
    g.N = (int)K;
    g.K = (int)N;
    map_line("nn (W^T)", M, K, N, "gemm4");
    ::mft::gemm4x(g, ::mft::GEMM_EPI_NONE, false, false, current_stream());
    return;
  }
  auto run_g8 = [&]() { gemm8_call(dy2, w, true, ::mft::GEMM_EPI_NONE, out); };
  auto run_lt = [&]() {
    Problem p;  // out^T [K, M] = W^T [K, N] . dy^T [N, M]
    p.dev = cur_dev();
    p.m = K;
    p.n = M;
    p.k = N;
    p.lda = w.stride(0);
    p.ldb = dy2.stride(0);
    p.ldd = out.stride(0);
    lt_run(p, w.data_ptr(), dy2.data_ptr(), out.data_ptr(), nullptr, 1.f, 0.f);
  };
  const bool g8_ok =
      N % 64 == 0 && K % 8 == 0 && dy2.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && out.stride(0) % 8 == 0;
  if (!g8_ok) return run_lt();
  // plain data-gradient GEMMs: the same static routing as the NT forwards (a library GEMM ->
  // hipBLASLt); MFT_NN=gemm8|lt forces one; deterministic mode and MFT_GEMM8_ALL=1 keep gemm8 (its
  // reduction order is fixed)
  static const char* env = std::getenv("MFT_NN");
  static const int forced = !env ? -1 : std::string(env) == "gemm8" ? 1 : std::string(env) == "lt" ? 0 : -1;
  const bool g8 = forced >= 0 ? forced == 1 : (deterministic() || gemm8_all());
  map_line("nn", M, K, N, g8 ? "gemm8" : "hipBLASLt");
  return g8 ? run_g8() : run_lt();
}

void gemm_wgrad(Tensor& buf, const Tensor& dy2, const Tensor& x2, float alpha) {
  MFT_CHECK(buf.dtype() == DType::F32 && buf.is_contiguous(), "gemm_wgrad: fp32 contiguous grad buffer");
  const long M = dy2.size(0), N = dy2.size(1), K = x2.size(1);
  MFT_CHECK(x2.size(0) == M && buf.numel() == N * K, "gemm_wgrad: shapes");
  // gemm8 (F32ACC epilogue straight into the flat grad, split-K over the tokens when the output
  // alone does not fill the CUs) for long token reductions: 0.9-1.1 PF/s on the GPT-2 shapes at
  // 65536 tokens, and the gpt2-full step 63.1 vs 66.5 ms with hipBLASLt's fp32-out kernels.  At
  // GPT-2 XL's 8192 tokens the 1600-6400-wide outputs need 7-way splits whose fp32 slabs cost more
  // than they save: hipBLASLt there (XL ZeRO-3 step 115.4 vs 121.9 ms; profiles/r3_wgrad_ab.jsonl).
  // MFT_WGRAD=gemm8|lt forces one (A/B).
  static const char* wg_env = std::getenv("MFT_WGRAD");
  static const int wg_mode = !wg_env ? 0 : std::string(wg_env) == "lt" ? 1 : std::string(wg_env) == "gemm8" ? 2 : 0;
  const bool want_g8 = wg_mode == 2 || (wg_mode == 0 && M >= 32768);
  if ((deterministic() || gemm8_all() || want_g8) && M % 64 == 0 && N % 8 == 0 && K % 8 == 0 && dy2.stride(0) % 8 == 0 &&
      x2.stride(0) % 8 == 0 && ::mft::gemm8_supported((int)N, (int)K, (int)M, true, true)) {
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
  map_line("wgrad", N, K, M, "hipBLASLt");
  // col-major: buf^T [K, N] += x^T [K, M] . dy [M, N]  (beta = 1)
  Problem p;
  p.dev = cur_dev();
  p.ta = 0;
  p.tb = 1;
  p.m = K;
  p.n = N;
  p.k = M;
  p.lda = x2.stride(0);
  p.ldb = dy2.stride(0);
  p.ldd = K;
  p.d = DType::F32;
  lt_run(p, x2.data_ptr(), dy2.data_ptr(), buf.data_ptr(), nullptr, alpha, 1.f);
}

void blas_gemm(const Tensor& a, bool ta, const Tensor& b, bool tb, Tensor& c, float alpha, float beta) {
  // row-major C[M, N] = op(A) op(B)  <=>  col-major C^T = op(B)^T op(A)^T
  MFT_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1,
            "blas_gemm: row-major 2-D operands");
  MFT_CHECK(a.dtype() == b.dtype(), "blas_gemm: operand dtypes differ");
  const long M = ta ? a.size(1) : a.size(0), K = ta ? a.size(0) : a.size(1);
  const long N = tb ? b.size(0) : b.size(1);
  MFT_CHECK((tb ? b.size(1) : b.size(0)) == K && c.size(0) == M && c.size(1) == N, "blas_gemm: shapes");
  map_line(ta ? (tb ? "blas TT" : "blas TN") : (tb ? "blas NT" : "blas NN"), M, N, K, "hipBLASLt");
  Problem p;
  p.dev = cur_dev();
  p.ta = tb;  // col-major A' = B^T stored as b (row-major [K,N] == col-major [N,K])
  p.tb = ta;
  p.m = N;
  p.n = M;
  p.k = K;
  p.lda = b.stride(0);
  p.ldb = a.stride(0);
  p.ldd = c.stride(0);
  p.ab = a.dtype();
  p.d = c.dtype();
  lt_run(p, b.data_ptr(), a.data_ptr(), c.data_ptr(), nullptr, alpha, beta);
}

}  // namespace eng
}  // namespace mft
