// hipBLASLt capability probe.
//
// Plain library GEMMs go through torch.mm / torch.addmm (hipBLASLt).  The fused-epilogue GEMMs are
// the hand-written kernels/gemm.hip because this ROCm build's gfx950 hipBLASLt has NO solutions for
// the GELU_AUX(_BIAS) / DGELU(_BGRAD) epilogues in bf16 (scripts/probe_lt.py: 0 solutions for
// every layout, while DEFAULT / BIAS / GELU / GELU_BIAS have 8).  lt_solutions() keeps that
// check reproducible on any box.  lt_wgrad_acc() is the one hipBLASLt call made directly: weight
// gradients accumulated in place into the fp32 grad buffer (beta = 1), which torch.mm cannot do
// for bf16 inputs.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <string>
#include <unordered_map>

namespace py = pybind11;
using torch::Tensor;

namespace {

#define LT_CHECK(expr)                                                                             \
  do {                                                                                             \
    hipblasStatus_t st_ = (expr);                                                                  \
    TORCH_CHECK(st_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt error ", (int)st_, " at ", #expr);       \
  } while (0)

constexpr size_t kWorkspace = 32u << 20;

struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
};

hipblasLtHandle_t handle_for(int dev) {
  static std::mutex mu;
  static std::unordered_map<int, hipblasLtHandle_t> handles;
  std::lock_guard<std::mutex> g(mu);
  auto it = handles.find(dev);
  if (it != handles.end()) return it->second;
  hipblasLtHandle_t h;
  LT_CHECK(hipblasLtCreate(&h));
  handles[dev] = h;
  return h;
}

// col-major problem: D (m x n, ld ldd) = op(A) (m x k) * op(B) (k x n)
struct Problem {
  int dev, ta, tb, epi, has_bias;
  long m, n, k, lda, ldb, ldd, ldaux;
  int d_f32 = 0;  // C/D in fp32 (weight-gradient accumulation) instead of bf16
  std::string key() const {
    char buf[256];
    snprintf(buf, sizeof(buf), "%d|%d|%d|%d|%d|%ld|%ld|%ld|%ld|%ld|%ld|%ld|%d", dev, ta, tb, epi, has_bias, m, n, k, lda,
             ldb, ldd, ldaux, d_f32);
    return buf;
  }
};

// A/B: the operands of the first call (timing candidates when the plan is created).
Plan& plan_for(const Problem& p, hipblasLtHandle_t h, const void* A = nullptr, const void* B = nullptr) {
  static std::mutex mu;
  static std::unordered_map<std::string, Plan> plans;
  std::lock_guard<std::mutex> g(mu);
  const std::string key = p.key();
  auto it = plans.find(key);
  if (it != plans.end()) return it->second;
  Plan pl;
  LT_CHECK(hipblasLtMatmulDescCreate(&pl.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t ta = p.ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = p.tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  hipblasLtEpilogue_t epi = (hipblasLtEpilogue_t)p.epi;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (p.has_bias) {
    hipDataType bt = HIP_R_16BF;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (p.ldaux > 0) {
    int64_t ld = p.ldaux;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
    hipDataType at = HIP_R_16BF;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
  }
  // A is (m x k) after op; stored (rows x cols) = ta ? (k x m) : (m x k)
  LT_CHECK(hipblasLtMatrixLayoutCreate(&pl.a, HIP_R_16BF, p.ta ? p.k : p.m, p.ta ? p.m : p.k, p.lda));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&pl.b, HIP_R_16BF, p.tb ? p.n : p.k, p.tb ? p.k : p.n, p.ldb));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&pl.d, p.d_f32 ? HIP_R_32F : HIP_R_16BF, p.m, p.n, p.ldd));
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t ws = kWorkspace;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
  constexpr int kCand = 16;
  hipblasLtMatmulHeuristicResult_t res[kCand];
  int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, pl.op, pl.a, pl.b, pl.d, pl.d, pref, kCand, res, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  TORCH_CHECK(st == HIPBLAS_STATUS_SUCCESS && got > 0, "hipBLASLt: no algorithm for epilogue ", p.epi, " m=", p.m,
              " n=", p.n, " k=", p.k);
  int best = 0;
  // Autotune: the heuristic's first pick is poor for some skinny shapes (weight gradients reduce
  // over M = B*S with few output tiles); time every candidate once on the real operands into a
  // scratch output.  Skipped while a hipGraph is being captured and with MFT_LT_TUNE=0.
  hipStream_t stream = c10::hip::getCurrentHIPStream().stream();
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(stream, &cap);
  const char* tune_env = getenv("MFT_LT_TUNE");
  if (got > 1 && A && B && cap == hipStreamCaptureStatusNone && !(tune_env && tune_env[0] == '0')) {
    const size_t esz = p.d_f32 ? 4 : 2;
    auto opts = torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, p.dev);
    Tensor scratch = torch::empty({(long)(p.ldd * p.n * esz)}, opts);
    size_t wmax = 0;
    for (int i = 0; i < got; ++i) wmax = std::max(wmax, (size_t)res[i].workspaceSize);
    Tensor wsb = torch::empty({(long)std::max<size_t>(wmax, 1)}, opts);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const float alpha = 1.f, beta = 0.f;
    float best_ms = 1e30f;
    for (int i = 0; i < got; ++i) {
      bool ok = true;
      for (int rep = 0; rep < 2 && ok; ++rep)
        ok = hipblasLtMatmul(h, pl.op, &alpha, A, pl.a, B, pl.b, &beta, scratch.data_ptr(), pl.d, scratch.data_ptr(),
                             pl.d, &res[i].algo, wsb.data_ptr(), res[i].workspaceSize, stream) == HIPBLAS_STATUS_SUCCESS;
      if (!ok) continue;
      (void)hipEventRecord(e0, stream);
      for (int rep = 0; rep < 5; ++rep)
        (void)hipblasLtMatmul(h, pl.op, &alpha, A, pl.a, B, pl.b, &beta, scratch.data_ptr(), pl.d, scratch.data_ptr(),
                              pl.d, &res[i].algo, wsb.data_ptr(), res[i].workspaceSize, stream);
      (void)hipEventRecord(e1, stream);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best_ms) {
        best_ms = ms;
        best = i;
      }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  pl.algo = res[best].algo;
  pl.ws = res[best].workspaceSize;
  return plans.emplace(key, pl).first->second;
}

void run(const Problem& p, const void* A, const void* B, void* D, const void* bias, void* aux, float alpha = 1.f,
         float beta = 0.f) {
  const int dev = p.dev;
  hipblasLtHandle_t h = handle_for(dev);
  Plan& pl = plan_for(p, h, A, B);
  if (bias) LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  if (aux) LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
  Tensor ws;
  void* wsp = nullptr;
  if (pl.ws) {
    ws = torch::empty({(long)pl.ws}, torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, dev));
    wsp = ws.data_ptr();
  }
  LT_CHECK(hipblasLtMatmul(h, pl.op, &alpha, A, pl.a, B, pl.b, &beta, D, pl.d, D, pl.d, &pl.algo, wsp, pl.ws,
                           c10::hip::getCurrentHIPStream().stream()));
}

// number of hipBLASLt solutions for a col-major problem (diagnostics / capability probing)
int lt_solutions(int64_t m, int64_t n, int64_t k, bool ta, bool tb, int64_t epi, bool bias, int64_t ldaux,
                 int64_t aux_dtype) {
  const int dev = c10::hip::current_device();
  hipblasLtHandle_t h = handle_for(dev);
  hipblasLtMatmulDesc_t op;
  LT_CHECK(hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa));
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob));
  hipblasLtEpilogue_t e = (hipblasLtEpilogue_t)epi;
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
  if (bias) {
    hipDataType bt = HIP_R_16BF;
    hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  }
  if (ldaux > 0) {
    int64_t ld = ldaux;
    hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
    if (aux_dtype >= 0) {
      hipDataType at = (hipDataType)aux_dtype;
      hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at));
    }
  }
  hipblasLtMatrixLayout_t a, b, d;
  hipblasLtMatrixLayoutCreate(&a, HIP_R_16BF, ta ? k : m, ta ? m : k, ta ? k : m);
  hipblasLtMatrixLayoutCreate(&b, HIP_R_16BF, tb ? n : k, tb ? k : n, tb ? n : k);
  hipblasLtMatrixLayoutCreate(&d, HIP_R_16BF, m, n, m);
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t ws = kWorkspace;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  hipblasLtMatmulHeuristicResult_t res[8];
  int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, op, a, b, d, d, pref, 8, res, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatrixLayoutDestroy(a);
  hipblasLtMatrixLayoutDestroy(b);
  hipblasLtMatrixLayoutDestroy(d);
  hipblasLtMatmulDescDestroy(op);
  return st == HIPBLAS_STATUS_SUCCESS ? got : -(int)st;
}

// out[N, K] (fp32) += alpha * dy[M, N]^T x[M, K]   (bf16 inputs, fp32 accumulate, beta = 1):
// weight gradients straight into the flat fp32 grad buffer -- no fp32 temporary + add pass.
void lt_wgrad_acc(Tensor x, Tensor dy, Tensor out, double alpha) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && dy.scalar_type() == torch::kBFloat16 &&
                  out.scalar_type() == torch::kFloat32, "lt_wgrad_acc: bf16 x/dy, fp32 out");
  TORCH_CHECK(x.dim() == 2 && dy.dim() == 2 && out.dim() == 2 && x.stride(1) == 1 && dy.stride(1) == 1 &&
                  out.stride(1) == 1, "lt_wgrad_acc: row-contiguous 2-D tensors");
  const long M = x.size(0), K = x.size(1), N = dy.size(1);
  TORCH_CHECK(dy.size(0) == M && out.size(0) == N && out.size(1) == K, "lt_wgrad_acc: shapes");
  c10::DeviceGuard g(x.device());
  // col-major: out^T [K, N] = x^T [K, M] . dy [M, N];  x row-major == col-major (K x M, ld K),
  // dy row-major == col-major (N x M, ld N) -> op(B) = T
  Problem p{x.get_device(), 0, 1, HIPBLASLT_EPILOGUE_DEFAULT, 0, K, N, M, x.stride(0), dy.stride(0), out.stride(0), 0};
  p.d_f32 = 1;
  run(p, x.data_ptr(), dy.data_ptr(), out.data_ptr(), nullptr, nullptr, (float)alpha, 1.f);
}

// y[M, N] = x[M, K] W[N, K]^T (+ bias[N])  -- autotuned hipBLASLt, bf16 out (BIAS epilogue)
Tensor lt_linear(Tensor x, Tensor w, c10::optional<Tensor> bias) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && w.scalar_type() == torch::kBFloat16 &&
                  x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && w.stride(1) == 1, "lt_linear: bf16 2-D row-major");
  const long M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "lt_linear: shapes");
  const bool hb = bias.has_value() && bias->defined();
  if (hb) TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->numel() == N && bias->is_contiguous(), "bias");
  c10::DeviceGuard g(x.device());
  auto y = torch::empty({M, N}, x.options());
  Problem p{x.get_device(), 1, 0, hb ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT, hb ? 1 : 0, N, M, K,
            w.stride(0), x.stride(0), N, 0};
  run(p, w.data_ptr(), x.data_ptr(), y.data_ptr(), hb ? bias->data_ptr() : nullptr, nullptr);
  return y;
}

// dx[M, K] = dy[M, N] W[N, K]  (data gradient of a Linear; W may be a row-strided view)
Tensor lt_mm_dx(Tensor dy, Tensor w, c10::optional<Tensor> out) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == torch::kBFloat16 && w.scalar_type() == torch::kBFloat16 &&
                  dy.dim() == 2 && w.dim() == 2 && dy.stride(1) == 1 && w.stride(1) == 1, "lt_mm_dx: bf16 2-D row-major");
  const long M = dy.size(0), N = dy.size(1), K = w.size(1);
  TORCH_CHECK(w.size(0) == N, "lt_mm_dx: shapes");
  c10::DeviceGuard g(dy.device());
  Tensor dx;
  if (out.has_value() && out->defined()) {
    dx = *out;
    TORCH_CHECK(dx.size(0) == M && dx.size(1) == K && dx.stride(1) == 1 && dx.scalar_type() == torch::kBFloat16,
                "lt_mm_dx: out must be [M, K] bf16 row-major");
  } else {
    dx = torch::empty({M, K}, dy.options());
  }
  Problem p{dy.get_device(), 0, 0, HIPBLASLT_EPILOGUE_DEFAULT, 0, K, M, N, w.stride(0), dy.stride(0), dx.stride(0), 0};
  run(p, w.data_ptr(), dy.data_ptr(), dx.data_ptr(), nullptr, nullptr);
  return dx;
}

}  // namespace

void register_gemm_lt(py::module_& m) {
  m.def("lt_linear", &lt_linear, "y = x W^T (+ b), autotuned hipBLASLt");
  m.def("lt_mm_dx", &lt_mm_dx, "dx = dy W, autotuned hipBLASLt");
  m.def("lt_wgrad_acc", &lt_wgrad_acc, "out[N,K] (fp32) += alpha * dy^T x (hipBLASLt, beta = 1)");
  m.def("lt_solutions", &lt_solutions, "number of hipBLASLt solutions for (m, n, k, ta, tb, epilogue, bias, ldaux, aux_dtype)");
}
