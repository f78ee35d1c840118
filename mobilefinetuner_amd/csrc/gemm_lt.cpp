// hipBLASLt capability probe.
//
// Plain library GEMMs go through torch.mm / torch.addmm (hipBLASLt).  The fused-epilogue GEMMs are
// the hand-written kernels/gemm.hip because this ROCm build's gfx950 hipBLASLt has NO solutions for
// the GELU_AUX(_BIAS) / DGELU(_BGRAD) epilogues in bf16 (scripts/probe_lt.py: 0 solutions for
// every layout, while DEFAULT / BIAS / GELU / GELU_BIAS have 8).  lt_solutions() keeps that
// check reproducible on any box; Plan/run() below are the cached-algorithm plumbing it shares.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <hipblaslt/hipblaslt.h>

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
  std::string key() const {
    char buf[256];
    snprintf(buf, sizeof(buf), "%d|%d|%d|%d|%d|%ld|%ld|%ld|%ld|%ld|%ld|%ld", dev, ta, tb, epi, has_bias, m, n, k, lda,
             ldb, ldd, ldaux);
    return buf;
  }
};

Plan& plan_for(const Problem& p, hipblasLtHandle_t h) {
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
  LT_CHECK(hipblasLtMatrixLayoutCreate(&pl.d, HIP_R_16BF, p.m, p.n, p.ldd));
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t ws = kWorkspace;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
  hipblasLtMatmulHeuristicResult_t res[4];
  int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, pl.op, pl.a, pl.b, pl.d, pl.d, pref, 4, res, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  TORCH_CHECK(st == HIPBLAS_STATUS_SUCCESS && got > 0, "hipBLASLt: no algorithm for epilogue ", p.epi, " m=", p.m,
              " n=", p.n, " k=", p.k);
  pl.algo = res[0].algo;
  pl.ws = res[0].workspaceSize;
  return plans.emplace(key, pl).first->second;
}

void run(const Problem& p, const void* A, const void* B, void* D, const void* bias, void* aux) {
  const int dev = p.dev;
  hipblasLtHandle_t h = handle_for(dev);
  Plan& pl = plan_for(p, h);
  if (bias) LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  if (aux) LT_CHECK(hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
  Tensor ws;
  void* wsp = nullptr;
  if (pl.ws) {
    ws = torch::empty({(long)pl.ws}, torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, dev));
    wsp = ws.data_ptr();
  }
  const float alpha = 1.f, beta = 0.f;
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

}  // namespace

void register_gemm_lt(py::module_& m) {
  m.def("lt_solutions", &lt_solutions, "number of hipBLASLt solutions for (m, n, k, ta, tb, epilogue, bias, ldaux, aux_dtype)");
}
