// Generic SIMT GEMM: the correctness fallback behind engine/gemm.cpp for the operands the MFMA kernels
// (gemm4 / gemm8) do not take -- fp32 operands, K not a multiple of 64, N not a multiple of 8,
// unaligned row strides.  No model of the benchmarks reaches it (their GEMMs all route to gemm4 /
// gemm8, profiles/r5_gemm_routing_map.txt); it keeps the engine's generic matmul / linear ops
// (engine/ops.cpp) complete without a vendor GEMM library.
//
//   D[M, N] = alpha op(A) op(B) (+ bias[N]) + beta Cin[M, N]      fp32 accumulation
//   op(A)[m, k] = ta ? A[k, m] : A[m, k]      op(B)[k, n] = tb ? B[n, k] : B[k, n]
//
// 64 x 64 output tile per 256-thread workgroup (4 x 4 per thread), K staged through LDS 16 at a time.
#include "common.h"
#include "kernels.h"

namespace mft {

namespace {

__device__ __forceinline__ float ld_any(const void* p, long i, int f32) {
  return f32 ? reinterpret_cast<const float*>(p)[i] : bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
}

__global__ __launch_bounds__(256) void gemm_simt_kernel(SimtGemmArgs a) {
  __shared__ float As[16][65], Bs[16][65];
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < a.K; k0 += 16) {
    for (int i = threadIdx.x; i < 16 * 64; i += 256) {
      const int kk = i >> 6, r = i & 63;
      const int k = k0 + kk, m = m0 + r, n = n0 + r;
      float av = 0.f, bv = 0.f;
      if (k < a.K && m < a.M) av = ld_any(a.A, a.ta ? (long)k * a.lda + m : (long)m * a.lda + k, a.a_f32);
      if (k < a.K && n < a.N) bv = ld_any(a.B, a.tb ? (long)n * a.ldb + k : (long)k * a.ldb + n, a.b_f32);
      As[kk][r] = av;
      Bs[kk][r] = bv;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float ar[4], br[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ar[i] = As[kk][ty * 4 + i];
        br[i] = Bs[kk][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(ar[i], br[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n >= a.N) continue;
      float v = a.alpha * acc[i][j];
      if (a.bias) v += bf2f(a.bias[n]);
      if (a.Cin && a.beta != 0.f) v += a.beta * ld_any(a.Cin, (long)m * a.ldcin + n, a.cin_f32);
      if (a.d_f32) reinterpret_cast<float*>(a.D)[(long)m * a.ldd + n] = v;
      else reinterpret_cast<bf16_t*>(a.D)[(long)m * a.ldd + n] = f2bf(v);
    }
  }
}

}  // namespace

void gemm_simt(const SimtGemmArgs& a, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0) return;
  const dim3 grid((a.N + 63) / 64, (a.M + 63) / 64);
  gemm_simt_kernel<<<grid, 256, 0, st>>>(a);
}

}  // namespace mft
