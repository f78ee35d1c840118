// Generic GEMM: the correctness path behind engine/gemm.cpp for the operands the bf16 MFMA kernels
// (gemm4 / gemm8 / gemm_s) do not take -- fp32 operands (the native --dtype fp32 mode), K not a multiple
// of 64, N not a multiple of 8, unaligned row strides.  No bf16 benchmark model reaches it (their GEMMs
// all route to gemm4 / gemm8 / gemm_s, profiles/r5_gemm_routing_map.txt); it keeps the engine's generic
// matmul / linear ops (engine/ops.cpp) complete without a vendor GEMM library.
//
//   D[M, N] = alpha op(A) op(B) (+ bias[N]) + beta Cin[M, N]      fp32 accumulation
//   op(A)[m, k] = ta ? A[k, m] : A[m, k]      op(B)[k, n] = tb ? B[n, k] : B[k, n]
//
// 64 x 64 output tile per 256-thread workgroup, K staged through LDS 16 at a time as fp32 (any operand
// dtype / layout / stride, range-checked).  The products run on the fp32 matrix cores:
// v_mfma_f32_16x16x4_f32, each wave a 32 x 32 quadrant (2 x 2 blocks, 4 k-steps per stage).  On gfx950
// that instruction is exact fp32 -- bitwise an fmaf chain over k (MI355X microarchitecture notes) -- so
// the result is the one of the VALU form kept below (MFT_GEMM_SIMT=valu, A/B and tests), at 16x the
// VALU's per-SIMD rate.
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <string>

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

// stage = 16 k of op(A) [16][64] and op(B) [16][64] as fp32, [k][m] / [k][n] (rows padded against bank conflicts)
__device__ __forceinline__ void simt_stage(const SimtGemmArgs& a, int m0, int n0, int k0, float (&As)[16][65],
                                           float (&Bs)[16][65]) {
  for (int i = threadIdx.x; i < 16 * 64; i += 256) {
    const int kk = i >> 6, r = i & 63;
    const int k = k0 + kk, m = m0 + r, n = n0 + r;
    float av = 0.f, bv = 0.f;
    if (k < a.K && m < a.M) av = ld_any(a.A, a.ta ? (long)k * a.lda + m : (long)m * a.lda + k, a.a_f32);
    if (k < a.K && n < a.N) bv = ld_any(a.B, a.tb ? (long)n * a.ldb + k : (long)k * a.ldb + n, a.b_f32);
    As[kk][r] = av;
    Bs[kk][r] = bv;
  }
}

__device__ __forceinline__ void simt_store(const SimtGemmArgs& a, int m, int n, float acc) {
  if (m >= a.M || n >= a.N) return;
  float v = a.alpha * acc;
  if (a.bias) v += bf2f(a.bias[n]);
  if (a.Cin && a.beta != 0.f) v += a.beta * ld_any(a.Cin, (long)m * a.ldcin + n, a.cin_f32);
  if (a.d_f32) reinterpret_cast<float*>(a.D)[(long)m * a.ldd + n] = v;
  else reinterpret_cast<bf16_t*>(a.D)[(long)m * a.ldd + n] = f2bf(v);
}

// v_mfma_f32_16x16x4_f32 operand maps: A lane l = A[m = l & 15][k = l >> 4], B lane l = B[k = l >> 4][n = l & 15],
// D lane l, reg i = D[4 (l >> 4) + i][l & 15]
__global__ __launch_bounds__(256) void gemm_f32mfma_kernel(SimtGemmArgs a) {
  __shared__ float As[16][65], Bs[16][65];
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;  // the wave's 32 x 32 quadrant
  const int li = l & 15, lk = l >> 4;
  f32x4_t acc[2][2] = {};
  for (int k0 = 0; k0 < a.K; k0 += 16) {
    simt_stage(a, m0, n0, k0, As, Bs);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kk = 4 * ks + lk;
      const float a0 = As[kk][wm + li], a1 = As[kk][wm + 16 + li];
      const float b0 = Bs[kk][wn + li], b1 = Bs[kk][wn + 16 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        simt_store(a, m0 + wm + 16 * bi + 4 * lk + i, n0 + wn + 16 * bj + li, acc[bi][bj][i]);
}

}  // namespace

void gemm_simt(const SimtGemmArgs& a, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0) return;
  const dim3 grid((a.N + 63) / 64, (a.M + 63) / 64);
  static const bool valu = getenv("MFT_GEMM_SIMT") && std::string(getenv("MFT_GEMM_SIMT")) == "valu";
  if (valu) gemm_simt_kernel<<<grid, 256, 0, st>>>(a);
  else gemm_f32mfma_kernel<<<grid, 256, 0, st>>>(a);
}

}  // namespace mft
