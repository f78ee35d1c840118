// MFMA fragment helpers for gfx950 (v_mfma_f32_16x16x32_bf16), shared by the attention and
// GEMM-epilogue kernels.
//
// Operand maps (CDNA HIP guide §3, verified layouts):
//   A[m][k]: lane l holds A[m = l&15][k = 8*(l>>4) + j], j = 0..7
//   B[k][n]: lane l holds B[k = 8*(l>>4) + j][n = l&15]
//   C/D   : lane l, reg i holds C[row = 4*(l>>4) + i][col = l&15]
// Every operand is read from a single ROW-MAJOR LDS image, either
//   * frag_row(): 16 contiguous bytes of one row (ds_read_b128), or
//   * frag_tr():  two ds_read_b64_tr_b16 hardware-transposed reads (T10), so no tile is ever
//                 stored twice (once per orientation) and no scalar transposing writes are needed.
#pragma once
#include "common.h"

namespace mft {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// lane holds M[r0 + (l&15)][c0 + 8*(l>>4) + j]
__device__ __forceinline__ bf16x8_t frag_row(const bf16_t* base, int ld, int r0, int c0) {
  const int l = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8_t*>(base + (r0 + (l & 15)) * ld + c0 + 8 * (l >> 4));
}

__device__ __forceinline__ s16x4_t ds_tr16(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

// lane holds M[r0 + 8*(l>>4) + j][c0 + (l&15)]   (EXEC must be full: call from converged code)
__device__ __forceinline__ bf16x8_t frag_tr(const bf16_t* base, int ld, int r0, int c0) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const bf16_t* a0 = base + (r0 + 8 * g + q) * ld + c0 + 4 * p;
  s16x4_t lo = ds_tr16(a0);
  s16x4_t hi = ds_tr16(a0 + 4 * ld);
  s16x8_t r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

__device__ __forceinline__ f32x4_t zero4() { return f32x4_t{0.f, 0.f, 0.f, 0.f}; }

}  // namespace mft
