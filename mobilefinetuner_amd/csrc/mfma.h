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

// Register-to-register operand reuse: two 16x16 C/D blocks c0, c1 whose COLUMNS index the next
// MFMA's m and whose ROWS index its k (k 0..15 in c0, 16..31 in c1) become an A operand without an
// LDS round trip if the k index is permuted consistently in both operands (the MFMA sums over k):
//   A lane l, element j  <-  k = 4*(l>>4) + j (j < 4, from c0) | 16 + 4*(l>>4) + (j - 4) (j >= 4, c1)
// pack_c2a builds that A fragment; frag_tr_perm reads the matching B fragment (rows permuted the
// same way) from a row-major LDS image with two ds_read_b64_tr_b16.
__device__ __forceinline__ bf16x8_t pack_c2a(f32x4_t c0, f32x4_t c1) {
  u16x8_t u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u[i] = f2bf(c0[i]);
    u[4 + i] = f2bf(c1[i]);
  }
  return __builtin_bit_cast(bf16x8_t, u);
}

// lane holds M[r0 + 4*(l>>4) + j][c0 + (l&15)] (j < 4) and M[r0 + 16 + 4*(l>>4) + j - 4][c0 + (l&15)] (j >= 4)
__device__ __forceinline__ bf16x8_t frag_tr_perm(const bf16_t* base, int ld, int r0, int c0) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const bf16_t* a0 = base + (r0 + 4 * g + q) * ld + c0 + 4 * p;
  s16x4_t lo = ds_tr16(a0);
  s16x4_t hi = ds_tr16(a0 + 16 * ld);
  s16x8_t r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

__device__ __forceinline__ f32x4_t zero4() { return f32x4_t{0.f, 0.f, 0.f, 0.f}; }

// cross-row-group exchanges as VALU permlane swaps (no LDS round trip, unlike ds_bpermute shuffles):
// value of lane l ^ 16 / l ^ 32
__device__ __forceinline__ float xor16_pl(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(((threadIdx.x >> 4) & 1) ? r[0] : r[1]);
}
__device__ __forceinline__ float xor32_pl(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(((threadIdx.x >> 5) & 1) ? r[0] : r[1]);
}

}  // namespace mft
