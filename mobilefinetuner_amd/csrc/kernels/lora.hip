// LoRA rank-r kernels: the skinny products around the frozen base GEMM.
//
// Replaces LoRALinear::forward/merge/unmerge (nn/lora_linear.cpp:47-178), whose partial-column
// slices were added without autograd, and the never-constructed
// LoRALinearBackward (core/backward_functions.cpp:1012-1226).
//
// Internal layouts: A is [R, K] (PEFT lora_A.weight), B is [R, N] (reference lora_B layout), so
// every rank-r operand is read along contiguous rows.  For y = x W^T + s (x A^T) B:
//   lora_rowdot : U[m, r] = s * sum_k X[m, k] Wt[r, k]           u = x A^T (Wt = A), v = s dy B^T (Wt = B)
//                 MFMA 16x16x32: one 16-row tile per 4-wave block, K split over the waves and
//                 reduced through LDS; X streamed once from HBM with 16-B loads.
//   lora_update : Y[m, n] = base[m, n] + s * sum_r U[m, r] W[r, n]  y += s u B (W = B), dx += v A (W = A)
//                 VALU; each thread keeps its 8 columns of W in registers for a strip of rows.
//   lora_wgrad  : out[k*osk + r*osr] += scale * sum_m X[m, k] Y[m, r]
//                 dA = v^T x, dB = s u^T dy.  MFMA with the X / Y tiles staged row-major in LDS
//                 and read transposed (ds_read_b64_tr_b16); one fp32 atomic per output element
//                 per 512-row chunk straight into the flat grad buffer (accumulation semantics).
//   lora_merge  : W[k, n] += s * sum_r A[r, k] B[r, n]                merge / unmerge (K10)
#include "mfma.h"
#include "kernels.h"

namespace mft {

// ------------------------------------------------------------------------------------ dropout
// PEFT applies dropout to the LoRA input: u = dropout(x) A^T (the reference stored lora_dropout but
// never applied it).  The mask is a counter-based hash of (step counter, layer salt,
// element index): recomputed wherever it is needed (u in forward, dA and the dx term in backward), so
// no mask tensor is ever written.  The step counter lives on the device (graph-replay safe).
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352dU;
  h ^= h >> 15;
  h *= 0x846ca68bU;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ float drop_mult(const LoraDrop& d, uint32_t seed, long m, int k, int K) {
  const uint64_t idx = (uint64_t)m * (uint64_t)K + (uint64_t)k;
  const uint32_t h = mix32((uint32_t)idx ^ mix32((uint32_t)(idx >> 32) ^ seed));
  return ((h >> 8) * (1.0f / 16777216.0f)) >= d.p ? 1.0f / (1.0f - d.p) : 0.0f;
}
__device__ __forceinline__ uint32_t drop_seed(const LoraDrop& d) {
  return mix32(d.salt * 0x9E3779B9U ^ (uint32_t)(d.ctr ? *d.ctr : 0) * 0x85EBCA6BU);
}
__device__ __forceinline__ bf16x8_t apply_drop8(bf16x8_t a, const LoraDrop& d, uint32_t seed, long m, int k, int K) {
  u16x8_t v = __builtin_bit_cast(u16x8_t, a);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) * drop_mult(d, seed, m, k + j, K));
  return __builtin_bit_cast(bf16x8_t, v);
}

// ------------------------------------------------------------------------------------ rowdot
// block = 4 waves; rows [16*blockIdx.x, +16); wave w handles k in [w*Kq, (w+1)*Kq).
// Each 16-col output tile covers ranks [16*t, 16*t+16) of R (RT tiles).
template <int RT>
__global__ __launch_bounds__(256) void lora_rowdot_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ Wt,
                                                          long ldw, bf16_t* __restrict__ U, long ldu, long M, int K, int R,
                                                          float s, LoraDrop drop) {
  __shared__ __attribute__((aligned(16))) float red[4][RT][64][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t dseed = drop.p > 0.f ? drop_seed(drop) : 0u;
  const long m0 = (long)blockIdx.x * 16;
  const long mr = m0 + (lane & 15);
  const bool row_ok = mr < M;
  const int nks = K / 32;
  const int per = (nks + 3) / 4;
  const int ks0 = w * per, ks1 = min(nks, ks0 + per);
  f32x4_t acc[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) acc[t] = zero4();
  for (int ks = ks0; ks < ks1; ++ks) {
    const int k = ks * 32 + 8 * (lane >> 4);
    bf16x8_t a = row_ok ? *reinterpret_cast<const bf16x8_t*>(X + mr * ldx + k) : bf16x8_t{};
    if (drop.p > 0.f) a = apply_drop8(a, drop, dseed, mr, k, K);
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const int r = t * 16 + (lane & 15);
      bf16x8_t b = r < R ? *reinterpret_cast<const bf16x8_t*>(Wt + (long)r * ldw + k) : bf16x8_t{};
      acc[t] = mfma16(a, b, acc[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w][t][lane][i] = acc[t][i];
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = red[0][t][lane][i] + red[1][t][lane][i] + red[2][t][lane][i] + red[3][t][lane][i];
        const long m = m0 + 4 * (lane >> 4) + i;
        const int r = t * 16 + (lane & 15);
        if (m < M && r < R) U[m * ldu + r] = f2bf(v * s);
      }
    }
  }
}

// ------------------------------------------------------------------------------------ update
// grid (ceil(N/8/blockDim), ceil(M/ROWS)); thread owns 8 columns, W[0..R)[n..n+8) in registers.
// With dropout (dx += mask * (v A) in backward) the mask of element (m, n) is re-derived.
template <int R>
__global__ __launch_bounds__(256) void lora_update_kernel(const bf16_t* base, long ldb, const bf16_t* __restrict__ U, long ldu,
                                                          const bf16_t* __restrict__ W, long ldw, bf16_t* Y, long ldy, long M,
                                                          int N, int rows, float s, LoraDrop drop) {
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (n >= N) return;
  const uint32_t dseed = drop.p > 0.f ? drop_seed(drop) : 0u;
  float wr[R][8];
#pragma unroll
  for (int r = 0; r < R; ++r) load8(W + (long)r * ldw + n, wr[r]);
  const long m0 = (long)blockIdx.y * rows;
  const long m1 = min(M, m0 + rows);
  for (long m = m0; m < m1; ++m) {
    float y[8], u[R], d[8];
    load8(base + m * ldb + n, y);
#pragma unroll
    for (int r = 0; r < R; ++r) u[r] = bf2f(U[m * ldu + r]) * s;
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] += u[r] * wr[r][j];
    if (drop.p > 0.f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] *= drop_mult(drop, dseed, m, n + j, N);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] += d[j];
    store8(Y + m * ldy + n, y);
  }
}

// ------------------------------------------------------------------------------------ wgrad
// Streaming VALU form (the reduction runs over M, the long axis; each X row is read once).
// block = 256 threads = 64 column-chunks of 8 x 4 row groups; each thread accumulates an 8 x RB
// fp32 outer-product tile over its rows; the 4 row groups are summed in LDS and one fp32 atomic per
// output element per block goes straight into the grad buffer.  RB <= 8 ranks per z-block.
template <int RB>
__global__ __launch_bounds__(256) void lora_wgrad_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ Y,
                                                         long ldy, float* __restrict__ out, long osk, long osr, long M, int K,
                                                         int R, long chunk, float scale, LoraDrop drop) {
  __shared__ __attribute__((aligned(16))) float red[3][64][8 * RB + 1];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int k = (blockIdx.x * 64 + c) * 8;
  const int r0 = blockIdx.z * RB;
  const long mbeg = (long)blockIdx.y * chunk;
  const long mend = min(M, mbeg + chunk);
  const bool kok = k < K;
  const uint32_t dseed = drop.p > 0.f ? drop_seed(drop) : 0u;
  float acc[8][RB];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[j][r] = 0.f;
#pragma unroll 2
  for (long m = mbeg + g; m < mend; m += 4) {
    float xv[8], yv[RB];
    if (kok) {
      load8(X + m * ldx + k, xv);
      if (drop.p > 0.f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j] *= drop_mult(drop, dseed, m, k + j, K);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[j] = 0.f;
    }
    const bf16_t* yr = Y + m * ldy + r0;  // wave-uniform address: one broadcast request
#pragma unroll
    for (int r = 0; r < RB; ++r) yv[r] = (r0 + r < R) ? bf2f(yr[r]) : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < RB; ++r) acc[j][r] += xv[j] * yv[r];
  }
  if (g > 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < RB; ++r) red[g - 1][c][j * RB + r] = acc[j][r];
  }
  __syncthreads();
  if (g == 0 && kok) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        if (r0 + r >= R) continue;
        const float v = acc[j][r] + red[0][c][j * RB + r] + red[1][c][j * RB + r] + red[2][c][j * RB + r];
        atomicAdd(out + (long)(k + j) * osk + (long)(r0 + r) * osr, v * scale);
      }
  }
}

template <typename T>
__global__ void lora_merge_kernel(T* W, long wsk, long wsn, const float* __restrict__ A, const float* __restrict__ B, int K,
                                  int N, int R, float s) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)K * N) return;
  const int k = t / N, n = t % N;
  float acc = 0.f;
  for (int r = 0; r < R; ++r) acc += A[(long)r * K + k] * B[(long)r * N + n];
  T* p = W + k * wsk + n * wsn;
  if constexpr (sizeof(T) == 2) {
    *p = f2bf(bf2f(*p) + s * acc);
  } else {
    *p = *p + s * acc;
  }
}

void lora_rowdot(const bf16_t* X, long ldx, const bf16_t* Wt, long ldw, bf16_t* U, long ldu, long M, int K, int R, float s,
                 LoraDrop drop, hipStream_t st) {
  const int grid = cdiv(M, 16);
  if (R <= 16) lora_rowdot_kernel<1><<<grid, 256, 0, st>>>(X, ldx, Wt, ldw, U, ldu, M, K, R, s, drop);
  else if (R <= 32) lora_rowdot_kernel<2><<<grid, 256, 0, st>>>(X, ldx, Wt, ldw, U, ldu, M, K, R, s, drop);
  else lora_rowdot_kernel<4><<<grid, 256, 0, st>>>(X, ldx, Wt, ldw, U, ldu, M, K, R, s, drop);
}

void lora_update(const bf16_t* base, long ldb, const bf16_t* U, long ldu, const bf16_t* W, long ldw, bf16_t* Y, long ldy,
                 long M, int N, int R, float s, LoraDrop drop, hipStream_t st) {
  const int nthreads_x = (N / 8 + 63) / 64 * 64;
  const int bx = nthreads_x < 256 ? nthreads_x : 256;
  const int gx = cdiv(N / 8, bx);
  // ~2k blocks in total, at least 16 rows per block to amortise the W register load
  long rows = (M * gx + 2047) / 2048;
  if (rows < 16) rows = 16;
  dim3 grid(gx, (unsigned)cdiv(M, rows));
  switch (R) {
#define MFT_UPD(RV) case RV: lora_update_kernel<RV><<<grid, bx, 0, st>>>(base, ldb, U, ldu, W, ldw, Y, ldy, M, N, (int)rows, s, drop); break;
    MFT_UPD(1) MFT_UPD(2) MFT_UPD(4) MFT_UPD(8) MFT_UPD(16)
#undef MFT_UPD
    default: {
      // larger ranks: apply in slices of 16 (in place after the first)
      for (int r0 = 0; r0 < R; r0 += 16) {
        const int rr = R - r0 < 16 ? R - r0 : 16;
        if (rr != 16) { fprintf(stderr, "lora_update: rank %d must be a multiple of 16 above 16\n", R); abort(); }
        lora_update_kernel<16><<<grid, bx, 0, st>>>(r0 == 0 ? base : Y, r0 == 0 ? ldb : ldy, U + r0, ldu,
                                                     W + (long)r0 * ldw, ldw, Y, ldy, M, N, (int)rows, s, drop);
      }
    }
  }
}

void lora_wgrad(const bf16_t* X, long ldx, const bf16_t* Y, long ldy, float* out, long osk, long osr, long M, int K, int R,
                float scale, LoraDrop drop, hipStream_t st) {
  const int rb = R <= 1 ? 1 : R <= 2 ? 2 : R <= 4 ? 4 : 8;
  const int gx = cdiv(K, 512);
  const int gz = cdiv(R, rb);
  // ~1k blocks; each block's 4 row groups stream >= 64 rows each
  long chunks = 1024 / (gx * gz);
  if (chunks < 1) chunks = 1;
  long chunk = (M + chunks - 1) / chunks;
  if (chunk < 256) chunk = 256;
  dim3 grid(gx, (unsigned)cdiv(M, chunk), gz);
  switch (rb) {
    case 1: lora_wgrad_kernel<1><<<grid, 256, 0, st>>>(X, ldx, Y, ldy, out, osk, osr, M, K, R, chunk, scale, drop); break;
    case 2: lora_wgrad_kernel<2><<<grid, 256, 0, st>>>(X, ldx, Y, ldy, out, osk, osr, M, K, R, chunk, scale, drop); break;
    case 4: lora_wgrad_kernel<4><<<grid, 256, 0, st>>>(X, ldx, Y, ldy, out, osk, osr, M, K, R, chunk, scale, drop); break;
    default: lora_wgrad_kernel<8><<<grid, 256, 0, st>>>(X, ldx, Y, ldy, out, osk, osr, M, K, R, chunk, scale, drop); break;
  }
}

void lora_merge(void* W, int w_is_bf16, long wsk, long wsn, const float* A, const float* B, int K, int N, int R, float s,
                hipStream_t st) {
  const long n = (long)K * N;
  if (w_is_bf16)
    lora_merge_kernel<bf16_t><<<cdiv(n, 256), 256, 0, st>>>((bf16_t*)W, wsk, wsn, A, B, K, N, R, s);
  else
    lora_merge_kernel<float><<<cdiv(n, 256), 256, 0, st>>>((float*)W, wsk, wsn, A, B, K, N, R, s);
}

}  // namespace mft
