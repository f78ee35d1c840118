// Small vectorised elementwise kernels: fp32<->bf16 casts (offload quantisation, master->shadow
// copies; replaces ops::cast core/ops.cpp:2705-2745 and the sharder's software fp16 conversion
// opt_ops/sharding/parameter_sharder.cpp:21-76), device-scalar scaling (loss / accumulation
// scaling without host sync), and residual adds.
#include "common.h"
#include "kernels.h"

namespace mft {

static inline int grid_for(long n8) {
  long g = (n8 + 255) / 256;
  return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const float4* x4 = reinterpret_cast<const float4*>(x + i * 8);
    float4 a = x4[0], b = x4[1];
    float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    store8(y + i * 8, f);
  }
  if (blockIdx.x == 0)
    for (long i = n8 * 8 + threadIdx.x; i < n; i += blockDim.x) y[i] = f2bf(x[i]);
}

__global__ void cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long n) {
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float f[8];
    load8(x + i * 8, f);
    float4* y4 = reinterpret_cast<float4*>(y + i * 8);
    y4[0] = make_float4(f[0], f[1], f[2], f[3]);
    y4[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
  if (blockIdx.x == 0)
    for (long i = n8 * 8 + threadIdx.x; i < n; i += blockDim.x) y[i] = bf2f(x[i]);
}

__global__ void scale_bf16_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long n,
                                  const float* __restrict__ sdev, float s) {
  const float sc = (sdev ? *sdev : 1.f) * s;
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float f[8];
    load8(x + i * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= sc;
    store8(y + i * 8, f);
  }
  if (blockIdx.x == 0)
    for (long i = n8 * 8 + threadIdx.x; i < n; i += blockDim.x) y[i] = f2bf(bf2f(x[i]) * sc);
}

__global__ void add_bf16_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, bf16_t* __restrict__ y, long n) {
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float f[8], g[8];
    load8(a + i * 8, f);
    load8(b + i * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] += g[j];
    store8(y + i * 8, f);
  }
  if (blockIdx.x == 0)
    for (long i = n8 * 8 + threadIdx.x; i < n; i += blockDim.x) y[i] = f2bf(bf2f(a[i]) + bf2f(b[i]));
}

void cast_f32_bf16(const float* x, bf16_t* y, long n, hipStream_t st) {
  cast_f32_bf16_kernel<<<grid_for(n / 8), 256, 0, st>>>(x, y, n);
}
void cast_bf16_f32(const bf16_t* x, float* y, long n, hipStream_t st) {
  cast_bf16_f32_kernel<<<grid_for(n / 8), 256, 0, st>>>(x, y, n);
}
// zero columns [c0, c0 + 8 * nch) of every row (16-B stores; the padding of augmented LoRA inputs)
__global__ void zero_cols_kernel(bf16_t* __restrict__ p, long ld, long M, int c0, int nch) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * nch) return;
  const long row = t / nch;
  const int ch = (int)(t % nch);
  *reinterpret_cast<u16x8_t*>(p + row * ld + c0 + ch * 8) = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
}

// part[blockIdx.y][n] = sum over this block's rows of x[m, n]  (bias gradients; 32 x 8-column chunks x
// 8 row lanes per block, combined through LDS; finished by reduce_rows)
__global__ __launch_bounds__(256) void colsum_partial_kernel(const bf16_t* __restrict__ x, long ld, long M, int N,
                                                             long rows_per_block, float* __restrict__ part) {
  __shared__ float red[8][32 * 8 + 1];
  const int cc = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int n = (blockIdx.x * 32 + cc) * 8;
  const long m0 = (long)blockIdx.y * rows_per_block, m1 = min(M, m0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (n < N) {
    // eight independent 16-B loads in flight per thread (one at a time left the pass latency-bound at
    // ~4.6 TB/s: ~1.5 MB in flight across the chip; the row-block count stays small for reduce_rows)
    long m = m0 + rl;
    for (; m + 56 < m1; m += 64) {
      u16x8_t q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] = *reinterpret_cast<const u16x8_t*>(x + (m + 8 * u) * ld + n);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(q[u][j]);
    }
    for (; m < m1; m += 8) {
      float v[8];
      load8(x + m * ld + n, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cc * 8 + j] = acc[j];
  __syncthreads();
  for (int t = threadIdx.x; t < 256; t += 256) {
    const int col = blockIdx.x * 256 + t;
    if (col < N) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += red[k][t];
      part[(long)blockIdx.y * N + col] = s;
    }
  }
}

int colsum_partial_blocks(long M) {
  const long nb = (M + 255) / 256;
  return (int)(nb < 128 ? nb : 128);
}

void colsum_partial(const bf16_t* x, long ld, long M, int N, float* part, hipStream_t st) {
  const int nb = colsum_partial_blocks(M);
  const long rows = (M + nb - 1) / nb;
  colsum_partial_kernel<<<dim3(cdiv(N, 256), nb), 256, 0, st>>>(x, ld, M, N, rows, part);
}

void zero_cols(bf16_t* p, long ld, long M, int c0, int ncols, hipStream_t st) {
  const int nch = ncols / 8;
  if (M <= 0 || nch <= 0) return;
  zero_cols_kernel<<<cdiv(M * nch, 256), 256, 0, st>>>(p, ld, M, c0, nch);
}

void scale_bf16(const bf16_t* x, bf16_t* y, long n, const float* scale_dev, float scale, hipStream_t st) {
  scale_bf16_kernel<<<grid_for(n / 8), 256, 0, st>>>(x, y, n, scale_dev, scale);
}
void add_bf16(const bf16_t* a, const bf16_t* b, bf16_t* y, long n, hipStream_t st) {
  add_bf16_kernel<<<grid_for(n / 8), 256, 0, st>>>(a, b, y, n);
}

}  // namespace mft
