// LoRA rank-r kernels (r <= 64): the skinny products around the frozen base GEMM.
//
// Replaces LoRALinear::forward/merge/unmerge (nn/lora_linear.cpp:47-178), whose partial-column
// slices were added without autograd, and the never-constructed
// LoRALinearBackward (core/backward_functions.cpp:1012-1226).
//
// For y = x W (+b) + s (x A) B with W frozen, the base GEMM runs on hipBLASLt and these kernels
// do the rank-r work:
//   lora_rowdot : u[m, r] = s * sum_k X[m, k] W[k, r]           (x A  and  s * dy B^T)
//   lora_update : Y[m, n] = base[m, n] (+ bias[n]) + s * sum_r U[m, r] W[r, n]
//                 (forward epilogue y = base + b + s u B, and dx += v A^T in backward; in place)
//   lora_wgrad  : out[k, r] += scale * sum_m X[m, k] Y[m, r]    (dA = x^T v, dB = s u^T dy),
//                 accumulated straight into the fp32 flat grad buffer with atomics (grad
//                 accumulation semantics).
//   lora_merge  : W[k, n] += s * sum_r A[k, r] B[r, n]           (merge / unmerge, K10)
// All row-streaming kernels use 16-B vector loads; the rank-r factor is tiny and L1/L2 resident.
#include "common.h"
#include "kernels.h"

namespace mft {

// one wave per row m; lanes stride over 8-wide k chunks; R partial sums per lane, wave-reduced.
template <int R>
__global__ __launch_bounds__(256) void lora_rowdot_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W,
                                                          long wsk, long wsr, bf16_t* __restrict__ U, long ldu, long M,
                                                          int K, float s) {
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (m >= M) return;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.f;
  for (int k = lane * 8; k < K; k += 512) {
    float xv[8];
    load8(X + m * ldx + k, xv);
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] += xv[j] * bf2f(W[(k + j) * wsk + r * wsr]);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (lane < R) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (lane == r) v = acc[r];
    U[m * ldu + lane] = f2bf(v * s);
  }
}

template <int R>
__global__ __launch_bounds__(256) void lora_update_kernel(const bf16_t* base, long ldb, const float* __restrict__ bias,
                                                          const bf16_t* __restrict__ U, long ldu, const bf16_t* __restrict__ W,
                                                          long wsr, long wsn, bf16_t* Y, long ldy, long M, int N, float s) {
  const int c8 = N / 8;
  const long total = M * c8;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const long m = t / c8;
    const int n = (int)(t % c8) * 8;
    float y[8], u[R];
    load8(base + m * ldb + n, y);
#pragma unroll
    for (int r = 0; r < R; ++r) u[r] = bf2f(U[m * ldu + r]) * s;
    if (bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] += bias[n + j];
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] += u[r] * bf2f(W[r * wsr + (n + j) * wsn]);
    store8(Y + m * ldy + n, y);
  }
}

// grid: (K/8/64 column groups, Mchunks); one thread = 8 columns k, R outputs each.
template <int R>
__global__ __launch_bounds__(64) void lora_wgrad_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ Y,
                                                        long ldy, float* __restrict__ out, long osk, long osr, long M, int K,
                                                        long rows_per_chunk, float scale) {
  const int k = (blockIdx.x * 64 + threadIdx.x) * 8;
  if (k >= K) return;
  const long m0 = blockIdx.y * rows_per_chunk;
  const int r0 = blockIdx.z * R;  // rank columns handled by this block
  Y += r0;
  out += r0 * osr;
  const long m1 = min(M, m0 + rows_per_chunk);
  float acc[8][R];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[j][r] = 0.f;
  for (long m = m0; m < m1; ++m) {
    float xv[8], yv[R];
    load8(X + m * ldx + k, xv);
#pragma unroll
    for (int r = 0; r < R; ++r) yv[r] = bf2f(Y[m * ldy + r]);
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[j][r] += xv[j] * yv[r];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int r = 0; r < R; ++r) atomicAdd(out + (k + j) * osk + r * osr, acc[j][r] * scale);
}

template <typename T>
__global__ void lora_merge_kernel(T* W, long wsk, long wsn, const float* __restrict__ A, const float* __restrict__ B, int K,
                                  int N, int R, float s) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)K * N) return;
  const int k = t / N, n = t % N;
  float acc = 0.f;
  for (int r = 0; r < R; ++r) acc += A[(long)k * R + r] * B[(long)r * N + n];
  T* p = W + k * wsk + n * wsn;
  if constexpr (sizeof(T) == 2) {
    *p = f2bf(bf2f(*p) + s * acc);
  } else {
    *p = *p + s * acc;
  }
}

#define MFT_RANK_DISPATCH(R, ...)                                                  \
  switch (R) {                                                                     \
    case 1: { constexpr int RR = 1; __VA_ARGS__; } break;                          \
    case 2: { constexpr int RR = 2; __VA_ARGS__; } break;                          \
    case 4: { constexpr int RR = 4; __VA_ARGS__; } break;                          \
    case 8: { constexpr int RR = 8; __VA_ARGS__; } break;                          \
    case 16: { constexpr int RR = 16; __VA_ARGS__; } break;                        \
    case 32: { constexpr int RR = 32; __VA_ARGS__; } break;                        \
    case 64: { constexpr int RR = 64; __VA_ARGS__; } break;                        \
    default: fprintf(stderr, "lora: unsupported rank %d (use 1,2,4,8,16,32,64)\n", R); abort(); \
  }

void lora_rowdot(const bf16_t* X, long ldx, const bf16_t* W, long wsk, long wsr, bf16_t* U, long ldu, long M, int K,
                 int R, float s, hipStream_t st) {
  MFT_RANK_DISPATCH(R, lora_rowdot_kernel<RR><<<cdiv(M, 4), 256, 0, st>>>(X, ldx, W, wsk, wsr, U, ldu, M, K, s));
}

void lora_update(const bf16_t* base, long ldb, const float* bias, const bf16_t* U, long ldu, const bf16_t* W, long wsr,
                 long wsn, bf16_t* Y, long ldy, long M, int N, int R, float s, hipStream_t st) {
  long g = (M * (N / 8) + 255) / 256;
  const int grid = (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
  MFT_RANK_DISPATCH(R, lora_update_kernel<RR><<<grid, 256, 0, st>>>(base, ldb, bias, U, ldu, W, wsr, wsn, Y, ldy, M, N, s));
}

void lora_wgrad(const bf16_t* X, long ldx, const bf16_t* Y, long ldy, float* out, long osk, long osr, long M, int K, int R,
                float scale, hipStream_t st) {
  const int gx = cdiv(K / 8, 64);
  // enough M-chunks for ~1k blocks, but at least 64 rows per chunk to amortise the atomics
  long chunks = 1024 / gx;
  if (chunks < 1) chunks = 1;
  long rows = (M + chunks - 1) / chunks;
  if (rows < 64) rows = 64;
  chunks = (M + rows - 1) / rows;
  const int rb = R < 8 ? R : 8;  // <= 64 fp32 accumulators per thread
  dim3 grid(gx, (unsigned)chunks, R / rb);
  MFT_RANK_DISPATCH(rb, lora_wgrad_kernel<RR><<<grid, 64, 0, st>>>(X, ldx, Y, ldy, out, osk, osr, M, K, rows, scale));
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
