// Activation kernels: GELU(tanh) and gated GeGLU / SwiGLU, forward + backward.
// Replaces ops::gelu / ops::swiglu and GeluBackward / SwiGLUBackward
// (core/ops.cpp:1055-1079, :2227-2263; core/backward_functions.cpp:155-177, :268-286) and the
// Gemma MLP composite gelu(gate)*up (graph/gemma_model.cpp:538-546).
// Memory-bound: 16-B vector loads/stores (8 x bf16 per lane), grid-stride, capped grid.
#include "common.h"
#include "kernels.h"

#include <cstdio>

namespace mft {

static inline int ew_grid(long n8) {
  long g = (n8 + 255) / 256;
  return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

// one block per row pair, capped at 16,384 blocks (64 per CU)
static inline int gated_grid(long M) {
  const long g = (M + 1) / 2;
  return (int)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float silu_grad(float x) {
  float s = 1.f / (1.f + __expf(-x));
  return s * (1.f + x * (1.f - s));
}

__global__ void gelu_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long n) {
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_tanh(v[j]);
    store8(y + i * 8, v);
  }
  if (blockIdx.x == 0)
    for (long i = n8 * 8 + threadIdx.x; i < n; i += blockDim.x) y[i] = f2bf(gelu_tanh(bf2f(x[i])));
}

__global__ void gelu_bwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                long n) {
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float v[8], g[8];
    load8(x + i * 8, v);
    load8(dy + i * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = g[j] * gelu_tanh_grad(v[j]);
    store8(dx + i * 8, v);
  }
  if (blockIdx.x == 0)
    for (long i = n8 * 8 + threadIdx.x; i < n; i += blockDim.x) dx[i] = f2bf(bf2f(dy[i]) * gelu_tanh_grad(bf2f(x[i])));
}

// Gated kernels: a block walks whole rows (blockIdx.x, stride gridDim.x) and its threads stride the row's
// 8-column groups, so no 64-bit division per element; two rows' loads are issued before either is used
// (3 x 16 B per lane in flight in the forward, 6 in the backward).
template <int ACT>
__global__ void gated_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ y, long M, int I, long ldy,
                                 int zpad) {
  for (long m0 = 2L * blockIdx.x; m0 < M; m0 += 2L * gridDim.x) {
    const bool two = m0 + 1 < M;
    for (int c = I + threadIdx.x * 8; c < I + zpad; c += blockDim.x * 8) {  // the widened output's zero columns
      *reinterpret_cast<uint4*>(y + m0 * ldy + c) = uint4{0u, 0u, 0u, 0u};
      if (two) *reinterpret_cast<uint4*>(y + (m0 + 1) * ldy + c) = uint4{0u, 0u, 0u, 0u};
    }
    for (int c = threadIdx.x * 8; c < I; c += blockDim.x * 8) {
      float g[2][8], u[2][8];
      load8(gu + m0 * 2 * I + c, g[0]);
      load8(gu + m0 * 2 * I + I + c, u[0]);
      if (two) {
        load8(gu + (m0 + 1) * 2 * I + c, g[1]);
        load8(gu + (m0 + 1) * 2 * I + I + c, u[1]);
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        if (r == 1 && !two) break;
#pragma unroll
        for (int j = 0; j < 8; ++j) g[r][j] = (ACT == 0 ? gelu_tanh(g[r][j]) : silu(g[r][j])) * u[r][j];
        store8(y + (m0 + r) * ldy + c, g[r]);
      }
    }
  }
}

template <int ACT>
__global__ void gated_bwd_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dy, bf16_t* __restrict__ dgu,
                                 long M, int I, long ldd) {
  for (long m0 = 2L * blockIdx.x; m0 < M; m0 += 2L * gridDim.x) {
    const bool two = m0 + 1 < M;
    for (int c = threadIdx.x * 8; c < I; c += blockDim.x * 8) {
      float g[2][8], u[2][8], d[2][8];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        if (r == 1 && !two) break;
        load8(gu + (m0 + r) * 2 * I + c, g[r]);
        load8(gu + (m0 + r) * 2 * I + I + c, u[r]);
        load8(dy + (m0 + r) * ldd + c, d[r]);
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        if (r == 1 && !two) break;
        float dg[8], du[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = ACT == 0 ? gelu_tanh(g[r][j]) : silu(g[r][j]);
          const float ag = ACT == 0 ? gelu_tanh_grad(g[r][j]) : silu_grad(g[r][j]);
          du[j] = d[r][j] * a;
          dg[j] = d[r][j] * u[r][j] * ag;
        }
        store8(dgu + (m0 + r) * 2 * I + c, dg);
        store8(dgu + (m0 + r) * 2 * I + I + c, du);
      }
    }
  }
}

void gelu_fwd(const bf16_t* x, bf16_t* y, long n, hipStream_t st) {
  gelu_fwd_kernel<<<ew_grid(n / 8), 256, 0, st>>>(x, y, n);
}
void gelu_bwd(const bf16_t* x, const bf16_t* dy, bf16_t* dx, long n, hipStream_t st) {
  gelu_bwd_kernel<<<ew_grid(n / 8), 256, 0, st>>>(x, dy, dx, n);
}
// ldy / ldd: row strides of y / dy (> I when y is the widened augmented-K input of a LoRA
// consumer, see bindings.cpp alloc_wide)
void gated_fwd(const bf16_t* gu, bf16_t* y, long M, int I, long ldy, int act, hipStream_t st, int zpad) {
  const int g = gated_grid(M);
  if (zpad % 8 || I + zpad > ldy || I % 8) {
    fprintf(stderr, "gated_fwd: zero padding %d after %d columns does not fit the row stride %ld\n", zpad, I, ldy);
    abort();
  }
  if (act == 0) gated_fwd_kernel<0><<<g, 256, 0, st>>>(gu, y, M, I, ldy, zpad);
  else gated_fwd_kernel<1><<<g, 256, 0, st>>>(gu, y, M, I, ldy, zpad);
}
void gated_bwd(const bf16_t* gu, const bf16_t* dy, long ldd, bf16_t* dgu, long M, int I, int act, hipStream_t st) {
  const int g = gated_grid(M);
  if (act == 0) gated_bwd_kernel<0><<<g, 256, 0, st>>>(gu, dy, dgu, M, I, ldd);
  else gated_bwd_kernel<1><<<g, 256, 0, st>>>(gu, dy, dgu, M, I, ldd);
}

}  // namespace mft
