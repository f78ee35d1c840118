// Activation kernels: GELU(tanh) and gated GeGLU / SwiGLU, forward + backward.
// Replaces ops::gelu / ops::swiglu and GeluBackward / SwiGLUBackward
// (core/ops.cpp:1055-1079, :2227-2263; core/backward_functions.cpp:155-177, :268-286) and the
// Gemma MLP composite gelu(gate)*up (graph/gemma_model.cpp:538-546).
// Memory-bound: 16-B vector loads/stores (8 x bf16 per lane), grid-stride, capped grid.
#include "common.h"
#include "kernels.h"

namespace mft {

static inline int ew_grid(long n8) {
  long g = (n8 + 255) / 256;
  return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
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

template <int ACT>
__global__ void gated_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ y, long M, int I, long ldy) {
  const int c8 = I / 8;
  const long n8 = M * c8;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += (long)gridDim.x * blockDim.x) {
    const long m = t / c8;
    const int c = (int)(t % c8) * 8;
    float g[8], u[8];
    load8(gu + m * 2 * I + c, g);
    load8(gu + m * 2 * I + I + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = (ACT == 0 ? gelu_tanh(g[j]) : silu(g[j])) * u[j];
    store8(y + m * ldy + c, g);
  }
}

template <int ACT>
__global__ void gated_bwd_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dy, bf16_t* __restrict__ dgu,
                                 long M, int I, long ldd) {
  const int c8 = I / 8;
  const long n8 = M * c8;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += (long)gridDim.x * blockDim.x) {
    const long m = t / c8;
    const int c = (int)(t % c8) * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    load8(gu + m * 2 * I + c, g);
    load8(gu + m * 2 * I + I + c, u);
    load8(dy + m * ldd + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = ACT == 0 ? gelu_tanh(g[j]) : silu(g[j]);
      const float ag = ACT == 0 ? gelu_tanh_grad(g[j]) : silu_grad(g[j]);
      du[j] = d[j] * a;
      dg[j] = d[j] * u[j] * ag;
    }
    store8(dgu + m * 2 * I + c, dg);
    store8(dgu + m * 2 * I + I + c, du);
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
void gated_fwd(const bf16_t* gu, bf16_t* y, long M, int I, long ldy, int act, hipStream_t st) {
  const int g = ew_grid(M * (I / 8));
  if (act == 0) gated_fwd_kernel<0><<<g, 256, 0, st>>>(gu, y, M, I, ldy);
  else gated_fwd_kernel<1><<<g, 256, 0, st>>>(gu, y, M, I, ldy);
}
void gated_bwd(const bf16_t* gu, const bf16_t* dy, long ldd, bf16_t* dgu, long M, int I, int act, hipStream_t st) {
  const int g = ew_grid(M * (I / 8));
  if (act == 0) gated_bwd_kernel<0><<<g, 256, 0, st>>>(gu, dy, dgu, M, I, ldd);
  else gated_bwd_kernel<1><<<g, 256, 0, st>>>(gu, dy, dgu, M, I, ldd);
}

}  // namespace mft
