// Shared device helpers for the gfx950 (CDNA4) kernels of mobilefinetuner_amd.
//
// Conventions used by every kernel in csrc/kernels:
//  * bf16 tensors are passed as raw uint16_t storage; math is done in fp32.
//  * wave64 everywhere (block sizes are multiples of 64, reductions use 64-lane shuffles).
//  * global loads/stores of bf16 are vectorised to 16 B per lane (8 x bf16) whenever the
//    row length allows it (Guideline 13 of the CDNA HIP guide).
//  * every launcher takes an explicit hipStream_t and never allocates or synchronises, so the
//    whole training step can be captured into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace mft {

typedef uint16_t bf16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8_t __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4_t __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);  // RNE; lowers to v_cvt_pk_bf16_f32 on gfx950
  return __bfloat16_as_ushort(h);
}

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (any multiple of 64). `smem` needs >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += smem[i];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, smem[i]);
  return r;
}

__device__ __forceinline__ void load8(const bf16_t* p, float* f) {
  u16x8_t v = *reinterpret_cast<const u16x8_t*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = bf2f(v[j]);
}

__device__ __forceinline__ void store8(bf16_t* p, const float* f) {
  u16x8_t v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(f[j]);
  *reinterpret_cast<u16x8_t*>(p) = v;
}

// store8 with the non-temporal hint (a streaming output nothing re-reads soon: keep it out of the caches)
__device__ __forceinline__ void store8_nt(bf16_t* p, const float* f) {
  u16x8_t v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(f[j]);
  __builtin_nontemporal_store(v, reinterpret_cast<u16x8_t*>(p));
}

// XCD-aware bijective remap of a 1-D block id (CDNA HIP guide §5 "XCD swizzle must be bijective"):
// consecutive logical tiles land on the same XCD (same L2) instead of being dealt round-robin.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// 2^x as ONE v_exp_f32.  exp2f() expands to a denormal-safe sequence (compare, select, add, exp,
// select, ldexp: ~6 VALU ops + hazard nops per element), which dominated the CE forward epilogue
// and the softmax of the attention kernels.  Every caller feeds x <= 0 (value minus a running or
// final max) or -inf: results below 2^-126 flush to 0, which a softmax sum cannot see.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// GELU (tanh form, GPT-2 "gelu_new") via 0.5 (1 + tanh(u)) = sigmoid(2u): one v_exp_f32 and one
// v_rcp_f32 instead of a libm tanhf (which dominated the fused GEMM epilogues).  Saturates
// correctly: exp -> inf gives sigmoid 0, exp -> 0 gives 1.
__device__ __forceinline__ float sigmoid_fast(float z) { return __builtin_amdgcn_rcpf(1.f + __expf(-z)); }

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  return x * sigmoid_fast(2.f * u);
}

// GELU(x) and GELU'(x) from one sigmoid
__device__ __forceinline__ void gelu_tanh_and_grad(float x, float& y, float& dy) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float s = sigmoid_fast(2.f * k0 * (x + k1 * x2 * x));
  y = x * s;
  dy = s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x2);
}

// Two elements at once in packed fp32 (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32 on gfx950: two lanes'
// worth per instruction), the constants folded: 10 packed ops + 2 v_exp_f32 + 2 v_rcp_f32 per pair
// instead of ~14 scalar ops + 2 transcendentals per element -- the GELU epilogue of the fused MLP GEMM
// was VALU-bound at one wave per SIMD (as many cycles as the tile's MFMAs).
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gelu_tanh_and_grad2(f32x2_t x, f32x2_t& y, f32x2_t& dy) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f, l2e = 1.4426950408889634f;
  const f32x2_t x2 = x * x;
  const f32x2_t in = __builtin_elementwise_fma(x2 * k1, x, x);       // x + k1 x^3
  const f32x2_t z = in * (-2.f * k0 * l2e);                            // -2u log2(e)
  const f32x2_t d = f32x2_t{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)} + 1.f;
  const f32x2_t s = f32x2_t{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};  // sigmoid(2u)
  y = x * s;
  const f32x2_t t = __builtin_elementwise_fma(-s, s, s);              // s (1 - s)
  const f32x2_t q = __builtin_elementwise_fma(x2, f32x2_t{6.f * k0 * k1, 6.f * k0 * k1}, f32x2_t{2.f * k0, 2.f * k0});
  dy = __builtin_elementwise_fma(x * t, q, s);                         // s + 2 k0 x s (1-s) (1 + 3 k1 x^2)
}

// d/dx: s + 2 x s (1 - s) k0 (1 + 3 k1 x^2), s = sigmoid(2u)   (0.5 (1 - tanh^2) = 2 s (1 - s))
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float u = k0 * (x + k1 * x2 * x);
  const float s = sigmoid_fast(2.f * u);
  return s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x2);
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace mft

#define MFT_HIP_CHECK(expr)                                                            \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
      abort();                                                                         \
    }                                                                                  \
  } while (0)
