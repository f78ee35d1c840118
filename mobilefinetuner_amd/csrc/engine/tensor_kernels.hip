// libmft engine: generic tensor kernels for gfx950 (see engine/kernels.h).
//
// These replace the reference's scalar CPU loops of core/ops.cpp (elementwise_binary_op :167-244
// with its per-element std::vector index on the broadcast path, unary math :1033-2651, softmax
// :1119-1230, reductions :1782-1939, dropout :2670-2704, casts :2705-2745).  Design: one grid-stride
// kernel per family; contiguous operands take a vectorised fast path (16 B per lane), strided /
// broadcast ones decompose the linear index over at most 8 dims (index math in 64-bit, strides 0 for
// broadcast).  Math is fp32 whatever the storage dtype.  Row kernels use one wave64 per row.
#include <hip/hip_fp16.h>
#include <math.h>

#include "common.h"
#include "engine/tensor_kernels.h"

namespace mft {
namespace eng {
namespace k {

namespace {

__device__ __forceinline__ float ld(const void* p, int dt, int64_t i) {
  switch (dt) {
    case F32: return ((const float*)p)[i];
    case BF16: return bf2f(((const uint16_t*)p)[i]);
    case F16: return __half2float(((const __half*)p)[i]);
    case I32: return (float)((const int32_t*)p)[i];
    case I64: return (float)((const int64_t*)p)[i];
    default: return (float)((const uint8_t*)p)[i];
  }
}

__device__ __forceinline__ void st(void* p, int dt, int64_t i, float v) {
  switch (dt) {
    case F32: ((float*)p)[i] = v; break;
    case BF16: ((uint16_t*)p)[i] = f2bf(v); break;
    case F16: ((__half*)p)[i] = __float2half(v); break;
    case I32: ((int32_t*)p)[i] = (int32_t)v; break;
    case I64: ((int64_t*)p)[i] = (int64_t)v; break;
    case BOOL: ((uint8_t*)p)[i] = v != 0.f; break;
    default: ((uint8_t*)p)[i] = (uint8_t)v; break;
  }
}

// exact integer copy path (int64 values do not survive a float round trip)
__device__ __forceinline__ int64_t ldi(const void* p, int dt, int64_t i) {
  switch (dt) {
    case I32: return ((const int32_t*)p)[i];
    case I64: return ((const int64_t*)p)[i];
    case U8:
    case BOOL: return ((const uint8_t*)p)[i];
    default: return (int64_t)ld(p, dt, i);
  }
}
__device__ __forceinline__ void sti(void* p, int dt, int64_t i, int64_t v) {
  switch (dt) {
    case I32: ((int32_t*)p)[i] = (int32_t)v; break;
    case I64: ((int64_t*)p)[i] = v; break;
    case U8: ((uint8_t*)p)[i] = (uint8_t)v; break;
    case BOOL: ((uint8_t*)p)[i] = v != 0; break;
    default: st(p, dt, i, (float)v); break;
  }
}
__device__ __forceinline__ bool is_int(int dt) { return dt == I32 || dt == I64 || dt == U8 || dt == BOOL; }

// element offset of linear index `lin` (row-major over `shape`) in a view with `stride`
__device__ __forceinline__ int64_t offset_of(int64_t lin, int ndim, const int64_t* shape, const int64_t* stride) {
  int64_t off = 0;
  for (int d = ndim - 1; d >= 0; --d) {
    const int64_t s = shape[d];
    const int64_t q = lin / s;
    off += (lin - q * s) * stride[d];
    lin = q;
  }
  return off;
}

__host__ __device__ inline int64_t numel(const Desc& d) {
  int64_t n = 1;
  for (int i = 0; i < d.ndim; ++i) n *= d.shape[i];
  return n;
}

bool contiguous(const Desc& d) {
  int64_t s = 1;
  for (int i = d.ndim - 1; i >= 0; --i) {
    if (d.shape[i] != 1 && d.stride[i] != s) return false;
    s *= d.shape[i];
  }
  return true;
}

int grid_for(int64_t n, int per_thread = 1) {
  int64_t b = (n + 256LL * per_thread - 1) / (256LL * per_thread);
  if (b < 1) b = 1;
  if (b > 65536) b = 65536;
  return (int)b;
}

// 64-bit mix (splitmix64 finaliser): the counter-based generator behind randn / uniform / dropout
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float u01(uint64_t h) { return ((h >> 40) + 0.5f) * (1.0f / 16777216.0f); }

__device__ __forceinline__ float unary_f(float x, int op, float a, float b) {
  switch (op) {
    case U_NEG: return -x;
    case U_RELU: return x > 0.f ? x : 0.f;
    case U_GELU_TANH: return gelu_tanh(x);
    case U_GELU_ERF: return 0.5f * x * (1.f + erff(x * 0.70710678f));
    case U_SILU: return x / (1.f + __expf(-x));
    case U_SIGMOID: return 1.f / (1.f + __expf(-x));
    case U_TANH: return tanhf(x);
    case U_EXP: return __expf(x);
    case U_LOG: return __logf(x);
    case U_SQRT: return sqrtf(x);
    case U_RSQRT: return rsqrtf(x);
    case U_ABS: return fabsf(x);
    case U_SQUARE: return x * x;
    case U_RECIP: return 1.f / x;
    case U_SIN: return sinf(x);
    case U_COS: return cosf(x);
    case U_POW: return powf(x, a);
    case U_AFFINE: return a * x + b;
    case U_CLAMP: return fminf(fmaxf(x, a), b);
    case U_STEP: return x > 0.f ? 1.f : 0.f;
    case U_SIGN: return (x > 0.f) - (x < 0.f);
  }
  return x;
}

// derivative of unary op at x
__device__ __forceinline__ float unary_d(float x, int op, float a, float b) {
  switch (op) {
    case U_NEG: return -1.f;
    case U_RELU: return x > 0.f ? 1.f : 0.f;
    case U_GELU_TANH: return gelu_tanh_grad(x);
    case U_GELU_ERF: return 0.5f * (1.f + erff(x * 0.70710678f)) + x * 0.3989422804f * __expf(-0.5f * x * x);
    case U_SILU: {
      const float s = 1.f / (1.f + __expf(-x));
      return s * (1.f + x * (1.f - s));
    }
    case U_SIGMOID: {
      const float s = 1.f / (1.f + __expf(-x));
      return s * (1.f - s);
    }
    case U_TANH: {
      const float t = tanhf(x);
      return 1.f - t * t;
    }
    case U_EXP: return __expf(x);
    case U_LOG: return 1.f / x;
    case U_SQRT: return 0.5f * rsqrtf(x);
    case U_RSQRT: return -0.5f * rsqrtf(x) / x;
    case U_ABS: return (x > 0.f) - (x < 0.f);
    case U_SQUARE: return 2.f * x;
    case U_RECIP: return -1.f / (x * x);
    case U_SIN: return cosf(x);
    case U_COS: return -sinf(x);
    case U_POW: return a * powf(x, a - 1.f);
    case U_AFFINE: return a;
    case U_CLAMP: return (x >= a && x <= b) ? 1.f : 0.f;
    default: return 0.f;
  }
}

__device__ __forceinline__ float binary_f(float x, float y, int op) {
  switch (op) {
    case B_ADD: return x + y;
    case B_SUB: return x - y;
    case B_MUL: return x * y;
    case B_DIV: return x / y;
    case B_MAX: return fmaxf(x, y);
    case B_MIN: return fminf(x, y);
    case B_POW: return powf(x, y);
    case B_EQ: return x == y;
    case B_NE: return x != y;
    case B_GT: return x > y;
    case B_LT: return x < y;
    case B_GE: return x >= y;
    case B_LE: return x <= y;
  }
  return 0.f;
}

// ---------------------------------------------------------------- kernels
__global__ void copy_kernel(Desc d, Desc s, int64_t n) {
  const bool ints = is_int(d.dtype) && is_int(s.dtype);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t od = offset_of(i, d.ndim, d.shape, d.stride);
    const int64_t os = offset_of(i, s.ndim, s.shape, s.stride);
    if (ints) sti(d.ptr, d.dtype, od, ldi(s.ptr, s.dtype, os));
    else st(d.ptr, d.dtype, od, ld(s.ptr, s.dtype, os));
  }
}

// 2-D transpose (same dtype): d [R, C] row-major (row stride ld) = the transpose of the row-major source
// S [C, R] (row stride ls), through a 64 x 64 LDS tile so both sides are read / written along rows --
// the per-step W^T copies of trainable weights (the element-wise strided copy_kernel ran them at
// ~0.7 TB/s: 12.5 ms of a gpt2-xl step)
template <typename T>
__global__ __launch_bounds__(256) void transpose2d_kernel(const T* __restrict__ s, int64_t ls, T* __restrict__ d,
                                                          int64_t ld, int64_t R, int64_t C) {
  __shared__ T tile[64][65];
  const int64_t i0 = (int64_t)blockIdx.x * 64, j0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int64_t j = j0 + r, i = i0 + tx;
    if (j < C && i < R) tile[r][tx] = s[j * ls + i];
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int64_t i = i0 + r, j = j0 + tx;
    if (i < R && j < C) d[i * ld + j] = tile[tx][r];
  }
}

// contiguous same-dtype fast path: 16-B vector copy
__global__ void copy16_kernel(const uint4* __restrict__ s, uint4* __restrict__ d, int64_t n16) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

__global__ void fill_kernel(Desc d, double v, int64_t n) {
  const bool ints = is_int(d.dtype);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t od = offset_of(i, d.ndim, d.shape, d.stride);
    if (ints) sti(d.ptr, d.dtype, od, (int64_t)v);
    else st(d.ptr, d.dtype, od, (float)v);
  }
}

__global__ void unary_kernel(Desc d, Desc s, int op, float a, float b, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = ld(s.ptr, s.dtype, offset_of(i, s.ndim, s.shape, s.stride));
    st(d.ptr, d.dtype, offset_of(i, d.ndim, d.shape, d.stride), unary_f(x, op, a, b));
  }
}

__global__ void unary_bwd_kernel(Desc dx, Desc dy, Desc x, int op, float a, float b, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float xv = ld(x.ptr, x.dtype, offset_of(i, x.ndim, x.shape, x.stride));
    const float g = ld(dy.ptr, dy.dtype, offset_of(i, dy.ndim, dy.shape, dy.stride));
    st(dx.ptr, dx.dtype, offset_of(i, dx.ndim, dx.shape, dx.stride), g * unary_d(xv, op, a, b));
  }
}

__global__ void binary_kernel(Desc d, Desc x, Desc y, int op, float alpha, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float xv = ld(x.ptr, x.dtype, offset_of(i, x.ndim, x.shape, x.stride));
    const float yv = ld(y.ptr, y.dtype, offset_of(i, y.ndim, y.shape, y.stride));
    st(d.ptr, d.dtype, offset_of(i, d.ndim, d.shape, d.stride), binary_f(xv, alpha * yv, op));
  }
}

__global__ void axpy_kernel(Desc d, Desc s, float alpha, int acc, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t od = offset_of(i, d.ndim, d.shape, d.stride);
    float v = alpha * ld(s.ptr, s.dtype, offset_of(i, s.ndim, s.shape, s.stride));
    if (acc) v += ld(d.ptr, d.dtype, od);
    st(d.ptr, d.dtype, od, v);
  }
}

// contiguous fp32 += alpha * fp32 (the gradient-accumulation hot case), float4 vectors
__global__ void axpy_f32_kernel(float* __restrict__ d, const float* __restrict__ s, float alpha, int acc, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(s)[i];
    float4 o = acc ? reinterpret_cast<float4*>(d)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    o.x += alpha * v.x;
    o.y += alpha * v.y;
    o.z += alpha * v.z;
    o.w += alpha * v.w;
    reinterpret_cast<float4*>(d)[i] = o;
  }
}

// one wave per row
__global__ void softmax_rows_kernel(const void* x, int xdt, void* y, int ydt, long rows, int n, long ldx, long ldy,
                                    int logm) {
  const long r = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float m = -INFINITY;
  for (int j = lane; j < n; j += 64) m = fmaxf(m, ld(x, xdt, r * ldx + j));
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < n; j += 64) s += __expf(ld(x, xdt, r * ldx + j) - m);
  s = wave_sum(s);
  const float ls = __logf(s);
  for (int j = lane; j < n; j += 64) {
    const float v = ld(x, xdt, r * ldx + j) - m;
    st(y, ydt, r * ldy + j, logm ? v - ls : __expf(v - ls));
  }
}

__global__ void softmax_rows_bwd_kernel(const void* y, const void* dy, void* dx, int dt, long rows, int n, int logm) {
  const long r = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const long base = r * n;
  float s = 0.f;
  for (int j = lane; j < n; j += 64) s += logm ? ld(dy, dt, base + j) : ld(dy, dt, base + j) * ld(y, dt, base + j);
  s = wave_sum(s);
  for (int j = lane; j < n; j += 64) {
    const float yv = ld(y, dt, base + j), g = ld(dy, dt, base + j);
    st(dx, dt, base + j, logm ? g - __expf(yv) * s : yv * (g - s));
  }
}

__global__ void sum_rows_kernel(const void* x, int xdt, void* out, int odt, long rows, int n, float scale) {
  const long r = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float s = 0.f;
  for (int j = lane; j < n; j += 64) s += ld(x, xdt, r * (long)n + j);
  s = wave_sum(s);
  if (lane == 0) st(out, odt, r, s * scale);
}

// stage 1: block b sums rows [b*rpb, (b+1)*rpb) of every column into part[b, :]
__global__ void sum_cols_part_kernel(const void* x, int xdt, float* part, long rows, int n, long rpb) {
  const long r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (long r = r0; r < r1; ++r) s += ld(x, xdt, r * n + j);
    part[blockIdx.y * (long)n + j] = s;
  }
}
__global__ void sum_cols_fin_kernel(const float* part, int nb, float* out, int n, float scale, int acc) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += part[(long)b * n + j];
  out[j] = (acc ? out[j] : 0.f) + s * scale;
}

__global__ void randn_kernel(void* d, int dt, long n, uint64_t seed, float stdev) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    // Box-Muller over two hashes of (seed, i): identical to the host generator in tensor.cpp
    const uint64_t h1 = mix64(seed * 0x2545F4914F6CDD1Dull + 2 * (uint64_t)i);
    const uint64_t h2 = mix64(seed * 0x2545F4914F6CDD1Dull + 2 * (uint64_t)i + 1);
    const float u1 = u01(h1), u2 = u01(h2);
    st(d, dt, i, stdev * sqrtf(-2.f * logf(u1)) * cosf(6.283185307f * u2));
  }
}

__global__ void uniform_kernel(void* d, int dt, long n, uint64_t seed, float lo, float hi) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    st(d, dt, i, lo + (hi - lo) * u01(mix64(seed * 0x2545F4914F6CDD1Dull + (uint64_t)i)));
}

__global__ void dropout_kernel(const void* x, void* y, uint8_t* mask, int dt, long n, uint64_t seed, float p) {
  const float inv = 1.f / (1.f - p);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const bool keep = u01(mix64(seed * 0x9E3779B97F4A7C15ull + (uint64_t)i)) >= p;
    mask[i] = keep;
    st(y, dt, i, keep ? ld(x, dt, i) * inv : 0.f);
  }
}

__global__ void dropout_bwd_kernel(const void* dy, const uint8_t* mask, void* dx, int dt, long n, float p) {
  const float inv = 1.f / (1.f - p);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    st(dx, dt, i, mask[i] ? ld(dy, dt, i) * inv : 0.f);
}

__global__ void nll_rows_kernel(const void* lp, int dt, const int64_t* t, float* out, long rows, int n, long ldl,
                                int ignore) {
  const long r = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const int64_t c = t[r];
  out[r] = (c == ignore || c < 0 || c >= n) ? 0.f : -ld(lp, dt, r * ldl + c);
}

__global__ void nll_rows_bwd_kernel(void* d, int dt, const int64_t* t, long rows, int n, long ldl, int ignore,
                                    const float* scale) {
  const float s = scale ? *scale : 1.f;
  const long total = rows * (long)n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / n;
    const int j = (int)(i - r * n);
    const int64_t c = t[r];
    st(d, dt, r * ldl + j, (j == c && c != ignore) ? -s : 0.f);
  }
}

// rows of a [V, C] table selected by idx (gather) / added back into an fp32 [V, C] table (scatter-add):
// one workgroup per row, the row's C values strided over its threads (embedding of the composite path)
__global__ void gather_rows_kernel(void* dst, int ddt, const void* src, int sdt, const int64_t* idx, long n, int C,
                                   long V) {
  const long r = blockIdx.x;
  if (r >= n) return;
  const int64_t row = idx[r];
  if (row < 0 || row >= V) return;  // (the host checks the ids; never read out of the table)
  for (int j = threadIdx.x; j < C; j += blockDim.x) st(dst, ddt, r * C + j, ld(src, sdt, row * (int64_t)C + j));
}

__global__ void scatter_add_rows_kernel(float* dst, const void* src, int sdt, const int64_t* idx, long n, int C, long V) {
  const long r = blockIdx.x;
  if (r >= n) return;
  const int64_t row = idx[r];
  if (row < 0 || row >= V) return;
  for (int j = threadIdx.x; j < C; j += blockDim.x) atomicAdd(dst + row * (int64_t)C + j, ld(src, sdt, r * C + j));
}

__global__ void count_valid_kernel(const int64_t* t, long n, int ignore, float* out) {
  __shared__ float sm[16];
  float c = 0.f;
  // 8 independent loads in flight per thread (one block: the step's 131,072 labels were a 60 us chain
  // of dependent-latency iterations); integer counts, so the sum is exact in any order
  long i = threadIdx.x;
  for (; i + 7 * (long)blockDim.x < n; i += 8 * (long)blockDim.x) {
    int64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = t[i + u * (long)blockDim.x];
#pragma unroll
    for (int u = 0; u < 8; ++u) c += (v[u] != ignore && v[u] >= 0) ? 1.f : 0.f;
  }
  for (; i < n; i += blockDim.x) c += (t[i] != ignore && t[i] >= 0) ? 1.f : 0.f;
  c = block_sum(c, sm);
  if (threadIdx.x == 0) out[0] = c;
}

// ema[0] = beta * ema[0] + (1 - beta) * loss (ema[0] = loss on the first finite loss, ema[1] = 1
// once initialised); a non-finite loss leaves both unchanged
__global__ void ema_update_kernel(float* ema, const float* loss, float beta) {
  if (threadIdx.x != 0) return;
  const float l = loss[0];
  if (!isfinite(l)) return;
  ema[0] = ema[1] > 0.f ? beta * ema[0] + (1.f - beta) * l : l;
  ema[1] = 1.f;
}

}  // namespace

// ---------------------------------------------------------------- launchers
static size_t dsize(int dt) { return dt == F32 || dt == I32 ? 4 : dt == I64 ? 8 : (dt == BF16 || dt == F16) ? 2 : 1; }

void copy(const Desc& d, const Desc& s, hipStream_t stm) {
  const int64_t n = numel(d);
  if (n == 0) return;
  if (d.dtype == s.dtype && contiguous(d) && contiguous(s) && numel(s) == n) {
    const size_t bytes = (size_t)n * dsize(d.dtype);
    if (bytes % 16 == 0 && ((uintptr_t)d.ptr % 16) == 0 && ((uintptr_t)s.ptr % 16) == 0) {
      const int64_t n16 = bytes / 16;
      copy16_kernel<<<grid_for(n16), 256, 0, stm>>>((const uint4*)s.ptr, (uint4*)d.ptr, n16);
      return;
    }
    MFT_HIP_CHECK(hipMemcpyAsync(d.ptr, s.ptr, bytes, hipMemcpyDeviceToDevice, stm));
    return;
  }
  // a transposed 2-D view into a row-major destination: the LDS-tiled transpose (MFT_COPY_T=0: off, A/B)
  static const bool tr_off = getenv("MFT_COPY_T") && getenv("MFT_COPY_T")[0] == '0';
  if (!tr_off && d.dtype == s.dtype && d.ndim == 2 && s.ndim == 2 && s.shape[0] == d.shape[0] && s.shape[1] == d.shape[1] &&
      d.stride[1] == 1 && d.stride[0] >= d.shape[1] && s.stride[0] == 1 && s.stride[1] >= s.shape[0] &&
      (dsize(d.dtype) == 2 || dsize(d.dtype) == 4) && (d.shape[0] + 63) / 64 < (1L << 31) && (d.shape[1] + 63) / 64 < 65536) {
    const dim3 grid((unsigned)((d.shape[0] + 63) / 64), (unsigned)((d.shape[1] + 63) / 64));
    if (dsize(d.dtype) == 2)
      transpose2d_kernel<uint16_t><<<grid, 256, 0, stm>>>((const uint16_t*)s.ptr, s.stride[1], (uint16_t*)d.ptr, d.stride[0],
                                                         d.shape[0], d.shape[1]);
    else
      transpose2d_kernel<uint32_t><<<grid, 256, 0, stm>>>((const uint32_t*)s.ptr, s.stride[1], (uint32_t*)d.ptr, d.stride[0],
                                                         d.shape[0], d.shape[1]);
    return;
  }
  copy_kernel<<<grid_for(n), 256, 0, stm>>>(d, s, n);
}

void fill(const Desc& d, double v, hipStream_t stm) {
  const int64_t n = numel(d);
  if (n == 0) return;
  if (v == 0.0 && contiguous(d)) {
    MFT_HIP_CHECK(hipMemsetAsync(d.ptr, 0, (size_t)n * dsize(d.dtype), stm));
    return;
  }
  fill_kernel<<<grid_for(n), 256, 0, stm>>>(d, v, n);
}

void unary(const Desc& d, const Desc& s, int op, float a, float b, hipStream_t stm) {
  const int64_t n = numel(d);
  if (n) unary_kernel<<<grid_for(n), 256, 0, stm>>>(d, s, op, a, b, n);
}

void unary_bwd(const Desc& dx, const Desc& dy, const Desc& x, int op, float a, float b, hipStream_t stm) {
  const int64_t n = numel(dx);
  if (n) unary_bwd_kernel<<<grid_for(n), 256, 0, stm>>>(dx, dy, x, op, a, b, n);
}

void binary(const Desc& d, const Desc& x, const Desc& y, int op, float alpha, hipStream_t stm) {
  const int64_t n = numel(d);
  if (n) binary_kernel<<<grid_for(n), 256, 0, stm>>>(d, x, y, op, alpha, n);
}

void axpy(const Desc& d, const Desc& s, float alpha, int acc, hipStream_t stm) {
  const int64_t n = numel(d);
  if (!n) return;
  if (d.dtype == F32 && s.dtype == F32 && contiguous(d) && contiguous(s) && numel(s) == n && n % 4 == 0 &&
      ((uintptr_t)d.ptr % 16) == 0 && ((uintptr_t)s.ptr % 16) == 0) {
    axpy_f32_kernel<<<grid_for(n / 4), 256, 0, stm>>>((float*)d.ptr, (const float*)s.ptr, alpha, acc, n / 4);
    return;
  }
  axpy_kernel<<<grid_for(n), 256, 0, stm>>>(d, s, alpha, acc, n);
}

void softmax_rows(const void* x, int xdt, void* y, int ydt, long rows, int n, long ldx, long ldy, int logm,
                  hipStream_t stm) {
  if (rows) softmax_rows_kernel<<<(int)((rows + 3) / 4), 256, 0, stm>>>(x, xdt, y, ydt, rows, n, ldx, ldy, logm);
}

void softmax_rows_bwd(const void* y, const void* dy, void* dx, int dt, long rows, int n, int logm, hipStream_t stm) {
  if (rows) softmax_rows_bwd_kernel<<<(int)((rows + 3) / 4), 256, 0, stm>>>(y, dy, dx, dt, rows, n, logm);
}

void sum_rows(const void* x, int xdt, void* out, int odt, long rows, int n, float scale, hipStream_t stm) {
  if (rows) sum_rows_kernel<<<(int)((rows + 3) / 4), 256, 0, stm>>>(x, xdt, out, odt, rows, n, scale);
}

void sum_cols(const void* x, int xdt, float* out, float* part, long rows, int n, float scale, int acc,
              hipStream_t stm) {
  if (!n) return;
  const int nb = (int)std::min<long>(256, std::max<long>(1, rows / 64));
  const long rpb = (rows + nb - 1) / nb;
  dim3 g1((unsigned)std::min(64, (n + 255) / 256), (unsigned)nb);
  sum_cols_part_kernel<<<g1, 256, 0, stm>>>(x, xdt, part, rows, n, rpb);
  sum_cols_fin_kernel<<<(n + 255) / 256, 256, 0, stm>>>(part, nb, out, n, scale, acc);
}

void randn(void* d, int dt, long n, uint64_t seed, float stdev, hipStream_t stm) {
  if (n) randn_kernel<<<grid_for(n), 256, 0, stm>>>(d, dt, n, seed, stdev);
}

void rand_uniform(void* d, int dt, long n, uint64_t seed, float lo, float hi, hipStream_t stm) {
  if (n) uniform_kernel<<<grid_for(n), 256, 0, stm>>>(d, dt, n, seed, lo, hi);
}

void dropout(const void* x, void* y, uint8_t* mask, int dt, long n, uint64_t seed, float p, hipStream_t stm) {
  if (n) dropout_kernel<<<grid_for(n), 256, 0, stm>>>(x, y, mask, dt, n, seed, p);
}

void dropout_bwd(const void* dy, const uint8_t* mask, void* dx, int dt, long n, float p, hipStream_t stm) {
  if (n) dropout_bwd_kernel<<<grid_for(n), 256, 0, stm>>>(dy, mask, dx, dt, n, p);
}

void nll_rows(const void* lp, int dt, const int64_t* t, float* out, long rows, int n, long ldl, int ignore,
              hipStream_t stm) {
  if (rows) nll_rows_kernel<<<(int)((rows + 255) / 256), 256, 0, stm>>>(lp, dt, t, out, rows, n, ldl, ignore);
}

void nll_rows_bwd(void* d, int dt, const int64_t* t, long rows, int n, long ldl, int ignore, const float* scale,
                  hipStream_t stm) {
  if (!rows) return;
  nll_rows_bwd_kernel<<<grid_for(rows * (int64_t)n), 256, 0, stm>>>(d, dt, t, rows, n, ldl, ignore, scale);
}

void gather_rows(void* dst, int ddt, const void* src, int sdt, const int64_t* idx, long n, int C, long V,
                 hipStream_t stm) {
  if (n) gather_rows_kernel<<<(unsigned)n, 256, 0, stm>>>(dst, ddt, src, sdt, idx, n, C, V);
}

void scatter_add_rows(float* dst, const void* src, int sdt, const int64_t* idx, long n, int C, long V, hipStream_t stm) {
  if (n) scatter_add_rows_kernel<<<(unsigned)n, 256, 0, stm>>>(dst, src, sdt, idx, n, C, V);
}

void count_valid(const int64_t* t, long n, int ignore, float* out, hipStream_t stm) {
  count_valid_kernel<<<1, 1024, 0, stm>>>(t, n, ignore, out);
}

void ema_update(float* ema, const float* loss, float beta, hipStream_t stm) {
  ema_update_kernel<<<1, 64, 0, stm>>>(ema, loss, beta);
}

}  // namespace k
}  // namespace eng
}  // namespace mft
