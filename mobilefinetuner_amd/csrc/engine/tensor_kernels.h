// libmft engine: launchers of the generic tensor kernels (engine/tensor_kernels.hip) -- the op catalog of
// the reference's core/ops.cpp that is not on the fused hot path (strided copies and
// casts, fills, broadcast binary ops, unary math, comparisons, row softmax / log-softmax,
// reductions, counter-based RNG, dropout).  Every launcher takes the stream explicitly and never
// allocates, so all of it is hipGraph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mft {
namespace eng {
namespace k {

constexpr int kMaxDims = 8;
// dtype codes (match eng::DType order)
enum : int { F32 = 0, BF16 = 1, F16 = 2, I32 = 3, I64 = 4, U8 = 5, BOOL = 6 };

struct Desc {  // a strided view: element pointer + geometry (strides in elements; 0 = broadcast)
  void* ptr;
  int dtype;
  int ndim;
  int64_t shape[kMaxDims];
  int64_t stride[kMaxDims];
};

enum Unary : int {
  U_NEG, U_RELU, U_GELU_TANH, U_GELU_ERF, U_SILU, U_SIGMOID, U_TANH, U_EXP, U_LOG, U_SQRT, U_RSQRT, U_ABS,
  U_SQUARE, U_RECIP, U_SIN, U_COS, U_POW, U_AFFINE /* a*x+b */, U_CLAMP /* [a, b] */, U_STEP /* x > 0 */,
  U_SIGN
};
enum Binary : int {
  B_ADD, B_SUB, B_MUL, B_DIV, B_MAX, B_MIN, B_POW, B_EQ, B_NE, B_GT, B_LT, B_GE, B_LE
};

// dst = cast(src) elementwise over dst's shape (src broadcast through zero strides)
void copy(const Desc& dst, const Desc& src, hipStream_t st);
void fill(const Desc& dst, double v, hipStream_t st);
// dst = f(src; a, b)
void unary(const Desc& dst, const Desc& src, int op, float a, float b, hipStream_t st);
// dx = dy * f'(x) (y = f(x) optionally used)   -- backward of the differentiable unary ops
void unary_bwd(const Desc& dx, const Desc& dy, const Desc& x, int op, float a, float b, hipStream_t st);
// dst = x (op) alpha * y   (broadcast through zero strides; comparisons write 0/1)
void binary(const Desc& dst, const Desc& x, const Desc& y, int op, float alpha, hipStream_t st);
// dst (+)= alpha * src  (accumulate when acc != 0)
void axpy(const Desc& dst, const Desc& src, float alpha, int acc, hipStream_t st);
// rows of length n (contiguous, row stride ld): softmax / log-softmax over the last dim
void softmax_rows(const void* x, int xdt, void* y, int ydt, long rows, int n, long ldx, long ldy, int log, hipStream_t st);
// dx = y * (dy - sum(dy * y))   (softmax) or dy - exp(y) * sum(dy)   (log-softmax)
void softmax_rows_bwd(const void* y, const void* dy, void* dx, int dt, long rows, int n, int log, hipStream_t st);
// sum over the last dim of contiguous rows: out[r] = scale * sum_j x[r, j]   (out fp32 or dtype)
void sum_rows(const void* x, int xdt, void* out, int odt, long rows, int n, float scale, hipStream_t st);
// column sums: out[j] = scale * sum_r x[r, j] (two-stage, deterministic); part >= 256 * n floats
void sum_cols(const void* x, int xdt, float* out, float* part, long rows, int n, float scale, int acc, hipStream_t st);
// counter-based RNG (splitmix/Philox-style hash of (seed, index)): normal(0, std) or uniform [lo, hi)
void randn(void* dst, int dt, long n, uint64_t seed, float stdev, hipStream_t st);
void rand_uniform(void* dst, int dt, long n, uint64_t seed, float lo, float hi, hipStream_t st);
// dropout with a counter hash: keep = hash(seed, i) >= p; y = keep ? x / (1 - p) : 0; mask stored as u8
void dropout(const void* x, void* y, uint8_t* mask, int dt, long n, uint64_t seed, float p, hipStream_t st);
void dropout_bwd(const void* dy, const uint8_t* mask, void* dx, int dt, long n, float p, hipStream_t st);
// per-row NLL from log-probs: out[r] = -lp[r, target[r]] (ignore_index -> 0), count of valid rows
void nll_rows(const void* lp, int dt, const int64_t* target, float* out, long rows, int n, long ld, int ignore,
              hipStream_t st);
// dlp[r, target[r]] = -scale (ignore rows 0), other entries 0
void nll_rows_bwd(void* dlp, int dt, const int64_t* target, long rows, int n, long ld, int ignore, const float* scale,
                  hipStream_t st);
// rows of a [V, C] table: dst[r, :] = src[idx[r], :] (any float dtypes; ids outside [0, V) skipped)
void gather_rows(void* dst, int ddt, const void* src, int sdt, const int64_t* idx, long n, int C, long V, hipStream_t st);
// dst[idx[r], :] += src[r, :] into an fp32 table (float atomics: the order of equal ids is not fixed)
void scatter_add_rows(float* dst, const void* src, int sdt, const int64_t* idx, long n, int C, long V, hipStream_t st);
// number of targets != ignore -> out[0] (fp32)
void count_valid(const int64_t* target, long n, int ignore, float* out, hipStream_t st);
// training-loss EMA on device: ema = {value, initialised}; non-finite losses are skipped
void ema_update(float* ema, const float* loss, float beta, hipStream_t st);

}  // namespace k
}  // namespace eng
}  // namespace mft
