// RoPE and fused per-head RMSNorm(1+w) + RoPE (Gemma-3 q_norm/k_norm -> rotary), fwd + bwd.
// Replaces ops::apply_rope + ApplyRoPEBackward (core/ops.cpp:2151-2225,
// core/backward_functions.cpp:718-763) and the q/k rms_norm calls of GemmaModel
// (graph/gemma_model.cpp:459-471).  Default pairing is HF rotate-half (d, d + D/2); the
// reference's interleaved pairs (2i, 2i+1) are available with interleaved=1.
// cos/sin come from host-built tables [S_max, D/2] fp32 (no on-device trig, Appendix B).
// One wave per (token, head) row; each lane owns PPL rotation pairs.
#include "common.h"
#include "kernels.h"

namespace mft {

__device__ __forceinline__ void pair_index(int p, int D, int interleaved, int& i0, int& i1) {
  if (interleaved) { i0 = 2 * p; i1 = 2 * p + 1; }
  else { i0 = p; i1 = p + D / 2; }
}

template <int PPL>
__global__ __launch_bounds__(256) void rope_kernel(bf16_t* x, long sb, long ss, long sh, int B, int S, int H, int D,
                                                   const float* __restrict__ cs, const float* __restrict__ sn, int pos0,
                                                   int interleaved, int inverse) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long)B * S * H) return;
  const int h = row % H, s = (row / H) % S, b = row / ((long)H * S);
  bf16_t* xr = x + b * sb + (long)s * ss + h * sh;
  const int half = D / 2;
  const float* c = cs + (long)(pos0 + s) * half;
  const float* n = sn + (long)(pos0 + s) * half;
#pragma unroll
  for (int t = 0; t < PPL; ++t) {
    const int p = lane * PPL + t;
    if (p < half) {
      int i0, i1;
      pair_index(p, D, interleaved, i0, i1);
      const float a = bf2f(xr[i0]), bb = bf2f(xr[i1]);
      const float cc = c[p], ss2 = inverse ? -n[p] : n[p];
      xr[i0] = f2bf(a * cc - bb * ss2);
      xr[i1] = f2bf(bb * cc + a * ss2);
    }
  }
}

// y = rope(x * rstd * (w + off)); x strided, y contiguous [rows, D]
template <int PPL>
__global__ __launch_bounds__(256) void qknorm_rope_fwd_kernel(const bf16_t* __restrict__ x, long sb, long ss, long sh,
                                                              bf16_t* __restrict__ y, float* __restrict__ rstd_out,
                                                              const float* __restrict__ w, int B, int S, int H, int D,
                                                              const float* __restrict__ cs, const float* __restrict__ sn,
                                                              int pos0, float eps, float off, int interleaved) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long)B * S * H) return;
  const int h = row % H, s = (row / H) % S, b = row / ((long)H * S);
  const bf16_t* xr = x + b * sb + (long)s * ss + h * sh;
  const int half = D / 2;
  float a[PPL], bb[PPL];
  float sq = 0.f;
#pragma unroll
  for (int t = 0; t < PPL; ++t) {
    const int p = lane * PPL + t;
    int i0 = 0, i1 = 0;
    if (p < half) pair_index(p, D, interleaved, i0, i1);
    a[t] = p < half ? bf2f(xr[i0]) : 0.f;
    bb[t] = p < half ? bf2f(xr[i1]) : 0.f;
    sq += a[t] * a[t] + bb[t] * bb[t];
  }
  const float rstd = rsqrtf(wave_sum(sq) / D + eps);
  const float* c = cs + (long)(pos0 + s) * half;
  const float* n = sn + (long)(pos0 + s) * half;
  bf16_t* yr = y + row * D;
#pragma unroll
  for (int t = 0; t < PPL; ++t) {
    const int p = lane * PPL + t;
    if (p < half) {
      int i0, i1;
      pair_index(p, D, interleaved, i0, i1);
      // HF Gemma3RMSNorm computes in fp32 and casts the normalised value once
      const float u0 = bf2f(f2bf(a[t] * rstd * (w[i0] + off)));
      const float u1 = bf2f(f2bf(bb[t] * rstd * (w[i1] + off)));
      yr[i0] = f2bf(u0 * c[p] - u1 * n[p]);
      yr[i1] = f2bf(u1 * c[p] + u0 * n[p]);
    }
  }
  if (lane == 0) rstd_out[row] = rstd;
}

// dx = rmsnorm_bwd(x, rope^T(dy)); dw partials per block (deterministic) when dw_part != null
template <int PPL>
__global__ __launch_bounds__(256) void qknorm_rope_bwd_kernel(const bf16_t* __restrict__ x, long sb, long ss, long sh,
                                                              const bf16_t* __restrict__ dy, const float* __restrict__ rstd_in,
                                                              const float* __restrict__ w, bf16_t* __restrict__ dx,
                                                              long dsb, long dss, long dsh, float* __restrict__ dw_part,
                                                              int B, int S, int H, int D, const float* __restrict__ cs,
                                                              const float* __restrict__ sn, int pos0, float off,
                                                              int interleaved) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int half = D / 2;
  float dwa[PPL], dwb[PPL];
#pragma unroll
  for (int t = 0; t < PPL; ++t) dwa[t] = dwb[t] = 0.f;
  const long rows = (long)B * S * H;
  for (long row = (long)blockIdx.x * 4 + wid; row < rows; row += (long)gridDim.x * 4) {
    const int h = row % H, s = (row / H) % S, b = row / ((long)H * S);
    const bf16_t* xr = x + b * sb + (long)s * ss + h * sh;
    const bf16_t* gr = dy + row * D;
    const float* c = cs + (long)(pos0 + s) * half;
    const float* n = sn + (long)(pos0 + s) * half;
    const float rstd = rstd_in[row];
    float xh0[PPL], xh1[PPL], g0[PPL], g1[PPL];
    float s2 = 0.f;
#pragma unroll
    for (int t = 0; t < PPL; ++t) {
      const int p = lane * PPL + t;
      xh0[t] = xh1[t] = g0[t] = g1[t] = 0.f;
      if (p < half) {
        int i0, i1;
        pair_index(p, D, interleaved, i0, i1);
        const float d0 = bf2f(gr[i0]), d1 = bf2f(gr[i1]);
        // rope^T
        const float u0 = d0 * c[p] + d1 * n[p];
        const float u1 = d1 * c[p] - d0 * n[p];
        xh0[t] = bf2f(xr[i0]) * rstd;
        xh1[t] = bf2f(xr[i1]) * rstd;
        if (dw_part) { dwa[t] += u0 * xh0[t]; dwb[t] += u1 * xh1[t]; }
        g0[t] = u0 * (w[i0] + off);
        g1[t] = u1 * (w[i1] + off);
        s2 += g0[t] * xh0[t] + g1[t] * xh1[t];
      }
    }
    s2 = wave_sum(s2) / D;
    bf16_t* dxr = dx + b * dsb + (long)s * dss + h * dsh;
#pragma unroll
    for (int t = 0; t < PPL; ++t) {
      const int p = lane * PPL + t;
      if (p < half) {
        int i0, i1;
        pair_index(p, D, interleaved, i0, i1);
        dxr[i0] = f2bf(rstd * (g0[t] - xh0[t] * s2));
        dxr[i1] = f2bf(rstd * (g1[t] - xh1[t] * s2));
      }
    }
  }
  if (dw_part) {
    extern __shared__ __attribute__((aligned(16))) float red[];  // [4][D]
#pragma unroll
    for (int t = 0; t < PPL; ++t) {
      const int p = lane * PPL + t;
      if (p < half) {
        int i0, i1;
        pair_index(p, D, interleaved, i0, i1);
        red[wid * D + i0] = dwa[t];
        red[wid * D + i1] = dwb[t];
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < D; i += blockDim.x)
      dw_part[(long)blockIdx.x * D + i] = red[i] + red[D + i] + red[2 * D + i] + red[3 * D + i];
  }
}

#define MFT_PPL_DISPATCH(D, ...)                                      \
  do {                                                                \
    const int ppl = ((D) / 2 + 63) / 64;                              \
    if (ppl <= 1) { constexpr int P = 1; __VA_ARGS__; }               \
    else if (ppl <= 2) { constexpr int P = 2; __VA_ARGS__; }          \
    else { constexpr int P = 4; __VA_ARGS__; }                        \
  } while (0)

void rope_apply(bf16_t* x, const long* st, int B, int S, int H, int D, const float* cos_t, const float* sin_t, int pos0,
                int interleaved, int inverse, hipStream_t stream) {
  const long rows = (long)B * S * H;
  MFT_PPL_DISPATCH(D, rope_kernel<P><<<cdiv(rows, 4), 256, 0, stream>>>(x, st[0], st[1], st[2], B, S, H, D, cos_t, sin_t,
                                                                         pos0, interleaved, inverse));
}

void qknorm_rope_fwd(const bf16_t* x, const long* st, bf16_t* y, float* rstd, const float* w, int B, int S, int H, int D,
                     const float* cos_t, const float* sin_t, int pos0, float eps, float off, int interleaved,
                     hipStream_t stream) {
  const long rows = (long)B * S * H;
  MFT_PPL_DISPATCH(D, qknorm_rope_fwd_kernel<P><<<cdiv(rows, 4), 256, 0, stream>>>(
                          x, st[0], st[1], st[2], y, rstd, w, B, S, H, D, cos_t, sin_t, pos0, eps, off, interleaved));
}

int qknorm_rope_bwd_blocks(long rows) {
  long nb = (rows + 3) / 4;
  return (int)(nb < 512 ? nb : 512);
}

void qknorm_rope_bwd(const bf16_t* x, const long* st, const bf16_t* dy, const float* rstd, const float* w, bf16_t* dx,
                     const long* dst, float* dw, float* work, int B, int S, int H, int D, const float* cos_t,
                     const float* sin_t, int pos0, float off, int interleaved, int accumulate, hipStream_t stream) {
  const long rows = (long)B * S * H;
  const int nb = dw ? qknorm_rope_bwd_blocks(rows) : cdiv(rows, 4);
  const size_t shm = dw ? sizeof(float) * 4 * D : 0;
  float* part = dw ? work : nullptr;
  MFT_PPL_DISPATCH(D, qknorm_rope_bwd_kernel<P><<<nb, 256, shm, stream>>>(
                          x, st[0], st[1], st[2], dy, rstd, w, dx, dst[0], dst[1], dst[2], part, B, S, H, D, cos_t,
                          sin_t, pos0, off, interleaved));
  if (dw) reduce_rows(part, dw, nb, D, accumulate, stream);
}

}  // namespace mft
