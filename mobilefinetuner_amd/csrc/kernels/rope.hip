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

// Vectorised rotate-half forms (the default pairing): a lane owns 4 consecutive rotation pairs, so
// x / dy / y move as 8-B pieces of each half and cos / sin / w as float4; LPR = D / 8 lanes per
// row, 64 / LPR rows per wave (D = 256: two rows per wave).  The scalar-per-pair kernels above
// stay for the interleaved layout.
template <int D>
__global__ __launch_bounds__(256) void qknorm_rope_fwd_v_kernel(const bf16_t* __restrict__ x, long sb, long ss, long sh,
                                                                bf16_t* __restrict__ y, float* __restrict__ rstd_out,
                                                                const float* __restrict__ w, int B, int S, int H,
                                                                const float* __restrict__ cs, const float* __restrict__ sn,
                                                                int pos0, float eps, float off) {
  constexpr int HALF = D / 2, LPR = HALF / 4, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane / LPR, li = lane % LPR, p0 = 4 * li;
  const long rows = (long)B * S * H;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + sub;
  const bool ok = row < rows;
  const long rr = ok ? row : rows - 1;
  const int h = rr % H, s = (rr / H) % S, b = rr / ((long)H * S);
  const bf16_t* xr = x + b * sb + (long)s * ss + h * sh;
  const u16x4_t va = *reinterpret_cast<const u16x4_t*>(xr + p0);
  const u16x4_t vb = *reinterpret_cast<const u16x4_t*>(xr + HALF + p0);
  float a[4], bb[4], sq = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    a[t] = bf2f(va[t]);
    bb[t] = bf2f(vb[t]);
    sq += a[t] * a[t] + bb[t] * bb[t];
  }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) sq += __shfl_xor(sq, o, 64);
  const float rstd = rsqrtf(sq / D + eps);
  const float4 c = *reinterpret_cast<const float4*>(cs + (long)(pos0 + s) * HALF + p0);
  const float4 n = *reinterpret_cast<const float4*>(sn + (long)(pos0 + s) * HALF + p0);
  const float4 w0 = *reinterpret_cast<const float4*>(w + p0);
  const float4 w1 = *reinterpret_cast<const float4*>(w + HALF + p0);
  const float cc[4] = {c.x, c.y, c.z, c.w}, nn[4] = {n.x, n.y, n.z, n.w};
  const float wa[4] = {w0.x, w0.y, w0.z, w0.w}, wb[4] = {w1.x, w1.y, w1.z, w1.w};
  u16x4_t ya, yb;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    // HF Gemma3RMSNorm computes in fp32 and casts the normalised value once
    const float u0 = bf2f(f2bf(a[t] * rstd * (wa[t] + off)));
    const float u1 = bf2f(f2bf(bb[t] * rstd * (wb[t] + off)));
    ya[t] = f2bf(u0 * cc[t] - u1 * nn[t]);
    yb[t] = f2bf(u1 * cc[t] + u0 * nn[t]);
  }
  if (ok) {
    bf16_t* yr = y + row * D;
    *reinterpret_cast<u16x4_t*>(yr + p0) = ya;
    *reinterpret_cast<u16x4_t*>(yr + HALF + p0) = yb;
    if (li == 0) rstd_out[row] = rstd;
  }
}

template <int D>
__global__ __launch_bounds__(256) void qknorm_rope_bwd_v_kernel(const bf16_t* __restrict__ x, long sb, long ss, long sh,
                                                                const bf16_t* __restrict__ dy,
                                                                const float* __restrict__ rstd_in,
                                                                const float* __restrict__ w, bf16_t* __restrict__ dx,
                                                                long dsb, long dss, long dsh, float* __restrict__ dw_part,
                                                                int B, int S, int H, const float* __restrict__ cs,
                                                                const float* __restrict__ sn, int pos0, float off) {
  constexpr int HALF = D / 2, LPR = HALF / 4, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, sub = lane / LPR, li = lane % LPR, p0 = 4 * li;
  const long rows = (long)B * S * H;
  const float4 w0 = *reinterpret_cast<const float4*>(w + p0);
  const float4 w1 = *reinterpret_cast<const float4*>(w + HALF + p0);
  const float wa[4] = {w0.x + off, w0.y + off, w0.z + off, w0.w + off};
  const float wb[4] = {w1.x + off, w1.y + off, w1.z + off, w1.w + off};
  float dwa[4] = {0.f, 0.f, 0.f, 0.f}, dwb[4] = {0.f, 0.f, 0.f, 0.f};
  const long step = (long)gridDim.x * 4 * RPW;
  for (long base = ((long)blockIdx.x * 4 + wid) * RPW; base < rows; base += step) {  // wave-uniform bound
    const long row = base + sub;
    const bool ok = row < rows;
    const long rr = ok ? row : rows - 1;
    const int h = rr % H, s = (rr / H) % S, b = rr / ((long)H * S);
    const bf16_t* xr = x + b * sb + (long)s * ss + h * sh;
    const bf16_t* gr = dy + rr * D;
    const u16x4_t xa = *reinterpret_cast<const u16x4_t*>(xr + p0);
    const u16x4_t xb = *reinterpret_cast<const u16x4_t*>(xr + HALF + p0);
    const u16x4_t da = *reinterpret_cast<const u16x4_t*>(gr + p0);
    const u16x4_t db = *reinterpret_cast<const u16x4_t*>(gr + HALF + p0);
    const float4 c = *reinterpret_cast<const float4*>(cs + (long)(pos0 + s) * HALF + p0);
    const float4 n = *reinterpret_cast<const float4*>(sn + (long)(pos0 + s) * HALF + p0);
    const float cc[4] = {c.x, c.y, c.z, c.w}, nn[4] = {n.x, n.y, n.z, n.w};
    const float rstd = ok ? rstd_in[row] : 0.f;
    float xh0[4], xh1[4], g0[4], g1[4], s2 = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float d0 = bf2f(da[t]), d1 = bf2f(db[t]);
      const float u0 = d0 * cc[t] + d1 * nn[t];  // rope^T
      const float u1 = d1 * cc[t] - d0 * nn[t];
      xh0[t] = bf2f(xa[t]) * rstd;
      xh1[t] = bf2f(xb[t]) * rstd;
      dwa[t] += u0 * xh0[t];
      dwb[t] += u1 * xh1[t];
      g0[t] = u0 * wa[t];
      g1[t] = u1 * wb[t];
      s2 += g0[t] * xh0[t] + g1[t] * xh1[t];
    }
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) s2 += __shfl_xor(s2, o, 64);
    s2 /= D;
    if (ok) {
      u16x4_t oa, ob;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        oa[t] = f2bf(rstd * (g0[t] - xh0[t] * s2));
        ob[t] = f2bf(rstd * (g1[t] - xh1[t] * s2));
      }
      bf16_t* dxr = dx + b * dsb + (long)s * dss + h * dsh;
      *reinterpret_cast<u16x4_t*>(dxr + p0) = oa;
      *reinterpret_cast<u16x4_t*>(dxr + HALF + p0) = ob;
    }
  }
  if (dw_part) {
    extern __shared__ __attribute__((aligned(16))) float red[];  // [4 * RPW][D]
    float* rr = red + (wid * RPW + sub) * D;
    *reinterpret_cast<float4*>(rr + p0) = float4{dwa[0], dwa[1], dwa[2], dwa[3]};
    *reinterpret_cast<float4*>(rr + HALF + p0) = float4{dwb[0], dwb[1], dwb[2], dwb[3]};
    __syncthreads();
    for (int i = threadIdx.x; i < D; i += blockDim.x) {
      float sacc = 0.f;
#pragma unroll
      for (int r = 0; r < 4 * RPW; ++r) sacc += red[r * D + i];
      dw_part[(long)blockIdx.x * D + i] = sacc;
    }
  }
}

static bool aligned16(const float* a, const float* b, const float* c) {
  return (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15) == 0;
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
  if (!interleaved && (D == 64 || D == 128 || D == 256) && st[0] % 4 == 0 && st[1] % 4 == 0 && st[2] % 4 == 0 &&
      aligned16(w, cos_t, sin_t) && ((uintptr_t)x & 7) == 0) {
    const int rpb = 4 * (64 / (D / 8));  // rows per 256-thread block
    switch (D) {
#define MFT_QKV(DD) case DD: qknorm_rope_fwd_v_kernel<DD><<<cdiv(rows, rpb), 256, 0, stream>>>( \
        x, st[0], st[1], st[2], y, rstd, w, B, S, H, cos_t, sin_t, pos0, eps, off); return;
      MFT_QKV(64) MFT_QKV(128) MFT_QKV(256)
#undef MFT_QKV
    }
  }
  MFT_PPL_DISPATCH(D, qknorm_rope_fwd_kernel<P><<<cdiv(rows, 4), 256, 0, stream>>>(
                          x, st[0], st[1], st[2], y, rstd, w, B, S, H, D, cos_t, sin_t, pos0, eps, off, interleaved));
}

int qknorm_rope_bwd_blocks(long rows) {
  long nb = (rows + 3) / 4;
  return (int)(nb < 1024 ? nb : 1024);
}

void qknorm_rope_bwd(const bf16_t* x, const long* st, const bf16_t* dy, const float* rstd, const float* w, bf16_t* dx,
                     const long* dst, float* dw, float* work, int B, int S, int H, int D, const float* cos_t,
                     const float* sin_t, int pos0, float off, int interleaved, int accumulate, hipStream_t stream) {
  const long rows = (long)B * S * H;
  if (!interleaved && (D == 64 || D == 128 || D == 256) && st[0] % 4 == 0 && st[1] % 4 == 0 && st[2] % 4 == 0 &&
      dst[0] % 4 == 0 && dst[1] % 4 == 0 && dst[2] % 4 == 0 && aligned16(w, cos_t, sin_t) &&
      ((uintptr_t)x & 7) == 0 && ((uintptr_t)dx & 7) == 0 && ((uintptr_t)dy & 7) == 0) {
    const int rpb = 4 * (64 / (D / 8));
    const int nb = dw ? qknorm_rope_bwd_blocks(rows) : (int)cdiv(rows, rpb);
    const size_t shm = dw ? sizeof(float) * 4 * (64 / (D / 8)) * D : 0;
    float* part = dw ? work : nullptr;
    switch (D) {
#define MFT_QKV(DD) case DD: qknorm_rope_bwd_v_kernel<DD><<<nb, 256, shm, stream>>>( \
        x, st[0], st[1], st[2], dy, rstd, w, dx, dst[0], dst[1], dst[2], part, B, S, H, cos_t, sin_t, pos0, off); break;
      MFT_QKV(64) MFT_QKV(128) MFT_QKV(256)
#undef MFT_QKV
    }
    if (dw) reduce_rows(part, dw, nb, D, accumulate, stream);
    return;
  }
  const int nb = dw ? qknorm_rope_bwd_blocks(rows) : cdiv(rows, 4);
  const size_t shm = dw ? sizeof(float) * 4 * D : 0;
  float* part = dw ? work : nullptr;
  MFT_PPL_DISPATCH(D, qknorm_rope_bwd_kernel<P><<<nb, 256, shm, stream>>>(
                          x, st[0], st[1], st[2], dy, rstd, w, dx, dst[0], dst[1], dst[2], part, B, S, H, D, cos_t,
                          sin_t, pos0, off, interleaved));
  if (dw) reduce_rows(part, dw, nb, D, accumulate, stream);
}

}  // namespace mft
