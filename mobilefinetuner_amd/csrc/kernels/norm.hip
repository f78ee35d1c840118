// LayerNorm / RMSNorm forward + backward for gfx950.
//
// Replaces the reference's scalar CPU loops ops::layer_norm / ops::rms_norm
// (operators/finetune_ops/core/ops.cpp:1404-1458, :1489-1574) and their backward classes
// (core/backward_functions.cpp:425-561).
//
// Design: one wave64 per row, 4 rows per 256-thread block; each lane owns CH chunks of 8
// contiguous bf16 (16-B vector loads), the row stays in registers between the statistics pass
// and the normalise pass, so the row is read from HBM exactly once.  Optional fused residual
// add (s = x + d; y = norm(s)) removes a separate elementwise pass per transformer sub-block.
// Statistics (mean/rstd) are saved in fp32 for the backward.  The affine weight is fp32.
// LoRA consumer fusion: when the output row is wider (augmented-K input of a LoRA projection,
// engine/nn.h lora_linear_aug) and an adapter matrix A [R, N] is given, the same pass also writes
// u = y A^T (the bf16-rounded normalised row, as the consumer reads it) into the appended columns
// N .. N+R-1 -- the separate pass over y (lora_rowdot) disappears.
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace mft {

template <int CH, bool RMS, bool RESID, int LR = 0>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ d,
                                                       bf16_t* __restrict__ s_out, const float* __restrict__ w,
                                                       const float* __restrict__ b, bf16_t* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int M, int N, float eps, float w_offset, long ldy,
                                                       const bf16_t* __restrict__ la = nullptr, long lda = 0,
                                                       int R = 0) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = N >> 3;
  const bf16_t* xr = x + (long)row * N;
  float v[CH][8];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      load8(xr + ch * 8, v[c]);
      if (RESID) {
        float dv[8];
        load8(d + (long)row * N + ch * 8, dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += dv[j];
        store8(s_out + (long)row * N + ch * 8, v[c]);
        // round like the stored residual so forward/backward see the same value
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(f2bf(v[c][j]));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += v[c][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
  float mean = 0.f;
  if (!RMS) mean = wave_sum(sum) / N;
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = v[c][j] - mean;
        sq += t * t;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) / N + eps);
  float up[LR > 0 ? LR : 1];  // LoRA: this lane's partial sums of y . A[r]
#pragma unroll
  for (int r = 0; r < (LR > 0 ? LR : 1); ++r) up[r] = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float o[8];
      const float4* w4 = reinterpret_cast<const float4*>(w + ch * 8);
      float4 wa = w4[0], wb = w4[1];
      float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
      if (RMS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[c][j] * rstd * (wv[j] + w_offset);
      } else {
        const float4* b4 = reinterpret_cast<const float4*>(b + ch * 8);
        float4 ba = b4[0], bb = b4[1];
        float bv[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * rstd * wv[j] + bv[j];
      }
      store8(y + (long)row * ldy + ch * 8, o);
      if constexpr (LR > 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(o[j]));  // the consumer reads the stored bf16 row
#pragma unroll
        for (int r = 0; r < LR; ++r) {
          if (r < R) {
            float av[8];
            load8(la + (long)r * lda + ch * 8, av);
#pragma unroll
            for (int j = 0; j < 8; ++j) up[r] = fmaf(o[j], av[j], up[r]);
          }
        }
      }
    }
  }
  if constexpr (LR > 0) {
#pragma unroll
    for (int r = 0; r < LR; ++r)
      if (r < R) up[r] = wave_sum(up[r]);
  }
  // a wider output row (appended LoRA columns, see kernels.h): u in the first R of them (LoRA
  // fusion), the rest zeroed
  for (long c = N + lane * 8; c < ldy; c += 64 * 8) {
    float z[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      z[j] = 0.f;
      if constexpr (LR > 0) {
        const long r = c - N + j;
#pragma unroll
        for (int q = 0; q < LR; ++q)
          if (r == q && q < R) z[j] = up[q];
      }
    }
    store8(y + (long)row * ldy + c, z);
  }
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Backward: dx = rstd * (w*dy - mean(w*dy) - xhat*mean(w*dy*xhat))  (LayerNorm)
//           dx = rstd * (w'*dy - xhat*mean(w'*dy*xhat))              (RMSNorm, w' = w + offset)
// plus optional dresid added in (residual branch of a fused add+norm).  dw/db partials are
// accumulated per block over its rows (grid-stride) into part[blockIdx][N] (fp32); a second tiny
// kernel sums the partials, so no float atomics are needed and the result is deterministic.
template <int CH, bool RMS, bool WGRAD, int U = WGRAD ? 4 : 1>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                       const float* __restrict__ w, const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in, const bf16_t* __restrict__ dresid,
                                                       bf16_t* __restrict__ dx, float* __restrict__ dw_part,
                                                       float* __restrict__ db_part, int M, int N, float w_offset,
                                                       long lddy) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = N >> 3;
  float dwa[CH][8], dba[CH][8];
  if (WGRAD) {
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) dwa[c][j] = dba[c][j] = 0.f;
  }
  // the lane's weights, once
  float wv[CH][8];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      const float4* w4 = reinterpret_cast<const float4*>(w + ch * 8);
      const float4 wa = w4[0], wb = w4[1];
      wv[c][0] = wa.x + w_offset, wv[c][1] = wa.y + w_offset, wv[c][2] = wa.z + w_offset, wv[c][3] = wa.w + w_offset;
      wv[c][4] = wb.x + w_offset, wv[c][5] = wb.y + w_offset, wv[c][6] = wb.z + w_offset, wv[c][7] = wb.w + w_offset;
    }
  }
  // U rows per wave per iteration, every load of the U rows issued before the first is used: the
  // weight-gradient form runs a bounded grid (512 blocks, one row at a time left it latency-bound at
  // ~2 TB/s: a few MB in flight across the chip)
  const int stride = gridDim.x * 4;
  for (int row0 = blockIdx.x * 4 + wid; row0 < M; row0 += stride * U) {
    u16x8_t xr[U][CH], dr[U][CH], rr[U][CH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = row0 + u * stride;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int ch = lane + c * 64;
        if (row < M && ch < nch) {
          xr[u][c] = *reinterpret_cast<const u16x8_t*>(x + (long)row * N + ch * 8);
          dr[u][c] = *reinterpret_cast<const u16x8_t*>(dy + (long)row * lddy + ch * 8);
          if (dresid) rr[u][c] = *reinterpret_cast<const u16x8_t*>(dresid + (long)row * N + ch * 8);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = row0 + u * stride;
      if (row >= M) break;  // (wave-uniform)
      const float mean = RMS ? 0.f : mean_in[row];
      const float rstd = rstd_in[row];
      float xh[CH][8], g[CH][8];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float dv = bf2f(dr[u][c][j]);
            xh[c][j] = (bf2f(xr[u][c][j]) - mean) * rstd;
            g[c][j] = dv * wv[c][j];
            s1 += g[c][j];
            s2 += g[c][j] * xh[c][j];
            if (WGRAD) {
              dwa[c][j] += dv * xh[c][j];
              dba[c][j] += dv;
            }
          }
        }
      }
      s1 = RMS ? 0.f : wave_sum(s1) / N;
      s2 = wave_sum(s2) / N;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = rstd * (g[c][j] - s1 - xh[c][j] * s2);
          if (dresid) {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] += bf2f(rr[u][c][j]);
          }
          store8(dx + (long)row * N + ch * 8, o);
        }
      }
    }
  }
  if (WGRAD) {
    // reduce the 4 waves of the block through LDS, then one row of partials per block
    extern __shared__ __attribute__((aligned(16))) float red[];  // [4][N] x2
    for (int c = 0; c < CH; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch)
        for (int j = 0; j < 8; ++j) {
          red[wid * N + ch * 8 + j] = dwa[c][j];
          red[4 * N + wid * N + ch * 8 + j] = dba[c][j];
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
      float a = red[i] + red[N + i] + red[2 * N + i] + red[3 * N + i];
      float bb = red[4 * N + i] + red[5 * N + i] + red[6 * N + i] + red[7 * N + i];
      dw_part[(long)blockIdx.x * N + i] = a;
      if (!RMS) db_part[(long)blockIdx.x * N + i] = bb;
    }
  }
}

// out[i] (+)= sum_b part[b][i].  256 threads = 32 columns x 8 row-lanes: each row-lane strides over
// the partial rows (coalesced 128-B column segments), the 8 lanes are combined through LDS.  (A
// thread-per-column loop over 512 partial rows was a 512-deep dependent chain: ~120 us per call.)
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ part, float* __restrict__ out, int nb,
                                                          int N, int accumulate) {
  __shared__ float red[8][33];
  const int c = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int i = blockIdx.x * 32 + c;
  float s = 0.f;
  if (i < N) {
#pragma unroll 4
    for (int b = rl; b < nb; b += 8) s += part[(long)b * N + i];
  }
  red[rl][c] = s;
  __syncthreads();
  if (rl == 0 && i < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][c];
    out[i] = accumulate ? out[i] + t : t;
  }
}

template <bool RMS>
static void norm_fwd_dispatch(const bf16_t* x, const bf16_t* d, bf16_t* s_out, const float* w, const float* b,
                              bf16_t* y, float* mean, float* rstd, int M, int N, float eps, float w_offset,
                              long ldy, hipStream_t st, const bf16_t* la = nullptr, long lda = 0, int R = 0) {
  const int nch = N / 8, ch = (nch + 63) / 64;
  dim3 grid(cdiv(M, 4)), block(256);
  if (la && R > 0) {  // fused LoRA input projection: R <= 32 ranks, appended columns hold them
    if (R > 32 || ldy < N + R) {
      fprintf(stderr, "mft::norm_fwd: LoRA fusion needs R <= 32 appended columns (R=%d, ldy=%ld, N=%d)\n", R, ldy, N);
      abort();
    }
#define MFT_NFL(CHV, LRV)                                                                                      \
  if (d)                                                                                                       \
    norm_fwd_kernel<CHV, RMS, true, LRV><<<grid, block, 0, st>>>(x, d, s_out, w, b, y, mean, rstd, M, N, eps, w_offset, ldy, la, lda, R); \
  else                                                                                                         \
    norm_fwd_kernel<CHV, RMS, false, LRV><<<grid, block, 0, st>>>(x, d, s_out, w, b, y, mean, rstd, M, N, eps, w_offset, ldy, la, lda, R);
#define MFT_NFR(LRV)                  \
  if (ch <= 1) { MFT_NFL(1, LRV) }    \
  else if (ch <= 2) { MFT_NFL(2, LRV) } \
  else if (ch <= 4) { MFT_NFL(4, LRV) } \
  else { MFT_NFL(8, LRV) }
    if (R <= 8) { MFT_NFR(8) }
    else if (R <= 16) { MFT_NFR(16) }
    else { MFT_NFR(32) }
#undef MFT_NFR
#undef MFT_NFL
    return;
  }
#define MFT_NF(CHV)                                                                                        \
  if (d)                                                                                                   \
    norm_fwd_kernel<CHV, RMS, true><<<grid, block, 0, st>>>(x, d, s_out, w, b, y, mean, rstd, M, N, eps, w_offset, ldy); \
  else                                                                                                     \
    norm_fwd_kernel<CHV, RMS, false><<<grid, block, 0, st>>>(x, d, s_out, w, b, y, mean, rstd, M, N, eps, w_offset, ldy);
  if (ch <= 1) { MFT_NF(1) }
  else if (ch <= 2) { MFT_NF(2) }
  else if (ch <= 4) { MFT_NF(4) }
  else { MFT_NF(8) }
#undef MFT_NF
}

template <bool RMS>
static void norm_bwd_dispatch(const bf16_t* x, const bf16_t* dy, const float* w, const float* mean, const float* rstd,
                              const bf16_t* dresid, bf16_t* dx, float* dw, float* db, float* work, int M, int N,
                              float w_offset, int accumulate, long lddy, hipStream_t st) {
  const int nch = N / 8, ch = (nch + 63) / 64;
  const bool wgrad = dw != nullptr;
  // with weight grads: a bounded grid so the partial buffer stays small (work: 2*nb*N floats)
  // without weight grads: U rows per wave (MFT_NORM_BWD_U=1|2, A/B), the grid covering M once
  static const int unw = getenv("MFT_NORM_BWD_U") && getenv("MFT_NORM_BWD_U")[0] == '2' ? 2 : 1;
  const int nb = wgrad ? norm_bwd_partial_blocks(M) : cdiv(M, 4 * unw);
  float* dw_part = work;
  float* db_part = work ? work + (long)nb * N : nullptr;
  const size_t shm = wgrad ? sizeof(float) * 8 * N : 0;
  dim3 grid(nb), block(256);
#define MFT_NB(CHV)                                                                                           \
  if (wgrad)                                                                                                  \
    norm_bwd_kernel<CHV, RMS, true><<<grid, block, shm, st>>>(x, dy, w, mean, rstd, dresid, dx, dw_part, db_part, M, N, w_offset, lddy); \
  else if (unw == 2)                                                                                          \
    norm_bwd_kernel<CHV, RMS, false, 2><<<grid, block, 0, st>>>(x, dy, w, mean, rstd, dresid, dx, dw_part, db_part, M, N, w_offset, lddy); \
  else                                                                                                        \
    norm_bwd_kernel<CHV, RMS, false><<<grid, block, 0, st>>>(x, dy, w, mean, rstd, dresid, dx, dw_part, db_part, M, N, w_offset, lddy);
  if (ch <= 1) { MFT_NB(1) }
  else if (ch <= 2) { MFT_NB(2) }
  else if (ch <= 4) { MFT_NB(4) }
  else { MFT_NB(8) }
#undef MFT_NB
  if (wgrad) {
    reduce_rows_kernel<<<cdiv(N, 32), 256, 0, st>>>(dw_part, dw, nb, N, accumulate);
    if (!RMS && db) reduce_rows_kernel<<<cdiv(N, 32), 256, 0, st>>>(db_part, db, nb, N, accumulate);
  }
}

void reduce_rows(const float* part, float* out, int nb, int N, int accumulate, hipStream_t st) {
  reduce_rows_kernel<<<cdiv(N, 32), 256, 0, st>>>(part, out, nb, N, accumulate);
}

int norm_bwd_partial_blocks(int M) {
  int nb = (M + 3) / 4;
  return nb < 512 ? nb : 512;
}

void layernorm_fwd(const bf16_t* x, const bf16_t* resid_delta, bf16_t* resid_out, const float* w, const float* b,
                   bf16_t* y, float* mean, float* rstd, int M, int N, float eps, long ldy, hipStream_t st,
                   const bf16_t* lora_a, long lda, int lora_r) {
  norm_fwd_dispatch<false>(x, resid_delta, resid_out, w, b, y, mean, rstd, M, N, eps, 0.f, ldy > 0 ? ldy : N, st,
                           lora_a, lda, lora_r);
}

void rmsnorm_fwd(const bf16_t* x, const bf16_t* resid_delta, bf16_t* resid_out, const float* w, bf16_t* y,
                 float* rstd, int M, int N, float eps, float w_offset, long ldy, hipStream_t st,
                 const bf16_t* lora_a, long lda, int lora_r) {
  norm_fwd_dispatch<true>(x, resid_delta, resid_out, w, nullptr, y, nullptr, rstd, M, N, eps, w_offset,
                          ldy > 0 ? ldy : N, st, lora_a, lda, lora_r);
}

void layernorm_bwd(const bf16_t* x, const bf16_t* dy, const float* w, const float* mean, const float* rstd,
                   const bf16_t* dresid, bf16_t* dx, float* dw, float* db, float* work, int M, int N, int accumulate,
                   long lddy, hipStream_t st) {
  norm_bwd_dispatch<false>(x, dy, w, mean, rstd, dresid, dx, dw, db, work, M, N, 0.f, accumulate,
                           lddy > 0 ? lddy : N, st);
}

void rmsnorm_bwd(const bf16_t* x, const bf16_t* dy, const float* w, const float* rstd, const bf16_t* dresid,
                 bf16_t* dx, float* dw, float* work, int M, int N, float w_offset, int accumulate, long lddy,
                 hipStream_t st) {
  norm_bwd_dispatch<true>(x, dy, w, nullptr, rstd, dresid, dx, dw, nullptr, work, M, N, w_offset, accumulate,
                          lddy > 0 ? lddy : N, st);
}

}  // namespace mft
