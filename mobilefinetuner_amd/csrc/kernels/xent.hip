// Fused softmax cross-entropy forward+backward over a (chunk of) bf16 logits rows.
// Replaces lm_cross_entropy + LMCrossEntropyBackward (core/lm_loss.cpp:19-210): the reference
// materialises fp32 logits [B,S,V], then recomputes the softmax per row in backward.  Here one
// workgroup per row does ONE online (max, sum-exp) pass and ONE pass that overwrites the logits
// in place with (softmax - onehot) * scale, so a chunk of logits sized to stay in the 256 MiB
// Infinity Cache is written by the LM-head GEMM, read twice here and consumed by the dgrad GEMM
// without a round trip to HBM (see ops/lm_head.py for the chunking).
#include "common.h"
#include "kernels.h"

namespace mft {

__global__ __launch_bounds__(256) void xent_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                   float* __restrict__ loss, int V, long ld,
                                                   const float* __restrict__ scale_ptr, float extra, int write_grad) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  bf16_t* x = logits + row * ld;
  const int64_t lab = labels[row];
  const int nv8 = V / 8;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < nv8; c += blockDim.x) {
    float v[8];
    load8(x + c * 8, v);
    float lm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
    if (lm > m) {
      s *= __expf(m - lm);
      m = lm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
  }
  for (int c = nv8 * 8 + threadIdx.x; c < V; c += blockDim.x) {
    const float v = bf2f(x[c]);
    if (v > m) {
      s *= __expf(m - v);
      m = v;
    }
    s += __expf(v - m);
  }
  const float gm = block_max(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  __syncthreads();
  const float gs = block_sum(s, red);
  const float lse = gm + __logf(gs);
  const bool valid = lab >= 0 && lab < V;
  if (threadIdx.x == 0) loss[row] = valid ? lse - bf2f(x[lab]) : 0.f;
  if (!write_grad) return;
  __syncthreads();  // the label logit must be read before anyone overwrites it
  const float sc = valid ? (scale_ptr ? *scale_ptr : 1.f) * extra : 0.f;
  for (int c = threadIdx.x; c < nv8; c += blockDim.x) {
    float v[8];
    load8(x + c * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(v[j] - lse);
      if (c * 8 + j == lab) p -= 1.f;
      v[j] = p * sc;
    }
    store8(x + c * 8, v);
  }
  for (long c = nv8 * 8 + threadIdx.x; c < ld; c += blockDim.x) {
    if (c < V) {
      float p = __expf(bf2f(x[c]) - lse);
      if (c == lab) p -= 1.f;
      x[c] = f2bf(p * sc);
    } else {
      x[c] = 0;
    }
  }
}

// (Measured: unrolling both passes to 4 independent 16-B loads per thread left the Gemma-3 bench
// unchanged, 483K vs 485K tok/s -- the two-pass form already streams at ~5.2 TB/s.)

// Register-resident variant for V <= 8 * CPT * 1024 (GPT-2: 50304 columns = 6.1 chunks of 8 per
// thread): a 1024-thread workgroup holds its whole row in VGPRs (packed bf16), so the logits are
// read from memory ONCE (the two-pass form above re-reads a 100 KB row that no longer sits in L2
// when 8k rows stream through) and the gradient is written once.
// Measured alternatives (GPT-2 bench, 65536 rows x 50304, MI355X): this form 2.99 ms (4.4 TB/s of
// read+write); 256 threads per row with 28 chunks each (4 rows in flight per CU) 3.47 ms (VGPR spills
// at 4 waves/SIMD); one fused (max, sum-exp) pair reduction instead of two block reductions 3.12 ms.
template <int CPT>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void xent_reg_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                        float* __restrict__ loss, int V, long ld,
                                                        const float* __restrict__ scale_ptr, float extra, int write_grad) {
  __shared__ float red[32];
  const long row = blockIdx.x;
  bf16_t* x = logits + row * ld;
  const int64_t lab = labels[row];
  const bool valid = lab >= 0 && lab < V;
  const float xl = (threadIdx.x == 0 && valid) ? bf2f(x[lab]) : 0.f;  // read before any overwrite
  const int nld8 = (int)(ld / 8);  // chunks incl. padding columns (written as 0 in the gradient)
  u16x8_t v[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 1024;
    v[i] = c < nld8 ? *reinterpret_cast<const u16x8_t*>(x + c * 8) : u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 1024;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c * 8 + j < V) m = fmaxf(m, bf2f(v[i][j]));
  }
  const float gm = block_max(m, red);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 1024;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c * 8 + j < V) s += __expf(bf2f(v[i][j]) - gm);
  }
  __syncthreads();
  const float gs = block_sum(s, red);
  const float lse = gm + __logf(gs);
  if (threadIdx.x == 0) loss[row] = valid ? lse - xl : 0.f;
  if (!write_grad) return;
  const float sc = valid ? (scale_ptr ? *scale_ptr : 1.f) * extra : 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 1024;
    if (c >= nld8) continue;
    float g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c * 8 + j;
      float p = col < V ? __expf(bf2f(v[i][j]) - lse) : 0.f;
      if (col == lab) p -= 1.f;
      g[j] = p * sc;
    }
    store8(x + c * 8, g);
  }
}

// out[m, c] = logits[m, idx[c]] - logsumexp(logits[m, :V])
__global__ __launch_bounds__(256) void logsoftmax_gather_kernel(const bf16_t* __restrict__ logits,
                                                                const int64_t* __restrict__ idx, float* __restrict__ out,
                                                                int V, long ld, int nidx) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < V; c += blockDim.x) {
    const float v = bf2f(x[c]);
    if (v > m) {
      s *= __expf(m - v);
      m = v;
    }
    s += __expf(v - m);
  }
  const float gm = block_max(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  __syncthreads();
  const float gs = block_sum(s, red);
  const float lse = gm + __logf(gs);
  for (int c = threadIdx.x; c < nidx; c += blockDim.x) out[row * nidx + c] = bf2f(x[idx[c]]) - lse;
}

// ------------------------------------------------------------------ fused LM head + CE (lm_head_ce)
// Row positions inside a 256-row tile in the order the CE dgrad main loop reads its row factors:
// lane (r16) of wave-row wm reads rows qa * 128 + wm * 64 + 16 i + r16 (i = 0..3) as one 16-B word.
__device__ __forceinline__ int ce_row_pos(int R) {
  const int rl = R & 255;
  return (R & ~255) + (rl >> 6) * 64 + (rl & 15) * 4 + ((rl >> 4) & 3);
}

// 64 rows per block.  Pass 1 (a wave per row, lanes over vocab tiles): row max of the tile maxima,
// lse = max + log sum_t s_t exp(m_t - max), loss, the dgrad's final factor and label weight.
// Pass 2: ratio[t][pos(R)] = exp(m'_{t-1} - m'_t), m'_t = max(m_t, rowmax - 60) (a tile 60 below
// the row max contributes < e^-60: clamping keeps every ratio and partial sum finite in fp32).
__global__ __launch_bounds__(256) void ce_finalize_kernel(const float2* __restrict__ stats, const float* __restrict__ lbl,
                                                          const int64_t* __restrict__ labels, int M, int T, int V,
                                                          long mpad, const float* __restrict__ scale, float extra,
                                                          float* __restrict__ loss, float* __restrict__ lse_out,
                                                          float* __restrict__ ratio, float* __restrict__ fin,
                                                          float* __restrict__ wlab) {
  __shared__ float s_mx[64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r0 = blockIdx.x * 64;
  for (int rr = w; rr < 64; rr += 4) {
    const int R = r0 + rr;
    if (R >= M) break;
    const float2* st = stats + (long)R * T;
    float m = -INFINITY;
    for (int t = lane; t < T; t += 64) m = fmaxf(m, st[t].x);
    m = wave_max(m);
    float s = 0.f;
    for (int t = lane; t < T; t += 64) {
      const float2 v = st[t];
      if (v.y > 0.f) s += v.y * __expf(v.x - m);
    }
    s = wave_sum(s);
    if (lane == 0) {
      const float l = m + __logf(s);
      const int64_t lab = labels[R];
      const bool valid = lab >= 0 && lab < V;
      loss[R] = valid ? l - lbl[R] : 0.f;
      if (lse_out) lse_out[R] = l;
      if (fin) {
        const float wv = valid ? (scale ? *scale : 1.f) * extra : 0.f;
        wlab[R] = wv;
        fin[R] = wv * __expf(fmaxf(st[T - 1].x, m - 60.f) - l);
      }
      s_mx[rr] = m;
    }
  }
  if (!ratio) return;
  // Pass 2 in chunks of 64 tiles through LDS: the waves stage the block's rows' (clamped) tile maxima
  // with lanes over tiles (coalesced reads), then every thread writes one row's ratios with lanes over
  // rows (one 256-B segment per tile).  Reading the stats row-per-lane instead (64 rows T * 8 B apart
  // per instruction) made this kernel 5-7x its bandwidth time at Gemma-3's 1,024 vocab tiles.
  __shared__ float s_m[64][65];  // [row][tile in chunk], +1 pad: the lanes-over-rows reads are conflict-free
  __syncthreads();
  const int nrow = min(64, M - r0);
  const int rr2 = threadIdx.x & 63;
  const long dst = ce_row_pos(r0 + rr2);
  for (int c0 = 0; c0 < T - 1; c0 += 63) {  // chunk = tiles c0 .. c0 + 63: ratios of tiles c0 + 1 ..
    const int cn = min(64, T - c0);
    for (int rr = w; rr < nrow; rr += 4)
      if (lane < cn) s_m[rr][lane] = fmaxf(stats[(long)(r0 + rr) * T + c0 + lane].x, s_mx[rr] - 60.f);
    __syncthreads();
    if (rr2 < nrow)
      for (int j = 1 + w; j < cn; j += 4) ratio[(long)(c0 + j) * mpad + dst] = __expf(s_m[rr2][j - 1] - s_m[rr2][j]);
    __syncthreads();
  }
}

// E (exp(logit - tile max)) -> dlogits = (softmax - onehot) * w in place; padding columns stay 0
__global__ __launch_bounds__(256) void ce_materialize_kernel(bf16_t* __restrict__ E, long lde, int N,
                                                             const float2* __restrict__ stats, int T,
                                                             const float* __restrict__ lse,
                                                             const int64_t* __restrict__ labels, int V,
                                                             const float* __restrict__ scale, float extra) {
  const long R = blockIdx.x;
  const int64_t lab = labels[R];
  const bool valid = lab >= 0 && lab < V;
  const float wv = valid ? (scale ? *scale : 1.f) * extra : 0.f;
  const float l = lse[R];
  bf16_t* e = E + R * lde;
  for (int c8 = threadIdx.x; c8 < N / 8; c8 += blockDim.x) {
    const int c = c8 * 8;
    const float f = wv * __expf(stats[R * T + (c >> 8)].x - l);
    float v[8];
    load8(e + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] *= f;
      if (c + j == lab) v[j] -= wv;
    }
    store8(e + c, v);
  }
}

long lm_head_ce_ws_floats(int M, int Vpad) {
  const long T = (Vpad + 255) / 256, mpad = (long)((M + 255) / 256) * 256;
  return 2 * (long)M * T + 4L * M + T * mpad + 64;
}

void lm_head_ce(const CeArgs& a, hipStream_t st) {
  if (a.M <= 0) return;
  const int T = (a.Vpad + 255) / 256;
  const long mpad = (long)((a.M + 255) / 256) * 256;
  float* p = a.ws;
  float* stats = p; p += 2 * (long)a.M * T;
  float* lbl = p; p += a.M;
  float* lse = a.lse ? a.lse : p; p += a.M;
  float* fin = p; p += a.M;
  float* wlab = p; p += a.M;
  float* ratio = a.ws + ((p - a.ws + 63) / 64) * 64;  // 256-B aligned: read by 16-B LDS-DMA
  const bool grad = a.dh != nullptr;
  if (grad && !a.E) {
    fprintf(stderr, "mft::lm_head_ce: the gradient needs the E workspace\n");
    abort();
  }
  GemmArgs f{};
  f.A = a.h; f.lda = a.ldh;
  f.B = a.W; f.ldb = a.ldw;
  f.C = a.E; f.ldc = a.lde;
  f.M = a.M; f.N = a.Vpad; f.K = a.K; f.alpha = 1.f;
  f.ce_labels = a.labels; f.ce_stats = stats; f.ce_lbl = lbl; f.ce_V = a.V;
  gemm8x(f, GEMM_EPI_CE_FWD, false, false, st);
  const bool fused = grad && !a.materialize;
  ce_finalize_kernel<<<(a.M + 63) / 64, 256, 0, st>>>(reinterpret_cast<const float2*>(stats), lbl, a.labels, a.M, T,
                                                       a.V, mpad, a.scale, a.extra, a.loss, lse,
                                                       fused ? ratio : nullptr, fused ? fin : nullptr, wlab);
  if (!grad) return;
  GemmArgs d{};
  d.A = a.E; d.lda = a.lde;
  d.B = a.W; d.ldb = a.ldw;
  d.C = a.dh; d.ldc = a.lddh;
  d.M = a.M; d.N = a.K; d.K = a.Vpad; d.alpha = 1.f;
  if (a.materialize) {
    ce_materialize_kernel<<<a.M, 256, 0, st>>>(a.E, a.lde, a.Vpad, reinterpret_cast<const float2*>(stats), T, lse,
                                               a.labels, a.V, a.scale, a.extra);
    gemm8x(d, GEMM_EPI_NONE, false, true, st);
  } else {
    d.ce_labels = a.labels; d.ce_ratio = ratio; d.ce_fin = fin; d.ce_wlab = wlab;
    gemm8x(d, GEMM_EPI_CE_DGRAD, false, true, st);
  }
}

void xent_fwd_bwd(bf16_t* logits, const int64_t* labels, float* loss, long M, int V, long ld, const float* scale,
                  float extra, int write_grad, hipStream_t st) {
  if (M <= 0) return;
  const long nld8 = ld / 8;
  if (ld % 8 == 0 && nld8 <= 8L * 1024) {
    const int cpt = (int)((nld8 + 1023) / 1024);
    switch (cpt) {
#define MFT_XR(CPT) case CPT: xent_reg_kernel<CPT><<<M, 1024, 0, st>>>(logits, labels, loss, V, ld, scale, extra, write_grad); return;
      MFT_XR(1) MFT_XR(2) MFT_XR(3) MFT_XR(4) MFT_XR(5) MFT_XR(6) MFT_XR(7) MFT_XR(8)
#undef MFT_XR
      default: break;
    }
  }
  xent_kernel<<<M, 256, 0, st>>>(logits, labels, loss, V, ld, scale, extra, write_grad);
}

void logsoftmax_gather(const bf16_t* logits, const int64_t* idx, float* out, long M, int V, long ld, int nidx,
                       hipStream_t st) {
  if (M <= 0) return;
  logsoftmax_gather_kernel<<<M, 256, 0, st>>>(logits, idx, out, V, ld, nidx);
}

}  // namespace mft
