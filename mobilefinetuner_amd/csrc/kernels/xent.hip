// Fused softmax cross-entropy forward+backward over a (chunk of) bf16 logits rows.
// Replaces lm_cross_entropy + LMCrossEntropyBackward (core/lm_loss.cpp:19-210): the reference
// materialises fp32 logits [B,S,V], then recomputes the softmax per row in backward.  Here one
// workgroup per row does ONE online (max, sum-exp) pass and ONE pass that overwrites the logits
// in place with (softmax - onehot) * scale, so a chunk of logits sized to stay in the 256 MiB
// Infinity Cache is written by the LM-head GEMM, read twice here and consumed by the dgrad GEMM
// without a round trip to HBM (see ops/lm_head.py for the chunking).
#include "common.h"
#include <cstdlib>

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

// RB rows per block (64, or 32 / 16 when M / 64 blocks would not fill the CUs twice: Gemma-3 at
// 8,192 rows and 1,024 vocab tiles ran 128 blocks at 293 us, latency-bound).  Pass 1 (a wave per row, lanes over vocab tiles): row max of the tile maxima,
// lse = max + log sum_t s_t exp(m_t - max), loss, the dgrad's final factor and label weight.
// Pass 2: ratio[t][pos(R)] = exp(m'_{t-1} - m'_t), m'_t = max(m_t, rowmax - 60) (a tile 60 below
// the row max contributes < e^-60: clamping keeps every ratio and partial sum finite in fp32).
template <int RB>
__global__ __launch_bounds__(256) void ce_finalize_kernel(const float2* __restrict__ stats, const float* __restrict__ lbl,
                                                          const int64_t* __restrict__ labels, int M, int T, int V,
                                                          long mpad, const float* __restrict__ scale, float extra,
                                                          float* __restrict__ loss, float* __restrict__ lse_out,
                                                          float* __restrict__ ratio, float* __restrict__ fin,
                                                          float* __restrict__ wlab, int nsplit, int tps) {
  __shared__ float s_mx[RB];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r0 = blockIdx.x * RB;
  for (int rr = w; rr < RB; rr += 4) {
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
    // (every lane holds the butterfly-reduced m and s)
    const float l = m + __logf(s);
    const int64_t lab = labels[R];
    const bool valid = lab >= 0 && lab < V;
    const float wv = valid ? (scale ? *scale : 1.f) * extra : 0.f;
    if (lane == 0) {
      loss[R] = valid ? l - lbl[R] : 0.f;
      if (lse_out) lse_out[R] = l;
      s_mx[rr] = m;
      if (fin) wlab[R] = wv;
    }
    // the dgrad's final factor per vocab split: relative to the split's last tile's (clamped) max
    if (fin) {
      for (int sp = lane; sp < nsplit; sp += 64) {
        const int te = min((sp + 1) * tps, T) - 1;
        fin[(long)sp * M + R] = wv * __expf(fmaxf(st[te].x, m - 60.f) - l);
      }
    }
  }
  if (!ratio) return;
  // Pass 2 in chunks of 64 tiles through LDS: the waves stage the block's rows' (clamped) tile maxima
  // with lanes over tiles (coalesced reads), then every thread writes one row's ratios with lanes over
  // rows (one 256-B segment per tile).  Reading the stats row-per-lane instead (64 rows T * 8 B apart
  // per instruction) made this kernel 5-7x its bandwidth time at Gemma-3's 1,024 vocab tiles.
  __shared__ float s_m[RB][65];  // [row][tile in chunk], +1 pad: the lanes-over-rows reads are conflict-free
  __syncthreads();
  const int nrow = min(RB, M - r0);
  const int rr2 = threadIdx.x % RB, jg = threadIdx.x / RB;  // 256 / RB tile groups
  const long dst = ce_row_pos(r0 + rr2);
  for (int c0 = 0; c0 < T - 1; c0 += 63) {  // chunk = tiles c0 .. c0 + 63: ratios of tiles c0 + 1 ..
    const int cn = min(64, T - c0);
    for (int rr = w; rr < nrow; rr += 4)
      if (lane < cn) s_m[rr][lane] = fmaxf(stats[(long)(r0 + rr) * T + c0 + lane].x, s_mx[rr] - 60.f);
    __syncthreads();
    if (rr2 < nrow)
      for (int j = 1 + jg; j < cn; j += 256 / RB) ratio[(long)(c0 + j) * mpad + dst] = __expf(s_m[rr2][j - 1] - s_m[rr2][j]);
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

// dh[row, col] = sum_s slab[s][row][col] in split order (deterministic), bf16 out; 8 columns per thread
__global__ __launch_bounds__(256) void ce_split_reduce_kernel(const float* __restrict__ ws, int S, int M, int N,
                                                              bf16_t* __restrict__ dh, long lddh) {
  const long i8 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  const long MN = (long)M * N;
  if (i8 >= MN) return;
  f32x4_t a = *reinterpret_cast<const f32x4_t*>(ws + i8), b = *reinterpret_cast<const f32x4_t*>(ws + i8 + 4);
  for (int sp = 1; sp < S; ++sp) {
    a += *reinterpret_cast<const f32x4_t*>(ws + (long)sp * MN + i8);
    b += *reinterpret_cast<const f32x4_t*>(ws + (long)sp * MN + i8 + 4);
  }
  const long row = i8 / N, col = i8 % N;
  const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  store8(dh + row * lddh + col, v);
}

static int ce_num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    MFT_HIP_CHECK(hipGetDevice(&dev));
    MFT_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    if (n <= 0) n = 256;
  }
  return n;
}

// Vocab splits of the CE dgrad.  Its output dh [M, d_model] has only ceil(M / 256) x ceil(d / 256)
// tiles (Gemma-3 at 8,192 rows: 96 for 256 CUs), so a row chunk alone leaves most CUs idle and
// bounding the E buffer by small chunks used to cost 17 % (profiles/r3_ce_budget_and_attn_nw_ab.txt).
// Split the vocab (the dgrad's K) so tiles x splits fills the CUs in as few, as full rounds as
// possible: time ~ rounds / splits, a split only for a > 5 % gain, >= 4 vocab tiles per split, whole
// vocab tiles per split (the per-tile rescale chain restarts at a split's first tile with acc = 0).
// The reference recipe's 512-row chunk (6 output tiles) takes 40 splits: +1.5 % over the old floor of
// 16 vocab tiles per split (11 splits, 66 workgroups; profiles/r6_ce_split_short_ab.txt).
// MFT_CE_SPLIT forces a count (1 = off).
int ce_dgrad_splits(int M, int K, int Vpad) {
  const int nk = (Vpad + 63) / 64, T = (Vpad + 255) / 256;
  const int tiles = ((M + 255) / 256) * ((K + 255) / 256);
  auto ok = [&](int sp) {
    const int kps = (nk + sp - 1) / sp;
    return kps % 4 == 0 && (long)(sp - 1) * kps < nk;
  };
  if (const char* e = getenv("MFT_CE_SPLIT")) {
    const int f = atoi(e);
    if (f >= 1 && f <= 64 && ok(f)) return f;
  }
  const int cus = ce_num_cus();
  int best = 1;
  double best_t = 1.0 * ((tiles + cus - 1) / cus);
  for (int sp = 2; sp <= 64 && T / sp >= 4; ++sp) {
    if (!ok(sp)) continue;
    const double t = (double)((tiles * sp + cus - 1) / cus) / sp;
    if (t < best_t * 0.95) {
      best_t = t;
      best = sp;
    }
  }
  return best;
}

namespace {
struct CeLayout {
  float *stats, *lbl, *lse, *fin, *wlab, *ratio, *slab;
  long total;
};
// stats [M][T] float2 | lbl [M] | lse [M] | wlab [M] | fin [S][M] | ratio [T][mpad] (256-B aligned:
// read by 16-B LDS-DMA) | split slabs [S][M][K] fp32 (S > 1)
CeLayout ce_layout(float* base, int M, int Vpad, int K, int S) {
  const long T = (Vpad + 255) / 256, mpad = (long)((M + 255) / 256) * 256;
  CeLayout L{};
  long o = 0;
  auto take = [&](long n, bool align) {
    if (align) o = (o + 63) / 64 * 64;
    float* p = base ? base + o : nullptr;
    o += n;
    return p;
  };
  L.stats = take(2 * (long)M * T, false);
  L.lbl = take(M, false);
  L.lse = take(M, false);
  L.wlab = take(M, false);
  L.fin = take((long)S * M, false);
  L.ratio = take(T * mpad, true);
  L.slab = S > 1 ? take((long)S * M * K, true) : nullptr;
  L.total = o + 64;
  return L;
}
}  // namespace

long lm_head_ce_ws_floats(int M, int Vpad, int K) {
  return ce_layout(nullptr, M, Vpad, K, K > 0 ? ce_dgrad_splits(M, K, Vpad) : 1).total;
}

void lm_head_ce(const CeArgs& a, hipStream_t st) {
  if (a.M <= 0) return;
  const int T = (a.Vpad + 255) / 256;
  const long mpad = (long)((a.M + 255) / 256) * 256;
  const bool grad = a.dh != nullptr;
  const int S = grad && !a.materialize ? ce_dgrad_splits(a.M, a.K, a.Vpad) : 1;
  const CeLayout L = ce_layout(a.ws, a.M, a.Vpad, a.K, S);
  float* lse = a.lse ? a.lse : L.lse;
  if (grad && !a.E) {
    fprintf(stderr, "mft::lm_head_ce: the gradient needs the E workspace\n");
    abort();
  }
  GemmArgs f{};
  f.A = a.h; f.lda = a.ldh;
  f.B = a.W; f.ldb = a.ldw;
  f.C = a.E; f.ldc = a.lde;
  f.M = a.M; f.N = a.Vpad; f.K = a.K; f.alpha = 1.f;
  f.ce_labels = a.labels; f.ce_stats = L.stats; f.ce_lbl = L.lbl; f.ce_V = a.V;
  // the logits GEMM + CE epilogue on gemm4 (4-wave hand-scheduled kernel) where it runs; MFT_CE_G4=0 -> gemm8
  const bool ce_g4 = !(getenv("MFT_CE_G4") && getenv("MFT_CE_G4")[0] == '0');
  if (ce_g4 && gemm4_supported(a.M, a.Vpad, a.K, false, false) && a.ldh % 8 == 0 && a.ldw % 8 == 0)
    gemm4x(f, GEMM_EPI_CE_FWD, false, false, st);
  else
    gemm8x(f, GEMM_EPI_CE_FWD, false, false, st);
  const bool fused = grad && !a.materialize;
  const int nk = (a.Vpad + 63) / 64, tps = ((nk + S - 1) / S) / 4;
  {
    auto fk = ce_finalize_kernel<64>;
    int rb = 64;
    for (; rb > 16 && (a.M + rb - 1) / rb < 2 * ce_num_cus(); rb /= 2) {}
    if (rb == 32) fk = ce_finalize_kernel<32>;
    if (rb == 16) fk = ce_finalize_kernel<16>;
    fk<<<(a.M + rb - 1) / rb, 256, 0, st>>>(reinterpret_cast<const float2*>(L.stats), L.lbl, a.labels, a.M, T, a.V,
                                            mpad, a.scale, a.extra, a.loss, lse, fused ? L.ratio : nullptr,
                                            fused ? L.fin : nullptr, L.wlab, S, S > 1 ? tps : T);
  }
  if (!grad) return;
  GemmArgs d{};
  d.A = a.E; d.lda = a.lde;
  d.B = a.W; d.ldb = a.ldw;
  d.C = a.dh; d.ldc = a.lddh;
  d.M = a.M; d.N = a.K; d.K = a.Vpad; d.alpha = 1.f;
  if (a.materialize) {
    ce_materialize_kernel<<<a.M, 256, 0, st>>>(a.E, a.lde, a.Vpad, reinterpret_cast<const float2*>(L.stats), T, lse,
                                               a.labels, a.V, a.scale, a.extra);
    // with the caller's W^T: the 4-wave NT kernel (K = Vpad contiguous in both operands) instead of the
    // 8-wave NN form (MFT_CE_NN8=1 keeps it, A/B)
    static const bool nn8 = getenv("MFT_CE_NN8") && getenv("MFT_CE_NN8")[0] == '1';
    if (!nn8 && a.Wt && a.ldwt % 8 == 0 && a.lde % 8 == 0 && gemm4_supported(a.M, a.K, a.Vpad, false, false)) {
      d.B = a.Wt;
      d.ldb = a.ldwt;
      gemm4x(d, GEMM_EPI_NONE, false, false, st);
    } else {
      gemm8x(d, GEMM_EPI_NONE, false, true, st);
    }
  } else {
    d.ce_labels = a.labels; d.ce_ratio = L.ratio; d.ce_fin = L.fin; d.ce_wlab = L.wlab;
    if (S > 1) {
      d.ksplit = S;
      d.ws = L.slab;
    }
    gemm8x(d, GEMM_EPI_CE_DGRAD, false, true, st);
    if (S > 1) {
      const long n8 = (long)a.M * a.K / 8;
      ce_split_reduce_kernel<<<(int)((n8 + 255) / 256), 256, 0, st>>>(L.slab, S, a.M, a.K, a.dh, a.lddh);
    }
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
