// LoRA rank-r kernels: the skinny products around the frozen base GEMM.
//
// Replaces LoRALinear::forward/merge/unmerge (nn/lora_linear.cpp:47-178), whose partial-column
// slices were added without autograd, and the never-constructed
// LoRALinearBackward (core/backward_functions.cpp:1012-1226).
//
// Internal layouts: A is [R, K] (PEFT lora_A.weight), B is [R, N] (reference lora_B layout), so
// every rank-r operand is read along contiguous rows.  For y = x W^T + s (x A^T) B:
//   lora_rowdot : U[m, r] = s * sum_k X[m, k] Wt[r, k]           u = x A^T (Wt = A), v = s dy B^T (Wt = B)
//                 MFMA 16x16x32: one 16-row tile and the whole K per wave (no LDS, no barrier);
//                 X streamed once from HBM with 16-B loads, two batches of k-steps in flight.
//   lora_update : Y[m, n] = base[m, n] + s * sum_r U[m, r] W[r, n]  y += s u B (W = B), dx += v A (W = A)
//                 VALU; each thread keeps its 8 columns of W in registers for a strip of rows.
//   lora_wgrad  : out[k*osk + r*osr] += scale * sum_m X[m, k] Y[m, r]
//                 dA = v^T x, dB = s u^T dy.  MFMA with the X / Y tiles staged row-major in LDS
//                 and read transposed (ds_read_b64_tr_b16); one fp32 atomic per output element
//                 per 512-row chunk straight into the flat grad buffer (accumulation semantics).
//   lora_merge  : W[k, n] += s * sum_r A[r, k] B[r, n]                merge / unmerge (K10)
#include <cstdlib>
#include "mfma.h"
#include "kernels.h"

namespace mft {

// ------------------------------------------------------------------------------------ dropout
// PEFT applies dropout to the LoRA input: u = dropout(x) A^T (the reference stored lora_dropout but
// never applied it).  The mask is a counter-based hash of (step counter, layer salt,
// element index): recomputed wherever it is needed (u in forward, dA and the dx term in backward), so
// no mask tensor is ever written.  The step counter lives on the device (graph-replay safe).
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352dU;
  h ^= h >> 15;
  h *= 0x846ca68bU;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ float drop_mult(const LoraDrop& d, uint32_t seed, long m, int k, int K) {
  const uint64_t idx = (uint64_t)m * (uint64_t)K + (uint64_t)k;
  const uint32_t h = mix32((uint32_t)idx ^ mix32((uint32_t)(idx >> 32) ^ seed));
  return ((h >> 8) * (1.0f / 16777216.0f)) >= d.p ? 1.0f / (1.0f - d.p) : 0.0f;
}
__device__ __forceinline__ uint32_t drop_seed(const LoraDrop& d) {
  return mix32(d.salt * 0x9E3779B9U ^ (uint32_t)(d.ctr ? *d.ctr : 0) * 0x85EBCA6BU);
}
__device__ __forceinline__ bf16x8_t apply_drop8(bf16x8_t a, const LoraDrop& d, uint32_t seed, long m, int k, int K) {
  u16x8_t v = __builtin_bit_cast(u16x8_t, a);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) * drop_mult(d, seed, m, k + j, K));
  return __builtin_bit_cast(bf16x8_t, v);
}

// ------------------------------------------------------------------------------------ rowdot
// U[m, r] = s * sum_k X[m, k] Wt[r, k] on v_mfma_f32_16x16x32_bf16.  A wave owns 16 rows and the WHOLE K --
// no cross-wave reduction, no LDS, no barrier.  X / Wt fragments come in batches of UNR k-steps, the next
// batch's loads issued before the current batch's MFMAs (two batches in flight); k past K (K % 8 == 0) and
// rows past M read as zeros.  (Round 5's form split K over the 4 waves of a 16-row workgroup and reduced
// through LDS behind a barrier, and silently dropped a K % 32 tail; this one measured the same end to end,
// profiles/r6_rowdot_wave_ab.txt.)
template <int RT>
__global__ __launch_bounds__(256) void lora_rowdot_kernel(const bf16_t* __restrict__ X, long ldx,
                                                            const bf16_t* __restrict__ Wt, long ldw, bf16_t* __restrict__ U,
                                                            long ldu, long M, int K, int R, float s, LoraDrop drop) {
  constexpr int UNR = RT == 1 ? 8 : RT == 2 ? 4 : 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long m0 = ((long)blockIdx.x * 4 + w) * 16;
  if (m0 >= M) return;  // (wave-uniform; nothing below synchronises the workgroup)
  const uint32_t dseed = drop.p > 0.f ? drop_seed(drop) : 0u;
  const long mr = m0 + (lane & 15);
  const bool row_ok = mr < M;
  const int nks = (K + 31) / 32;
  f32x4_t acc[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) acc[t] = zero4();
  bf16x8_t a[2][UNR], b[2][UNR][RT];
  auto load = [&](int buf, int kb) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int k = (kb + u) * 32 + 8 * (lane >> 4);
      const bool ok = k < K;  // (K % 8 == 0: an 8-column chunk is in or out as a whole)
      a[buf][u] = (ok && row_ok) ? *reinterpret_cast<const bf16x8_t*>(X + mr * ldx + k) : bf16x8_t{};
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const int r = t * 16 + (lane & 15);
        b[buf][u][t] = (ok && r < R) ? *reinterpret_cast<const bf16x8_t*>(Wt + (long)r * ldw + k) : bf16x8_t{};
      }
    }
  };
  auto mul = [&](int buf, int kb) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      bf16x8_t x = a[buf][u];
      if (drop.p > 0.f) x = apply_drop8(x, drop, dseed, mr, (kb + u) * 32 + 8 * (lane >> 4), K);
#pragma unroll
      for (int t = 0; t < RT; ++t) acc[t] = mfma16(x, b[buf][u][t], acc[t]);
    }
  };
  load(0, 0);
  for (int kb = 0; kb < nks; kb += 2 * UNR) {
    load(1, kb + UNR);
    mul(0, kb);
    if (kb + 2 * UNR < nks) load(0, kb + 2 * UNR);
    if (kb + UNR < nks) mul(1, kb + UNR);
  }
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long m = m0 + 4 * (lane >> 4) + i;
      const int r = t * 16 + (lane & 15);
      if (m < M && r < R) U[m * ldu + r] = f2bf(acc[t][i] * s);
    }
}

// ------------------------------------------------------------------------------------ update
// grid (ceil(N/8/blockDim), ceil(M/ROWS)); thread owns 8 columns, W[0..R)[n..n+8) in registers.
// With dropout (dx += mask * (v A) in backward) the mask of element (m, n) is re-derived.
template <int R>
__global__ __launch_bounds__(256) void lora_update_kernel(const bf16_t* base, long ldb, const bf16_t* __restrict__ U, long ldu,
                                                          const bf16_t* __restrict__ W, long ldw, bf16_t* Y, long ldy, long M,
                                                          int N, int rows, float s, LoraDrop drop) {
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (n >= N) return;
  const uint32_t dseed = drop.p > 0.f ? drop_seed(drop) : 0u;
  float wr[R][8];
#pragma unroll
  for (int r = 0; r < R; ++r) load8(W + (long)r * ldw + n, wr[r]);
  const long m0 = (long)blockIdx.y * rows;
  const long m1 = min(M, m0 + rows);
  for (long m = m0; m < m1; ++m) {
    float y[8], u[R], d[8];
    load8(base + m * ldb + n, y);
#pragma unroll
    for (int r = 0; r < R; ++r) u[r] = bf2f(U[m * ldu + r]) * s;
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] += u[r] * wr[r][j];
    if (drop.p > 0.f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] *= drop_mult(drop, dseed, m, n + j, N);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] += d[j];
    store8(Y + m * ldy + n, y);
  }
}

// ------------------------------------------------------------------------------------ wgrad
// Streaming VALU form: the reduction runs over M (the long axis) so every X element is read
// exactly once with fully coalesced 8-B/lane loads.  A 1024-thread block = 16 waves that share one
// 256-column strip (4 columns per lane) and split the block's row chunk round-robin; each lane keeps
// a 4 x RB fp32 outer-product tile in registers and issues U independent row loads before using any
// (the kernel is pure HBM streaming: bytes in flight, not FLOPs, set its speed).  The 16 wave tiles
// are folded in LDS (16 -> 8 -> final sum) and each output element gets ONE fp32 atomic per block,
// straight into the grad buffer.  The launcher picks the row chunk so that ~4 waves per SIMD are
// live while atomics stay a small fraction of the X traffic.
template <int RB, bool YVEC, bool DROP>
__global__ __launch_bounds__(1024) void lora_wgrad_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ Y,
                                                          long ldy, float* __restrict__ out, long osk, long osr, long M, int K,
                                                          int R, long chunk, float scale, LoraDrop drop, WgradOuts outs,
                                                          float* __restrict__ det_ws, long det_kp) {
  constexpr int U = DROP ? 6 : 12;
  __shared__ __attribute__((aligned(16))) float red[8][RB][256];
  __shared__ __attribute__((aligned(16))) bf16_t ysh[2][16 * U][RB];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int k = blockIdx.x * 256 + lane * 4;
  const int r0 = blockIdx.z * RB;
  const long mbeg = (long)blockIdx.y * chunk;
  const long mend = min(M, mbeg + chunk);
  const bool kok = k < K;
  const uint32_t dseed = DROP ? drop_seed(drop) : 0u;
  float acc[4][RB];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[j][r] = 0.f;
  // all X loads are unconditional (row / column indices clamped into range; out-of-range rows are
  // zeroed after the load) so the U row loads issue back to back.  Y rows of the block's current
  // 16*U-row tile are staged once in LDS (double-buffered: one barrier per tile) and read back as
  // wave-uniform broadcasts.
  const int kc = kok ? k : K - 4;
  int t = 0;
  for (long mb0 = mbeg; mb0 < mend; mb0 += 16 * U, ++t) {
    bf16_t* ys = ysh[t & 1][0];
    // Y tile load first (its wait then covers only itself), X loads next, then the LDS store
    const long my = mb0 + threadIdx.x;
    const bool ystage = threadIdx.x < 16 * U;
    const bf16_t* yp = Y + (ystage && my < mend ? my : mbeg) * ldy + r0;
    u16x8_t yv8{0, 0, 0, 0, 0, 0, 0, 0};
    if (ystage) {
      if constexpr (YVEC && RB == 8) {
        yv8 = *reinterpret_cast<const u16x8_t*>(yp);
      } else if constexpr (YVEC && RB == 4) {
        const u16x4_t v = *reinterpret_cast<const u16x4_t*>(yp);
        yv8 = u16x8_t{v[0], v[1], v[2], v[3], 0, 0, 0, 0};
      } else {
#pragma unroll
        for (int r = 0; r < RB; ++r) yv8[r] = (r0 + r < R) ? yp[r] : (bf16_t)0;
      }
      if (my >= mend) yv8 = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
    u16x4_t xr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long m = mb0 + w + 16 * u;
      const long mc = m < mend ? m : mend - 1;
      xr[u] = *reinterpret_cast<const u16x4_t*>(X + mc * ldx + kc);
    }
    if (ystage) {
      bf16_t* yd = ys + threadIdx.x * RB;
      if constexpr (RB == 8) {
        *reinterpret_cast<u16x8_t*>(yd) = yv8;
      } else {
#pragma unroll
        for (int r = 0; r < RB; ++r) yd[r] = yv8[r];
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long m = mb0 + w + 16 * u;
      float xv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[j] = bf2f(xr[u][j]);
      if constexpr (DROP) {
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[j] *= drop_mult(drop, dseed, m, kc + j, K);
      }
      const bf16_t* yrow = ys + (w + 16 * u) * RB;
      float yv[RB];
      if constexpr (RB == 8) {
        load8(yrow, yv);
      } else {
#pragma unroll
        for (int r = 0; r < RB; ++r) yv[r] = bf2f(yrow[r]);
      }
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j][r] += xv[j] * yv[r];
    }
  }
  // 16 -> 8 wave tiles.  LDS image per wave: [r][256 columns] so the final pass reads columns
  // contiguously and every atomic wave-instruction covers 256 contiguous bytes when osk == 1
  // (MI355X_MICROARCH.md "Global float atomics": scattered 4-B lanes run ~17x slower).
  if (w >= 8) {
#pragma unroll
    for (int r = 0; r < RB; ++r)
      *reinterpret_cast<f32x4_t*>(&red[w - 8][r][lane * 4]) = f32x4_t{acc[0][r], acc[1][r], acc[2][r], acc[3][r]};
  }
  __syncthreads();
  if (w < 8) {
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      f32x4_t* q = reinterpret_cast<f32x4_t*>(&red[w][r][lane * 4]);
      *q = *q + f32x4_t{acc[0][r], acc[1][r], acc[2][r], acc[3][r]};
    }
  }
  __syncthreads();
  // final 8-way sum over RB x 256 outputs; lane order follows the unit-stride output axis
  float* const dst = outs.n ? outs.p[blockIdx.z] : out;  // segmented: this rank block's own buffer
  const int rdst = outs.n ? 0 : r0;
  for (int o = threadIdx.x; o < RB * 256; o += 1024) {
    int r, c;
    if (osk == 1) { r = o >> 8; c = o & 255; }
    else { c = o / RB; r = o % RB; }
    const int kk = blockIdx.x * 256 + c;
    if (kk >= K || r0 + r >= R) continue;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) v += red[i][r][c];
    if (det_ws) {  // deterministic mode: this row chunk's partial, summed in a fixed order later
      det_ws[((long)blockIdx.y * R + r0 + r) * det_kp + kk] = v * scale;
      continue;
    }
    atomicAdd(dst + (long)kk * osk + (long)(rdst + r) * osr, v * scale);
  }
}

// deterministic-mode reduction of lora_wgrad partials: out(rank r, column k) += sum_y ws[y][r][k]
// in ascending y (row-chunk) order; segmented outputs map rank r to outs.p[r / 8], local rank r % 8
__global__ void lora_wgrad_reduce_kernel(const float* __restrict__ ws, int ny, int R, int K, long kp, float* out,
                                         long osk, long osr, WgradOuts outs) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)R * K) return;
  const int r = (int)(t / K), k = (int)(t % K);
  float acc = 0.f;
  for (int y = 0; y < ny; ++y) acc += ws[((long)y * R + r) * kp + k];
  float* dst = outs.n ? outs.p[r >> 3] : out;
  const int rl = outs.n ? (r & 7) : r;
  dst[(long)k * osk + (long)rl * osr] += acc;
}

// ------------------------------------------------------------------------------------ dy pass
// lora_dy (rank 8): ONE streaming pass over dy [M, N] for both rank-r products that read it
//   v[m, r]   = s * sum_n dy[m, n] B[r, n]    (reduction over N)
//   dB[r, n] += s * sum_m u[m, r] dy[m, n]    (reduction over M)
// replacing lora_rowdot(dy, B) + lora_wgrad(dy, u), which each streamed dy (the largest LoRA operand:
// M x 2304 for the fused qkv projection) from HBM.
//
// Both products run on MFMA (v_mfma_f32_16x16x32_bf16).  A wave owns 32-row tiles of one 256-column
// strip.  Its dy tile is loaded ONCE from HBM with 16-B loads straight into A-operand fragments
// (lane: row l&15, 8 contiguous columns), which
//   * feed v += dy B^T directly (B^T fragments of the strip stay in registers), and
//   * are written to the wave's own padded LDS image, read back transposed (ds_read_b64_tr_b16) as
//     the B operand of dB^T-tile += u^T dy, with u^T staged through a tiny [32][16] LDS image.
// dB accumulates over the wave's tiles in 16 f32x4 registers; the 4 waves of the block fold through
// LDS and issue one fp32 atomic per (rank, column) per block (256-B contiguous per wave instruction).
// v partial sums per 256-column strip go to an fp32 scratch [strip][M][8] summed by lora_dy_finish (one
// strip, N <= 256: v is written directly).
constexpr int kDyLd = 256 + 8;  // padded LDS row (elements): transposed reads conflict-free

// several adapters in one launch (lora_dy_multi): strip blockIdx.x belongs to adapter a with
// strip0[a] <= x < strip0[a + 1]; its operands replace the single-adapter arguments
struct LoraDyTable {
  int n;
  int strip0[5];
  const bf16_t* B[4];
  long ldb[4];
  const bf16_t* u[4];
  long ldu[4];
  float* dB[4];
  long ldd[4];
  int N[4];
};

__global__ __launch_bounds__(256, 2) void lora_dy_kernel(const bf16_t* __restrict__ dy, long ldy,
                                                         const bf16_t* __restrict__ B, long ldb,
                                                         const bf16_t* __restrict__ u, long ldu, float* __restrict__ dB,
                                                         long ldd, float* __restrict__ vpart, long M, int N, long chunk,
                                                         float s, float* __restrict__ det_ws, long det_np,
                                                         bf16_t* __restrict__ vout, long ldv, LoraDyTable tb) {
  // per wave: dy image [32][kDyLd] + u^T image [32][16]; block reduction buffer aliases the images
  __shared__ __attribute__((aligned(16))) bf16_t lds[4][32 * kDyLd + 32 * 16];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  int n0 = blockIdx.x * 256;
  if (tb.n > 0) {  // (workgroup-uniform)
    int a = 0;
    for (int i = 1; i < tb.n; ++i) a = (int)blockIdx.x >= tb.strip0[i] ? i : a;
    dy += (long)tb.strip0[a] * 256;
    B = tb.B[a], ldb = tb.ldb[a], u = tb.u[a], ldu = tb.ldu[a], dB = tb.dB[a], ldd = tb.ldd[a], N = tb.N[a];
    n0 = ((int)blockIdx.x - tb.strip0[a]) * 256;
  }
  bf16_t* img = lds[w];
  bf16_t* uimg = lds[w] + 32 * kDyLd;
  // B^T fragments of the strip: lane holds B[r = l&15][n0 + 32 cg + 8g + j] (zero for r >= 8 / n >= N)
  bf16x8_t bt[8];
#pragma unroll
  for (int cg = 0; cg < 8; ++cg) {
    const int n = n0 + 32 * cg + 8 * g;
    bt[cg] = (c16 < 8 && n < N) ? *reinterpret_cast<const bf16x8_t*>(B + (long)c16 * ldb + n) : bf16x8_t{};
  }
  // zero ranks 8..15 of the u^T image once (rows are rewritten per tile, ranks 0..7 only)
  if (lane < 32) *reinterpret_cast<u16x8_t*>(uimg + lane * 16 + 8) = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  f32x4_t db[16];
#pragma unroll
  for (int cb = 0; cb < 16; ++cb) db[cb] = zero4();
  const long mbeg = (long)blockIdx.y * chunk;
  const long mend = min(M, mbeg + chunk);
  // The tile's dy fragments are dead once the v MFMAs and the LDS image have consumed them, so the
  // NEXT tile's loads are issued into the same registers right there: they stream in under this
  // tile's dB MFMAs / transposed reads / v stores (no extra VGPRs; the loads used to start only after
  // the whole tile was done).
  bf16x8_t a[2][8];
  u16x8_t ur;
  auto load_tile = [&](long t0) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const long m = t0 + 16 * rb + c16;
      const bool rok = m < mend;
      const bf16_t* rowp = dy + (rok ? m : mbeg) * ldy;
#pragma unroll
      for (int cg = 0; cg < 8; ++cg) {
        const int n = n0 + 32 * cg + 8 * g;
        a[rb][cg] = (rok && n < N) ? *reinterpret_cast<const bf16x8_t*>(rowp + n) : bf16x8_t{};
      }
    }
    ur = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    if (lane < 32 && t0 + lane < mend) ur = *reinterpret_cast<const u16x8_t*>(u + (t0 + lane) * ldu);
  };
  if (mbeg + 32 * w < mend) load_tile(mbeg + 32 * w);
  for (long t0 = mbeg + 32 * w; t0 < mend; t0 += 128) {
    // ---- v partials: D[row][rank] += dy[row][32 cols] . B^T[32 cols][rank]
    f32x4_t vacc[2] = {zero4(), zero4()};
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cg = 0; cg < 8; ++cg) vacc[rb] = mfma16(a[rb][cg], bt[cg], vacc[rb]);
    // ---- dy tile -> LDS (row-major, padded), u rows -> u^T image
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cg = 0; cg < 8; ++cg)
        *reinterpret_cast<bf16x8_t*>(img + (16 * rb + c16) * kDyLd + 32 * cg + 8 * g) = a[rb][cg];
    if (lane < 32) *reinterpret_cast<u16x8_t*>(uimg + lane * 16) = ur;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (t0 + 128 < mend) load_tile(t0 + 128);
    // ---- dB^T tiles: D[rank][16 cols] += u^T[rank][32 rows] . dy[32 rows][16 cols]
    const bf16x8_t ua = frag_tr(uimg, 16, 0, 0);  // lane: u[row 8g + j][rank l&15]
#pragma unroll
    for (int cb = 0; cb < 16; ++cb) db[cb] = mfma16(ua, frag_tr(img, kDyLd, 0, 16 * cb), db[cb]);
    // v partial rows 4g+i of each 16-row block, rank l&15 (< 8)
    if (c16 < 8) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const long m = t0 + 16 * rb + 4 * g + i;
          if (m >= mend) continue;
          if (vout)  // a single 256-column strip (N <= 256): v directly, no partials to sum
            vout[m * ldv + c16] = f2bf(vacc[rb][i] * s);
          else
            vpart[((long)blockIdx.x * M + m) * 8 + c16] = vacc[rb][i];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // tr-reads done before the next tile's writes
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // ---- block fold of dB (ranks 0..7 live in lane groups g = 0, 1) and one atomic per element
  __syncthreads();
  float* red = reinterpret_cast<float*>(&lds[0][0]);  // [4 waves][8 ranks][256 cols] fp32 = 32 KB
  if (g < 2) {
#pragma unroll
    for (int cb = 0; cb < 16; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(w * 8 + 4 * g + i) * 256 + 16 * cb + c16] = db[cb][i];
  }
  __syncthreads();
  for (int o = threadIdx.x; o < 8 * 256; o += 256) {
    const int r = o >> 8, c = o & 255;
    if (n0 + c >= N) continue;
    const float v = red[r * 256 + c] + red[(8 + r) * 256 + c] + red[(16 + r) * 256 + c] + red[(24 + r) * 256 + c];
    if (det_ws) {  // deterministic mode: per-row-chunk partial, fixed-order sum in lora_dy_reduce
      det_ws[((long)blockIdx.y * 8 + r) * det_np + n0 + c] = v * s;
      continue;
    }
    atomicAdd(dB + (long)r * ldd + n0 + c, v * s);
  }
}

// the adapters' v from their strips' partials: adapter blockIdx.y, strips [strip0, strip1)
struct LoraDyFinTable {
  int strip0[5];
  bf16_t* v[4];
  long ldv[4];
  int vz[4];
};
__global__ void lora_dy_finish_multi_kernel(const float* __restrict__ vpart, long M, float s, LoraDyFinTable ft) {
  const int a = blockIdx.y;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * 8) return;
  float acc = 0.f;
  for (int k = ft.strip0[a]; k < ft.strip0[a + 1]; ++k) acc += vpart[(long)k * M * 8 + t];
  bf16_t* v = ft.v[a];
  const long ldv = ft.ldv[a];
  v[(t >> 3) * ldv + (t & 7)] = f2bf(acc * s);
  const int c = (int)(t & 7), vz = ft.vz[a];
  if (c >= 1 && 8 * c < 8 + vz) *reinterpret_cast<uint4*>(v + (t >> 3) * ldv + 8 * c) = uint4{0u, 0u, 0u, 0u};
}

// v[m, r] = s * sum over strips of vpart[strip, m, r]   (bf16 out, row stride ldv)
// vz > 0: also zero v's columns 8 .. 8 + vz - 1 (vz % 8 == 0; 16-B stores, ldv % 8 == 0) -- the zero padding
// of the gemm4 second K segment (engine/nn.cpp), without a launch of its own
__global__ void lora_dy_finish_kernel(const float* __restrict__ vpart, int nstrip, long M, float s, bf16_t* __restrict__ v,
                                      long ldv, int vz) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * 8) return;
  float a = 0.f;
  for (int k = 0; k < nstrip; ++k) a += vpart[(long)k * M * 8 + t];
  v[(t >> 3) * ldv + (t & 7)] = f2bf(a * s);
  const int c = (int)(t & 7);
  if (c >= 1 && 8 * c < 8 + vz) *reinterpret_cast<uint4*>(v + (t >> 3) * ldv + 8 * c) = uint4{0u, 0u, 0u, 0u};
}

__global__ void lora_dy_reduce_kernel(const float* __restrict__ ws, int ny, int N, long np, float* __restrict__ dB,
                                      long ldd) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 8L * N) return;
  const int r = (int)(t / N), n = (int)(t % N);
  float acc = 0.f;
  for (int y = 0; y < ny; ++y) acc += ws[((long)y * 8 + r) * np + n];
  dB[(long)r * ldd + n] += acc;
}

static long dy_chunks(long M, int N, long* chunk_out) {
  const int gx = cdiv(N, 256);
  // 2 resident blocks per CU (68 KB LDS each): at most 512 blocks, so the whole grid is ONE round.  (The
  // round-3 sizing, ny = ceil(512 / gx), gave 513 blocks for gx = 3 and 9 -- GPT-2's 768 / 2304 and
  // Gemma-3's 640-wide strips -- and the 513th block ran alone after the first round.)  Row chunks are
  // whole 128-row quads (4 waves x 32 rows) split as evenly as the quads allow.
  long ny = 512 / gx;
  const long quads = cdiv(M, 128);
  if (ny > quads) ny = quads;
  if (ny < 1) ny = 1;
  const long chunk = cdiv(quads, ny) * 128;
  if (chunk_out) *chunk_out = chunk;
  return cdiv(M, chunk);
}

bool lora_dy_multi_ok(const LoraDyAdapter* ads, int n) {
  if (n < 1 || n > 4) return false;
  int next = 0;  // first free strip
  for (int i = 0; i < n; ++i) {
    const LoraDyAdapter& a = ads[i];
    if (a.col0 % 256 || a.col0 / 256 < next || a.N <= 0 || a.N % 8 || a.ldb % 8 || a.ldu % 8 || a.vz % 8 || a.vz > 56 ||
        a.ldv % 8 || !a.dB || (reinterpret_cast<uintptr_t>(a.B) | reinterpret_cast<uintptr_t>(a.u)) % 16)
      return false;
    next = a.col0 / 256 + cdiv(a.N, 256);
  }
  return true;
}

long lora_dy_multi_vpart_floats(const LoraDyAdapter* ads, int n, long M) {
  return (long)(ads[n - 1].col0 / 256 + cdiv(ads[n - 1].N, 256)) * M * 8;
}

void lora_dy_multi(const bf16_t* dy, long ldy, const LoraDyAdapter* ads, int n, float* vpart, long M, float s,
                   hipStream_t st) {
  if (!lora_dy_multi_ok(ads, n) || ldy % 8 || reinterpret_cast<uintptr_t>(dy) % 16) {
    fprintf(stderr, "lora_dy_multi: unsupported adapter set\n");
    abort();
  }
  if (M <= 0) return;
  LoraDyTable tb{};
  LoraDyFinTable ft{};
  tb.n = n;
  for (int i = 0; i < n; ++i) {
    const LoraDyAdapter& a = ads[i];
    tb.strip0[i] = ft.strip0[i] = a.col0 / 256;
    tb.B[i] = a.B, tb.ldb[i] = a.ldb, tb.u[i] = a.u, tb.ldu[i] = a.ldu, tb.dB[i] = a.dB, tb.ldd[i] = a.ldd, tb.N[i] = a.N;
    ft.v[i] = a.v, ft.ldv[i] = a.ldv, ft.vz[i] = a.vz;
  }
  const int gx = ads[n - 1].col0 / 256 + cdiv(ads[n - 1].N, 256);
  tb.strip0[n] = ft.strip0[n] = gx;
  long chunk = 0;
  const long ny = dy_chunks(M, gx * 256, &chunk);
  // strips between adapters (none for adjacent ranges) run the first adapter past its N: masked, no output
  lora_dy_kernel<<<dim3(gx, (unsigned)ny), 256, 0, st>>>(dy, ldy, ads[0].B, ads[0].ldb, ads[0].u, ads[0].ldu, ads[0].dB,
                                                           ads[0].ldd, vpart, M, ads[0].N, chunk, s, nullptr, 0, nullptr, 0,
                                                           tb);
  lora_dy_finish_multi_kernel<<<dim3((unsigned)cdiv(M * 8, 256), n), 256, 0, st>>>(vpart, M, s, ft);
}

long lora_dy_ws_floats(long M, int N) { return dy_chunks(M, N, nullptr) * 8L * cdiv(N, 256) * 256; }
long lora_dy_grid_blocks(long M, int N) { return dy_chunks(M, N, nullptr) * cdiv(N, 256); }

void lora_dy(const bf16_t* dy, long ldy, const bf16_t* B, long ldb, const bf16_t* u, long ldu, float* dB, long ldd,
             float* vpart, bf16_t* v, long ldv, long M, int N, float s, hipStream_t st, float* det_ws, int vzero) {
  if ((N % 8) || (ldy % 8) || (ldb % 8) || (ldu % 8) || (reinterpret_cast<uintptr_t>(dy) % 16) ||
      (reinterpret_cast<uintptr_t>(B) % 16) || (reinterpret_cast<uintptr_t>(u) % 16)) {
    fprintf(stderr, "lora_dy: N and the row strides must be multiples of 8, dy/B/u 16-B aligned\n");
    abort();
  }
  if (M <= 0 || N <= 0) return;
  const int gx = cdiv(N, 256);
  long chunk = 0;
  const long ny = dy_chunks(M, N, &chunk);
  const long np = (long)gx * 256;
  dim3 grid(gx, (unsigned)ny);
  lora_dy_kernel<<<grid, 256, 0, st>>>(dy, ldy, B, ldb, u, ldu, dB, ldd, vpart, M, N, chunk, s, det_ws, np,
                                       gx == 1 ? v : nullptr, ldv, LoraDyTable{});
  if (gx > 1) {
    lora_dy_finish_kernel<<<cdiv(M * 8, 256), 256, 0, st>>>(vpart, gx, M, s, v, ldv, vzero);
  } else if (vzero > 0) {
    zero_cols(v, ldv, M, 8, vzero, st);
  }
  if (det_ws) lora_dy_reduce_kernel<<<cdiv(8L * N, 256), 256, 0, st>>>(det_ws, (int)ny, N, np, dB, ldd);
}

template <typename T>
__global__ void lora_merge_kernel(T* W, long wsk, long wsn, const float* __restrict__ A, const float* __restrict__ B, int K,
                                  int N, int R, float s) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)K * N) return;
  const int k = t / N, n = t % N;
  float acc = 0.f;
  for (int r = 0; r < R; ++r) acc += A[(long)r * K + k] * B[(long)r * N + n];
  T* p = W + k * wsk + n * wsn;
  if constexpr (sizeof(T) == 2) {
    *p = f2bf(bf2f(*p) + s * acc);
  } else {
    *p = *p + s * acc;
  }
}

void lora_rowdot(const bf16_t* X, long ldx, const bf16_t* Wt, long ldw, bf16_t* U, long ldu, long M, int K, int R, float s,
                 LoraDrop drop, hipStream_t st) {
  if (K % 8 || ldx % 8 || ldw % 8 || R > 64 || (reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Wt)) % 16) {
    fprintf(stderr, "lora_rowdot: K and the row strides must be multiples of 8, X / Wt 16-B aligned, R <= 64\n");
    abort();
  }
  if (M <= 0) return;
  const int grid = cdiv(M, 64);
  if (R <= 16) lora_rowdot_kernel<1><<<grid, 256, 0, st>>>(X, ldx, Wt, ldw, U, ldu, M, K, R, s, drop);
  else if (R <= 32) lora_rowdot_kernel<2><<<grid, 256, 0, st>>>(X, ldx, Wt, ldw, U, ldu, M, K, R, s, drop);
  else lora_rowdot_kernel<4><<<grid, 256, 0, st>>>(X, ldx, Wt, ldw, U, ldu, M, K, R, s, drop);
}

void lora_update(const bf16_t* base, long ldb, const bf16_t* U, long ldu, const bf16_t* W, long ldw, bf16_t* Y, long ldy,
                 long M, int N, int R, float s, LoraDrop drop, hipStream_t st) {
  const int nthreads_x = (N / 8 + 63) / 64 * 64;
  const int bx = nthreads_x < 256 ? nthreads_x : 256;
  const int gx = cdiv(N / 8, bx);
  // ~2k blocks in total, at least 16 rows per block to amortise the W register load
  long rows = (M * gx + 2047) / 2048;
  if (rows < 16) rows = 16;
  dim3 grid(gx, (unsigned)cdiv(M, rows));
  switch (R) {
#define MFT_UPD(RV) case RV: lora_update_kernel<RV><<<grid, bx, 0, st>>>(base, ldb, U, ldu, W, ldw, Y, ldy, M, N, (int)rows, s, drop); break;
    MFT_UPD(1) MFT_UPD(2) MFT_UPD(4) MFT_UPD(8) MFT_UPD(16)
#undef MFT_UPD
    default: {
      // larger ranks: apply in slices of 16 (in place after the first)
      for (int r0 = 0; r0 < R; r0 += 16) {
        const int rr = R - r0 < 16 ? R - r0 : 16;
        if (rr != 16) { fprintf(stderr, "lora_update: rank %d must be a multiple of 16 above 16\n", R); abort(); }
        lora_update_kernel<16><<<grid, bx, 0, st>>>(r0 == 0 ? base : Y, r0 == 0 ? ldb : ldy, U + r0, ldu,
                                                     W + (long)r0 * ldw, ldw, Y, ldy, M, N, (int)rows, s, drop);
      }
    }
  }
}

// lora_xty (weight-gradient of a rank-r factor on MFMA):  out[k, r] (+)= scale * sum_m X[m, k] Y[m, r]
// for R % 8 == 0, R <= 32 -- dA = v^T x (X = the layer input, Y = v) and dB = u^T dy (X = dy, Y = u)
// of every adapter sharing X in ONE pass over X.  The dB half of lora_dy with up to 32 ranks: a wave
// owns 32-row tiles of one 256-column strip, loads its X tile once with 16-B loads, writes it to its
// padded LDS image and reads it back transposed (ds_read_b64_tr_b16) as the B operand of
// D[rank][16 cols] += Y^T[rank][32 rows] . X[32 rows][16 cols]; the Y rows of the tile go through a
// [32][16 NR] image read back transposed as the A operand.  The VALU form (lora_wgrad_kernel) does
// R fp32 FMAs per X element and was VALU-bound (Gemma q|k|v dA: 60 us for 84 MB).
template <int NR>  // rank blocks of 16
__global__ __launch_bounds__(256, 2) void lora_xty_kernel(const bf16_t* __restrict__ X, long ldx,
                                                          const bf16_t* __restrict__ Y, long ldy, int R,
                                                          float* __restrict__ out, long osk, long osr, WgradOuts outs,
                                                          long M, int K, long chunk, float scale) {
  constexpr int YL = 16 * NR;
  __shared__ __attribute__((aligned(16))) bf16_t lds[4][32 * kDyLd + 32 * YL];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int k0 = blockIdx.x * 256;
  bf16_t* img = lds[w];
  bf16_t* yimg = lds[w] + 32 * kDyLd;
  f32x4_t acc[NR][16];
#pragma unroll
  for (int nr = 0; nr < NR; ++nr)
#pragma unroll
    for (int cb = 0; cb < 16; ++cb) acc[nr][cb] = zero4();
  const long mbeg = (long)blockIdx.y * chunk;
  const long mend = min(M, mbeg + chunk);
  // as lora_dy: the next tile's X / Y loads go out as soon as this tile sits in LDS
  bf16x8_t a[2][8];
  u16x8_t yr[2 * NR];
  auto load_tile = [&](long t0) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const long m = t0 + 16 * rb + c16;
      const bool rok = m < mend;
      const bf16_t* rowp = X + (rok ? m : mbeg) * ldx;
#pragma unroll
      for (int cg = 0; cg < 8; ++cg) {
        const int k = k0 + 32 * cg + 8 * g;
        a[rb][cg] = (rok && k < K) ? *reinterpret_cast<const bf16x8_t*>(rowp + k) : bf16x8_t{};
      }
    }
    // Y rows of the tile: lane < 32 -> row t0 + lane, 8 ranks per 16-B load (zero past R / mend)
#pragma unroll
    for (int j = 0; j < 2 * NR; ++j) {
      yr[j] = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      if (lane < 32 && t0 + lane < mend && 8 * j < R) yr[j] = *reinterpret_cast<const u16x8_t*>(Y + (t0 + lane) * ldy + 8 * j);
    }
  };
  // (the early load needs the 64 fragment VGPRs live across the MFMAs: with NR = 2's 128 accumulators
  // it spills, so NR = 2 keeps the load at the top of each tile)
  constexpr bool kEarly = NR == 1;
  if (kEarly && mbeg + 32 * w < mend) load_tile(mbeg + 32 * w);
  for (long t0 = mbeg + 32 * w; t0 < mend; t0 += 128) {
    if (!kEarly) load_tile(t0);
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cg = 0; cg < 8; ++cg)
        *reinterpret_cast<bf16x8_t*>(img + (16 * rb + c16) * kDyLd + 32 * cg + 8 * g) = a[rb][cg];
    if (lane < 32) {
#pragma unroll
      for (int j = 0; j < 2 * NR; ++j) *reinterpret_cast<u16x8_t*>(yimg + lane * YL + 8 * j) = yr[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (kEarly && t0 + 128 < mend) load_tile(t0 + 128);
#pragma unroll
    for (int nr = 0; nr < NR; ++nr) {
      const bf16x8_t ya = frag_tr(yimg, YL, 0, 16 * nr);  // lane: Y[row 8g + j][rank 16 nr + (l & 15)]
#pragma unroll
      for (int cb = 0; cb < 16; ++cb) acc[nr][cb] = mfma16(ya, frag_tr(img, kDyLd, 0, 16 * cb), acc[nr][cb]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // tr-reads done before the next tile's writes
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // block fold per 16-rank block through LDS ([4 waves][16 ranks][256 cols] fp32 = 64 KB), one fp32
  // atomic per (rank, column) per block
  float* red = reinterpret_cast<float*>(&lds[0][0]);
#pragma unroll
  for (int nr = 0; nr < NR; ++nr) {
    __syncthreads();
#pragma unroll
    for (int cb = 0; cb < 16; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(w * 16 + 4 * g + i) * 256 + 16 * cb + c16] = acc[nr][cb][i];
    __syncthreads();
    for (int o = threadIdx.x; o < 16 * 256; o += 256) {
      const int rl16 = o >> 8, c = o & 255;
      const int r = 16 * nr + rl16;
      if (r >= R || k0 + c >= K) continue;
      const float v = red[rl16 * 256 + c] + red[(16 + rl16) * 256 + c] + red[(32 + rl16) * 256 + c] +
                      red[(48 + rl16) * 256 + c];
      float* dst = outs.n ? outs.p[r >> 3] : out;
      const int rr = outs.n ? (r & 7) : r;
      atomicAdd(dst + (long)(k0 + c) * osk + (long)rr * osr, v * scale);
    }
  }
}

// MFT_WGRAD_VALU=1: every lora_wgrad on the VALU kernel (A/B switch)
static bool wgrad_valu() {
  static const int v = [] {
    const char* e = getenv("MFT_WGRAD_VALU");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return v == 1;
}

static long wgrad_chunks(long M, int K, int R, long* chunk_out) {
  const int rb = R <= 1 ? 1 : R <= 2 ? 2 : R <= 4 ? 4 : 8;
  const int gx = cdiv(K, 256);
  const int gz = cdiv(R, rb);
  // ~4 live waves per SIMD (4096 waves = 256 blocks of 16) but at least U=8 rows per wave; the
  // chunk is a multiple of 16 rows so every wave streams the same number of rows
  static const long target = getenv("MFT_WGRAD_BLOCKS") ? atol(getenv("MFT_WGRAD_BLOCKS")) : 256;
  long nrc = cdiv(target, (long)gx * gz);
  const long max_nrc = cdiv(M, 16 * 8);  // >= 8 rows per wave
  if (nrc > max_nrc) nrc = max_nrc;
  if (nrc < 1) nrc = 1;
  long chunk = cdiv(M, nrc);
  chunk = cdiv(chunk, 16) * 16;
  if (chunk_out) *chunk_out = chunk;
  return cdiv(M, chunk);
}

long lora_wgrad_ws_floats(long M, int K, int R) { return wgrad_chunks(M, K, R, nullptr) * R * (long)cdiv(K, 256) * 256; }

void lora_wgrad(const bf16_t* X, long ldx, const bf16_t* Y, long ldy, float* out, long osk, long osr, long M, int K, int R,
                float scale, LoraDrop drop, hipStream_t st, const WgradOuts* outs, float* det_ws) {
  WgradOuts so{};
  if (outs) {
    if (outs->n < 1 || outs->n > 8 || R != 8 * outs->n) {
      fprintf(stderr, "lora_wgrad: segmented output needs R == 8 * n (R=%d, n=%d)\n", R, outs ? outs->n : 0);
      abort();
    }
    so = *outs;
  }
  if ((K % 4) || (ldx % 4) || (reinterpret_cast<uintptr_t>(X) % 8)) {
    fprintf(stderr, "lora_wgrad: K (%d) and ldx (%ld) must be multiples of 4 and X 8-byte aligned\n", K, ldx);
    abort();
  }
  // MFMA form: no dropout mask on X, ranks in whole 8-blocks up to 32, 16-B aligned rows, fp32 atomics
  // (the deterministic mode keeps the VALU kernel's fixed-order partials)
  if (!det_ws && drop.p <= 0.f && R % 8 == 0 && R <= 32 && K % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 &&
      reinterpret_cast<uintptr_t>(X) % 16 == 0 && reinterpret_cast<uintptr_t>(Y) % 16 == 0 && !wgrad_valu()) {
    long chunk = 0;
    const long ny = dy_chunks(M, K, &chunk);
    dim3 grid(cdiv(K, 256), (unsigned)ny);
    if (R <= 16)
      lora_xty_kernel<1><<<grid, 256, 0, st>>>(X, ldx, Y, ldy, R, out, osk, osr, so, M, K, chunk, scale);
    else
      lora_xty_kernel<2><<<grid, 256, 0, st>>>(X, ldx, Y, ldy, R, out, osk, osr, so, M, K, chunk, scale);
    return;
  }
  const int rb = R <= 1 ? 1 : R <= 2 ? 2 : R <= 4 ? 4 : 8;
  const int gx = cdiv(K, 256);
  const int gz = cdiv(R, rb);
  long chunk = 0;
  const long ny = wgrad_chunks(M, K, R, &chunk);
  const long kp = (long)gx * 256;
  dim3 grid(gx, (unsigned)ny, gz);
  // vector Y loads need every rank block complete and 2*RB-byte aligned rows
  const bool yvec = (rb == 8 || rb == 4) && R % rb == 0 && ldy % rb == 0 &&
                    reinterpret_cast<uintptr_t>(Y) % (2 * rb) == 0;
#define MFT_WG(RBV, YV)                                                                                         \
  do {                                                                                                          \
    if (drop.p > 0.f)                                                                                           \
      lora_wgrad_kernel<RBV, YV, true><<<grid, 1024, 0, st>>>(X, ldx, Y, ldy, out, osk, osr, M, K, R, chunk, scale, drop, so, \
                                                              det_ws, kp);                                     \
    else                                                                                                        \
      lora_wgrad_kernel<RBV, YV, false><<<grid, 1024, 0, st>>>(X, ldx, Y, ldy, out, osk, osr, M, K, R, chunk, scale, drop, \
                                                               so, det_ws, kp);                                \
  } while (0)
  switch (rb) {
    case 1: MFT_WG(1, false); break;
    case 2: MFT_WG(2, false); break;
    case 4: if (yvec) MFT_WG(4, true); else MFT_WG(4, false); break;
    default: if (yvec) MFT_WG(8, true); else MFT_WG(8, false); break;
  }
#undef MFT_WG
  if (det_ws)
    lora_wgrad_reduce_kernel<<<cdiv((long)R * K, 256), 256, 0, st>>>(det_ws, (int)ny, R, K, kp, out, osk, osr, so);
}

void lora_merge(void* W, int w_is_bf16, long wsk, long wsn, const float* A, const float* B, int K, int N, int R, float s,
                hipStream_t st) {
  const long n = (long)K * N;
  if (w_is_bf16)
    lora_merge_kernel<bf16_t><<<cdiv(n, 256), 256, 0, st>>>((bf16_t*)W, wsk, wsn, A, B, K, N, R, s);
  else
    lora_merge_kernel<float><<<cdiv(n, 256), 256, 0, st>>>((float*)W, wsk, wsn, A, B, K, N, R, s);
}

__global__ __launch_bounds__(256) void lora_prep_kernel(const LoraPrepEntry* __restrict__ es) {
  const LoraPrepEntry e = es[blockIdx.x];
  const long n = (long)e.rows * e.cols;
  for (long t = threadIdx.x; t < n; t += blockDim.x) {
    const long r = t / e.cols, c = t % e.cols;
    e.dst[r * e.dld + c] = f2bf(e.scale * bf2f(e.src[r * e.srs + c * e.scs]));
  }
}

void lora_prep_batched(const LoraPrepEntry* dev_entries, int n, hipStream_t st) {
  if (n > 0) lora_prep_kernel<<<n, 256, 0, st>>>(dev_entries);
}

}  // namespace mft
