// 256 x 128 x 32 bf16 MFMA GEMM, FOUR waves per workgroup and TWO workgroups per CU (gfx950):
//
//   C[M, N] = epi(alpha * A . B^T)      A [M, K] K-contiguous (activations), B [N, K] (weights, "NT")
//
// Why a second GEMM beside gemm8 (the 256 x 256, one-workgroup-per-CU 8-phase kernel): at the
// training shapes K is short (768 / 832 for GPT-2, 640-2112 for Gemma-3), so a 256 x 256 tile is
// only 12-13 K-tiles of MFMA work between a prologue (first tiles fetched from HBM / MALL) and an
// epilogue (128 KB of bf16 stored from registers, issue-bound) -- and with one workgroup per CU and
// every CU finishing its tiles in lockstep, the whole chip alternates between a compute phase and a
// memory phase.  Here two independent workgroups share each CU (72 KB of LDS and <= 256 VGPRs per
// wave each), so one workgroup's epilogue stores and next-tile prologue loads overlap the other's
// MFMA main loop, and the store traffic spreads over the whole kernel instead of arriving in bursts.
//
// Structure (CDNA HIP guide §5: glds staging with the swizzle on the SOURCE address, rule 21;
// counted vmcnt and raw s_barrier so the LDS-DMA prefetch stays in flight across the barrier, T4;
// XCD-aware grouped tile order, T1):
//   * waves 2 (M) x 2 (N), each a 128 x 64 piece: 8 x 4 accumulator blocks of 16 x 16 (128 fp32
//     registers), 8 A + 4 B ds_read_b128 fragments and 32 MFMA 16x16x32 per 32-deep K-step;
//   * LDS: a ring of 3 stages x (A 256 x 32 + B 128 x 32) bf16 = 3 x 24 KB, each stage filled by
//     6 global_load_lds_dwordx4 per thread; K-step t prefetches stage t + 2 while computing stage t,
//     waits vmcnt(6) (only that prefetch still in flight) and passes ONE barrier;
//   * 64-byte LDS rows: the 16-byte chunk index is XOR-swizzled with a function of row bits 2-3
//     (swz below), so the 16 (row, chunk) pairs of one ds_read_b128 lane group hit 16 distinct
//     bank slots (conflict-free);
//   * the MFMAs run with the operands swapped (C^T blocks), so after one v_permlane16_swap per
//     register pair every lane owns 8 contiguous output columns of one row: the epilogue is 16-byte
//     vector loads / stores straight from registers (same epilogue family as gemm8).
#include <stdlib.h>

#include "kernels.h"
#include "mfma.h"

namespace mft {

namespace {

constexpr int WBM = 256, WBN = 128, WBK = 32, WNS = 3;
constexpr int W_A = WBM * WBK, W_B = WBN * WBK, W_STAGE = W_A + W_B;  // elements
constexpr int W_THREADS = 256;

typedef __attribute__((address_space(3))) void lds_void_w;
typedef const __attribute__((address_space(1))) void g_void_w;

__device__ __forceinline__ void glds16w(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((g_void_w*)src, (lds_void_w*)lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ void raw_barrier_w() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait_w() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16-byte chunk swizzle of a 64-byte row: g((row >> 2) & 3) with g = (0, 2, 3, 1).  A ds_read_b128
// lane group ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and their +32 twins) reads rows 0-15 of a
// fragment at chunks q / q^1 (lanes 16-31 read chunk 1); with this g the 16 (row, chunk) pairs of
// every group land in 16 distinct 16-byte bank slots.  (row >> 2) & 3 alone leaves 2-way conflicts.
__device__ __forceinline__ int swz(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }

// stage rows r0.. (clamped to rmax - 1) x k0..k0+31 of a K-contiguous operand into a [ROWS][32]
// LDS image; ROWS / 16 glds per wave-instruction set: thread t of instruction i moves chunk
// c = i * 256 + t -> row c >> 2, LDS chunk c & 3 holds global chunk (c & 3) ^ swz(row)
template <int ROWS>
__device__ __forceinline__ void stage_rows(bf16_t* lds, const bf16_t* src, long ld, int r0, int rmax, int k0) {
  const int tid = threadIdx.x, w = tid >> 6;
  const int rb = min(r0, rmax - 1);
  const char* base = reinterpret_cast<const char*>(src + (long)rb * ld + k0);
#pragma unroll
  for (int i = 0; i < ROWS / 64; ++i) {
    const int c = i * W_THREADS + tid;
    const int r = c >> 2, ch = c & 3;
    const int gr = min(r0 + r, rmax - 1) - rb;
    const uint32_t off = (uint32_t)((gr * (int)ld + ((ch ^ swz(r)) << 3)) * 2);
    glds16w(base + off, lds + (i * W_THREADS + w * 64) * 8);
  }
}

// fragment of a swizzled [ROWS][32] image: lane holds T[r0 + (l & 15)][8 * (l >> 4) + j]
__device__ __forceinline__ bf16x8_t fragw(const bf16_t* t, int r0) {
  const int l = threadIdx.x & 63;
  const int r = r0 + (l & 15), q = l >> 4;
  return *reinterpret_cast<const bf16x8_t*>(t + r * 32 + ((q ^ swz(r)) << 3));
}

}  // namespace

// ------------------------------------------------------------------ epilogue (registers only)
// acc[i][j]: C^T block of rows wm*128 + 16 i, columns wn*64 + 16 j.  Pieces (i, p): after the swap
// of blocks (2p, 2p+1) lane l owns row wm*128 + 16 i + (l & 15), columns wn*64 + 32 p + cofs .. +7.
template <int EPI>
__device__ __forceinline__ void epilogue_w(const GemmArgs& g, f32x4_t (&acc)[8][4], int m0, int n0, int wm, int wn,
                                           int lane) {
  const int g4 = lane >> 4;
  const int cofs = (g4 & 1) * 16 + (g4 >> 1) * 8;
  constexpr bool kAux = EPI == GEMM_EPI_DGELU || EPI == GEMM_EPI_MUL_AUX;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int col = n0 + wn * 64 + p * 32 + cofs;
    const bool col_ok = col < g.N;
    const int colc = min(col, g.N - 8);
    float bias_v[8];
    if constexpr (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU || EPI == GEMM_EPI_BIAS_GELU_D)
      load8(g.bias + colc, bias_v);
    u16x8_t wv[8];  // LoRA: the lane's 8 columns x 8 ranks of lora_w (rank <= 8 per pass)
#pragma unroll
    for (int ih = 0; ih < 2; ++ih) {  // two halves of 4 row blocks: bounded live registers
      u16x8_t auxv[4];
      if constexpr (kAux) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const int row = min(m0 + wm * 128 + (ih * 4 + ii) * 16 + (lane & 15), g.M - 1);
          auxv[ii] = *reinterpret_cast<const u16x8_t*>(g.aux + (long)row * g.ldaux + colc);
        }
      }
      float o[4][8];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = ih * 4 + ii;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * p][r]),
                                                           __float_as_uint(acc[i][2 * p + 1][r]), false, false);
          o[ii][r] = __uint_as_float(sw[0]);
          o[ii][4 + r] = __uint_as_float(sw[1]);
        }
      }
      if constexpr (EPI == GEMM_EPI_LORA) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int e = 0; e < 8; ++e) o[ii][e] *= g.alpha;
#pragma unroll 1
        for (int t8 = 0; t8 < g.lora_r; t8 += 8) {
#pragma unroll
          for (int t = 0; t < 8; ++t) wv[t] = *reinterpret_cast<const u16x8_t*>(g.lora_w + (long)(t8 + t) * g.ld_lw + colc);
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) {
            const int row = min(m0 + wm * 128 + (ih * 4 + ii) * 16 + (lane & 15), g.M - 1);
            float u[8];
            load8(g.lora_u + (long)row * g.ld_lu + t8, u);
#pragma unroll
            for (int t = 0; t < 8; ++t)
#pragma unroll
              for (int e = 0; e < 8; ++e) o[ii][e] += u[t] * bf2f(wv[t][e]);
          }
        }
      }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int row = m0 + wm * 128 + (ih * 4 + ii) * 16 + (lane & 15);
        const bool ok = col_ok && row < g.M;
        float* v = o[ii];
        if constexpr (EPI == GEMM_EPI_F32ACC) {
          if (ok) {
            float* C = reinterpret_cast<float*>(g.C) + (long)row * g.ldc + col;
            f32x4_t c0 = *reinterpret_cast<f32x4_t*>(C), c1 = *reinterpret_cast<f32x4_t*>(C + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              c0[e] += g.alpha * v[e];
              c1[e] += g.alpha * v[4 + e];
            }
            *reinterpret_cast<f32x4_t*>(C) = c0;
            *reinterpret_cast<f32x4_t*>(C + 4) = c1;
          }
          continue;
        }
        if constexpr (EPI != GEMM_EPI_LORA) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            v[e] *= g.alpha;
            if constexpr (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU || EPI == GEMM_EPI_BIAS_GELU_D)
              v[e] += bias_v[e];
          }
        }
        if constexpr (EPI == GEMM_EPI_DGELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= gelu_tanh_grad(bf2f(auxv[ii][e]));
        }
        if constexpr (EPI == GEMM_EPI_MUL_AUX) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= bf2f(auxv[ii][e]);
        }
        if constexpr (EPI == GEMM_EPI_BIAS_GELU) {
          if (ok) store8(g.aux + (long)row * g.ldaux + col, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
        }
        if constexpr (EPI == GEMM_EPI_BIAS_GELU_D) {
          float d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) gelu_tanh_and_grad(v[e], v[e], d[e]);
          if (ok) store8(g.aux + (long)row * g.ldaux + col, d);
        }
        if (ok) store8(reinterpret_cast<bf16_t*>(g.C) + (long)row * g.ldc + col, v);
      }
    }
  }
}

template <int EPI>
__global__ __launch_bounds__(256, 2) void gemmw_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smemw[];
  const int tiles_m = (g.M + WBM - 1) / WBM, tiles_n = (g.N + WBN - 1) / WBN;
  const int ntiles = tiles_m * tiles_n;
  // XCD remap, then grouped order: GROUP_M row panels sweep the column tiles together, so the
  // workgroups an XCD holds at once share A panels and B column tiles through its L2
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 4;
  const int group = bid / (GM * tiles_n), first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int in_g = bid - group * GM * tiles_n;
  const int tm = first_m + in_g % gsz, tn = in_g / gsz;
  if (bid >= ntiles) return;
  const int m0 = tm * WBM, n0 = tn * WBN;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int nk = g.K / WBK;

  auto stage = [&](int s, int kt) {
    const int k0 = min(kt, nk - 1) * WBK;  // past the end: re-read the last K-step (uniform counts)
    bf16_t* base = smemw + s * W_STAGE;
    stage_rows<WBM>(base, g.A, g.lda, m0, g.M, k0);
    stage_rows<WBN>(base + W_A, g.B, g.ldb, n0, g.N, k0);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero4();

  stage(0, 0);
  stage(1, 1);
  vm_wait_w<6>();  // stage 0 landed (this wave's share); the barrier makes it everyone's
  raw_barrier_w();

  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // prefetch K-step kt + 2 into the slot computed at kt - 1 (every wave passed that step's barrier)
    const int nxt = cur == 0 ? 2 : cur - 1;
    stage(nxt, kt + 2);
    const bf16_t* sa = smemw + cur * W_STAGE;
    const bf16_t* sb = sa + W_A;
    bf16x8_t bfr[4], afr[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = fragw(sb, wn * 64 + j * 16);
#pragma unroll
    for (int i = 0; i < 8; ++i) afr[i] = fragw(sa, wm * 128 + i * 16);
    // every fragment read issued before the first MFMA (the scheduling barrier stops hipcc from
    // re-using two A registers in a read -> wait -> 8 MFMA chain); its waitcnt pass then waits for
    // each A fragment just before that fragment's first MFMA (lgkmcnt 7, 6, ..., 0)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], afr[i], acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);  // the MFMA cluster stays ahead of the wait + barrier
    vm_wait_w<6>();  // K-step kt + 1 landed; only the kt + 2 prefetch still in flight
    raw_barrier_w();
    cur = cur == 2 ? 0 : cur + 1;
  }
  vm_wait_w<0>();  // drain the clamped tail prefetches (LDS-DMA must not outlive the workgroup)
  epilogue_w<EPI>(g, acc, m0, n0, wm, wn, lane);
}

// ================================================================== gemm4: 256 x 256 x 64, 4 waves
// One workgroup per CU, ONE wave per SIMD, each wave a 128 x 128 quadrant of the tile: 8 x 8
// accumulator blocks = 256 fp32 registers per lane, which the 512-entry unified register file of a
// lone wave holds in AGPRs beside the VGPR fragments.  Against gemm8 (8 waves of 64 x 32 pieces,
// 16 barriers per K-tile) a wave re-reads each LDS fragment for 8 MFMAs instead of 2-4: 32
// ds_read_b128 per 128 MFMAs and only 2 barriers per 64-deep K-tile.  Latency is hidden inside the
// wave by register double-buffering of the two 32-deep k-steps:
//
//   top of K-tile t (buffer c = t & 1 holds it; k-step-0 fragments of t already requested):
//     seg 1: request the k-step-1 fragments of t (16 ds_read_b128) | 64 MFMAs of k-step 0
//     lgkmcnt(0); barrier M   -- every wave is done reading buffer c
//     issue the LDS-DMA of K-tile t + 2 into buffer c (16 global_load_lds_dwordx4 per lane)
//     seg 2: 32 MFMAs of k-step 1
//     vmcnt(16) (K-tile t + 1 landed: only t + 2 still in flight); barrier E
//     seg 3: request the k-step-0 fragments of t + 1 from buffer c ^ 1 | 32 MFMAs of k-step 1
//
// so a K-tile's loads are in flight for ~1.5 K-tiles of MFMA work, never drained inside the loop
// (raw s_barrier, counted waits; guide §5 "Pipelining across barriers").  LDS images as gemm8: 128-B
// rows, the 16-B chunk index XOR-swizzled with (row & 7) on the SOURCE address (rule 21).
namespace {
constexpr int G4_HALF = 256 * 64;  // elements of one operand's K-tile image (32 KB)

__device__ __forceinline__ void g4_raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One operand's K-tile (256 rows x 64 k) is 8 LDS-DMA pieces per lane: piece t of wave w moves
// chunk c = t * 256 + tid -> row 32 t + (tid >> 3), 16-B chunk (tid & 7) ^ (row & 7) (the swizzle
// term (tid >> 3) & 7 does not depend on t).  Through a buffer descriptor whose base is the tile's
// row r0 at column k0 and whose size ends at the last valid row: rows past the matrix are dropped
// by the range check (their LDS rows only feed output rows / columns that are never stored), and
// each piece is one 32-bit VGPR offset (voff + t * 64 ld bytes) -- no 64-bit address math.
struct G4Src {
  __amdgpu_buffer_rsrc_t rsrc;
};
__device__ __forceinline__ G4Src g4_src(const bf16_t* src, long ld, int r0, int rmax, int k0, bool none = false) {
  const long rows = (long)rmax - r0;  // >= 1
  const long bytes = none ? 0 : ((rows - 1) * ld + 64) * 2;
  return G4Src{__builtin_amdgcn_make_buffer_rsrc((void*)(src + (long)r0 * ld + k0), (short)0,
                                                 (int)min(bytes, 0x7FFFFFFFL), 0x00020000)};
}
__device__ __forceinline__ uint32_t g4_voff(long ld) {
  const int tid = threadIdx.x, r = tid >> 3, s = tid & 7;
  return (uint32_t)((r * (int)ld + ((s ^ (r & 7)) << 3)) * 2);
}
__device__ __forceinline__ void g4_piece(const G4Src& s, uint32_t voff, long ld, int t, bf16_t* lds_img, int w) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(s.rsrc, (__attribute__((address_space(3))) void*)(lds_img + (t * 256 + w * 64) * 8),
                                           16, voff + (uint32_t)(t * 64 * ld), 0, 0, 0);
}

// lane holds T[r0 + (l & 15)][8 * kc + 8 * (l >> 4) + j] of a swizzled [256][64] image
__device__ __forceinline__ bf16x8_t g4_frag(const bf16_t* t, int r0, int kc) {
  const int l = threadIdx.x & 63;
  const int r = r0 + (l & 15), q = kc + (l >> 4);
  return *reinterpret_cast<const bf16x8_t*>(t + r * 64 + ((q ^ (r & 7)) << 3));
}

// acc += b^T-swapped product: inline asm with the accumulator tied "+a" so it stays in place in the
// AGPR file (hipcc's own MFMA selection rotates accumulators between iterations: ~370 v_accvgpr
// copies per K-tile).  Hazards: an accumulator is next read by an MFMA 63 MFMAs later (none), the
// fragments come from ds_read waited by hipcc's own lgkmcnt, and g4_mfma_drain pads the last MFMA
// before any compiler code reads the AGPRs.
__device__ __forceinline__ void g4_mfma(f32x4_t& c, const bf16x8_t& b, const bf16x8_t& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}
}  // namespace

// DBG (timing diagnostics only, results invalid): 1 = every LDS-DMA dropped by a zero-size
// descriptor (same instruction stream, no memory traffic), 2 = no barriers in the loop, 4 = no
// LDS-DMA instructions in the loop
// A3: asymmetric LDS ring -- THREE 32 KB slots for the A (activation) K-tiles, two for B (weights,
// L2-resident): the A loads are issued three K-tiles ahead (in flight ~2 K-tiles of MFMA work instead
// of ~1), B two ahead; 5 x 32 KB = the whole 160 KB LDS.
template <int EPI, int DBG = 0, bool A3 = false>
__global__ __launch_bounds__(256, 1) void gemm4_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem4[];
  const int tiles_n = (g.N + 255) / 256;
  const int ntiles = ((g.M + 255) / 256) * tiles_n;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  if (tile >= ntiles) return;
  // grouped order: GM row panels sweep the column tiles together, so the 32 workgroups an XCD holds
  // at once (consecutive ids after the remap) form a compact block sharing A and B panels in its L2
  // (8192^3: 980 -> 1432 TF/s; fc forward 895 -> 943)
  constexpr int GM = 8;
  const int tiles_m = (g.M + 255) / 256;
  const int group = tile / (GM * tiles_n), first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int in_g = tile - group * GM * tiles_n;
  const int m0 = (first_m + in_g % gsz) * 256, n0 = (in_g / gsz) * 256;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nk = g.K / 64;
  // A3: A slot s at smem + s HALF (s < 3), B slot s at smem + (3 + s) HALF; else buffer b = {A, B}
  auto sa = [&](int b) { return A3 ? smem4 + b * G4_HALF : smem4 + b * 2 * G4_HALF; };
  auto sb = [&](int b) { return A3 ? smem4 + (3 + b) * G4_HALF : smem4 + b * 2 * G4_HALF + G4_HALF; };
  const uint32_t voa = g4_voff(g.lda), vob = g4_voff(g.ldb);
  // piece p (0..15) of K-tile kt into buffer b: p < 8 -> A piece p, else B piece p - 8
  G4Src srcA, srcB;
  auto set_src = [&](int kt) {
    const int k0 = min(kt, nk - 1) * 64;  // past the end: re-read the last K-tile (uniform counts)
    srcA = g4_src(g.A, g.lda, m0, g.M, k0, DBG == 1 && kt >= 2);
    srcB = g4_src(g.B, g.ldb, n0, g.N, k0, DBG == 1 && kt >= 2);
  };
  auto piece = [&](int b, int p) {
    if (p < 8) g4_piece(srcA, voa, g.lda, p, sa(b), w);
    else g4_piece(srcB, vob, g.ldb, p - 8, sb(b), w);
  };

  f32x4_t acc[2][8][4];  // [column half][i: 16-row block][j: 16-column block]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = zero4();
  bf16x8_t a0[8], b0[8], a1[8], b1[8];
  // fragment r (0..15) of k-step ks: r < 8 -> B fragment r, else A fragment r - 8
  auto frag = [&](bf16x8_t (&af)[8], bf16x8_t (&bf)[8], int b, int ks, int r) {
    if (r < 8) bf[r] = g4_frag(sb(b), wc * 128 + r * 16, ks * 4);
    else af[r - 8] = g4_frag(sa(b), wr * 128 + (r - 8) * 16, ks * 4);
  };
  // MFMA number m (0..63) of a k-step: i = m / 8, j = m % 8
  auto mma = [&](const bf16x8_t (&af)[8], const bf16x8_t (&bf)[8], int m) {
    const int i = m >> 3, j = m & 7;
    g4_mfma(acc[j >> 2][i][j & 3], bf[j], af[i]);
  };

  if constexpr (A3) {
    auto src_a = [&](int kt) { srcA = g4_src(g.A, g.lda, m0, g.M, min(kt, nk - 1) * 64); };
    auto src_b = [&](int kt) { srcB = g4_src(g.B, g.ldb, n0, g.N, min(kt, nk - 1) * 64); };
    // issue order B(0) A(0) B(1) A(1) A(2), then per K-tile kt: B(kt + 2) A(kt + 3) -- so "B(kt + 1)
    // and A(kt + 1) landed" is always vmcnt(24): A(kt + 2), B(kt + 2), A(kt + 3) may still fly
    src_b(0);
    src_a(0);
#pragma unroll
    for (int p = 0; p < 8; ++p) g4_piece(srcB, vob, g.ldb, p, sb(0), w);
#pragma unroll
    for (int p = 0; p < 8; ++p) g4_piece(srcA, voa, g.lda, p, sa(0), w);
    src_b(1);
    src_a(1);
#pragma unroll
    for (int p = 0; p < 8; ++p) g4_piece(srcB, vob, g.ldb, p, sb(1), w);
#pragma unroll
    for (int p = 0; p < 8; ++p) g4_piece(srcA, voa, g.lda, p, sa(1), w);
    src_a(2);
#pragma unroll
    for (int p = 0; p < 8; ++p) g4_piece(srcA, voa, g.lda, p, sa(2), w);
    vm_wait_w<24>();
    g4_raw_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (r < 8) b0[r] = g4_frag(sb(0), wc * 128 + r * 16, 0);
      else a0[r - 8] = g4_frag(sa(0), wr * 128 + (r - 8) * 16, 0);
    }
    int ca = 0;  // kt % 3
    for (int kt = 0; kt < nk; ++kt) {
      const int cb = kt & 1, ca1 = ca == 2 ? 0 : ca + 1;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r < 8) b1[r] = g4_frag(sb(cb), wc * 128 + r * 16, 4);
        else a1[r - 8] = g4_frag(sa(ca), wr * 128 + (r - 8) * 16, 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) mma(a0, b0, 4 * r + q);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      g4_raw_barrier();  // M: A slot ca and B slot cb fully read by every wave
      src_b(kt + 2);
      src_a(kt + 3);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r < 8) g4_piece(srcB, vob, g.ldb, r, sb(cb), w);
        else g4_piece(srcA, voa, g.lda, r - 8, sa(ca), w);
#pragma unroll
        for (int q = 0; q < 2; ++q) mma(a1, b1, 2 * r + q);
      }
      vm_wait_w<24>();   // B(kt + 1), A(kt + 1) landed
      g4_raw_barrier();  // E
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r < 8) b0[r] = g4_frag(sb(cb ^ 1), wc * 128 + r * 16, 0);
        else a0[r - 8] = g4_frag(sa(ca1), wr * 128 + (r - 8) * 16, 0);
#pragma unroll
        for (int q = 0; q < 2; ++q) mma(a1, b1, 32 + 2 * r + q);
      }
      ca = ca1;
    }
  } else {
  set_src(0);
#pragma unroll
  for (int p = 0; p < 16; ++p) piece(0, p);
  set_src(1);
#pragma unroll
  for (int p = 0; p < 16; ++p) piece(1, p);
  vm_wait_w<16>();  // K-tile 0 landed (this wave's share); the barrier makes it everyone's
  g4_raw_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) frag(a0, b0, 0, 0, r);
  for (int kt = 0; kt < nk; ++kt) {
    const int c = kt & 1;
    // seg 1: k-step-1 fragments of K-tile kt | 64 MFMAs of k-step 0
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      frag(a1, b1, c, 1, r);
#pragma unroll
      for (int q = 0; q < 4; ++q) mma(a0, b0, 4 * r + q);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (DBG != 2) g4_raw_barrier();  // M: every wave is done reading buffer c
    // seg 2: LDS-DMA of K-tile kt + 2 into buffer c | 32 MFMAs of k-step 1
    set_src(kt + 2);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if constexpr (DBG != 4) piece(c, r);
#pragma unroll
      for (int q = 0; q < 2; ++q) mma(a1, b1, 2 * r + q);
    }
    if constexpr (DBG == 4) vm_wait_w<0>();
    else vm_wait_w<16>();  // K-tile kt + 1 landed (only kt + 2 still in flight)
    if constexpr (DBG != 2) g4_raw_barrier();  // E: ... for every wave
    // seg 3: k-step-0 fragments of K-tile kt + 1 | the other 32 MFMAs of k-step 1
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      frag(a0, b0, c ^ 1, 0, r);
#pragma unroll
      for (int q = 0; q < 2; ++q) mma(a1, b1, 32 + 2 * r + q);
    }
  }
  }
  vm_wait_w<0>();  // drain the clamped tail prefetches (LDS-DMA must not outlive the workgroup)
  // MFMA result -> first compiler read of the AGPR: 8-pass XDL needs >= 12 wait states, which hipcc
  // does not insert after an asm MFMA.  The pad "redefines" the accumulators of the last 8 MFMAs
  // (i = 7), so no read or copy of them (hipcc emits AGPR copies right after the loop) can be
  // scheduled above it; every earlier MFMA is >= 8 MFMA issues old.
  asm volatile("s_nop 15\n\ts_nop 7"
               : "+a"(acc[0][7][0]), "+a"(acc[0][7][1]), "+a"(acc[0][7][2]), "+a"(acc[0][7][3]), "+a"(acc[1][7][0]),
                 "+a"(acc[1][7][1]), "+a"(acc[1][7][2]), "+a"(acc[1][7][3])
               :
               : "memory");
  epilogue_w<EPI>(g, acc[0], m0, n0 + wc * 128, wr, 0, lane);
  epilogue_w<EPI>(g, acc[1], m0, n0 + wc * 128, wr, 1, lane);
}

template <int EPI>
static void launch4(const GemmArgs& g, hipStream_t st) {
  constexpr size_t shm = sizeof(bf16_t) * 4 * G4_HALF;  // 128 KB: 2 K-tile buffers of A and B
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm4_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)shm));
    attr = true;
  }
  const int tiles = ((g.M + 255) / 256) * ((g.N + 255) / 256);
  {
    const char* a3 = getenv("MFT_G4_A3");  // re-read per call (bench A/B)
    if (a3 && a3[0] == '1') {
      static bool attr3 = false;
      if (!attr3) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm4_kernel<EPI, 0, true>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 5 * G4_HALF * (int)sizeof(bf16_t)));
        attr3 = true;
      }
      gemm4_kernel<EPI, 0, true><<<tiles, 256, 5 * G4_HALF * sizeof(bf16_t), st>>>(g);
      return;
    }
  }
  if constexpr (EPI == GEMM_EPI_NONE) {
    static const int dbg = getenv("MFT_G4_DBG") ? atoi(getenv("MFT_G4_DBG")) : 0;
    if (dbg) {
      static bool attr_d = false;
      if (!attr_d) {
        for (const void* f : {(const void*)gemm4_kernel<EPI, 1>, (const void*)gemm4_kernel<EPI, 2>,
                              (const void*)gemm4_kernel<EPI, 4>})
          MFT_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        attr_d = true;
      }
      const int v = getenv("MFT_G4_DBG_V") ? atoi(getenv("MFT_G4_DBG_V")) : 0;  // re-read per call
      if (v == 1) { gemm4_kernel<EPI, 1><<<tiles, 256, shm, st>>>(g); return; }
      if (v == 2) { gemm4_kernel<EPI, 2><<<tiles, 256, shm, st>>>(g); return; }
      if (v == 4) { gemm4_kernel<EPI, 4><<<tiles, 256, shm, st>>>(g); return; }
    }
  }
  gemm4_kernel<EPI><<<tiles, 256, shm, st>>>(g);
}

bool gemm4_supported(int M, int N, int K) { return M > 0 && K > 0 && K % 64 == 0 && N >= 8 && N % 8 == 0; }

void gemm4(const GemmArgs& g, int epi, hipStream_t st) {
  if (!gemm4_supported(g.M, g.N, g.K) || g.lda > (1L << 23) || g.ldb > (1L << 23) || g.lda % 8 || g.ldb % 8) {
    fprintf(stderr, "mft::gemm4: unsupported shape M=%d N=%d K=%d lda=%ld ldb=%ld\n", g.M, g.N, g.K, g.lda, g.ldb);
    abort();
  }
  switch (epi) {
    case GEMM_EPI_NONE: launch4<GEMM_EPI_NONE>(g, st); break;
    case GEMM_EPI_BIAS: launch4<GEMM_EPI_BIAS>(g, st); break;
    case GEMM_EPI_BIAS_GELU: launch4<GEMM_EPI_BIAS_GELU>(g, st); break;
    case GEMM_EPI_DGELU: launch4<GEMM_EPI_DGELU>(g, st); break;
    case GEMM_EPI_BIAS_GELU_D: launch4<GEMM_EPI_BIAS_GELU_D>(g, st); break;
    case GEMM_EPI_MUL_AUX: launch4<GEMM_EPI_MUL_AUX>(g, st); break;
    case GEMM_EPI_F32ACC: launch4<GEMM_EPI_F32ACC>(g, st); break;
    case GEMM_EPI_LORA:
      if (g.lora_r <= 0 || g.lora_r > 32 || g.lora_r % 8 || g.ld_lu % 8) {
        fprintf(stderr, "mft::gemm4: LoRA epilogue needs rank %% 8 == 0, <= 32 (got %d)\n", g.lora_r);
        abort();
      }
      launch4<GEMM_EPI_LORA>(g, st);
      break;
    default: fprintf(stderr, "mft::gemm4: unsupported epilogue %d\n", epi); abort();
  }
}

template <int EPI>
static void launchw(const GemmArgs& g, hipStream_t st) {
  constexpr size_t shm = sizeof(bf16_t) * WNS * W_STAGE;  // 72 KB: two workgroups per CU
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemmw_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)shm));
    attr = true;
  }
  const int tiles = ((g.M + WBM - 1) / WBM) * ((g.N + WBN - 1) / WBN);
  gemmw_kernel<EPI><<<tiles, W_THREADS, shm, st>>>(g);
}

bool gemmw_supported(int M, int N, int K) { return M > 0 && K > 0 && K % WBK == 0 && N >= 8 && N % 8 == 0; }

void gemmw(const GemmArgs& g, int epi, hipStream_t st) {
  if (!gemmw_supported(g.M, g.N, g.K) || g.lda > (1L << 23) || g.ldb > (1L << 23) || g.lda % 8 || g.ldb % 8) {
    fprintf(stderr, "mft::gemmw: unsupported shape M=%d N=%d K=%d lda=%ld ldb=%ld\n", g.M, g.N, g.K, g.lda, g.ldb);
    abort();
  }
  switch (epi) {
    case GEMM_EPI_NONE: launchw<GEMM_EPI_NONE>(g, st); break;
    case GEMM_EPI_BIAS: launchw<GEMM_EPI_BIAS>(g, st); break;
    case GEMM_EPI_BIAS_GELU: launchw<GEMM_EPI_BIAS_GELU>(g, st); break;
    case GEMM_EPI_DGELU: launchw<GEMM_EPI_DGELU>(g, st); break;
    case GEMM_EPI_BIAS_GELU_D: launchw<GEMM_EPI_BIAS_GELU_D>(g, st); break;
    case GEMM_EPI_MUL_AUX: launchw<GEMM_EPI_MUL_AUX>(g, st); break;
    case GEMM_EPI_F32ACC: launchw<GEMM_EPI_F32ACC>(g, st); break;
    case GEMM_EPI_LORA:
      if (g.lora_r <= 0 || g.lora_r > 32 || g.lora_r % 8 || g.ld_lu % 8) {
        fprintf(stderr, "mft::gemmw: LoRA epilogue needs rank %% 8 == 0, <= 32 (got %d)\n", g.lora_r);
        abort();
      }
      launchw<GEMM_EPI_LORA>(g, st);
      break;
    default: fprintf(stderr, "mft::gemmw: unsupported epilogue %d\n", epi); abort();
  }
}

}  // namespace mft
