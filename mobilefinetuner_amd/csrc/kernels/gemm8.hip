// 256 x 256 x 64 bf16 MFMA GEMM with an 8-phase software pipeline (gfx950), every operand layout:
//
//   C[M, N] = epi(alpha * op(A) . op(B))
//   A: AT = false  [M, K] K-contiguous (activations)      AT = true  [K, M] M-contiguous
//   B: BT = false  [N, K] K-contiguous ("NT": y = x W^T)  BT = true  [K, N] N-contiguous ("NN": dx = dy W)
//   TN weight gradient dW[N_out, K_in] = dy^T x: AT = BT = true (both operands token-major), split
//   over the token (K) dimension into fp32 slabs reduced deterministically by gemm_splitk_reduce.
//
// K-contiguous half-tiles are [128 rows][64 k] (ds_read_b128 fragments); token-major half-tiles are
// [64 k][128 rows] read with ds_read_b64_tr_b16 (CDNA HIP guide T10) -- no transposed copies of any
// operand (the weight_t copies of round 1 are gone).  Structure after the CDNA HIP guide §5 "256² 8-phase template" (T1 XCD remap, T2 LDS
// XOR swizzle, T3+T4 8-phase interleave with counted vmcnt, T5 setprio):
//
//   * 8 waves; each 64-wide ds_read/MFMA phase works on ONE 128 x 128 quadrant of the block tile
//     (every wave a 64 x 32 piece of it: 4 x 2 fragments x 2 k-steps = 16 MFMAs).  Quadrants are
//     visited (A0,B0) (A0,B1) (A1,B1) (A1,B0) so consecutive phases reuse either the A or the B
//     fragments in registers.  A K-tile = 4 phases; an iteration = 2 K-tiles (even/odd LDS
//     buffer) = 8 phases.
//   * LDS: 2 buffers x {A0, A1, B0, B1} half-tiles of 128 x 64 bf16 (16 KB each) = 128 KB, filled
//     by global_load_lds_dwordx4 (2 per thread per half-tile) straight from HBM/L2; the 16-B chunk
//     index is XOR-swizzled with (row & 7) on the SOURCE address so the lane-linear LDS image reads
//     back conflict-light with ds_read_b128.
//   * Each half-tile is restaged ONE phase after its last read (every phase ends its reads with
//     lgkmcnt(0) before the barrier), one half-tile per phase, so the next K-tile of a buffer streams
//     in while the other buffer is multiplied; the waits are counted (vmcnt(4): two half-tiles stay
//     in flight across the barrier), never vmcnt(0) inside the loop, and the barriers are raw
//     s_barrier (a __syncthreads() would drain the LDS-DMA queue).
//
// Half-tile staging schedule (phase -> half-tile, K-tile of iteration i):
//   1: O.A1 (2i+1)  2: O.B0 (2i+1)  3: E.A0 (2i+2)  4: E.B1 (2i+2)
//   5: E.A1 (2i+2)  6: E.B0 (2i+2)  7: O.A0 (2i+3)  8: O.B1 (2i+3)
// with vmcnt(4) before the barriers of phases 4 (retires O for phases 5-8) and 8 (retires E for
// the next phases 1-4).  Loads of K-tiles past the end are clamped onto the last tile (harmless
// re-reads) so every wave issues the same count and the counted waits stay exact.
#include <stdlib.h>

#include "mfma.h"
#include "kernels.h"

namespace mft {

namespace {

constexpr int kHalf = 128 * 64;  // elements in a half-tile

typedef __attribute__((address_space(3))) void lds_void8;
typedef const __attribute__((address_space(1))) void g_void8;

__device__ __forceinline__ void glds16_8(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((g_void8*)src, (lds_void8*)lds_wave_base, 16, 0, 0);
}


// v_max3_f32 as asm (see epilogue_ce_fwd)
__device__ __forceinline__ float max3_f32(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Addresses are a wave-uniform base plus a 32-bit per-lane byte offset (the SGPR-base "saddr" form
// of global_load_lds): 1 VGPR per load instead of a 64-bit VGPR pair, which keeps the 256-VGPR
// budget of two waves per SIMD free for the epilogue variants.
__device__ __forceinline__ void glds16_off(const bf16_t* base, uint32_t off_bytes, void* lds_wave_base) {
  glds16_8(reinterpret_cast<const char*>(base) + off_bytes, lds_wave_base);
}

// stage one 128 x 64 half-tile: rows r0.. of src (clamped to rmax-1), columns k0..k0+63
__device__ __forceinline__ void stage_half(bf16_t* lds, const bf16_t* src, long ld, int r0, int rmax, int k0) {
  const int tid = threadIdx.x, w = tid >> 6;
  const int rb = min(r0, rmax - 1);
  const bf16_t* base = src + (long)rb * ld + k0;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c = t * 512 + tid;
    const int r = c >> 3, s = c & 7;
    const int gr = min(r0 + r, rmax - 1) - rb;
    glds16_off(base, (uint32_t)((gr * (int)ld + ((s ^ (r & 7)) << 3)) * 2), lds + (t * 512 + w * 64) * 8);
  }
}

// per-lane byte offsets of stage_half's two loads for an interior half-tile (no row clamping): they
// depend only on the lane and the row stride, so a kernel that moves between tiles computes them
// once and each staging is one scalar base + these offsets
__device__ __forceinline__ void stage_offsets(long ld, uint32_t (&off)[2]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c = t * 512 + tid;
    const int r = c >> 3, s = c & 7;
    off[t] = (uint32_t)((r * (int)ld + ((s ^ (r & 7)) << 3)) * 2);
  }
}
__device__ __forceinline__ void stage_half_fast(bf16_t* lds, const bf16_t* src, long ld, int r0, int rmax, int k0,
                                                const uint32_t (&off)[2]) {
  if (r0 + 128 <= rmax) {
    const int w = threadIdx.x >> 6;
    const bf16_t* base = src + (long)r0 * ld + k0;
#pragma unroll
    for (int t = 0; t < 2; ++t) glds16_off(base, off[t], lds + (t * 512 + w * 64) * 8);
  } else {
    stage_half(lds, src, ld, r0, rmax, k0);
  }
}

// stage one [64 k][128 cols] half-tile of a k-major operand: rows k0..k0+63 of src, columns
// c0..c0+127 (clamped to cmax-8; cmax % 8 == 0).  256-B rows; the 16-B chunk index is XOR-swizzled
// with tsw(k) (even, so 32-B pairs stay together) on the SOURCE address: the 8 rows one 32-lane half
// of ds_read_b64_tr_b16 touches ({0..3, 8..11} or {4..7, 12..15} mod 16) land in 8 distinct 32-B
// bank slots -> conflict-free transposed reads.
__device__ __forceinline__ int tsw(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

__device__ __forceinline__ void stage_half_t(bf16_t* lds, const bf16_t* src, long ld, int c0, int cmax, int k0) {
  const int tid = threadIdx.x, w = tid >> 6;
  const int cb = min(c0, cmax - 8);
  const bf16_t* base = src + (long)k0 * ld + cb;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c = t * 512 + tid;
    const int r = c >> 4, s = c & 15;
    const int gc = min(c0 + ((s ^ tsw(r)) << 3), cmax - 8) - cb;
    glds16_off(base, (uint32_t)((r * (int)ld + gc) * 2), lds + (t * 512 + w * 64) * 8);
  }
}

// ds_read_b64_tr_b16 as inline asm: the builtin makes hipcc (ROCm 7.2) assume it may alias the
// in-flight LDS-DMA and emit s_waitcnt vmcnt(0) before every transposed read, draining the
// 8-phase prefetch (measured: NN 2.6x the wave-cycles of NT).  The asm result is only valid after
// the explicit lgkmcnt(0) + sched_barrier of each phase (lds_sync below, guide §5.4 rule 18).
__device__ __forceinline__ s16x4_t ds_tr16_asm(const bf16_t* p) {
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
  s16x4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}

// fragment of a swizzled [64 k][128] half-tile: lane holds T[k = 8*kc + 8*(l>>4) + j][c = r0 + (l&15)]
// (the same register image frag8 produces from a K-contiguous tile)
__device__ __forceinline__ bf16x8_t frag8_t(const bf16_t* t, int r0, int kc) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int k = 8 * kc + 8 * g + q;        // rows k (lo) and k + 4 (hi)
  const int col = r0 + 4 * p;              // 4 columns per lane of the 16-lane group
  const int ch = col >> 3, off = col & 7;  // logical 16-B chunk, element offset inside it
  const bf16_t* a0 = t + k * 128 + ((ch ^ tsw(k)) << 3) + off;
  const bf16_t* a1 = t + (k + 4) * 128 + ((ch ^ tsw(k + 4)) << 3) + off;
  s16x4_t lo = ds_tr16_asm(a0);
  s16x4_t hi = ds_tr16_asm(a1);
  s16x8_t r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

// fragment of a swizzled half-tile: lane holds T[r0 + (l&15)][8*kc + 8*(l>>4) + j]
__device__ __forceinline__ bf16x8_t frag8(const bf16_t* t, int r0, int kc) {
  const int l = threadIdx.x & 63;
  const int r = r0 + (l & 15), q = kc + (l >> 4);
  return *reinterpret_cast<const bf16x8_t*>(t + r * 64 + ((q ^ (r & 7)) << 3));
}

}  // namespace

// ------------------------------------------------------------------ epilogue (registers only)
template <int EPI>
__device__ __forceinline__ void epilogue8(const GemmArgs& g, f32x4_t (&acc)[4][4][2], int m0, int n0, int wm, int wn,
                                          int lane, int split) {
  // The MFMAs ran with the operands swapped, so each 16 x 16 accumulator block is C^T: lane l holds
  // row (l & 15) of the block, columns 4 * (l >> 4) .. +3.  One v_permlane16_swap per dword pairs
  // the two column blocks of the wave's 32-column piece so every lane then owns EIGHT CONTIGUOUS
  // columns of one row: lane group g = l >> 4 -> column offset {0, 16, 8, 24}[g].  Every epilogue
  // is then 16-B vector loads/stores straight from registers (no LDS staging, no wave syncs).
  const int g4 = lane >> 4;
  const int cofs = (g4 & 1) * 16 + (g4 >> 1) * 8;
  // epilogues that read an [M, N] operand: every load of the lane's 16 pieces is issued before the
  // first store (the stores may alias it, so the compiler would otherwise wait on each load in turn)
  constexpr bool kAux = EPI == GEMM_EPI_DGELU || EPI == GEMM_EPI_MUL_AUX || EPI == GEMM_EPI_BIAS_ADD;
  u16x8_t auxv[4][4];
  if constexpr (kAux) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int qa = (q == 2 || q == 3) ? 1 : 0, qb = (q == 1 || q == 2) ? 1 : 0;
      const int colc = min(n0 + qb * 128 + wn * 32 + cofs, g.N - 8);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = min(m0 + qa * 128 + wm * 64 + i * 16 + (lane & 15), g.M - 1);
        auxv[q][i] = *reinterpret_cast<const u16x8_t*>(g.aux + (long)row * g.ldaux + colc);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int qa = (q == 2 || q == 3) ? 1 : 0, qb = (q == 1 || q == 2) ? 1 : 0;
    const int rbase = m0 + qa * 128 + wm * 64, col = n0 + qb * 128 + wn * 32 + cofs;
    const bool col_ok = col < g.N;
    const int colc = min(col, g.N - 8);
    float bias_v[8];
    if constexpr (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU || EPI == GEMM_EPI_BIAS_GELU_D ||
                  EPI == GEMM_EPI_BIAS_ADD)
      load8(g.bias + colc, bias_v);
    float o[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[q][i][0][r]),
                                                         __float_as_uint(acc[q][i][1][r]), false, false);
        o[i][r] = __uint_as_float(sw[0]);
        o[i][4 + r] = __uint_as_float(sw[1]);
      }
    }
    if constexpr (EPI == GEMM_EPI_LORA) {
      // rank-r update: the lane's 8 x r slice of lora_w is loaded once per 8 ranks per quadrant,
      // each row of lora_u is one 16-B load per 8 ranks (r <= 32, multiple of 8)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[i][e] *= g.alpha;
      // (ranks in groups of 4: the lane's 4 x 8 slice of lora_w is 16 VGPRs, which keeps the kernel
      // inside 256 VGPRs with the B0 fragments held across phases (KEEPB))
#pragma unroll 1
      for (int t4 = 0; t4 < g.lora_r; t4 += 4) {
        u16x8_t wv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) wv[t] = *reinterpret_cast<const u16x8_t*>(g.lora_w + (long)(t4 + t) * g.ld_lw + colc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = min(rbase + i * 16 + (lane & 15), g.M - 1);
          const uint2 ur = *reinterpret_cast<const uint2*>(g.lora_u + (long)row * g.ld_lu + t4);
          const float u[4] = {__uint_as_float(ur.x << 16), __uint_as_float(ur.x & 0xffff0000u),
                              __uint_as_float(ur.y << 16), __uint_as_float(ur.y & 0xffff0000u)};
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int e = 0; e < 8; ++e) o[i][e] += u[t] * bf2f(wv[t][e]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = rbase + i * 16 + (lane & 15);
      const bool ok = col_ok && row < g.M;
      float* v = o[i];
      if constexpr (EPI == GEMM_EPI_F32PART) {  // split-K slab: plain fp32 store, reduced later
        if (ok) {
          float* P = g.ws + ((long)split * g.M + row) * g.N + col;
          *reinterpret_cast<f32x4_t*>(P) = f32x4_t{v[0], v[1], v[2], v[3]};
          *reinterpret_cast<f32x4_t*>(P + 4) = f32x4_t{v[4], v[5], v[6], v[7]};
        }
        continue;
      }
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
          if constexpr (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU || EPI == GEMM_EPI_BIAS_GELU_D ||
                        EPI == GEMM_EPI_BIAS_ADD)
            v[e] += bias_v[e];
          if constexpr (EPI == GEMM_EPI_BIAS_ADD) v[e] += bf2f(auxv[q][i][e]);
        }
      }
      if constexpr (EPI == GEMM_EPI_DGELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= gelu_tanh_grad(bf2f(auxv[q][i][e]));
      }
      if constexpr (EPI == GEMM_EPI_MUL_AUX) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= bf2f(auxv[q][i][e]);
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

// ------------------------------------------------------------------ LM-head CE dgrad epilogue
// dh = fin * acc - wlab * W[label] (B = W stored [Vpad, N]).  Every per-row operand of the lane's
// 8 rows is loaded before the first store (the stores could alias them, so the compiler would
// otherwise serialise 16 dependent load chains behind them).
// Vocab-split form (ksplit > 1, a row chunk too short to fill the CUs with its 256 x 256 output
// tiles): split s covers whole vocab tiles, applies its own final factor ce_fin[s][row] (the
// accumulator is relative to its LAST tile's max), only split 0 subtracts the label row, and the
// result goes to the fp32 slab ws[s][M][N] reduced in split order by ce_split_reduce.
__device__ __forceinline__ void epilogue_ce_dgrad(const GemmArgs& g, f32x4_t (&acc)[4][4][2], int m0, int n0, int wm,
                                                  int wn, int lane, int split) {
  const int g4 = lane >> 4;
  const int cofs = (g4 & 1) * 16 + (g4 >> 1) * 8;
  const bool slab = g.ksplit > 1;
  float fin[2][4], wl[2][4];
  long lab[2][4];
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = min(m0 + qa * 128 + wm * 64 + i * 16 + (lane & 15), g.M - 1);
      fin[qa][i] = g.ce_fin[(long)split * g.M + rr];
      wl[qa][i] = split == 0 ? g.ce_wlab[rr] : 0.f;
      lab[qa][i] = g.ce_labels[rr];
    }
#pragma unroll
  for (int qa = 0; qa < 2; ++qa) {
    u16x8_t wv[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = n0 + h * 128 + wn * 32 + cofs, colc = min(col, g.N - 8);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long l = wl[qa][i] != 0.f ? lab[qa][i] : 0;
        wv[h][i] = *reinterpret_cast<const u16x8_t*>(g.B + l * g.ldb + colc);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = qa ? (h ? 2 : 3) : (h ? 1 : 0);  // quadrant (qa, qb = h)
      const int col = n0 + h * 128 + wn * 32 + cofs;
      float o[4][8];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[q][i][0][r]),
                                                           __float_as_uint(acc[q][i][1][r]), false, false);
          o[i][r] = __uint_as_float(sw[0]);
          o[i][4 + r] = __uint_as_float(sw[1]);
        }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + qa * 128 + wm * 64 + i * 16 + (lane & 15);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[i][e] = o[i][e] * fin[qa][i] - wl[qa][i] * bf2f(wv[h][i][e]);
        if (col < g.N && row < g.M) {
          if (slab) {
            float* P = g.ws + ((long)split * g.M + row) * g.N + col;
            *reinterpret_cast<f32x4_t*>(P) = f32x4_t{o[i][0], o[i][1], o[i][2], o[i][3]};
            *reinterpret_cast<f32x4_t*>(P + 4) = f32x4_t{o[i][4], o[i][5], o[i][6], o[i][7]};
          } else {
            store8(reinterpret_cast<bf16_t*>(g.C) + (long)row * g.ldc + col, o[i]);
          }
        }
      }
    }
  }
}

// Workgroup barrier for an LDS exchange only: this wave's LDS operations retired, then a raw
// s_barrier.  __syncthreads() is a workgroup fence as well, for which the compiler waits on
// vmcnt(0) -- every global store still in flight (the CE forward's 128 KB tile of E) would stall
// each wave at the barrier (measured: 30.5 vs 25.6 ms for Gemma's LM-head forward without E).
__device__ __forceinline__ void lds_barrier() {
  lgkm_wait0();
  raw_barrier();
}

// ------------------------------------------------------------------ LDS-staged epilogues
// The register epilogue stores 16 rows x 64 B per wave instruction, which the store path moves at
// ~13 B/cycle per CU; whole-row segments (>= 128 B per row) move at ~48 B/cycle per CU when not
// every CU stores at once (profiles/r4_store_probe.txt).  Here the finished bf16 tile goes through
// the (now idle) LDS operand buffers -- 16-B chunks XOR-swizzled by (row & 31): conflict-free
// writes and reads -- and leaves as 2 full 512-B tile rows per wave instruction.  Epilogues with an
// [M, N] operand (dGELU, MUL_AUX) bring it in the same way: one LDS-DMA of whole tile rows into the
// image, then every lane reads back its own fragment positions and overwrites them in place.
// BIAS_GELU_D has two outputs: two rounds through the one 128 KB image.
__device__ __forceinline__ int lds_tile_off(int rowt, int chunk) { return rowt * 256 + ((chunk ^ (rowt & 31)) << 3); }

// the whole [256 x 256] bf16 tile image -> C rows (bounds-checked), 16 x 16 B per lane
__device__ __forceinline__ void lds_tile_store(const bf16_t* lds, bf16_t* C, long ldc, int m0, int n0, int M, int N) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = k * 512 + tid;
    const int rowt = c >> 5, chunk = c & 31;
    const uint4 pk = *reinterpret_cast<const uint4*>(lds + lds_tile_off(rowt, chunk));
    const int row = m0 + rowt, col = n0 + chunk * 8;
    if (row < M && col < N) *reinterpret_cast<uint4*>(C + (long)row * ldc + col) = pk;
  }
}

// X rows [m0, m0 + 256) x cols [n0, n0 + 256) (clamped at the edges) -> the swizzled tile image by
// LDS-DMA (lane-linear destination; the swizzle is applied on the source column), then waited
__device__ __forceinline__ void lds_tile_load(bf16_t* lds, const bf16_t* X, long ldx, int m0, int n0, int M, int N) {
  const int tid = threadIdx.x, w = tid >> 6;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = k * 512 + tid;           // destination chunk of the image (lane-linear)
    const int rowt = c >> 5, dch = c & 31;  // image row, swizzled chunk slot
    const int chunk = dch ^ (rowt & 31);    // the logical column chunk stored at that slot
    const int row = min(m0 + rowt, M - 1), col = min(n0 + chunk * 8, N - 8);
    glds16_8(X + (long)row * ldx + col, lds + (k * 512 + w * 64) * 8);
  }
  vm_wait<0>();
  lds_barrier();
}

template <int EPI>
__device__ __forceinline__ void epilogue_lds(const GemmArgs& g, f32x4_t (&acc)[4][4][2], int m0, int n0, int wm, int wn,
                                             int lane, bf16_t* lds) {
  constexpr bool kAux = EPI == GEMM_EPI_DGELU || EPI == GEMM_EPI_MUL_AUX;
  constexpr bool kBias = EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU_D;
  constexpr int kRounds = EPI == GEMM_EPI_BIAS_GELU_D ? 2 : 1;
  const int g4 = lane >> 4;
  const int cofs = (g4 & 1) * 16 + (g4 >> 1) * 8;
  if constexpr (kAux) lds_tile_load(lds, g.aux, g.ldaux, m0, n0, g.M, g.N);
#pragma unroll
  for (int rnd = 0; rnd < kRounds; ++rnd) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int qa = (q == 2 || q == 3) ? 1 : 0, qb = (q == 1 || q == 2) ? 1 : 0;
      const int colt = qb * 128 + wn * 32 + cofs;
      float bias_v[8];
      if constexpr (kBias) load8(g.bias + min(n0 + colt, g.N - 8), bias_v);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[q][i][0][r]),
                                                           __float_as_uint(acc[q][i][1][r]), false, false);
          v[r] = __uint_as_float(sw[0]);
          v[4 + r] = __uint_as_float(sw[1]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] *= g.alpha;
          if constexpr (kBias) v[e] += bias_v[e];
        }
        const int rowt = qa * 128 + wm * 64 + i * 16 + (lane & 15);
        uint4* slot = reinterpret_cast<uint4*>(lds + lds_tile_off(rowt, colt >> 3));
        if constexpr (kAux) {
          const u16x8_t av = __builtin_bit_cast(u16x8_t, *slot);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= EPI == GEMM_EPI_DGELU ? gelu_tanh_grad(bf2f(av[e])) : bf2f(av[e]);
        }
        if constexpr (EPI == GEMM_EPI_BIAS_GELU_D) {
          float d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) gelu_tanh_and_grad(v[e], v[e], d[e]);
          if (rnd == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = d[e];
          }
        }
        *slot = uint4{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
      }
    }
    lds_barrier();
    bf16_t* dst = (EPI == GEMM_EPI_BIAS_GELU_D && rnd == 1) ? g.aux : reinterpret_cast<bf16_t*>(g.C);
    const long ldd = (EPI == GEMM_EPI_BIAS_GELU_D && rnd == 1) ? g.ldaux : g.ldc;
    lds_tile_store(lds, dst, ldd, m0, n0, g.M, g.N);
    if (rnd + 1 < kRounds) lds_barrier();  // every wave's reads of the image done before round 2 writes
  }
}

// ------------------------------------------------------------------ LM-head CE forward epilogue
// Logits tile (fp32 accumulators) -> per-row tile max and sum-exp, label logit, and (optionally)
// E = exp(logit - tile max) in bf16.  A row's 256 tile columns are spread over the lane's 2 x 8
// columns (quadrants qb = 0, 1), the 4 lane groups of the wave (shuffles) and the 4 wn-waves (LDS).
// Numerics: the loss comes from fp32 logits; E is relative to its tile max, so every softmax term
// keeps bf16's relative precision whatever the logit magnitude (raw bf16 logits of a pretrained
// model, |logit| ~ 100, would be quantised to 0.5).
// LDSE: the E tile goes through an LDS image (after the 4 KB reduction scratch) and leaves as whole
// tile rows (lds_tile_store) instead of 16-row x 64-B register stores.
template <bool LDSE = false>
__device__ __forceinline__ void epilogue_ce_fwd(const GemmArgs& g, f32x4_t (&acc)[4][4][2], int m0, int n0, int wm,
                                                int wn, int lane, float* red) {
  bf16_t* img = reinterpret_cast<bf16_t*>(red) + 4096;  // 8 KB past the scratch (LDSE)
  const int g4 = lane >> 4, r16 = lane & 15;
  const int cofs = (g4 & 1) * 16 + (g4 >> 1) * 8;
  const int T = (g.N + 255) / 256, tn = n0 >> 8;
  float o[4][4][8];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[q][i][0][r]),
                                                         __float_as_uint(acc[q][i][1][r]), false, false);
        o[q][i][r] = __uint_as_float(sw[0]);
        o[q][i][4 + r] = __uint_as_float(sw[1]);
      }
  // quadrants: 0 = (A0, B0), 1 = (A0, B1), 2 = (A1, B1), 3 = (A1, B0); row half qa holds q = 2qa, 2qa+1
  auto qcol = [&](int q) { return n0 + ((q == 1 || q == 2) ? 128 : 0) + wn * 32 + cofs; };
  // only the last vocab tile has padding columns: the mask is a uniform branch elsewhere
  const bool full = n0 + 256 <= g.ce_V;
  const int rl0 = wm * 64 + r16;  // tile row = qa * 128 + rl0 + 16 i
  // the rows' labels are fetched first: their global-load latency hides under the max reduction
  long labs[2][4];
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int i = 0; i < 4; ++i) labs[qa][i] = g.ce_labels[min(m0 + qa * 128 + rl0 + i * 16, g.M - 1)];
  float mt[2][4];
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float m;
      if (full) {
        // 16 values in 8 v_max3_f32 (asm: fmaxf on MFMA results makes hipcc insert a canonicalising
        // v_max_f32 per operand -- the epilogue measured 3.8 VALU per MFMA of the whole kernel)
        const float* a = o[2 * qa][i];
        const float* b = o[2 * qa + 1][i];
        m = max3_f32(a[0], a[1], a[2]);
        m = max3_f32(m, a[3], a[4]);
        m = max3_f32(m, a[5], a[6]);
        m = max3_f32(m, a[7], b[0]);
        m = max3_f32(m, b[1], b[2]);
        m = max3_f32(m, b[3], b[4]);
        m = max3_f32(m, b[5], b[6]);
        m = fmaxf(m, b[7]);
      } else {
        // padding columns become -inf here, so the exp pass below needs no mask (exp2(-inf) = 0)
        m = -INFINITY;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int q = 2 * qa + h, c = qcol(q);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if (c + e >= g.ce_V) o[q][i][e] = -INFINITY;
            m = fmaxf(m, o[q][i][e]);
          }
        }
      }
      m = fmaxf(m, xor16_pl(m));
      m = fmaxf(m, xor32_pl(m));
      mt[qa][i] = m;
    }
  if (g4 == 0) {
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(qa * 128 + rl0 + i * 16) * 4 + wn] = mt[qa][i];
  }
  lds_barrier();
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(red + (qa * 128 + rl0 + i * 16) * 4);
      mt[qa][i] = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));  // -inf only for an all-padding tile
    }
  lds_barrier();  // red is reused for the sums
  float st[2][4];
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int R = m0 + qa * 128 + rl0 + i * 16;
      const bool rok = R < g.M;
      const int lab = (int)labs[qa][i];  // vocab < 2^31; -100 (ignored) never matches a column
      // an all-padding tile (max -inf) must not turn exp(-inf - -inf) into NaN
      const float mb = (mt[qa][i] == -INFINITY ? 0.f : mt[qa][i]) * 1.4426950408889634f;
      float s = 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int q = 2 * qa + h, c = qcol(q);
        const unsigned d = (unsigned)(lab - c);
        // the label column: a branch the wave almost never takes (one row's label in this lane's 8
        // columns of a 256-column tile), instead of a branch-free 64-bit select chain over every value
        if (__builtin_expect(rok && d < 8u, 0)) {
          float xl = o[q][i][0];
#pragma unroll
          for (int e = 1; e < 8; ++e) xl = d == (unsigned)e ? o[q][i][e] : xl;
          g.ce_lbl[R] = xl;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = fast_exp2(fmaf(o[q][i][e], 1.4426950408889634f, -mb));
          o[q][i][e] = x;
          s += x;
        }
        if constexpr (LDSE) {
          const int rowt = R - m0, colt = c - n0;
          const float* ov = o[q][i];
          *reinterpret_cast<uint4*>(img + lds_tile_off(rowt, colt >> 3)) =
              uint4{pack_bf2(ov[0], ov[1]), pack_bf2(ov[2], ov[3]), pack_bf2(ov[4], ov[5]), pack_bf2(ov[6], ov[7])};
        } else {
          // non-temporal: E is re-read only by the dgrad after the whole chunk (GBs later), far beyond
          // L2 / MALL reach -- streaming stores keep it from evicting the operand tiles
          if (g.C && rok && c < g.N) store8_nt(reinterpret_cast<bf16_t*>(g.C) + (long)R * g.ldc + c, o[q][i]);
        }
      }
      s += xor16_pl(s);
      s += xor32_pl(s);
      st[qa][i] = s;
    }
  if (g4 == 0) {
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(qa * 128 + rl0 + i * 16) * 4 + wn] = st[qa][i];
  }
  lds_barrier();
  if (wn == 0 && g4 == 0) {
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int R = m0 + qa * 128 + rl0 + i * 16;
        if (R >= g.M) continue;
        const f32x4_t v = *reinterpret_cast<const f32x4_t*>(red + (qa * 128 + rl0 + i * 16) * 4);
        float* p = g.ce_stats + ((long)R * T + tn) * 2;
        p[0] = mt[qa][i];
        p[1] = (v[0] + v[1]) + (v[2] + v[3]);
      }
  }
  if constexpr (LDSE) {
    if (g.C) lds_tile_store(img, reinterpret_cast<bf16_t*>(g.C), g.ldc, m0, n0, g.M, g.N);  // (the image was
    // complete at the lds_barrier above: every wave wrote its E pieces before it)
  }
}

#ifdef MFT_G8_STAMPS  // diagnostic build only (scripts/g8_stamps.hip): s_memtime per phase per WG
__device__ unsigned long long* g8_stamps;
#ifdef MFT_G8_STAMPS_RT  // 100 MHz constant clock instead of the shader clock
#define G8_STAMP(k) \
  if (threadIdx.x == 0) g8_stamps[blockIdx.x * 4 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define G8_STAMP(k) \
  if (threadIdx.x == 0) g8_stamps[blockIdx.x * 4 + (k)] = __builtin_amdgcn_s_memtime()
#endif
#else
#define G8_STAMP(k)
#endif

// LATE (default): each phase arrives at its first barrier with its fragment reads still in flight
// and waits for them after it (the guide §5 template order: s_barrier; lgkmcnt(0); MFMAs), the B
// fragments read before the A fragments -- the read latency then overlaps the barrier skew instead
// of adding to it: +1-4 % on every NT shape measured (profiles/r3_g8late.txt).  (Reads complete
// before the phase's MFMAs; the half-tile they read is restaged only after the phase's second
// barrier, so the order is safe.)  LATE = false keeps the earlier order for A/B runs.
// KEEPB defaults on where the 16 extra VGPRs fit without spilling (not the TT wgrad form or the CE
// dgrad, which spill 2-7 VGPRs with it; the LoRA epilogue fits since it walks the ranks 4 at a time)
template <int EPI, bool AT, bool BT, bool LATE = true,
          bool KEEPB = !(AT && BT) && EPI != GEMM_EPI_CE_DGRAD, bool LDSEPI = false>
__global__ __launch_bounds__(512, 1) void gemm8_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  if (g.stagger > 0 && blockIdx.x < 256) {  // first round: spread each XCD's CUs over a tile round
    for (int c = (int)(blockIdx.x >> 3) * g.stagger; c > 0; c -= 8000) __builtin_amdgcn_s_sleep(125);
  }
  G8_STAMP(0);
  // buffer b (0 = even, 1 = odd): half-tiles A0, A1, B0, B1 at smem + (b * 4 + h) * kHalf
  const int tiles_n = (g.N + 255) / 256;
  const int ntiles = ((g.M + 255) / 256) * tiles_n;
  const int ksplit = g.ksplit > 1 ? g.ksplit : 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // split-major: the workgroups an XCD holds at once work on the SAME K (token) slab for different
  // output tiles, so each slab of both operands is fetched into that XCD's L2 once and shared (a
  // tile's splits share no data; tile-major ordering measured 2.8x the cycles per K-tile in TN)
  const int tile = bid % ntiles, split = bid / ntiles;
  const int m0 = (tile / tiles_n) * 256, n0 = (tile % tiles_n) * 256;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;  // wave's 64 x 32 piece inside each 128 x 128 quadrant
  const int nk_all = g.K / 64;
  const int kps = (nk_all + ksplit - 1) / ksplit;  // K-tiles per split
  const int kbase = split * kps;
  const int nk = max(0, min(nk_all - kbase, kps));
  const int last = max(nk - 1, 0);

  auto half_ptr = [&](int buf, int h) { return smem + (buf * 4 + h) * kHalf; };
  // h: 0 = A0, 1 = A1, 2 = B0, 3 = B1
  auto stage = [&](int buf, int h, int kt) {
    const int k0 = min(kbase + min(kt, last), nk_all - 1) * 64;  // an empty split still stores zeros
    if (h < 2) {
      if constexpr (AT) stage_half_t(half_ptr(buf, h), g.A, g.lda, m0 + h * 128, g.M, k0);
      else stage_half(half_ptr(buf, h), g.A, g.lda, m0 + h * 128, g.M, k0);
    } else {
      if constexpr (BT) stage_half_t(half_ptr(buf, h), g.B, g.ldb, n0 + (h - 2) * 128, g.N, k0);
      else stage_half(half_ptr(buf, h), g.B, g.ldb, n0 + (h - 2) * 128, g.N, k0);
    }
  };

  f32x4_t acc[4][4][2];  // [quadrant][i][j]
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[q][i][j] = zero4();

  // B fragments per 128-column half: with KEEPB the (A1, B0) phase reuses the B0 fragments its
  // (A0, B0) phase read (+16 VGPRs, 4 of the 28 ds_read_b128 per wave and K-tile saved)
  bf16x8_t af[4][2], bfr2[2][2][2];
  auto read_a = [&](int buf, int ah) {
    const bf16_t* t = half_ptr(buf, ah);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (AT) af[i][ks] = frag8_t(t, wm * 64 + i * 16, ks * 4);
        else af[i][ks] = frag8(t, wm * 64 + i * 16, ks * 4);
      }
  };
  auto read_b = [&](int buf, int bh) {
    const bf16_t* t = half_ptr(buf, 2 + bh);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (BT) bfr2[KEEPB ? bh : 0][j][ks] = frag8_t(t, wn * 32 + j * 16, ks * 4);
        else bfr2[KEEPB ? bh : 0][j][ks] = frag8(t, wn * 32 + j * 16, ks * 4);
      }
  };
  auto mma = [&](int q) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[q][i][j] = mfma16(bfr2[KEEPB && (q == 1 || q == 2)][j][ks], af[i][ks], acc[q][i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // end of a phase's fragment reads: every ds_read retired; with asm transposed reads the compiler
  // must not move the MFMAs that consume them above this point
  auto lds_sync = [&]() {
    lgkm_wait0();
    if constexpr (AT || BT) __builtin_amdgcn_sched_barrier(0);
  };

  // CE_DGRAD: the A operand E holds exp(logit - tile max) per 256-column vocab tile (4 K-tiles); at
  // each tile start the accumulator is rescaled by exp(m'_prev - m'_cur) (ratios precomputed per
  // row by ce_finalize), so after the last tile acc = sum_t exp(m'_t - m'_last) E_t W_t and the
  // epilogue's factor exp(m'_last - lse) turns it into softmax . W -- no elementwise pass over E.
  // The 256 row factors of a tile arrive by one LDS-DMA of wave 0 (1 KB, 2 slots after the half-
  // tile buffers), issued in phase 5 two iterations ahead: it is older than the 4 in-flight
  // half-tiles at the phase-8 vm_wait, so the counted waits retire it with no extra wait.
  float* const rslot = reinterpret_cast<float*>(smem + 8 * kHalf);
  auto ce_dma = [&](int kt) {
    if constexpr (EPI == GEMM_EPI_CE_DGRAD) {
      const int tt = kt / 4 + 1;  // local vocab tile of this split (kbase is a whole number of tiles)
      if ((kt & 3) == 0 && tt * 4 < nk && w == 0) {
        const long mpad = (long)((g.M + 255) / 256) * 256;
        glds16_8(g.ce_ratio + (long)(kbase / 4 + tt) * mpad + m0 + lane * 4, rslot + (tt & 1) * 256);
      }
    }
  };
  // the phase's 4 row factors: read with its fragments (before lds_sync), applied after it
  auto ce_read = [&](int q, int kt) -> f32x4_t {
    if constexpr (EPI == GEMM_EPI_CE_DGRAD) {
      if ((kt & 3) == 0 && kt > 0)
        return *reinterpret_cast<const f32x4_t*>(rslot + ((kt / 4) & 1) * 256 + (q < 2 ? 0 : 128) + wm * 64 +
                                                 (lane & 15) * 4);
    }
    return f32x4_t{1.f, 1.f, 1.f, 1.f};
  };
  // The rescale of each accumulator block is issued right before its first MFMA of the even
  // K-tile, inside the MFMA cluster: 4 v_mul_f32 fit the 16-cycle issue gap of the MFMA before (the
  // same multiplies placed in the load segment cost ~15% of the kernel: VALU there competes with
  // the partner wave's prio-1 MFMA cluster).  Branch-free (factor 1 off the tile starts): a
  // second MFMA code path for the tile starts spills.  Scalar asm multiplies: left to the
  // compiler they become v_pk_mul_f32, which costs extra cycles beside MFMAs.
  auto mma_ce = [&](int q, const f32x4_t& r) {
    if constexpr (EPI == GEMM_EPI_CE_DGRAD) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (ks == 0) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                float x = acc[q][i][j][e];
                asm("v_mul_f32 %0, %1, %2" : "=v"(x) : "v"(x), "v"(r[i]));
                acc[q][i][j][e] = x;
              }
            }
            acc[q][i][j] = mfma16(bfr2[KEEPB && (q == 1 || q == 2)][j][ks], af[i][ks], acc[q][i][j]);
          }
      __builtin_amdgcn_s_setprio(0);
    } else {
      mma(q);
    }
  };

  // prologue: E <- K-tile 0 (all halves), O <- K-tile 1 (A0, B1); retire E
  stage(0, 0, 0);
  stage(0, 3, 0);
  stage(0, 1, 0);
  stage(0, 2, 0);
  stage(1, 0, 1);
  stage(1, 3, 1);
  vm_wait<4>();
  raw_barrier();
  G8_STAMP(1);
  // Ping-pong the two wave groups (wm = 0 / 1; each SIMD holds one wave of each): group 1 runs one
  // barrier behind, so on every SIMD one wave issues its ds_reads + glds while the other one runs
  // its MFMA cluster (guide §5 template, "if(wr==1) s_barrier").  Staging stays correct: a half-tile
  // is restaged >= 1 phase after its last read and read >= 1 phase after the wait that retires it,
  // which holds for both groups with a one-barrier offset.
  if (wm == 1) raw_barrier();
  // N tail: when the tile's upper 128 columns lie wholly past N (N % 256 in (0, 128], e.g. Gemma-3's
  // d_model 640 -> 3rd column tile, or GPT-2's 50304-wide LM head), the (A*, B1) quadrants only
  // produce columns that are never stored: their B1 fragment reads and MFMAs are skipped (a
  // workgroup-uniform branch; staging and the counted waits are unchanged).  Not in the CE dgrad:
  // there the three column tiles of a row block stream the same 34 GB E operand in lockstep through
  // L2, and a faster third tile breaks that sharing (measured 21.9 -> 23.2 ms at Gemma-3's shape).
  const bool b1_ok = EPI == GEMM_EPI_CE_DGRAD || g.ntail_full || n0 + 128 < g.N;

  // a phase's first barrier: fragment-read wait before (default) or after (LATE) it
  auto pre_sync = [&]() {
    if constexpr (LATE) {
      raw_barrier();
      lds_sync();
    } else {
      lds_sync();
      raw_barrier();
    }
  };
  auto pre_sync_vm = [&]() {  // phases 4 / 8: + retire the other buffer's half-tiles
    if constexpr (LATE) {
      vm_wait<4>();
      raw_barrier();
      lds_sync();
    } else {
      lds_sync();
      vm_wait<4>();
      raw_barrier();
    }
  };

  for (int kt = 0; kt < nk; kt += 2) {
    const bool odd_ok = kt + 1 < nk;  // the odd K-tile of this iteration exists
    // ---- phases 1-4: even buffer, K-tile kt
    // phase 1: quadrant (A0, B0); stage O.A1 (kt+1)
    if constexpr (LATE) {
      read_b(0, 0);
      read_a(0, 0);
    } else {
      read_a(0, 0);
      read_b(0, 0);
    }
    const f32x4_t rq0 = ce_read(0, kt);
    stage(1, 1, kt + 1);
    pre_sync();
    mma_ce(0, rq0);
    raw_barrier();
    // phase 2: (A0, B1); stage O.B0 (kt+1)
    if (b1_ok) read_b(0, 1);
    const f32x4_t rq1 = ce_read(1, kt);
    stage(1, 2, kt + 1);
    pre_sync();
    if (b1_ok) mma_ce(1, rq1);
    raw_barrier();
    // phase 3: (A1, B1); stage E.A0 (kt+2)
    read_a(0, 1);
    const f32x4_t rq2 = ce_read(2, kt);
    stage(0, 0, kt + 2);
    pre_sync();
    if (b1_ok) mma_ce(2, rq2);
    raw_barrier();
    // phase 4: (A1, B0); stage E.B1 (kt+2); retire the odd buffer
    if constexpr (!KEEPB) read_b(0, 0);
    const f32x4_t rq3 = ce_read(3, kt);
    stage(0, 3, kt + 2);
    pre_sync_vm();
    mma_ce(3, rq3);
    raw_barrier();
    // ---- phases 5-8: odd buffer, K-tile kt+1 (MFMAs skipped past the end; loads/waits stay uniform)
    // phase 5: (A0, B0); stage E.A1 (kt+2)
    if constexpr (LATE) {
      read_b(1, 0);
      read_a(1, 0);
    } else {
      read_a(1, 0);
      read_b(1, 0);
    }
    ce_dma(kt);
    stage(0, 1, kt + 2);
    pre_sync();
    if (odd_ok) mma(0);
    raw_barrier();
    // phase 6: (A0, B1); stage E.B0 (kt+2)
    if (b1_ok) read_b(1, 1);
    stage(0, 2, kt + 2);
    pre_sync();
    if (odd_ok && b1_ok) mma(1);
    raw_barrier();
    // phase 7: (A1, B1); stage O.A0 (kt+3)
    read_a(1, 1);
    stage(1, 0, kt + 3);
    pre_sync();
    if (odd_ok && b1_ok) mma(2);
    raw_barrier();
    // phase 8: (A1, B0); stage O.B1 (kt+3); retire the even buffer
    if constexpr (!KEEPB) read_b(1, 0);
    stage(1, 3, kt + 3);
    pre_sync_vm();
    if (odd_ok) mma(3);
    raw_barrier();
  }
  if (wm == 0) raw_barrier();  // re-align the groups' barrier counts
  vm_wait<0>();  // drain the clamped tail prefetches (LDS-DMA must not outlive the workgroup)
  G8_STAMP(2);

  if constexpr (EPI == GEMM_EPI_CE_FWD) {
    if constexpr (LDSEPI) raw_barrier();  // every wave's tail LDS-DMA retired before the image overwrites LDS
    epilogue_ce_fwd<LDSEPI>(g, acc, m0, n0, wm, wn, lane, reinterpret_cast<float*>(smem));
  }
  else if constexpr (EPI == GEMM_EPI_CE_DGRAD) epilogue_ce_dgrad(g, acc, m0, n0, wm, wn, lane, split);
  else if constexpr (LDSEPI && (EPI == GEMM_EPI_NONE || EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU_D ||
                                 EPI == GEMM_EPI_DGELU || EPI == GEMM_EPI_MUL_AUX)) {
    raw_barrier();  // every wave's tail LDS-DMA retired (vm_wait<0> above) before the tile overwrites LDS
    epilogue_lds<EPI>(g, acc, m0, n0, wm, wn, lane, smem);
  } else epilogue8<EPI>(g, acc, m0, n0, wm, wn, lane, split);
  G8_STAMP(3);
}

// ------------------------------------------------------------------ 4-phase form (32-MFMA segments)
// The same tile, waves, LDS image and epilogues as gemm8_kernel, with HALF the barriers: a K-tile is
// TWO compute segments of 32 MFMAs -- quadrants (A0,B0)+(A0,B1) sharing the A0 fragments, then
// (A1,B1)+(A1,B0) reusing both B halves' fragments -- so an iteration (2 K-tiles) is 4 phases and 8
// barriers instead of 8 phases and 16.  Each barrier interval costs ~100 cycles beyond its MFMAs
// (profiles/r4_*): fewer, longer intervals.  Per phase 2 half-tiles are restaged, one phase after
// their last read (reads retire with lgkmcnt(0) BEFORE the phase's first barrier, so the 1-phase WAR
// distance is strict):
//   P1 (E, kt):   read E.B0 E.B1 E.A0   stage O.B1 O.A1 (kt+1)
//   P2 (E, kt):   read E.A1             stage E.A0 E.B0 (kt+2)   vmcnt(4): O (kt+1) retired
//   P3 (O, kt+1): read O.B0 O.B1 O.A0   stage E.B1 E.A1 (kt+2)
//   P4 (O, kt+1): read O.A1             stage O.A0 O.B0 (kt+3)   vmcnt(4): E (kt+2) retired
// A half-tile is read >= 1 phase after the (per-wave) wait + barrier that retires it, for both
// ping-pong groups (group 1 one barrier behind).
template <int EPI, bool AT, bool BT>
__global__ __launch_bounds__(512, 1) void gemm8p2_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int tiles_n = (g.N + 255) / 256;
  const int ntiles = ((g.M + 255) / 256) * tiles_n;
  const int ksplit = g.ksplit > 1 ? g.ksplit : 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntiles, split = bid / ntiles;
  const int m0 = (tile / tiles_n) * 256, n0 = (tile % tiles_n) * 256;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int nk_all = g.K / 64;
  const int kps = (nk_all + ksplit - 1) / ksplit;
  const int kbase = split * kps;
  const int nk = max(0, min(nk_all - kbase, kps));
  const int last = max(nk - 1, 0);

  auto half_ptr = [&](int buf, int h) { return smem + (buf * 4 + h) * kHalf; };
  auto stage = [&](int buf, int h, int kt) {
    const int k0 = min(kbase + min(kt, last), nk_all - 1) * 64;
    if (h < 2) {
      if constexpr (AT) stage_half_t(half_ptr(buf, h), g.A, g.lda, m0 + h * 128, g.M, k0);
      else stage_half(half_ptr(buf, h), g.A, g.lda, m0 + h * 128, g.M, k0);
    } else {
      if constexpr (BT) stage_half_t(half_ptr(buf, h), g.B, g.ldb, n0 + (h - 2) * 128, g.N, k0);
      else stage_half(half_ptr(buf, h), g.B, g.ldb, n0 + (h - 2) * 128, g.N, k0);
    }
  };

  f32x4_t acc[4][4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[q][i][j] = zero4();

  bf16x8_t af[4][2], bfr[2][2][2];  // A fragments of one A half; B fragments of both B halves
  auto read_a = [&](int buf, int ah) {
    const bf16_t* t = half_ptr(buf, ah);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (AT) af[i][ks] = frag8_t(t, wm * 64 + i * 16, ks * 4);
        else af[i][ks] = frag8(t, wm * 64 + i * 16, ks * 4);
      }
  };
  auto read_b = [&](int buf, int bh) {
    const bf16_t* t = half_ptr(buf, 2 + bh);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (BT) bfr[bh][j][ks] = frag8_t(t, wn * 32 + j * 16, ks * 4);
        else bfr[bh][j][ks] = frag8(t, wn * 32 + j * 16, ks * 4);
      }
  };
  // two quadrants sharing the A fragments: qa (with B half ba) and qb (with B half bb)
  auto mma2 = [&](int qa, int ba, int qb, int bb, bool do_b) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[qa][i][j] = mfma16(bfr[ba][j][ks], af[i][ks], acc[qa][i][j]);
          if (do_b) acc[qb][i][j] = mfma16(bfr[bb][j][ks], af[i][ks], acc[qb][i][j]);
        }
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_reads = [&]() {
    lgkm_wait0();
    if constexpr (AT || BT) __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: E <- K-tile 0 (all halves), O.A0 O.B0 <- K-tile 1; retire E
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 3, 0);
  stage(0, 1, 0);
  stage(1, 0, 1);
  stage(1, 2, 1);
  vm_wait<4>();
  raw_barrier();
  if (wm == 1) raw_barrier();  // ping-pong: group 1 one barrier behind
  const bool b1_ok = g.ntail_full || n0 + 128 < g.N;

  for (int kt = 0; kt < nk; kt += 2) {
    const bool odd_ok = kt + 1 < nk;
    // P1: (A0,B0) + (A0,B1) of K-tile kt
    read_b(0, 0);
    if (b1_ok) read_b(0, 1);
    read_a(0, 0);
    stage(1, 3, kt + 1);
    stage(1, 1, kt + 1);
    sync_reads();
    raw_barrier();
    mma2(0, 0, 1, 1, b1_ok);
    raw_barrier();
    // P2: (A1,B1) + (A1,B0)
    read_a(0, 1);
    stage(0, 0, kt + 2);
    stage(0, 2, kt + 2);
    sync_reads();
    vm_wait<4>();
    raw_barrier();
    mma2(3, 0, 2, 1, b1_ok);
    raw_barrier();
    // P3: odd buffer, K-tile kt+1 (MFMAs skipped past the end; loads / waits stay uniform)
    read_b(1, 0);
    if (b1_ok) read_b(1, 1);
    read_a(1, 0);
    stage(0, 3, kt + 2);
    stage(0, 1, kt + 2);
    sync_reads();
    raw_barrier();
    if (odd_ok) mma2(0, 0, 1, 1, b1_ok);
    raw_barrier();
    // P4
    read_a(1, 1);
    stage(1, 0, kt + 3);
    stage(1, 2, kt + 3);
    sync_reads();
    vm_wait<4>();
    raw_barrier();
    if (odd_ok) mma2(3, 0, 2, 1, b1_ok);
    raw_barrier();
  }
  if (wm == 0) raw_barrier();
  vm_wait<0>();
  epilogue8<EPI>(g, acc, m0, n0, wm, wn, lane, split);
}

// ------------------------------------------------------------------ persistent streaming form
// One quadrant of the deferred epilogue (NONE / BIAS / BIAS_GELU_D): acc[q] of the finished tile
// (rows m0 + qa*128 + wm*64 + 16 i, columns n0 + qb*128 + wn*32 ..) -> 4 (GELU_D: 8) 16-B stores per
// lane, then acc[q] = 0 for the next tile.  bias_q: the lane's 8 bias values of that column half,
// loaded when the tile started (no load -- hence no vmcnt wait -- inside the pipeline).
template <int EPI>
__device__ __forceinline__ void epi_quad8(const GemmArgs& g, f32x4_t (&aq)[4][2], int q, int m0, int n0, int wm,
                                          int wn, int lane, const u16x8_t& bias_q) {
  const int g4 = lane >> 4;
  const int cofs = (g4 & 1) * 16 + (g4 >> 1) * 8;
  const int qa = (q == 2 || q == 3) ? 1 : 0, qb = (q == 1 || q == 2) ? 1 : 0;
  const int col = n0 + qb * 128 + wn * 32 + cofs;
  const bool col_ok = col < g.N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(aq[i][0][r]), __float_as_uint(aq[i][1][r]),
                                                       false, false);
      v[r] = __uint_as_float(sw[0]);
      v[4 + r] = __uint_as_float(sw[1]);
    }
    const int row = m0 + qa * 128 + wm * 64 + i * 16 + (lane & 15);
    const bool ok = col_ok && row < g.M;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] *= g.alpha;
      if constexpr (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU_D) v[e] += bf2f(bias_q[e]);
    }
    if constexpr (EPI == GEMM_EPI_BIAS_GELU_D) {
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) gelu_tanh_and_grad(v[e], v[e], d[e]);
      if (ok) store8(g.aux + (long)row * g.ldaux + col, d);
    }
    if (ok) store8(reinterpret_cast<bf16_t*>(g.C) + (long)row * g.ldc + col, v);
    aq[i][0] = zero4();
    aq[i][1] = zero4();
  }
}

// Persistent streaming form (ksplit == 1; epilogues NONE / BIAS / BIAS_GELU_D): one workgroup per
// CU walks its tiles (logical ids b, b + grid, ..., XCD-remapped) as ONE continuous stream of
// K-tiles, so the 8-phase pipeline never restarts -- the prefetches issued near the end of a tile
// already fetch the next tile's first K-tiles (no prologue fill, no workgroup relaunch).
// The finished tile's epilogue is DEFERRED by one quadrant-phase each: during the 4 phases after a
// tile's last K-tile, the phase that is about to accumulate quadrant q of the NEW tile first
// converts and stores quadrant q of the OLD one (and zeroes it), after that phase's staging loads.
// So the 128 KB of stores leave in four 32 KB pieces interleaved with MFMA work instead of one
// issue-bound burst, and -- vmcnt being in order -- the stores are always YOUNGER than the loads
// the next counted wait needs except for the first quadrant's: that wait allows the 3 later
// quadrants' stores in flight (vm_wait<4 + 3 S>, S stores per lane per quadrant).
template <int EPI, bool AT, bool BT>
__global__ __launch_bounds__(512, 1) void gemm8s_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  constexpr int S = EPI == GEMM_EPI_BIAS_GELU_D ? 8 : 4;  // stores per lane per quadrant
  constexpr bool kBias = EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU_D;
  const int tiles_n = (g.N + 255) / 256;
  const int ntiles = ((g.M + 255) / 256) * tiles_n;
  const int b = blockIdx.x, grid = gridDim.x;
  const int n_my = (ntiles - b + grid - 1) / grid;
  const int nk = g.K / 64;
  const int NG = n_my * nk;  // K-tiles this workgroup streams
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int g4 = lane >> 4;
  const int cofs = (g4 & 1) * 16 + (g4 >> 1) * 8;

  // position in the stream: K-tile Gk = (tile number i of this workgroup, k-tile kk of it); the
  // iterator advances with scalar adds, dividing only when it crosses into the next tile; past the
  // end it stays on the last K-tile (uniform re-reads keep the counted waits exact)
  struct It {
    int Gk, i, kk, m0, n0;
  };
  auto tile_origin = [&](It& t) {
    const int tile = xcd_remap(b + t.i * grid, ntiles);
    t.m0 = (tile / tiles_n) * 256;
    t.n0 = (tile % tiles_n) * 256;
  };
  auto adv = [&](It t) {
    if (t.Gk + 1 < NG) {
      ++t.Gk;
      if (++t.kk == nk) {
        t.kk = 0;
        ++t.i;
        tile_origin(t);
      }
    }
    return t;
  };
  uint32_t offA[2], offB[2];
  stage_offsets(g.lda, offA);
  stage_offsets(g.ldb, offB);
  auto half_ptr = [&](int buf, int h) { return smem + (buf * 4 + h) * kHalf; };
  auto stage_at = [&](int buf, int h, const It& t) {
    const int k0 = t.kk * 64;
    if (h < 2) stage_half_fast(half_ptr(buf, h), g.A, g.lda, t.m0 + h * 128, g.M, k0, offA);
    else stage_half_fast(half_ptr(buf, h), g.B, g.ldb, t.n0 + (h - 2) * 128, g.N, k0, offB);
  };

  f32x4_t acc[4][4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[q][i][j] = zero4();

  bf16x8_t af[4][2], bfr[2][2];
  auto read_a = [&](int buf, int ah) {
    const bf16_t* t = half_ptr(buf, ah);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (AT) af[i][ks] = frag8_t(t, wm * 64 + i * 16, ks * 4);
        else af[i][ks] = frag8(t, wm * 64 + i * 16, ks * 4);
      }
  };
  auto read_b = [&](int buf, int bh) {
    const bf16_t* t = half_ptr(buf, 2 + bh);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (BT) bfr[j][ks] = frag8_t(t, wn * 32 + j * 16, ks * 4);
        else bfr[j][ks] = frag8(t, wn * 32 + j * 16, ks * 4);
      }
  };
  auto mma = [&](int q) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[q][i][j] = mfma16(bfr[j][ks], af[i][ks], acc[q][i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto lds_sync = [&]() {
    lgkm_wait0();
    if constexpr (AT || BT) __builtin_amdgcn_sched_barrier(0);
  };

  // the deferred tile: its origin, its bias (the lane's 8 columns of each column half)
  int pm0 = 0, pn0 = 0;
  bool pend = false;
  u16x8_t bias_c[2] = {}, bias_p[2] = {};  // current tile's, pending tile's
  auto load_bias = [&](int n0) {
    if constexpr (kBias) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
        bias_c[h] = *reinterpret_cast<const u16x8_t*>(g.bias + min(n0 + h * 128 + wn * 32 + cofs, g.N - 8));
    }
  };
  // after the last quadrant of K-tile t: a finished tile becomes the pending one
  auto finish = [&](const It& t) {
    if (t.kk == nk - 1) {
      pm0 = t.m0, pn0 = t.n0, pend = true;
      bias_p[0] = bias_c[0], bias_p[1] = bias_c[1];
      if (t.Gk + 1 < NG) load_bias(adv(t).n0);
    }
  };
  auto epi = [&](int q) {
    if (pend) epi_quad8<EPI>(g, acc[q], q, pm0, pn0, wm, wn, lane, bias_p[(q == 1 || q == 2) ? 1 : 0]);
  };

  It t0{0, 0, 0, 0, 0};
  tile_origin(t0);
  It t1 = adv(t0);  // stream position of the odd buffer's K-tile
  {  // prologue: E <- K-tile 0 (all halves), O <- K-tile 1 (A0, B1); retire E
    load_bias(t0.n0);
    stage_at(0, 0, t0);
    stage_at(0, 3, t0);
    stage_at(0, 1, t0);
    stage_at(0, 2, t0);
    stage_at(1, 0, t1);
    stage_at(1, 3, t1);
  }
  vm_wait<4>();
  raw_barrier();
  if (wm == 1) raw_barrier();

  for (int G = 0; G < NG; G += 2) {
    const bool odd_ok = G + 1 < NG;
    // staging targets: K-tiles G+1 (= t1), G+2, G+3; t0 = K-tile G
    const It t2 = adv(t1), t3 = adv(t2);
    // ---- phases 1-4: even buffer, K-tile G (the pending tile's quadrants leave in order)
    const bool ep0 = pend;
    read_a(0, 0);
    read_b(0, 0);
    stage_at(1, 1, t1);
    epi(0);
    lds_sync();
    raw_barrier();
    mma(0);
    raw_barrier();
    read_b(0, 1);
    stage_at(1, 2, t1);
    epi(1);
    lds_sync();
    raw_barrier();
    mma(1);
    raw_barrier();
    read_a(0, 1);
    stage_at(0, 0, t2);
    epi(2);
    lds_sync();
    raw_barrier();
    mma(2);
    raw_barrier();
    read_b(0, 0);
    stage_at(0, 3, t2);
    epi(3);
    pend = false;
    lds_sync();
    if (ep0) vm_wait<4 + 3 * S>();  // the 3 later quadrants' stores may stay in flight
    else vm_wait<4>();
    raw_barrier();
    mma(3);
    finish(t0);
    raw_barrier();
    // ---- phases 5-8: odd buffer, K-tile G+1
    const bool ep1 = pend;
    read_a(1, 0);
    read_b(1, 0);
    stage_at(0, 1, t2);
    epi(0);
    lds_sync();
    raw_barrier();
    if (odd_ok) mma(0);
    raw_barrier();
    read_b(1, 1);
    stage_at(0, 2, t2);
    epi(1);
    lds_sync();
    raw_barrier();
    if (odd_ok) mma(1);
    raw_barrier();
    read_a(1, 1);
    stage_at(1, 0, t3);
    epi(2);
    lds_sync();
    raw_barrier();
    if (odd_ok) mma(2);
    raw_barrier();
    read_b(1, 0);
    stage_at(1, 3, t3);
    epi(3);
    pend = false;
    lds_sync();
    if (ep1) vm_wait<4 + 3 * S>();
    else vm_wait<4>();
    raw_barrier();
    if (odd_ok) {
      mma(3);
      finish(t1);
    }
    raw_barrier();
    t0 = t2;
    t1 = t3;
  }
  if (wm == 0) raw_barrier();
  vm_wait<0>();
  if (pend) {  // the last tile
#pragma unroll
    for (int q = 0; q < 4; ++q) epi_quad8<EPI>(g, acc[q], q, pm0, pn0, wm, wn, lane, bias_p[(q == 1 || q == 2) ? 1 : 0]);
  }
}

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    MFT_HIP_CHECK(hipGetDevice(&dev));
    MFT_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    if (n <= 0) n = 256;
  }
  return n;
}

// MFT_GEMM8_STREAM=1: the persistent streaming kernel with the deferred epilogue for NT NONE / BIAS /
// BIAS_GELU_D whenever every CU gets >= 2 tiles.  Off by default: measured within +-5 % of one tile
// per workgroup at K = 704-832 and 9-18 % slower at K = 2112-3072 and with the GELU epilogue
// (profiles/r3_gemm_stream_ab.txt) -- the per-tile cost at short K is not the prologue fill, the
// relaunch or the store burst, which this form removes.
static int g_stream = -1;
static bool gemm8_stream() {
  if (g_stream < 0) {
    const char* e = getenv("MFT_GEMM8_STREAM");
    g_stream = (e && e[0] >= '1' && e[0] <= '5') ? e[0] - '0' : 0;
  }
  return g_stream == 1;
}
// 0 default, 1 streaming form, 2 early-wait phase order, 3 LATE without B0 reuse (NT A/Bs)
void gemm8_set_stream(int on) { g_stream = on; }
static bool gemm8_early() {
  gemm8_stream();
  return g_stream == 2;
}
static bool gemm8_nokeepb() {
  gemm8_stream();
  return g_stream == 3;
}
static bool gemm8_p2() {  // 4 (MFT_GEMM8_STREAM=4): the 4-phase form (32-MFMA segments)
  gemm8_stream();
  return g_stream == 4;
}
static bool gemm8_ldsepi() {  // 5: LDS-staged whole-row epilogue stores (NONE / BIAS)
  gemm8_stream();
  return g_stream == 5;
}
static int g_stagger = -1;
void gemm8_set_stagger(int cycles) { g_stagger = cycles; }
static int gemm8_stagger() {
  if (g_stagger < 0) {
    const char* e = getenv("MFT_G8_STAGGER");
    g_stagger = e ? atoi(e) : 0;
  }
  return g_stagger;
}

template <int EPI, bool AT, bool BT>
static void launch8(const GemmArgs& g, hipStream_t st) {
  // 128 KB of half-tile buffers (+ 2 KB of row-factor slots for the CE dgrad)
  constexpr size_t shm = sizeof(bf16_t) * 8 * kHalf + (EPI == GEMM_EPI_CE_DGRAD ? 2048 : 0);
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm8_kernel<EPI, AT, BT>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    attr = true;
  }
  const int tiles = ((g.M + 255) / 256) * ((g.N + 255) / 256);
  const int ks = g.ksplit > 1 ? g.ksplit : 1;
  // streaming form: epilogues without per-element operand loads (NONE / BIAS / BIAS_GELU_D)
  if constexpr (!AT && !BT && (EPI == GEMM_EPI_NONE || EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU_D)) {
    if (ks == 1 && gemm8_stream() && tiles >= 2 * num_cus()) {
      static bool attr_s = false;
      if (!attr_s) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm8s_kernel<EPI, AT, BT>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        attr_s = true;
      }
      gemm8s_kernel<EPI, AT, BT><<<num_cus(), 512, shm, st>>>(g);
      return;
    }
  }
  if constexpr (EPI != GEMM_EPI_CE_FWD && EPI != GEMM_EPI_CE_DGRAD) {
    if (gemm8_p2()) {
      static bool attr_p = false;
      if (!attr_p) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm8p2_kernel<EPI, AT, BT>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        attr_p = true;
      }
      gemm8p2_kernel<EPI, AT, BT><<<tiles * ks, 512, shm, st>>>(g);
      return;
    }
  }
  if constexpr (!AT && (EPI == GEMM_EPI_NONE || EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU_D ||
                        EPI == GEMM_EPI_DGELU || EPI == GEMM_EPI_MUL_AUX || EPI == GEMM_EPI_CE_FWD)) {
    if (gemm8_ldsepi()) {
      constexpr size_t shm_e = EPI == GEMM_EPI_CE_FWD ? shm + 8192 : shm;  // + the CE reduction scratch
      static bool attr_e = false;
      if (!attr_e) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm8_kernel<EPI, AT, BT, true, true, true>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm_e));
        attr_e = true;
      }
      gemm8_kernel<EPI, AT, BT, true, true, true><<<tiles * ks, 512, shm_e, st>>>(g);
      return;
    }
  }
  if constexpr (!AT && !BT && EPI == GEMM_EPI_NONE) {
    if (gemm8_early()) {
      static bool attr_l = false;
      if (!attr_l) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm8_kernel<EPI, AT, BT, false, false>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        attr_l = true;
      }
      gemm8_kernel<EPI, AT, BT, false, false><<<tiles * ks, 512, shm, st>>>(g);
      return;
    }
    if (gemm8_nokeepb()) {
      static bool attr_k = false;
      if (!attr_k) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm8_kernel<EPI, AT, BT, true, false>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        attr_k = true;
      }
      gemm8_kernel<EPI, AT, BT, true, false><<<tiles * ks, 512, shm, st>>>(g);
      return;
    }
  }
  gemm8_kernel<EPI, AT, BT><<<tiles * ks, 512, shm, st>>>(g);
}

template <int EPI>
static void launch8_layout(const GemmArgs& g, bool a_t, bool b_t, hipStream_t st) {
  if (a_t && b_t) launch8<EPI, true, true>(g, st);
  else if (b_t) launch8<EPI, false, true>(g, st);
  else if (a_t) launch8<EPI, true, false>(g, st);
  else launch8<EPI, false, false>(g, st);
}

// C (+)= alpha * sum_s ws[s]   (fp32, [M, N] slabs; deterministic split order)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int ksplit, long MN, int N,
                                                            float* __restrict__ C, long ldc, float alpha, int accumulate) {
  const long i4 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 * 4 >= MN) return;
  const long i = i4 * 4;
  f32x4_t s = *reinterpret_cast<const f32x4_t*>(ws + i);
  for (int k = 1; k < ksplit; ++k) s += *reinterpret_cast<const f32x4_t*>(ws + (long)k * MN + i);
  const long row = i / N, col = i % N;
  float* c = C + row * ldc + col;
  f32x4_t o = s * alpha;
  if (accumulate) o += *reinterpret_cast<f32x4_t*>(c);
  *reinterpret_cast<f32x4_t*>(c) = o;
}

void gemm_splitk_reduce(const float* ws, int ksplit, int M, int N, float* C, long ldc, float alpha, int accumulate,
                        hipStream_t st) {
  const long MN = (long)M * N;
  splitk_reduce_kernel<<<(int)((MN / 4 + 255) / 256), 256, 0, st>>>(ws, ksplit, MN, N, C, ldc, alpha, accumulate);
}

int gemm8_pick_ksplit(int M, int N, int K) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int nk = K / 64;
  const int cus = num_cus();
  // split the K (token) dimension so tiles * ks fills the CUs in as few, as full waves as possible,
  // each split keeping >= 16 K-tiles (the 8-phase prologue/epilogue amortised); near-ties -> fewer splits
  int best = 1;
  double best_eff = 0.0;
  for (int ks = 1; ks <= 32 && nk / ks >= 16; ++ks) {
    const int wgs = tiles * ks;
    const int waves = (wgs + cus - 1) / cus;
    // a wave of workgroups costs ~ nk / ks K-tiles; minimise total time ~ waves * nk / ks
    const double t = (double)waves * ((nk + ks - 1) / ks);
    const double eff = 1.0 / t;
    if (eff > best_eff * 1.05) {  // more splits cost fp32 slab traffic: only for a clear win
      best_eff = eff;
      best = ks;
    }
  }
  return best;
}

bool gemm8_supported(int M, int N, int K, bool a_t, bool b_t) {
  if (K % 64 || K <= 0 || M <= 0 || N < 8 || N % 8) return false;
  if (a_t && (M % 8 || M < 8)) return false;
  return true;
}

// MFT_GEMM8_NTAIL=0 turns the N-tail quadrant skip off (A/B runs)
static int gemm8_ntail_full() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MFT_GEMM8_NTAIL");
    v = (e && e[0] == '0') ? 1 : 0;
  }
  return v;
}

void gemm8x(const GemmArgs& g0, int epi, bool a_t, bool b_t, hipStream_t st) {
  GemmArgs g = g0;
  g.ntail_full = gemm8_ntail_full();
  g.stagger = gemm8_stagger();
  // per-lane staging offsets are 32-bit byte offsets from a uniform base (128 rows x ld x 2 B)
  if (!gemm8_supported(g.M, g.N, g.K, a_t, b_t) || g.lda > (1L << 23) || g.ldb > (1L << 23)) {
    fprintf(stderr, "mft::gemm8: unsupported shape M=%d N=%d K=%d (a_t=%d b_t=%d)\n", g.M, g.N, g.K, a_t, b_t);
    abort();
  }
  switch (epi) {
    case GEMM_EPI_NONE: launch8_layout<GEMM_EPI_NONE>(g, a_t, b_t, st); break;
    case GEMM_EPI_BIAS: launch8_layout<GEMM_EPI_BIAS>(g, a_t, b_t, st); break;
    case GEMM_EPI_BIAS_GELU: launch8_layout<GEMM_EPI_BIAS_GELU>(g, a_t, b_t, st); break;
    case GEMM_EPI_DGELU: launch8_layout<GEMM_EPI_DGELU>(g, a_t, b_t, st); break;
    case GEMM_EPI_BIAS_GELU_D: launch8_layout<GEMM_EPI_BIAS_GELU_D>(g, a_t, b_t, st); break;
    case GEMM_EPI_MUL_AUX: launch8_layout<GEMM_EPI_MUL_AUX>(g, a_t, b_t, st); break;
    case GEMM_EPI_BIAS_ADD:
      if (!g.bias || !g.aux) {
        fprintf(stderr, "mft::gemm8: BIAS_ADD needs the bias and the residual (aux)\n");
        abort();
      }
      launch8_layout<GEMM_EPI_BIAS_ADD>(g, a_t, b_t, st);
      break;
    case GEMM_EPI_F32ACC:
      // fp32 weight-gradient accumulate: split over K into slabs (g.ws, ksplit * M * N floats) when
      // the output has few tiles, then one deterministic reduce into C; else accumulate in place
      if (g.ksplit > 1) {
        if (!g.ws) {
          fprintf(stderr, "mft::gemm8: split-K needs a workspace\n");
          abort();
        }
        launch8_layout<GEMM_EPI_F32PART>(g, a_t, b_t, st);
        gemm_splitk_reduce(g.ws, g.ksplit, g.M, g.N, reinterpret_cast<float*>(g.C), g.ldc, g.alpha, 1, st);
      } else {
        launch8_layout<GEMM_EPI_F32ACC>(g, a_t, b_t, st);
      }
      break;
    case GEMM_EPI_LORA:
      if (g.lora_r <= 0 || g.lora_r > 32 || g.lora_r % 8 || g.ld_lu % 8) {
        fprintf(stderr, "mft::gemm8: LoRA epilogue needs rank %% 8 == 0, <= 32 (got %d)\n", g.lora_r);
        abort();
      }
      launch8_layout<GEMM_EPI_LORA>(g, a_t, b_t, st);
      break;
    case GEMM_EPI_CE_FWD:  // NT only (logits = h W^T)
      if (a_t || b_t || g.ksplit > 1 || !g.ce_labels || !g.ce_stats || !g.ce_lbl || g.ce_V <= 0 || g.ce_V > g.N) {
        fprintf(stderr, "mft::gemm8: CE forward epilogue needs the NT layout, labels/stats/lbl, 0 < V <= N\n");
        abort();
      }
      launch8<GEMM_EPI_CE_FWD, false, false>(g, st);
      break;
    case GEMM_EPI_CE_DGRAD:  // NN only (dh = dlogits W, W stored [V, N])
      if (a_t || !b_t || !g.ce_labels || !g.ce_ratio || !g.ce_fin || !g.ce_wlab ||
          (g.ksplit > 1 && (!g.ws || ((g.K / 64 + g.ksplit - 1) / g.ksplit) % 4 != 0))) {
        fprintf(stderr, "mft::gemm8: CE dgrad needs the NN layout, ratio/fin/wlab/labels, and for a vocab split a "
                        "slab workspace and whole vocab tiles per split\n");
        abort();
      }
      launch8<GEMM_EPI_CE_DGRAD, false, true>(g, st);
      break;
    default: fprintf(stderr, "mft::gemm8: bad epilogue %d\n", epi); abort();
  }
}

void gemm8(const GemmArgs& g, int epi, hipStream_t st) { gemm8x(g, epi, false, false, st); }

}  // namespace mft
