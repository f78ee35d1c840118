// gemm_s: the short-token GEMM (NT, C = epi(alpha A B^T [+ A2 B2^T])) for products whose 256 x 256 tile
// count cannot fill the chip -- the reference's own recipe, 4 x 128 tokens per micro-batch
// (reference README.md:133-141), where gemm4 launches 6 workgroups for a 512 x 768 output and every
// product is one long serial K-loop (47 us for 0.6 GFLOP, profiles/r5_kernel_tables.txt).
//
// Design for latency, not throughput:
//   * 64 x 64 output tile per 256-thread workgroup, and the K-loop SPLIT ACROSS THE 4 WAVES: wave w
//     takes K-tiles w, w + 4, ... (each a full 64 x 64 x 64 product, 4 x 4 blocks of
//     v_mfma_f32_16x16x32_bf16), so a K = 768 product is 3 dependent K-tiles per wave, not 12;
//   * operands straight from global memory into MFMA fragments (one 16-B load per lane per fragment:
//     both NT operands are K-contiguous), the next K-tile's 16 fragments in flight while the current
//     one multiplies -- no LDS staging, no barriers in the loop;
//   * the 4 partial tiles meet once in LDS (fp32, padded rows), each wave reduces 16 rows and runs the
//     fused epilogue on 16 contiguous columns per lane (16-B loads / stores).
// The MFMAs run with the operands swapped (C^T = B A^T) so each lane's accumulators are 4 contiguous
// columns of one row.
// Split-K across workgroups (S > 1, long K with few tiles, e.g. 512 x 768 x 3072): the S workgroups of a
// tile take interleaved K-tile shares, write their reduced fp32 partial tile to a workspace and count in on
// a per-tile counter; the last to arrive sums the S partials in split order (deterministic) and runs the
// epilogue, then re-arms the counter.  Partials and counter are agent-scope relaxed atomics (sc1 stores /
// loads through to the coherence point; the writers wait for their stores before counting in), and the S
// workgroups of a tile sit on one XCD (block ids congruent mod 8).
#include "common.h"
#include "kernels.h"
#include "mfma.h"

#include <algorithm>
#include <mutex>
#include <unordered_map>

namespace mft {

namespace {

constexpr int kLdr = 68;  // fp32 row pitch of the reduction image (64 + 4: float4 writes spread over banks)
constexpr int kMaxSplit = 4;  // K-splits across workgroups (gemm_s split-K)
constexpr int kNW = 4;    // waves per workgroup, each a 1/kNW share of the K-tiles (8 measured slower: 139 KB LDS, one WG per CU)


template <int TM>  // output rows per tile: 64 (4 row blocks) or 32 (2)
struct Frags {
  bf16x8_t a[2][TM / 16], b[2][4];  // [k-step][block]
};

// fragments of one K-tile (64 columns) through range-checked buffer descriptors: A rows m0 + 16 i + (l & 15),
// B rows n0 + 16 j + (l & 15), columns k0 + 32 ks + 8 (l >> 4) .. + 7.  Rows past M / N, and a whole K-tile
// moved out of range by its scalar offset (a wave's tiles past its last), read as zeros -- no branch and
// no clamp around any load, so the compiler keeps the next K-tile's loads in flight under the MFMAs.
typedef int i32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <int TM>
__device__ __forceinline__ void load_frags(Frags<TM>& f, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb,
                                           const uint32_t (&oa)[4], const uint32_t (&ob)[4], uint32_t soff) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
    for (int i = 0; i < TM / 16; ++i)
      f.a[ks][i] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(ra, oa[i] + 64 * ks, soff, 0));
#pragma unroll
    for (int j = 0; j < 4; ++j)
      f.b[ks][j] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(rb, ob[j] + 64 * ks, soff, 0));
  }
}

// Builtin MFMAs (not asm): the compiler must see them to place the wait states between an MFMA still reading
// its source VGPRs and the next write of those registers (with two waves per SIMD part of the fragments live
// in AGPRs and are copied to VGPRs right before their MFMA -- an asm MFMA there read clobbered operands).
template <int TM>
__device__ __forceinline__ void mma(f32x4_t (&acc)[TM / 16][4], const Frags<TM>& f) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < TM / 16; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(f.b[ks][j], f.a[ks][i], acc[i][j]);
}

// TM = 32 (short products with few 64-row tiles): twice the workgroups, and a 3-deep fragment ring -- the
// 3 K-tiles of a K = 768 wave all in flight before its first MFMA (one memory latency, not two)
template <int EPI, bool SEG2, int TM>
__global__ __launch_bounds__(64 * kNW) void gemm_s_kernel(GemmArgs g, int S, float* __restrict__ ws, int* __restrict__ cnt) {
  constexpr int RB = TM / 16;                // row blocks per tile
  constexpr int kDepth = TM == 32 ? 3 : 2;   // K-tiles in flight per wave
  extern __shared__ __attribute__((aligned(16))) float red[];  // [kNW waves][TM rows][kLdr]
  __shared__ int last;
  const int tiles_n = (g.N + 63) / 64, tiles = ((g.M + TM - 1) / TM) * tiles_n;
  // block -> (tile t, split s): the S splits of a tile on one XCD (block ids congruent mod 8)
  const int bx = blockIdx.x & 7, bq = blockIdx.x >> 3, sp = bq % S, t = (bq / S) * 8 + bx;
  if (t >= tiles) return;
  const int m0 = (t / tiles_n) * TM, n0 = (t % tiles_n) * 64;
  const int w = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;  // (uniform: scalar loop)
  const int nk = g.K / 64, nkt = nk + (SEG2 ? g.K2 / 64 : 0);
  const int slot = sp * kNW + w, P = S * kNW;  // this wave's K-tiles: slot, slot + P, ...
  f32x4_t acc[RB][4];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero4();
  // the wave's it-th K-tile is slot + P it; past its last one the loads are out of range (zeros: a multiply
  // that adds nothing), so the MFMA chain is unconditional and the accumulators stay in place
  const int n_my = slot < nkt ? (nkt - slot + P - 1) / P : 0;
  // operand panels of this tile: base + byte count (rows past M / N: VGPR offsets beyond the records -> 0)
  auto recs = [](long bytes) { return (int)__builtin_amdgcn_readfirstlane((uint32_t)min(bytes, 0x7fff0000L)); };
  const bf16_t* pa1 = g.A + (long)m0 * g.lda;
  const bf16_t* pb1 = g.B + (long)n0 * g.ldb;
  const int na1 = recs((long)(g.M - m0) * g.lda * 2), nb1 = recs((long)(g.N - n0) * g.ldb * 2);
  const bf16_t* pa2 = pa1;
  const bf16_t* pb2 = pb1;
  int na2 = 0, nb2 = 0;
  if constexpr (SEG2) {
    pa2 = g.A2 + (long)m0 * g.lda2, pb2 = g.B2 + (long)n0 * g.ldb2;
    na2 = recs((long)(g.M - m0) * g.lda2 * 2), nb2 = recs((long)(g.N - n0) * g.ldb2 * 2);
  }
  uint32_t oa1[4], ob1[4], oa2[4], ob2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 16 * i + (l & 15), c = 8 * (l >> 4);
    oa1[i] = (uint32_t)((r * g.lda + c) * 2), ob1[i] = (uint32_t)((r * g.ldb + c) * 2);
    if constexpr (SEG2) oa2[i] = (uint32_t)((r * g.lda2 + c) * 2), ob2[i] = (uint32_t)((r * g.ldb2 + c) * 2);
  }
  // (the SGPR offset is not range-checked -- only the VGPR offset is -- so a K-tile past the wave's last
  // reads through a 0-record descriptor, not through a large soffset; scalar selects of base and count,
  // the descriptor built per load: a select between descriptor values went through scratch)
  auto load = [&](Frags<TM>& f, int it) {  // (selects only: a branch here would make the compiler wait early)
    const int kt = slot + P * it;
    const bool ok = it < n_my && !g.stagger, s2 = SEG2 && kt >= nk;
    const uint32_t off = (uint32_t)(s2 ? kt - nk : min(kt, nk - 1)) * 128u;
    const bf16_t* pa = s2 ? pa2 : pa1;
    const bf16_t* pb = s2 ? pb2 : pb1;
    const int na = !ok ? 0 : s2 ? na2 : na1, nb = !ok ? 0 : s2 ? nb2 : nb1;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(pa), (short)0, na, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(pb), (short)0, nb, 0x00020000);
    if constexpr (SEG2) {
      uint32_t oa[4], ob[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) oa[i] = s2 ? oa2[i] : oa1[i], ob[i] = s2 ? ob2[i] : ob1[i];
      load_frags(f, ra, rb, oa, ob, off);
    } else {
      load_frags(f, ra, rb, oa1, ob1, off);
    }
  };
  // (sched_barrier: the scheduler would otherwise sink each load next to its first use -- load, wait, MFMA;
  // a third K-tile in flight measured no faster and spilled: the product is bound by the MFMA time of
  // the ~100 busy CUs and the launch / reduction floor, not by the load chain)
  if constexpr (kDepth == 2) {
    Frags<TM> f0, f1;
    load(f0, 0);
    for (int it = 0; it < max(n_my, 1); it += 2) {  // (a wave without K-tiles multiplies zeros once: acc = 0)
      load(f1, it + 1);
      __builtin_amdgcn_sched_barrier(0);
      mma<TM>(acc, f0);
      __builtin_amdgcn_sched_barrier(0);
      load(f0, it + 2);
      __builtin_amdgcn_sched_barrier(0);
      mma<TM>(acc, f1);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    Frags<TM> f0, f1, f2;
    load(f0, 0);
    load(f1, 1);
    for (int it = 0; it < max(n_my, 1); it += 3) {
      load(f2, it + 2);
      __builtin_amdgcn_sched_barrier(0);
      mma<TM>(acc, f0);
      __builtin_amdgcn_sched_barrier(0);
      load(f0, it + 3);
      __builtin_amdgcn_sched_barrier(0);
      mma<TM>(acc, f1);
      __builtin_amdgcn_sched_barrier(0);
      load(f1, it + 4);
      __builtin_amdgcn_sched_barrier(0);
      mma<TM>(acc, f2);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // partial tile of this wave -> LDS: lane holds row 16 i + (l & 15), columns 16 j + 4 (l >> 4) .. + 3
  float* mine = red + w * TM * kLdr;
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<f32x4_t*>(mine + (16 * i + (l & 15)) * kLdr + 16 * j + 4 * (l >> 4)) = acc[i][j];
  __syncthreads();
  // wave w reduces rows kRows w .. + kRows - 1: lane -> one row, kCols contiguous columns
  constexpr int kRows = TM / kNW, kLpr = 64 / kRows, kCols = 64 / kLpr;
  const int rt = kRows * w + l / kLpr, ct = kCols * (l % kLpr);
  const int row = m0 + rt;
  float v[kCols];
#pragma unroll
  for (int q = 0; q < kCols / 4; ++q) {
    f32x4_t s = *reinterpret_cast<const f32x4_t*>(red + rt * kLdr + ct + 4 * q);
#pragma unroll
    for (int p = 1; p < kNW; ++p) {
      const f32x4_t t = *reinterpret_cast<const f32x4_t*>(red + (p * TM + rt) * kLdr + ct + 4 * q);
      s[0] += t[0], s[1] += t[1], s[2] += t[2], s[3] += t[3];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * q + e] = s[e];
  }
  if (S > 1) {  // split-K: partial out, count in; the last workgroup of the tile sums the S partials
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(ws, (short)0, 0x7fffffff, 0x00020000);
    const uint32_t o0 = (uint32_t)(((long)t * S * (TM * 64) + rt * 64 + ct) * 4);
#pragma unroll
    for (int q = 0; q < kCols / 4; ++q)  // (aux 16 = sc1: through to the agent coherence point)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, f32x4_t{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]}),
                                             rw, o0 + (uint32_t)sp * (TM * 256u) + 16u * q, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this lane's partial is at the coherence point
    __syncthreads();
    // The hand-off: every partial stored sc1 and drained (vmcnt(0)) by every wave before the barrier, ONE
    // lane's agent-scope add, the last arriver told by the returned value, then sc1 loads only behind a
    // workgroup barrier -- the measured-valid form of the MI355X guide's Valid-forms table (row 1), which
    // is not an architectural guarantee of the memory model.  handoff_fence adds the agent release before
    // the add and the acquire after it (~1.7 us each on the critical path of a ~16 us call).
    if (threadIdx.x == 0) {
      if (g.handoff_fence) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-back done before the add
      }
      last = __hip_atomic_fetch_add(cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
      if (last && g.handoff_fence) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate done before the barrier
      }
    }
    __syncthreads();
    if (!last) return;
    // every split's loads issued before the first add (S <= kMaxSplit; splits past S re-read the last one,
    // weighted 0), in split order
    f32x4_t pv[kMaxSplit][kCols / 4];
#pragma unroll
    for (int p = 0; p < kMaxSplit; ++p)
#pragma unroll
      for (int q = 0; q < kCols / 4; ++q)
        pv[p][q] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rw, o0 + (uint32_t)min(p, S - 1) * (TM * 256u) + 16u * q, 0, 16));
#pragma unroll
    for (int q = 0; q < kCols / 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = pv[0][q][e];
#pragma unroll
        for (int p = 1; p < kMaxSplit; ++p) a += p < S ? pv[p][q][e] : 0.f;
        v[4 * q + e] = a;
      }
    if (threadIdx.x == 0) __hip_atomic_store(cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }
#pragma unroll
  for (int e = 0; e < kCols; ++e) v[e] *= g.alpha;
  if (row >= g.M) return;
  constexpr bool kBias = EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU_D || EPI == GEMM_EPI_BIAS_ADD;
  constexpr bool kAux = EPI == GEMM_EPI_MUL_AUX || EPI == GEMM_EPI_DGELU || EPI == GEMM_EPI_BIAS_ADD;
#pragma unroll
  for (int h = 0; h < kCols / 8; ++h) {
    const int col = n0 + ct + 8 * h;
    if (col >= g.N) break;  // (N % 8 == 0: an 8-column group is in or out as a whole)
    float* x = v + 8 * h;
    if constexpr (kBias) {
      float b[8];
      load8(g.bias + col, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] += b[e];
    }
    if constexpr (kAux) {
      float a[8];
      load8(g.aux + (long)row * g.ldaux + col, a);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if constexpr (EPI == GEMM_EPI_MUL_AUX) x[e] *= a[e];
        else if constexpr (EPI == GEMM_EPI_DGELU) x[e] *= gelu_tanh_grad(a[e]);
        else x[e] += a[e];
      }
    }
    if constexpr (EPI == GEMM_EPI_BIAS_GELU_D) {
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        f32x2_t y2, d2;
        gelu_tanh_and_grad2(f32x2_t{x[e], x[e + 1]}, y2, d2);
        x[e] = y2.x, x[e + 1] = y2.y, d[e] = d2.x, d[e + 1] = d2.y;
      }
      store8(g.aux + (long)row * g.ldaux + col, d);
    }
    store8(reinterpret_cast<bf16_t*>(g.C) + (long)row * g.ldc + col, x);
  }
}

// split-K workspace of a stream: kWsTiles fp32 64 x 64 partials + kCnt tile counters (zeroed once; the
// kernels re-arm them), allocated on first use outside graph capture
constexpr int kWsTiles = 2048, kCnt = 16384;
struct SplitWs {
  float* ws = nullptr;
  int* cnt = nullptr;
};
static SplitWs split_ws(hipStream_t st) {
  static std::mutex mu;
  static std::unordered_map<hipStream_t, SplitWs> m;
  std::lock_guard<std::mutex> lk(mu);
  auto it = m.find(st);
  if (it != m.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  MFT_HIP_CHECK(hipStreamIsCapturing(st, &cs));
  if (cs != hipStreamCaptureStatusNone) return SplitWs{};  // (no allocation inside a capture: S = 1)
  SplitWs w;
  MFT_HIP_CHECK(hipMalloc(&w.ws, sizeof(float) * 4096 * kWsTiles));
  MFT_HIP_CHECK(hipMalloc(&w.cnt, sizeof(int) * kCnt));
  MFT_HIP_CHECK(hipMemsetAsync(w.cnt, 0, sizeof(int) * kCnt, st));
  m[st] = w;
  return w;
}

// K-splits: enough workgroups for ~1.5 per CU, every wave at least 2 K-tiles (MFT_GS_SPLIT=0: off, A/B)
// (MFT_GS_SPLIT_TILES: the tile count from which no product splits, A/B)
static int pick_split(int tiles, int nkt, int tm) {
  static const int on = getenv("MFT_GS_SPLIT") ? atoi(getenv("MFT_GS_SPLIT")) : 1;
  static const int lim = getenv("MFT_GS_SPLIT_TILES") ? atoi(getenv("MFT_GS_SPLIT_TILES")) : 192;
  if (!on || tiles >= lim) return 1;
  int S = std::min((384 + tiles - 1) / tiles, nkt / (2 * kNW));
  S = std::max(1, std::min({S, kMaxSplit, kWsTiles * (64 / tm) / std::max(tiles, 1)}));
  return tiles > kCnt ? 1 : S;
}

template <int EPI, bool SEG2, int TM>
void launch_s_tm(const GemmArgs& g, hipStream_t st) {
  constexpr size_t shm = kNW * TM * kLdr * sizeof(float);
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm_s_kernel<EPI, SEG2, TM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)shm));
    attr = true;
  }
  const int tiles = ((g.M + TM - 1) / TM) * ((g.N + 63) / 64);
  int S = pick_split(tiles, g.K / 64 + (SEG2 ? g.K2 / 64 : 0), TM);
  SplitWs w;
  if (S > 1) {
    w = split_ws(st);
    if (!w.ws) S = 1;
  }
  const int blocks = S > 1 ? (tiles + 7) / 8 * 8 * S : tiles;
  static const int strict = getenv("MFT_STRICT_HANDOFF") && getenv("MFT_STRICT_HANDOFF")[0] == '1';
  GemmArgs gs = g;
  gs.handoff_fence = strict;
  gemm_s_kernel<EPI, SEG2, TM><<<blocks, 64 * kNW, shm, st>>>(gs, S, w.ws, w.cnt);
}

// 32-row tiles while the 64-row tiles would leave more than half the CUs idle (MFT_GS_TM=64 | 32 forces one)
template <int EPI, bool SEG2>
void launch_s(const GemmArgs& g, hipStream_t st) {
  static const int force = getenv("MFT_GS_TM") ? atoi(getenv("MFT_GS_TM")) : 0;
  const long tiles64 = (long)((g.M + 63) / 64) * ((g.N + 63) / 64);
  const bool t32 = force == 32 || (force != 64 && tiles64 < 128);
  if (t32) launch_s_tm<EPI, SEG2, 32>(g, st);
  else launch_s_tm<EPI, SEG2, 64>(g, st);
}

}  // namespace

bool gemm_s_supported(int M, int N, int K, int epi) {
  const bool epi_ok = epi == GEMM_EPI_NONE || epi == GEMM_EPI_BIAS || epi == GEMM_EPI_BIAS_GELU_D ||
                      epi == GEMM_EPI_MUL_AUX || epi == GEMM_EPI_DGELU || epi == GEMM_EPI_BIAS_ADD;
  return epi_ok && M > 0 && N >= 8 && N % 8 == 0 && K >= 64 && K % 64 == 0;
}

// short-token rule: the 256 x 256 tiles of gemm4 would fill less than half the CUs
bool gemm_s_preferred(int M, int N, int K) {
  const long tiles256 = (long)((M + 255) / 256) * ((N + 255) / 256);
  return tiles256 * 2 < 256 && (long)M * N * K < (1L << 33);
}

void gemm_s(const GemmArgs& g, int epi, hipStream_t st) {
  if (!gemm_s_supported(g.M, g.N, g.K, epi) || (g.K2 > 0 && (epi != GEMM_EPI_NONE || g.K2 % 64)) || g.lda % 8 ||
      g.ldb % 8 || g.ldc % 8) {
    fprintf(stderr, "mft::gemm_s: unsupported M=%d N=%d K=%d K2=%d epi=%d\n", g.M, g.N, g.K, g.K2, epi);
    abort();
  }
  if (g.K2 > 0) return launch_s<GEMM_EPI_NONE, true>(g, st);
  static const int diag = getenv("MFT_GS_DIAG") ? atoi(getenv("MFT_GS_DIAG")) : 0;  // 1: every operand load out of range
  if (diag) {
    GemmArgs d = g;
    d.stagger = 1;
    return launch_s<GEMM_EPI_BIAS, false>(d, st);
  }
  switch (epi) {
    case GEMM_EPI_NONE: return launch_s<GEMM_EPI_NONE, false>(g, st);
    case GEMM_EPI_BIAS: return launch_s<GEMM_EPI_BIAS, false>(g, st);
    case GEMM_EPI_BIAS_GELU_D: return launch_s<GEMM_EPI_BIAS_GELU_D, false>(g, st);
    case GEMM_EPI_MUL_AUX: return launch_s<GEMM_EPI_MUL_AUX, false>(g, st);
    case GEMM_EPI_DGELU: return launch_s<GEMM_EPI_DGELU, false>(g, st);
    case GEMM_EPI_BIAS_ADD: return launch_s<GEMM_EPI_BIAS_ADD, false>(g, st);
    default: break;
  }
}

}  // namespace mft
