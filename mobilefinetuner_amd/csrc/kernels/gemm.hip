// Hand-written MFMA GEMM for gfx950 with fused epilogues.
//
//   C[M, N] = epi(alpha * A[M, K] . op(B))       A row-major (K contiguous)
//   op(B) = B^T for B [N, K] ("NT": nn.Linear forward, y = x W^T)
//         = B   for B [K, N] ("NN": data-grad, dx = dy W)
//
// Epilogues (the reason this kernel exists next to hipBLASLt, whose gfx950 build has no AUX/DGELU
// solutions): bias; bias + GELU(tanh) writing BOTH the pre-activation (for backward) and the
// activation; dGELU (multiply by GELU'(pre) read from an aux tensor); fp32 accumulate (weight
// gradients straight into the fp32 grad buffer, beta = 1).  Reference ops replaced: core/ops.cpp
// matmul/linear (:61-250), gelu (:1121-1180) and their backward pairs in the autograd tape.
//
// Structure (CDNA HIP guide §5): 256 x 256 (or 128 x 256) block tile, BK = 64, 8 waves as 2 (M) x 4
// (N), each wave a (BM/2) x 64 sub-tile of 16x16 MFMA accumulators (v_mfma_f32_16x16x32_bf16).
// Operands go global -> LDS with global_load_lds_dwordx4 (no VGPR round trip), double-buffered, the
// next K-tile in flight while the current one is multiplied (counted vmcnt + raw s_barrier, never
// a vmcnt(0) in the loop).  K-contiguous tiles are stored with an XOR swizzle of the 16-B chunk
// index (chunk ^ (row & 7)) applied on the GLOBAL source address, so the LDS image stays
// lane-linear for the DMA and ds_read_b128 fragment reads spread over the banks.  NN B tiles
// ([64 k][BN n]) are read with ds_read_b64_tr_b16.  The epilogue stages each wave's tile through
// LDS so every global store is a 16-B row piece.  Tiles are mapped XCD-aware (consecutive tiles,
// which share A rows, land on one XCD's L2).
#include "mfma.h"
#include "kernels.h"

namespace mft {

namespace {

constexpr int kBK = 64;

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void g_void;

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)lds_wave_base, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void block_sync_raw() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// K-contiguous tile [ROWS][64] from src rows r0.. (clamped to rmax-1), swizzled chunks.
template <int ROWS, int NT>
__device__ __forceinline__ void stage_k(bf16_t* lds, const bf16_t* src, long ld, int r0, int rmax, int k0) {
  const int tid = threadIdx.x, w = tid >> 6;
#pragma unroll
  for (int t = 0; t < ROWS * 8 / NT; ++t) {
    const int c = t * NT + tid;
    const int r = c >> 3, s = c & 7;
    const int gr = min(r0 + r, rmax - 1);
    const bf16_t* p = src + (long)gr * ld + k0 + ((s ^ (r & 7)) << 3);
    glds16(p, lds + (t * NT + w * 64) * 8);
  }
}

// N-contiguous tile [64 k][COLS] from src rows k0.., columns c0.. (clamped), plain layout.
template <int COLS, int NT>
__device__ __forceinline__ void stage_n(bf16_t* lds, const bf16_t* src, long ld, int k0, int c0, int cmax) {
  const int tid = threadIdx.x, w = tid >> 6;
  constexpr int CPR = COLS / 8;
#pragma unroll
  for (int t = 0; t < 64 * CPR / NT; ++t) {
    const int c = t * NT + tid;
    const int r = c / CPR, s = c % CPR;
    const int gc = min(c0 + s * 8, cmax - 8);
    glds16(src + (long)(k0 + r) * ld + gc, lds + (t * NT + w * 64) * 8);
  }
}

// A-operand fragment of a swizzled [.][64] tile: lane holds T[r0 + (l&15)][kc*8 + 8*(l>>4) + j]
__device__ __forceinline__ bf16x8_t frag_swz(const bf16_t* t, int r0, int kc) {
  const int l = threadIdx.x & 63;
  const int r = r0 + (l & 15), q = kc + (l >> 4);
  return *reinterpret_cast<const bf16x8_t*>(t + r * 64 + ((q ^ (r & 7)) << 3));
}

__device__ __forceinline__ float gelu_grad_tanh(float x) { return gelu_tanh_grad(x); }

}  // namespace

template <int BM, int BN, int WM, int WN, bool BNN, int EPI>
__global__ __launch_bounds__(64 * WM * WN) void gemm_kernel(GemmArgs g) {
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, MR = TM / 16, NR = TN / 16;
  constexpr int A_ELEMS = BM * kBK, B_ELEMS = BN * kBK;
  constexpr int NA = BM * 8 / NT, NB = BN * 8 / NT;  // glds instructions per thread per K-tile
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  // buffer b: A image at smem + b * (A_ELEMS + B_ELEMS), B image right after it

  const int tiles_n = (g.N + BN - 1) / BN;
  const int nblk = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nblk);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w / WN, wn = w % WN;
  const int nk = g.K / kBK;

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = zero4();

  auto stage = [&](int kt, int buf) {
    bf16_t* a_dst = smem + buf * (A_ELEMS + B_ELEMS);
    stage_k<BM, NT>(a_dst, g.A, g.lda, m0, g.M, kt * kBK);
    if constexpr (BNN) stage_n<BN, NT>(a_dst + A_ELEMS, g.B, g.ldb, kt * kBK, n0, g.N);
    else stage_k<BN, NT>(a_dst + A_ELEMS, g.B, g.ldb, n0, g.N, kt * kBK);
  };

  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      stage(kt + 1, cur ^ 1);
      wait_vm<NA + NB>();
    } else {
      wait_vm<0>();
    }
    block_sync_raw();
    const bf16_t* a_t = smem + cur * (A_ELEMS + B_ELEMS);
    const bf16_t* b_t = a_t + A_ELEMS;
#pragma unroll
    for (int ks = 0; ks < kBK / 32; ++ks) {
      bf16x8_t af[MR], bfr[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) af[i] = frag_swz(a_t, wm * TM + i * 16, ks * 4);
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        if constexpr (BNN) bfr[j] = frag_tr(b_t, BN, ks * 32, wn * TN + j * 16);
        else bfr[j] = frag_swz(b_t, wn * TN + j * 16, ks * 4);
      }
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    block_sync_raw();
  }

  // ------------------------------------------------------------------ epilogue
  const int rbase = m0 + wm * TM, cbase = n0 + wn * TN;
  if constexpr (EPI == GEMM_EPI_F32ACC) {
    float* C = reinterpret_cast<float*>(g.C);
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int col = cbase + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + i * 16 + 4 * (lane >> 4) + r;
          if (row < g.M && col < g.N) {
            float* p = C + (long)row * g.ldc + col;
            *p += g.alpha * acc[i][j][r];
          }
        }
      }
    return;
  } else {
    // per-wave staging tile [TM][TN] bf16 (stride TN + 8 to break bank aliasing of the column writes)
    constexpr int LDT = TN + 8;
    bf16_t* T = smem + w * TM * LDT;
    constexpr int CPR = TN / 8;
    auto tile_to_global = [&](bf16_t* dst, long ldd) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 4
      for (int c = lane; c < TM * CPR; c += 64) {
        const int r = c / CPR, ch = c % CPR;
        const int row = rbase + r, col = cbase + ch * 8;
        if (row < g.M && col < g.N)
          *reinterpret_cast<u16x8_t*>(dst + (long)row * ldd + col) = *reinterpret_cast<const u16x8_t*>(T + r * LDT + ch * 8);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    if constexpr (EPI == GEMM_EPI_DGELU) {
      // aux (pre-activation) tile -> LDS with coalesced 16-B loads, then read per C-layout element
#pragma unroll 4
      for (int c = lane; c < TM * CPR; c += 64) {
        const int r = c / CPR, ch = c % CPR;
        const int row = min(rbase + r, g.M - 1), col = min(cbase + ch * 8, g.N - 8);
        *reinterpret_cast<u16x8_t*>(T + r * LDT + ch * 8) =
            *reinterpret_cast<const u16x8_t*>(g.aux + (long)row * g.ldaux + col);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    float bias_v[NR];
    if constexpr (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU) {
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int col = min(cbase + j * 16 + (lane & 15), g.N - 1);
        bias_v[j] = bf2f(g.bias[col]);
      }
    }
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int tr = i * 16 + 4 * (lane >> 4) + r, tc = j * 16 + (lane & 15);
          float v = acc[i][j][r] * g.alpha;
          if constexpr (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU) v += bias_v[j];
          if constexpr (EPI == GEMM_EPI_DGELU) v *= gelu_grad_tanh(bf2f(T[tr * LDT + tc]));
          if constexpr (EPI == GEMM_EPI_BIAS_GELU) acc[i][j][r] = v;  // keep pre-activation
          T[tr * LDT + tc] = f2bf(v);
        }
    if constexpr (EPI == GEMM_EPI_BIAS_GELU) {
      tile_to_global(g.aux, g.ldaux);  // pre-activation
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int tr = i * 16 + 4 * (lane >> 4) + r, tc = j * 16 + (lane & 15);
            T[tr * LDT + tc] = f2bf(gelu_tanh(acc[i][j][r]));
          }
    }
    tile_to_global(reinterpret_cast<bf16_t*>(g.C), g.ldc);
  }
}

template <int BM, int BN, int WM, int WN, bool BNN, int EPI>
static void launch_t(const GemmArgs& g, hipStream_t st) {
  constexpr size_t shm_loop = sizeof(bf16_t) * 2 * (BM + BN) * kBK;
  constexpr size_t shm_epi = sizeof(bf16_t) * WM * WN * (BM / WM) * (BN / WN + 8);
  constexpr size_t shm = shm_loop > shm_epi ? shm_loop : shm_epi;
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, WM, WN, BNN, EPI>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    attr = true;
  }
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  gemm_kernel<BM, BN, WM, WN, BNN, EPI><<<tiles, 64 * WM * WN, shm, st>>>(g);
}

// tile configurations: 0 = 256x256 (8 waves, 1 block/CU), 1 = 128x256 (8 waves),
//                      2 = 128x128 (4 waves, 2 blocks/CU), 3 = 256x128 (8 waves)
template <bool BNN, int EPI>
static void launch_e(const GemmArgs& g, int cfg, hipStream_t st) {
  switch (cfg) {
    case 1: launch_t<128, 256, 2, 4, BNN, EPI>(g, st); break;
    case 2: launch_t<128, 128, 2, 2, BNN, EPI>(g, st); break;
    case 3: launch_t<256, 128, 4, 2, BNN, EPI>(g, st); break;
    default: launch_t<256, 256, 2, 4, BNN, EPI>(g, st); break;
  }
}

bool gemm_supported(int M, int N, int K) { return K % kBK == 0 && N % 8 == 0 && M > 0 && N >= 8 && K > 0; }

void gemm(const GemmArgs& g, bool b_nn, int epi, int cfg, hipStream_t st) {
  if (!gemm_supported(g.M, g.N, g.K)) {
    fprintf(stderr, "mft::gemm: unsupported shape M=%d N=%d K=%d (K %% 64, N %% 8)\n", g.M, g.N, g.K);
    abort();
  }
#define MFT_GEMM_EPI(E)                           \
  case E:                                         \
    if (b_nn) launch_e<true, E>(g, cfg, st);      \
    else launch_e<false, E>(g, cfg, st);          \
    break;
  switch (epi) {
    MFT_GEMM_EPI(GEMM_EPI_NONE)
    MFT_GEMM_EPI(GEMM_EPI_BIAS)
    MFT_GEMM_EPI(GEMM_EPI_BIAS_GELU)
    MFT_GEMM_EPI(GEMM_EPI_DGELU)
    MFT_GEMM_EPI(GEMM_EPI_F32ACC)
    default:
      fprintf(stderr, "mft::gemm: bad epilogue %d\n", epi);
      abort();
  }
#undef MFT_GEMM_EPI
}

}  // namespace mft
