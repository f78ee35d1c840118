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
#include "common.h"
#include "kernels.h"
#include "mfma.h"

namespace mft {

namespace {

constexpr int kLdr = 68;  // fp32 row pitch of the reduction image (64 + 4: float4 writes spread over banks)

struct Frags {
  bf16x8_t a[2][4], b[2][4];  // [k-step][block]
};

// fragments of K-tile kt (64 columns) for the tile (m0, n0): A rows m0 + 16 i + (l & 15), B rows
// n0 + 16 j + (l & 15), columns 32 ks + 8 (l >> 4) .. + 7; rows past M / N read the last row
__device__ __forceinline__ void load_frags(Frags& f, const bf16_t* A, long lda, const bf16_t* B, long ldb, int m0,
                                           int n0, int M, int N, int k0) {
  const int l = threadIdx.x & 63, r = l & 15, c = k0 + 8 * (l >> 4);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ra = min(m0 + 16 * i + r, M - 1), rb = min(n0 + 16 * i + r, N - 1);
      f.a[ks][i] = *reinterpret_cast<const bf16x8_t*>(A + (long)ra * lda + c + 32 * ks);
      f.b[ks][i] = *reinterpret_cast<const bf16x8_t*>(B + (long)rb * ldb + c + 32 * ks);
    }
}

__device__ __forceinline__ void mma(f32x4_t (&acc)[4][4], const Frags& f) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(f.b[ks][j], f.a[ks][i], acc[i][j]);
}

template <int EPI, bool SEG2>
__global__ __launch_bounds__(256) void gemm_s_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4 waves][64 rows][kLdr]
  const int tiles_n = (g.N + 63) / 64;
  const int m0 = (blockIdx.x / tiles_n) * 64, n0 = (blockIdx.x % tiles_n) * 64;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int nk = g.K / 64, nkt = nk + (SEG2 ? g.K2 / 64 : 0);
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero4();
  auto load = [&](Frags& f, int kt) {
    if (SEG2 && kt >= nk) load_frags(f, g.A2, g.lda2, g.B2, g.ldb2, m0, n0, g.M, g.N, (kt - nk) * 64);
    else load_frags(f, g.A, g.lda, g.B, g.ldb, m0, n0, g.M, g.N, kt * 64);
  };
  Frags f0, f1;
  int kt = w;
  if (kt < nkt) load(f0, kt);
  while (kt < nkt) {  // two K-tiles per trip: one in flight while the other multiplies
    if (kt + 4 < nkt) load(f1, kt + 4);
    mma(acc, f0);
    kt += 4;
    if (kt >= nkt) break;
    if (kt + 4 < nkt) load(f0, kt + 4);
    mma(acc, f1);
    kt += 4;
  }
  // partial tile of this wave -> LDS: lane holds row 16 i + (l & 15), columns 16 j + 4 (l >> 4) .. + 3
  float* mine = red + w * 64 * kLdr;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<f32x4_t*>(mine + (16 * i + (l & 15)) * kLdr + 16 * j + 4 * (l >> 4)) = acc[i][j];
  __syncthreads();
  // wave w reduces rows 16 w .. + 15: lane -> row 16 w + (l >> 2), columns 16 (l & 3) .. + 15
  const int rt = 16 * w + (l >> 2), ct = 16 * (l & 3);
  const int row = m0 + rt, col = n0 + ct;
  float v[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4_t s = *reinterpret_cast<const f32x4_t*>(red + rt * kLdr + ct + 4 * q);
#pragma unroll
    for (int p = 1; p < 4; ++p) {
      const f32x4_t t = *reinterpret_cast<const f32x4_t*>(red + (p * 64 + rt) * kLdr + ct + 4 * q);
      s[0] += t[0], s[1] += t[1], s[2] += t[2], s[3] += t[3];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * q + e] = s[e] * g.alpha;
  }
  if (row >= g.M || col >= g.N) return;  // (N % 8 == 0: a lane's two 8-column halves are in or out together)
  const bool hi_ok = col + 8 < g.N;
  constexpr bool kBias = EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_GELU_D || EPI == GEMM_EPI_BIAS_ADD;
  constexpr bool kAux = EPI == GEMM_EPI_MUL_AUX || EPI == GEMM_EPI_DGELU || EPI == GEMM_EPI_BIAS_ADD;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 1 && !hi_ok) break;
    float* x = v + 8 * h;
    const int c = col + 8 * h;
    if constexpr (kBias) {
      float b[8];
      load8(g.bias + c, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] += b[e];
    }
    if constexpr (kAux) {
      float a[8];
      load8(g.aux + (long)row * g.ldaux + c, a);
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
      for (int e = 0; e < 8; ++e) gelu_tanh_and_grad(x[e], x[e], d[e]);
      store8(g.aux + (long)row * g.ldaux + c, d);
    }
    store8(reinterpret_cast<bf16_t*>(g.C) + (long)row * g.ldc + c, x);
  }
}

template <int EPI, bool SEG2>
void launch_s(const GemmArgs& g, hipStream_t st) {
  constexpr size_t shm = 4 * 64 * kLdr * sizeof(float);
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)gemm_s_kernel<EPI, SEG2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)shm));
    attr = true;
  }
  const int tiles = ((g.M + 63) / 64) * ((g.N + 63) / 64);
  gemm_s_kernel<EPI, SEG2><<<tiles, 256, shm, st>>>(g);
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
