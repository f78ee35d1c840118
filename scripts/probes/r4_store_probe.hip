// Diagnostic: is a GEMM tile's 128 KB bf16 epilogue store (and its 128 KB prologue fill) bound by the
// chip's HBM bandwidth when every CU does it at once (lockstep tile rounds), or by the per-CU store
// issue rate?  Each 512-thread workgroup writes R consecutive 256 x 256 bf16 tiles of a row-major
// [M, 3072] output exactly like gemm8's epilogue (16 x 16-B stores per lane), stamping s_memtime
// around each tile.  Grids of 256 (one per CU), 64 and 16 workgroups; per-tile median cycles.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/r4_store_probe.hip -o gpurun_out/r4_store_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// pattern 0: gemm8's epilogue (per instruction 16 rows x 64 B), 1: 8 rows x 128 B, 2: 4 rows x 256 B,
// 3: 2 rows x 512 B (whole tile rows)
__global__ __launch_bounds__(512, 1) void store_tiles(unsigned short* C, int N, int tiles_n, int R,
                                                       unsigned long long* st, int spread, int pat) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 2, wn = w & 3;
  const int g4 = lane >> 4, cofs = (g4 & 1) * 16 + (g4 >> 1) * 8;
  f32x4 v = {__int_as_float(0x3f803f80 + lane), __int_as_float(0x3f813f81 + w), 1.f, 2.f};
  for (int r = 0; r < R; ++r) {
    if (threadIdx.x == 0) st[(blockIdx.x * R + r) * 2] = __builtin_amdgcn_s_memtime();
    const int tile = r * gridDim.x + blockIdx.x;
    const int m0 = (tile / tiles_n) * 256, n0 = (tile % tiles_n) * 256;
    if (pat == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int qa = (q == 2 || q == 3), qb = (q == 1 || q == 2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + qa * 128 + wm * 64 + i * 16 + (lane & 15);
          const int col = n0 + qb * 128 + wn * 32 + cofs;
          *reinterpret_cast<f32x4*>(C + (long)row * N + col) = v;
          v[2] += 1.f;
          if (spread) __builtin_amdgcn_s_sleep(4);
        }
      }
    } else {
      // per instruction: RW rows x (1024 / RW) bytes; the wave's 16 instructions cover 32 rows x 512 B
      const int lpr = 64 >> (pat == 1 ? 3 : pat == 2 ? 2 : 1);  // lanes per row segment
      const int rw = 64 / lpr;                                   // rows per instruction
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int seg = k % (32 / lpr * 0 + (256 * 2 / (lpr * 16)));  // segments per tile row
        const int nseg = 512 / (lpr * 16);
        const int s2 = k % nseg, rblk = k / nseg;
        const int row = m0 + w * 32 + rblk * rw + lane / lpr;
        const int col = n0 + s2 * lpr * 8 + (lane % lpr) * 8;
        (void)seg;
        *reinterpret_cast<f32x4*>(C + (long)row * N + col) = v;
        v[2] += 1.f;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) st[(blockIdx.x * R + r) * 2 + 1] = __builtin_amdgcn_s_memtime();
  }
}

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void g_void;

// 128 KB per tile: rows m0.. of a [M, K] bf16 operand, the first 128 k-columns (two 64-deep K-tiles
// of A; the B operand is L2-resident in a GEMM), 16 x 1 KB LDS-DMA pieces per wave
__global__ __launch_bounds__(512, 1) void load_tiles(const unsigned short* A, int K, int R, unsigned long long* st) {
  // A: [131072, K]; tile t -> row block t % 512, column block t / 512 (cold bytes on every tile)
  extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
  const int tid = threadIdx.x, w = tid >> 6;
  for (int r = 0; r < R; ++r) {
    if (threadIdx.x == 0) st[(blockIdx.x * R + r) * 2] = __builtin_amdgcn_s_memtime();
    const int tile = r * gridDim.x + blockIdx.x;
    const long m0 = (long)(tile % 512) * 256;
    const int k0 = (tile / 512) * 128;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int c = t * 512 + tid;  // 16-B chunk of the 256 x 128 tile
      const int row = c >> 4, s = c & 15;
      const unsigned short* src = A + (m0 + row) * K + k0 + s * 8;
      __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(smem + (t * 512 + w * 64) * 8), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) st[(blockIdx.x * R + r) * 2 + 1] = __builtin_amdgcn_s_memtime();
  }
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const int M = 131072, N = 3072, K = 768;
  unsigned short *C, *A;
  hipMalloc(&C, (size_t)M * N * 2);
  hipMalloc(&A, (size_t)M * K * 2);
  hipMemset(A, 0x3c, (size_t)M * K * 2);
  unsigned long long* st;
  hipMalloc(&st, (size_t)6144 * 2 * 8);
  const int tiles_n = N / 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int pat : {0, 1, 2, 3}) {
    const int spread = 0;
    for (int grid : {256, 16}) {
      const int R = 8;
      for (int it = 0; it < 3; ++it) store_tiles<<<grid, 512>>>(C, N, tiles_n, R, st, spread, pat);
      hipEventRecord(e0, 0);
      store_tiles<<<grid, 512>>>(C, N, tiles_n, R, st, spread, pat);
      hipEventRecord(e1, 0);
      hipDeviceSynchronize();
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      std::vector<unsigned long long> h((size_t)grid * R * 2);
      hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
      std::vector<double> d;
      for (int b = 0; b < grid * R; ++b) d.push_back(double(h[b * 2 + 1] - h[b * 2]));
      const double bytes = (double)grid * R * 256 * 256 * 2;
      printf("store  pattern=%d grid=%3d spread=%d: %.1f us, %.2f TB/s chip, median %.0f cycles per 128 KB tile (%.1f B/cycle/CU)\n",
             pat, grid, spread, ms * 1e3, bytes / (ms * 1e-3) / 1e12, med(d), 131072.0 / med(d));
    }
  }
  for (int grid : {256, 128, 64, 16}) {
    const int R = 8;
    for (int it = 0; it < 3; ++it) load_tiles<<<grid, 512, 65536>>>(C, N, R, st);
    hipEventRecord(e0, 0);
    load_tiles<<<grid, 512, 65536>>>(C, N, R, st);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h((size_t)grid * R * 2);
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> d;
    for (int b = 0; b < grid * R; ++b) d.push_back(double(h[b * 2 + 1] - h[b * 2]));
    const double bytes = (double)grid * R * 256 * 128 * 2;
    printf("glds   grid=%3d: %.1f us, %.2f TB/s chip, median %.0f cycles per 64 KB fill (%.1f B/cycle/CU)\n", grid,
           ms * 1e3, bytes / (ms * 1e-3) / 1e12, med(d), 65536.0 / med(d));
  }
  hipFree(C);
  hipFree(A);
  hipFree(st);
  return 0;
}
