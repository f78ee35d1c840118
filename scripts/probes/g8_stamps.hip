// Diagnostic: per-workgroup s_memtime stamps of gemm8 (start / after prologue / after main loop /
// after epilogue) at one shape, to split a tile's time into prologue, MFMA loop and epilogue.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMFT_G8_STAMPS -I mobilefinetuner_amd/csrc \
//          scripts/probes/g8_stamps.hip -o gpurun_out/g8_stamps
#include "../../mobilefinetuner_amd/csrc/kernels/gemm8.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace mft;
namespace mft {
bool gemm_supported(int M, int N, int K) { return K % 64 == 0 && N % 8 == 0; }
}

__global__ void fill(bf16_t* p, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995; h ^= h >> 15;
    p[i] = f2bf(((h & 0xffff) / 32768.0f - 1.0f) * scale);
  }
}

static void run(int M, int N, int K, int epi) {
  bf16_t *A, *B, *C, *aux, *bias;
  hipMalloc(&A, (size_t)M * K * 2); hipMalloc(&B, (size_t)N * K * 2);
  hipMalloc(&C, (size_t)M * N * 2); hipMalloc(&aux, (size_t)M * N * 2); hipMalloc(&bias, N * 2);
  fill<<<1024, 256>>>(A, (long)M * K, 1, 1.f);
  fill<<<1024, 256>>>(B, (long)N * K, 2, 0.05f);
  fill<<<64, 256>>>(bias, N, 3, 0.1f);
  fill<<<1024, 256>>>(aux, (long)M * N, 4, 1.f);
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  unsigned long long* st;
  hipMalloc(&st, (size_t)tiles * 4 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g8_stamps), &st, sizeof(st));
  GemmArgs g{};
  g.A = A; g.lda = K; g.B = B; g.ldb = K; g.C = C; g.ldc = N; g.bias = bias; g.aux = aux; g.ldaux = N;
  g.M = M; g.N = N; g.K = K; g.alpha = 1.f;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 5; ++i) gemm8(g, epi, 0);
  hipEventRecord(e0, 0);
  for (int i = 0; i < 10; ++i) gemm8(g, epi, 0);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h((size_t)tiles * 4);
  hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> pro, loop, epil, tot;
  unsigned long long t_min = ~0ull, t_max = 0;
  for (int b = 0; b < tiles; ++b) {
    auto* s = &h[b * 4];
    pro.push_back(double(s[1] - s[0])); loop.push_back(double(s[2] - s[1]));
    epil.push_back(double(s[3] - s[2])); tot.push_back(double(s[3] - s[0]));
    t_min = std::min(t_min, s[0]); t_max = std::max(t_max, s[3]);
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  const double us = ms * 1e3 / 10;
  const double span = double(t_max - t_min);
  double sum_tot = 0; for (double x : tot) sum_tot += x;
  printf("  per-CU busy (sum of tile totals / 256) = %.0f ticks; t_min=%llu t_max=%llu\n", sum_tot / 256, t_min, t_max);
  printf("M=%d N=%d K=%d epi=%d: %.1f us/call, %d tiles; median cycles per tile: prologue %.0f, main loop %.0f, "
         "epilogue %.0f, total %.0f; last call span %.0f cycles (-> %.2f GHz if span ~ call time)\n",
         M, N, K, epi, us, tiles, med(pro), med(loop), med(epil), med(tot), span, span / (us * 1e3));
  hipFree(A); hipFree(B); hipFree(C); hipFree(aux); hipFree(bias); hipFree(st);
}

// TN weight gradient: dW[P, Q] += dy[T, P]^T x[T, Q] (split-K over the T tokens)
static void run_tn(int T, int P, int Q, int ks) {
  bf16_t *dy, *x;
  float *dw, *ws;
  hipMalloc(&dy, (size_t)T * P * 2); hipMalloc(&x, (size_t)T * Q * 2);
  hipMalloc(&dw, (size_t)P * Q * 4); hipMalloc(&ws, (size_t)ks * P * Q * 4);
  fill<<<1024, 256>>>(dy, (long)T * P, 1, 1.f);
  fill<<<1024, 256>>>(x, (long)T * Q, 2, 1.f);
  const int tiles = ((P + 255) / 256) * ((Q + 255) / 256) * ks;
  unsigned long long* st;
  hipMalloc(&st, (size_t)tiles * 4 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g8_stamps), &st, sizeof(st));
  GemmArgs g{};
  g.A = dy; g.lda = P; g.B = x; g.ldb = Q; g.C = dw; g.ldc = Q; g.M = P; g.N = Q; g.K = T; g.alpha = 1.f;
  g.ksplit = ks; g.ws = ws;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) gemm8x(g, GEMM_EPI_F32ACC, true, true, 0);
  hipEventRecord(e0, 0);
  for (int i = 0; i < 10; ++i) gemm8x(g, GEMM_EPI_F32ACC, true, true, 0);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h((size_t)tiles * 4);
  hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> pro, loop, epil;
  for (int b = 0; b < tiles; ++b) {
    auto* s = &h[b * 4];
    pro.push_back(double(s[1] - s[0])); loop.push_back(double(s[2] - s[1])); epil.push_back(double(s[3] - s[2]));
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  printf("TN T=%d P=%d Q=%d ks=%d: %.1f us/call (incl. reduce), %d WGs, %d K-tiles/WG; median ticks: prologue %.0f, "
         "main loop %.0f, epilogue %.0f\n", T, P, Q, ks, ms * 1e3 / 10, tiles, T / 64 / ks, med(pro), med(loop), med(epil));
  hipFree(dy); hipFree(x); hipFree(dw); hipFree(ws); hipFree(st);
}

int main() {
  run_tn(65536, 2304, 768, 8);
  run_tn(65536, 2304, 768, 9);
  run_tn(65536, 3072, 768, 8);
  run_tn(65536, 3072, 768, 7);
  run(131072, 3072, 768, GEMM_EPI_NONE);
  run(131072, 2304, 832, GEMM_EPI_NONE);
  run(65536, 768, 3072, GEMM_EPI_NONE);
  run(65536, 3072, 768, GEMM_EPI_NONE);
  run(65536, 3072, 768, GEMM_EPI_BIAS_GELU);
  run(65536, 768, 2304, GEMM_EPI_NONE);
  run(65536, 3072, 3072, GEMM_EPI_NONE);
  return 0;
}
