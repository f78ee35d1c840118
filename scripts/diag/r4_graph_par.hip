// Do independent branches of a captured hipGraph run concurrently on this ROCm?  Two 20 ms spin
// kernels (one workgroup each) on two forked streams: eager, then as a captured graph.  ~20 ms =
// concurrent, ~40 ms = serialised.  Run under different runtime settings from the shell.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                         \
    }                                                                                       \
  } while (0)

__global__ void spin(long long ticks, int* out) {
  const long long t0 = wall_clock64();
  long long t = t0;
  while (t - t0 < ticks) t = wall_clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = (int)(t - t0);  // vector store
}

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const long long ticks = (long long)khz * 20;  // 20 ms
  int* out;
  CK(hipMalloc(&out, 64 * sizeof(int)));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t f, j;
  CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
  auto body = [&]() {
    CK(hipEventRecord(f, s0));
    CK(hipStreamWaitEvent(s1, f, 0));
    spin<<<1, 64, 0, s0>>>(ticks, out);
    spin<<<1, 64, 0, s1>>>(ticks, out + 1);
    CK(hipEventRecord(j, s1));
    CK(hipStreamWaitEvent(s0, j, 0));
  };
  body();  // warm-up
  CK(hipStreamSynchronize(s0));
  auto t = std::chrono::steady_clock::now();
  for (int r = 0; r < 3; ++r) body();
  CK(hipStreamSynchronize(s0));
  std::printf("eager two streams: %.1f ms per iteration (20 = concurrent, 40 = serialised)\n", ms_since(t) / 3);
  hipGraph_t g;
  hipGraphExec_t x;
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
  body();
  CK(hipStreamEndCapture(s0, &g));
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, s0));
  CK(hipStreamSynchronize(s0));
  t = std::chrono::steady_clock::now();
  for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(x, s0));
  CK(hipStreamSynchronize(s0));
  std::printf("graph, two branches: %.1f ms per launch\n", ms_since(t) / 3);
  return 0;
}
