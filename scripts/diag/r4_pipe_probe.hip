// Cross-queue pipelining: stream A runs a chain of N 'updates' (spin kernels), recording an event after
// each; stream B runs N 'compute' kernels, the k-th waiting on A's event k.  Overlapped: ~N x 2.5 + 2 ms;
// serialised: ~N x 4.5 ms.  Variants: 1 = A and B both default priority; 2 = A low priority; 3 = B's
// waits routed through a third stream C (B waits on C's event, C waits on A's) like the ZeRO-3 gathers.
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
  if (threadIdx.x == 0) out[blockIdx.x] = (int)(t - t0);
}

int main(int argc, char** argv) {
  const int v = argc > 1 ? std::atoi(argv[1]) : 1;
  const int N = 20, grid = argc > 2 ? std::atoi(argv[2]) : 64;
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  int* out;
  CK(hipMalloc(&out, 4096 * sizeof(int)));
  hipStream_t A, B, C;
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  if (v == 2) CK(hipStreamCreateWithPriority(&A, hipStreamNonBlocking, least));
  else CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
  hipEvent_t ev[N], cev[N], f;
  for (int k = 0; k < N; ++k) {
    CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&cev[k], hipEventDisableTiming));
  }
  CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
  auto run = [&]() {
    CK(hipEventRecord(f, B));
    CK(hipStreamWaitEvent(A, f, 0));
    for (int k = 0; k < N; ++k) {  // host order interleaved like the forward: update k, then compute k - 2
      spin<<<grid, 256, 0, A>>>((long long)khz * 25 / 10, out);
      CK(hipEventRecord(ev[k], A));
      if (k >= 2) {
        if (v == 3) {
          CK(hipStreamWaitEvent(C, ev[k - 2], 0));
          CK(hipEventRecord(cev[k - 2], C));
          CK(hipStreamWaitEvent(B, cev[k - 2], 0));
        } else {
          CK(hipStreamWaitEvent(B, ev[k - 2], 0));
        }
        spin<<<grid, 256, 0, B>>>((long long)khz * 2, out + 2048);
      }
    }
    CK(hipEventRecord(f, A));
    CK(hipStreamWaitEvent(B, f, 0));
    CK(hipStreamSynchronize(B));
  };
  run();
  auto t = std::chrono::steady_clock::now();
  run();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  std::printf("variant %d grid %d: %.1f ms (overlapped ~%.0f, serialised ~%.0f)\n", v, grid, ms, N * 2.5 + 2.0,
              N * 2.5 + (N - 2) * 2.0);
  return 0;
}
