// Which part of the staged ZeRO-3 host-moment step's stream pattern (engine/zero3.cpp, staged_ = true)
// makes hipStreamEndCapture crash?  The pattern per captured step, streams M (capture origin), S (the
// communication stream: gathers, the device-resident AdamW update), C (the copy stream: SDMA moment
// write-back / prefetch):
//   for each unit u:  M -> S (event), S: update(u); S -> C (event); C: D2H write-back (+ H2D prefetch);
//                     S: all-gather(u) [a kernel here]; S -> M (event)
//   finish:           C -> S (event), S -> M (event)
// Variants (one per process): 1 the full pattern; 2 no memcpy (a kernel on C instead); 3 D2H only;
// 4 H2D only; 5 copies on S (no C); 6 C joined straight to M (not through S); 7 = 1 with the S -> C
// event re-recorded per unit (one event object), 8 = 1 with C never waited on before its last copy.
// Prints "variant N ok" after EndCapture + instantiate + 2 replays.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

__global__ void add1(float* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.f;
}

int main(int argc, char** argv) {
  const int v = argc > 1 ? std::atoi(argv[1]) : 1;
  const int n = 1 << 16, U = 4;
  const size_t bytes = n * sizeof(float);
  hipStream_t M, S, C;
  CK(hipStreamCreateWithFlags(&M, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
  float *d, *slot, *h;
  CK(hipMalloc(&d, bytes * U));
  CK(hipMalloc(&slot, bytes * U));
  CK(hipHostMalloc(&h, bytes * U, hipHostMallocDefault));
  CK(hipMemset(d, 0, bytes * U));
  CK(hipMemset(slot, 0, bytes * U));
  hipEvent_t order, upd[U], h2d[U], cjoin, join, single;
  CK(hipEventCreateWithFlags(&order, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&cjoin, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&single, hipEventDisableTiming));
  for (int u = 0; u < U; ++u) {
    CK(hipEventCreateWithFlags(&upd[u], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&h2d[u], hipEventDisableTiming));
  }
  const dim3 g((n + 255) / 256);
  CK(hipStreamBeginCapture(M, hipStreamCaptureModeRelaxed));
  add1<<<g, 256, 0, M>>>(d, n);
  for (int u = 0; u < U; ++u) {
    CK(hipEventRecord(order, M));
    CK(hipStreamWaitEvent(S, order, 0));
    add1<<<g, 256, 0, S>>>(slot + u * n, n);  // the update
    hipStream_t cs = v == 5 ? S : C;
    hipEvent_t e = v == 7 ? single : upd[u];
    if (v != 5) {
      CK(hipEventRecord(e, S));
      CK(hipStreamWaitEvent(C, e, 0));
    }
    if (v == 2) {
      add1<<<g, 256, 0, C>>>(slot + u * n, n);
    } else {
      if (v != 4) CK(hipMemcpyAsync(h + u * n, slot + u * n, bytes, hipMemcpyDeviceToHost, cs));
      if (v != 3) CK(hipMemcpyAsync(slot + ((u + 1) % U) * n, h + ((u + 1) % U) * n, bytes, hipMemcpyHostToDevice, cs));
    }
    add1<<<g, 256, 0, S>>>(d + u * n, n);  // the all-gather
    CK(hipEventRecord(join, S));
    CK(hipStreamWaitEvent(M, join, 0));
    add1<<<g, 256, 0, M>>>(d, n);  // the block's compute
  }
  if (v != 5) {
    CK(hipEventRecord(cjoin, C));
    if (v == 6) {
      CK(hipStreamWaitEvent(M, cjoin, 0));
    } else {
      CK(hipStreamWaitEvent(S, cjoin, 0));
    }
  }
  CK(hipEventRecord(join, S));
  CK(hipStreamWaitEvent(M, join, 0));
  add1<<<g, 256, 0, M>>>(d, n);
  std::fprintf(stderr, "variant %d: ending capture\n", v);
  hipGraph_t graph;
  CK(hipStreamEndCapture(M, &graph));
  hipGraphExec_t exec;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  for (int r = 0; r < 2; ++r) CK(hipGraphLaunch(exec, M));
  CK(hipStreamSynchronize(M));
  std::printf("variant %d ok\n", v);
  return 0;
}
