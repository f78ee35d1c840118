// Which part of the staged ZeRO-3 host-moment step's stream pattern (engine/zero3.cpp, staged_ = true)
// makes hipStreamEndCapture crash?  The pattern per captured step, streams M (capture origin), S (the
// communication stream: gathers, the device-resident AdamW update), C (the copy stream: SDMA moment
// write-back / prefetch):
//   for each unit u:  M -> S (event), S: update(u); S -> C (event); C: D2H write-back (+ H2D prefetch);
//                     S: all-gather(u) [a kernel here]; S -> M (event)
//   finish:           C -> S (event), S -> M (event)
// Variants (one per process): 1 the full pattern; 2 no memcpy (a kernel on C instead); 3 D2H only;
// 4 H2D only; 5 copies on S (no C); 6 C joined straight to M (not through S); 7 = 1 with the S -> C
// event re-recorded per unit (one event object), 8 = 1 with C never waited on before its last copy,
// 9 = the engine's slot ring (2 slots: C prefetches unit u + 2's moments after u's write-back and S waits
// on that H2D event before u + 2's update), 10 = 1 with S also waiting on an event recorded BEFORE
// the capture began (state carried over from an eager step), 11 = 1 with S also waiting on an event it
// recorded itself (the staged engine's gather waited on the update event of its own stream).
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
  hipEvent_t pre;
  CK(hipEventCreateWithFlags(&pre, hipEventDisableTiming));
  add1<<<g, 256, 0, C>>>(slot, n);
  CK(hipEventRecord(pre, C));  // recorded outside the capture (variant 10 waits on it inside)
  CK(hipStreamSynchronize(C));
  bool h2d_pending[U] = {};
  CK(hipStreamBeginCapture(M, hipStreamCaptureModeRelaxed));
  add1<<<g, 256, 0, M>>>(d, n);
  for (int u = 0; u < U; ++u) {
    CK(hipEventRecord(order, M));
    CK(hipStreamWaitEvent(S, order, 0));
    if (v == 10 && u == 0) CK(hipStreamWaitEvent(S, pre, 0));
    if (v == 9 && h2d_pending[u]) CK(hipStreamWaitEvent(S, h2d[u], 0));
    add1<<<g, 256, 0, S>>>(slot + u * n, n);  // the update
    hipStream_t cs = v == 5 ? S : C;
    hipEvent_t e = v == 7 ? single : upd[u];
    if (v != 5) {
      CK(hipEventRecord(e, S));
      CK(hipStreamWaitEvent(C, e, 0));
    }
    if (v == 2) {
      add1<<<g, 256, 0, C>>>(slot + u * n, n);
    } else if (v == 9) {  // 2 slots: write u back, prefetch u + 2 into the same slot, S waits on it later
      CK(hipMemcpyAsync(h + u * n, slot + (u % 2) * n, bytes, hipMemcpyDeviceToHost, C));
      if (u + 2 < U) {
        CK(hipMemcpyAsync(slot + (u % 2) * n, h + (u + 2) * n, bytes, hipMemcpyHostToDevice, C));
        CK(hipEventRecord(h2d[u + 2], C));
        h2d_pending[u + 2] = true;
      }
    } else {
      if (v != 4) CK(hipMemcpyAsync(h + u * n, slot + u * n, bytes, hipMemcpyDeviceToHost, cs));
      if (v != 3) CK(hipMemcpyAsync(slot + ((u + 1) % U) * n, h + ((u + 1) % U) * n, bytes, hipMemcpyHostToDevice, cs));
    }
    if (v == 11) CK(hipStreamWaitEvent(S, e, 0));  // e was recorded on S itself, just above
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
