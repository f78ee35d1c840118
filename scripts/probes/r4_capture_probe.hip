// Which stream-capture construction makes hipStreamEndCapture crash?  One variant per process:
//   1  fork a side stream (event), a kernel on it, join back
//   2  + H2D hipMemcpyAsync from hipHostMalloc memory on the side stream
//   3  + D2H hipMemcpyAsync to hipHostMalloc memory on a second side stream
//   4  + one join event recorded on three side streams in turn
//   5  + the side streams ran unsynchronised eager work just before the capture
//   6  + an event recorded twice on one side stream, waited on by another stream in between
//   7  4 + a stream waits on another's event and is joined with no node of its own after the wait
//   9  8 with a fresh event for the second record
//  10  3 + a back edge: stream a waits on an event of b (which waited on a) and adds a kernel
//   8  4 + an event re-recorded (recorded, waited on, recorded on another stream, waited on), every
//      waiting stream adding a node before its own join
// Prints "variant N ok" after instantiate + 2 replays + a check of the copied data.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                         \
    }                                                                                       \
  } while (0)

__global__ void add1(float* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.f;
}

int main(int argc, char** argv) {
  const int v = argc > 1 ? std::atoi(argv[1]) : 1;
  const int n = 1 << 16;
  const size_t bytes = n * sizeof(float);
  hipStream_t s0, a, b, c;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  hipEvent_t fork, join, e1, e2, ev[3];
  for (hipEvent_t* e : {&fork, &join, &e1, &e2, &ev[0], &ev[1], &ev[2]})
    CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  float *d, *d2, *h;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&d2, bytes));
  CK(hipHostMalloc((void**)&h, bytes, hipHostMallocDefault));
  for (int i = 0; i < n; ++i) h[i] = (float)i;
  CK(hipMemset(d, 0, bytes));
  CK(hipDeviceSynchronize());
  if (v >= 5) {  // eager side-stream work left running
    CK(hipMemcpyAsync(d2, h, bytes, hipMemcpyHostToDevice, a));
    add1<<<n / 256, 256, 0, c>>>(d2, n);
    CK(hipMemcpyAsync(h, d2, bytes, hipMemcpyDeviceToHost, b));
    CK(hipStreamSynchronize(b));
    CK(hipStreamSynchronize(a));
    CK(hipStreamSynchronize(c));
    for (int i = 0; i < n; ++i) h[i] = (float)i;
    CK(hipMemcpyAsync(d2, h, bytes, hipMemcpyHostToDevice, a));  // still in flight at capture start
  }
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
  add1<<<n / 256, 256, 0, s0>>>(d, n);
  CK(hipEventRecord(fork, s0));
  CK(hipStreamWaitEvent(a, fork, 0));
  if (v >= 2) {
    CK(hipMemcpyAsync(d2, h, bytes, hipMemcpyHostToDevice, a));
    CK(hipEventRecord(e1, a));
  }
  add1<<<n / 256, 256, 0, a>>>(v >= 2 ? d2 : d, n);
  if (v >= 3) {
    CK(hipEventRecord(e2, a));
    CK(hipStreamWaitEvent(b, fork, 0));
    CK(hipStreamWaitEvent(b, e2, 0));
    CK(hipMemcpyAsync(h, d2, bytes, hipMemcpyDeviceToHost, b));
  }
  if (v == 10) {
    CK(hipEventRecord(ev[2], b));
    CK(hipStreamWaitEvent(a, ev[2], 0));
    add1<<<n / 256, 256, 0, a>>>(d, n);
  }
  if (v == 7) {
    CK(hipStreamWaitEvent(c, fork, 0));
    add1<<<n / 256, 256, 0, c>>>(d, n);
    CK(hipEventRecord(ev[0], c));
    CK(hipStreamWaitEvent(a, ev[0], 0));  // a's tail: its own kernel + c's kernel
  }
  if (v == 8 || v == 9) {
    CK(hipStreamWaitEvent(c, fork, 0));
    CK(hipEventRecord(ev[0], b));
    CK(hipStreamWaitEvent(c, ev[0], 0));
    add1<<<n / 256, 256, 0, c>>>(d, n);
    hipEvent_t e = v == 9 ? ev[2] : ev[0];
    CK(hipEventRecord(e, c));
    CK(hipStreamWaitEvent(a, e, 0));
    add1<<<n / 256, 256, 0, a>>>(d2, n);
  }
  if (v == 6) {  // event reuse: recorded, waited on, recorded again
    CK(hipStreamWaitEvent(c, fork, 0));
    CK(hipEventRecord(ev[0], b));
    CK(hipStreamWaitEvent(c, ev[0], 0));
    add1<<<n / 256, 256, 0, c>>>(d, n);
    CK(hipEventRecord(ev[0], c));
    CK(hipStreamWaitEvent(a, ev[0], 0));
  }
  if (v >= 4) {
    for (hipStream_t s : {a, b, c}) {
      if (s == c && v < 6) continue;  // (c joins in 6-8)
      CK(hipEventRecord(join, s));
      CK(hipStreamWaitEvent(s0, join, 0));
    }
  } else {
    CK(hipEventRecord(join, a));
    CK(hipStreamWaitEvent(s0, join, 0));
    if (v >= 3) {
      CK(hipEventRecord(ev[1], b));
      CK(hipStreamWaitEvent(s0, ev[1], 0));
    }
  }
  std::fprintf(stderr, "variant %d: ending capture\n", v);
  hipGraph_t g;
  CK(hipStreamEndCapture(s0, &g));
  std::fprintf(stderr, "variant %d: instantiating\n", v);
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  for (int r = 0; r < 2; ++r) CK(hipGraphLaunch(x, s0));
  CK(hipStreamSynchronize(s0));
  CK(hipDeviceSynchronize());
  if (v >= 3 && v != 8 && v != 9 && h[7] != 9.f) {
    std::fprintf(stderr, "variant %d: h[7] = %g (expected 9)\n", v, h[7]);
    return 1;
  }
  std::printf("variant %d ok\n", v);
  return 0;
}
