// Fused softmax cross-entropy forward+backward over a (chunk of) bf16 logits rows.
// Replaces lm_cross_entropy + LMCrossEntropyBackward (core/lm_loss.cpp:19-210): the reference
// materialises fp32 logits [B,S,V], then recomputes the softmax per row in backward.  Here one
// workgroup per row does ONE online (max, sum-exp) pass and ONE pass that overwrites the logits
// in place with (softmax - onehot) * scale, so a chunk of logits sized to stay in the 256 MiB
// Infinity Cache is written by the LM-head GEMM, read twice here and consumed by the dgrad GEMM
// without a round trip to HBM (see ops/lm_head.py for the chunking).
#include "common.h"
#include "kernels.h"

namespace mft {

__global__ __launch_bounds__(256) void xent_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                   float* __restrict__ loss, int V, long ld,
                                                   const float* __restrict__ scale_ptr, float extra, int write_grad) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  bf16_t* x = logits + row * ld;
  const int64_t lab = labels[row];
  const int nv8 = V / 8;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < nv8; c += blockDim.x) {
    float v[8];
    load8(x + c * 8, v);
    float lm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
    if (lm > m) {
      s *= __expf(m - lm);
      m = lm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
  }
  for (int c = nv8 * 8 + threadIdx.x; c < V; c += blockDim.x) {
    const float v = bf2f(x[c]);
    if (v > m) {
      s *= __expf(m - v);
      m = v;
    }
    s += __expf(v - m);
  }
  const float gm = block_max(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  __syncthreads();
  const float gs = block_sum(s, red);
  const float lse = gm + __logf(gs);
  const bool valid = lab >= 0 && lab < V;
  if (threadIdx.x == 0) loss[row] = valid ? lse - bf2f(x[lab]) : 0.f;
  if (!write_grad) return;
  __syncthreads();  // the label logit must be read before anyone overwrites it
  const float sc = valid ? (scale_ptr ? *scale_ptr : 1.f) * extra : 0.f;
  for (int c = threadIdx.x; c < nv8; c += blockDim.x) {
    float v[8];
    load8(x + c * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(v[j] - lse);
      if (c * 8 + j == lab) p -= 1.f;
      v[j] = p * sc;
    }
    store8(x + c * 8, v);
  }
  for (long c = nv8 * 8 + threadIdx.x; c < ld; c += blockDim.x) {
    if (c < V) {
      float p = __expf(bf2f(x[c]) - lse);
      if (c == lab) p -= 1.f;
      x[c] = f2bf(p * sc);
    } else {
      x[c] = 0;
    }
  }
}

// out[m, c] = logits[m, idx[c]] - logsumexp(logits[m, :V])
__global__ __launch_bounds__(256) void logsoftmax_gather_kernel(const bf16_t* __restrict__ logits,
                                                                const int64_t* __restrict__ idx, float* __restrict__ out,
                                                                int V, long ld, int nidx) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < V; c += blockDim.x) {
    const float v = bf2f(x[c]);
    if (v > m) {
      s *= __expf(m - v);
      m = v;
    }
    s += __expf(v - m);
  }
  const float gm = block_max(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  __syncthreads();
  const float gs = block_sum(s, red);
  const float lse = gm + __logf(gs);
  for (int c = threadIdx.x; c < nidx; c += blockDim.x) out[row * nidx + c] = bf2f(x[idx[c]]) - lse;
}

void xent_fwd_bwd(bf16_t* logits, const int64_t* labels, float* loss, long M, int V, long ld, const float* scale,
                  float extra, int write_grad, hipStream_t st) {
  if (M <= 0) return;
  xent_kernel<<<M, 256, 0, st>>>(logits, labels, loss, V, ld, scale, extra, write_grad);
}

void logsoftmax_gather(const bf16_t* logits, const int64_t* idx, float* out, long M, int V, long ld, int nidx,
                       hipStream_t st) {
  if (M <= 0) return;
  logsoftmax_gather_kernel<<<M, 256, 0, st>>>(logits, idx, out, V, ld, nidx);
}

}  // namespace mft
