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

// (Measured: unrolling both passes to 4 independent 16-B loads per thread left the Gemma-3 bench
// unchanged, 483K vs 485K tok/s -- the two-pass form already streams at ~5.2 TB/s.)

// Register-resident variant for V <= 8 * CPT * 1024 (GPT-2: 50304 columns = 6.1 chunks of 8 per
// thread): a 1024-thread workgroup holds its whole row in VGPRs (packed bf16), so the logits are
// read from memory ONCE (the two-pass form above re-reads a 100 KB row that no longer sits in L2
// when 8k rows stream through) and the gradient is written once.
// Measured alternatives (GPT-2 bench, 65536 rows x 50304, MI355X): this form 2.99 ms (4.4 TB/s of
// read+write); 256 threads per row with 28 chunks each (4 rows in flight per CU) 3.47 ms (VGPR spills
// at 4 waves/SIMD); one fused (max, sum-exp) pair reduction instead of two block reductions 3.12 ms.
template <int CPT>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void xent_reg_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                        float* __restrict__ loss, int V, long ld,
                                                        const float* __restrict__ scale_ptr, float extra, int write_grad) {
  __shared__ float red[32];
  const long row = blockIdx.x;
  bf16_t* x = logits + row * ld;
  const int64_t lab = labels[row];
  const bool valid = lab >= 0 && lab < V;
  const float xl = (threadIdx.x == 0 && valid) ? bf2f(x[lab]) : 0.f;  // read before any overwrite
  const int nld8 = (int)(ld / 8);  // chunks incl. padding columns (written as 0 in the gradient)
  u16x8_t v[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 1024;
    v[i] = c < nld8 ? *reinterpret_cast<const u16x8_t*>(x + c * 8) : u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 1024;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c * 8 + j < V) m = fmaxf(m, bf2f(v[i][j]));
  }
  const float gm = block_max(m, red);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 1024;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c * 8 + j < V) s += __expf(bf2f(v[i][j]) - gm);
  }
  __syncthreads();
  const float gs = block_sum(s, red);
  const float lse = gm + __logf(gs);
  if (threadIdx.x == 0) loss[row] = valid ? lse - xl : 0.f;
  if (!write_grad) return;
  const float sc = valid ? (scale_ptr ? *scale_ptr : 1.f) * extra : 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 1024;
    if (c >= nld8) continue;
    float g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c * 8 + j;
      float p = col < V ? __expf(bf2f(v[i][j]) - lse) : 0.f;
      if (col == lab) p -= 1.f;
      g[j] = p * sc;
    }
    store8(x + c * 8, g);
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
  const long nld8 = ld / 8;
  if (ld % 8 == 0 && nld8 <= 8L * 1024) {
    const int cpt = (int)((nld8 + 1023) / 1024);
    switch (cpt) {
#define MFT_XR(CPT) case CPT: xent_reg_kernel<CPT><<<M, 1024, 0, st>>>(logits, labels, loss, V, ld, scale, extra, write_grad); return;
      MFT_XR(1) MFT_XR(2) MFT_XR(3) MFT_XR(4) MFT_XR(5) MFT_XR(6) MFT_XR(7) MFT_XR(8)
#undef MFT_XR
      default: break;
    }
  }
  xent_kernel<<<M, 256, 0, st>>>(logits, labels, loss, V, ld, scale, extra, write_grad);
}

void logsoftmax_gather(const bf16_t* logits, const int64_t* idx, float* out, long M, int V, long ld, int nidx,
                       hipStream_t st) {
  if (M <= 0) return;
  logsoftmax_gather_kernel<<<M, 256, 0, st>>>(logits, idx, out, V, ld, nidx);
}

}  // namespace mft
