// Token (+ position) embedding gather and its scatter-add backward.
// Replaces GPT2Model::embedding_lookup + the in-place wpe add (graph/gpt2_model.cpp:346-381,
// :500-528; no autograd there — SURVEY §8 Q5) and Gemma's embed*sqrt(H) (graph/gemma_model.cpp:222-259).
// Forward: one wave per token row, 16-B vector copies.  Backward: fp32 atomics for the token table
// (rows are ~random, one 256-B contiguous atomic wave-instruction per chunk group) and a
// deterministic per-position column reduction over the batch for wpe.
#include "common.h"
#include "kernels.h"

namespace mft {

__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ wte,
                                                        const bf16_t* __restrict__ wpe, bf16_t* __restrict__ out, long M,
                                                        int C, int S, int pos0, float scale) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const long id = ids[row];
  const int pos = pos0 + (int)(row % S);
  for (int c = lane * 8; c < C; c += 64 * 8) {
    float a[8];
    load8(wte + id * C + c, a);
    if (scale != 1.f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = bf2f(f2bf(a[j] * scale));
    }
    if (wpe) {
      float p[8];
      load8(wpe + (long)pos * C + c, p);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += p[j];
    }
    store8(out + row * C + c, a);
  }
}

__global__ __launch_bounds__(256) void embed_bwd_wte_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ dout,
                                                            float* __restrict__ dwte, long M, int C, float scale) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const long id = ids[row];
  for (int c = lane; c < C; c += 64) atomicAdd(dwte + id * C + c, bf2f(dout[row * C + c]) * scale);
}

// dwpe[pos0 + s, c] += sum_b dout[b*S + s, c]: block (s, 256-column strip) = 32 x 8-column chunks x 8
// batch lanes, each lane with 8 independent 16-B loads in flight, folded through LDS in a fixed order
// (deterministic).  (A thread per column walking all nb rows one 2-B load at a time: 1.13 ms per
// gpt2-full step for 201 MB.)  C % 8 == 0.
__global__ __launch_bounds__(256) void embed_bwd_wpe_kernel(const bf16_t* __restrict__ dout, float* __restrict__ dwpe,
                                                            long M, int C, int S, int pos0) {
  __shared__ float red[8][256 + 4];
  const int s = blockIdx.x, cc = threadIdx.x & 31, bl = threadIdx.x >> 5;
  const int c = blockIdx.y * 256 + cc * 8;
  const long nb = M / S;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < C) {
    long b = bl;
    for (; b + 56 < nb; b += 64) {
      u16x8_t q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] = *reinterpret_cast<const u16x8_t*>(dout + ((b + 8 * u) * S + s) * C + c);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(q[u][j]);
    }
    for (; b < nb; b += 8) {
      float v[8];
      load8(dout + (b * S + s) * C + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[bl][cc * 8 + j] = acc[j];
  __syncthreads();
  const int col = blockIdx.y * 256 + threadIdx.x;
  if (col < C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][threadIdx.x];
    dwpe[(long)(pos0 + s) * C + col] += t;
  }
}

// Deterministic token-table gradient: block b owns vocab rows [b*16, b*16 + 16) and walks ALL token
// rows in ascending order, adding the rows whose id it owns (fp32, LDS accumulators) -- every
// dwte element is summed in the same order on every run.  Only for the deterministic mode (it reads
// the id list once per block: V/16 passes over M int64 ids, L2-resident).
constexpr int kDetRows = 16;
__global__ __launch_bounds__(256) void embed_bwd_wte_det_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ dout,
                                                                float* __restrict__ dwte, long M, int C, long V, float scale) {
  extern __shared__ float acc[];  // [kDetRows][C]
  const long v0 = (long)blockIdx.x * kDetRows;
  for (int i = threadIdx.x; i < kDetRows * C; i += blockDim.x) acc[i] = 0.f;
  __syncthreads();
  for (long m0 = 0; m0 < M; m0 += 256) {
    const long m = m0 + threadIdx.x;
    const long id = m < M ? ids[m] : -1;
    const bool mine = id >= v0 && id < v0 + kDetRows;
    // the block's rows of this 256-token window, processed in token order (one row at a time)
    __shared__ int hit[256];
    hit[threadIdx.x] = mine ? (int)(id - v0) : -1;
    __syncthreads();
    for (int t = 0; t < 256 && m0 + t < M; ++t) {
      const int r = hit[t];
      if (r < 0) continue;
      const bf16_t* src = dout + (m0 + t) * C;
      for (int c = threadIdx.x; c < C; c += blockDim.x) acc[r * C + c] += bf2f(src[c]) * scale;
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < kDetRows * C; i += blockDim.x) {
    const long v = v0 + i / C;
    if (v < V) dwte[v * C + (i % C)] += acc[i];
  }
}

void embed_fwd(const int64_t* ids, const bf16_t* wte, const bf16_t* wpe, bf16_t* out, long M, int C, int S, int pos0,
               float scale, hipStream_t st) {
  embed_fwd_kernel<<<cdiv(M, 4), 256, 0, st>>>(ids, wte, wpe, out, M, C, S, pos0, scale);
}

void embed_bwd(const int64_t* ids, const bf16_t* dout, float* dwte, float* dwpe, long M, int C, int S, int pos0,
               float scale, hipStream_t st, long det_vocab) {
  if (dwte && det_vocab > 0) {
    const size_t shm = sizeof(float) * kDetRows * C;
    embed_bwd_wte_det_kernel<<<cdiv(det_vocab, kDetRows), 256, shm, st>>>(ids, dout, dwte, M, C, det_vocab, scale);
  } else if (dwte) {
    embed_bwd_wte_kernel<<<cdiv(M, 4), 256, 0, st>>>(ids, dout, dwte, M, C, scale);
  }
  if (dwpe) {
    if (C % 8) {
      fprintf(stderr, "mft::embed_bwd: the position-table gradient needs C %% 8 == 0 (C=%d)\n", C);
      abort();
    }
    embed_bwd_wpe_kernel<<<dim3(S, cdiv(C, 256)), 256, 0, st>>>(dout, dwpe, M, C, S, pos0);
  }
}

}  // namespace mft
