// Flash attention forward / backward on MFMA (gfx950, wave64, v_mfma_f32_16x16x32_bf16).
//
// Replaces the reference's attention paths:
//   * core/memory_efficient_attention.cpp:40-185 (two-pass per-row online softmax, fwd only,
//     backward returns zeros — SURVEY §8 Q3),
//   * graph/gpt2_model.cpp:679-711 and graph/gemma_model.cpp:481-508 (dense S x S scores,
//     masks, softmax, repeat_kv for GQA, core/ops.cpp:2072-2149).
// Supported: causal, sliding window (Gemma-3 local layers), right padding via per-batch key
// lengths, GQA (kv head = q head / group) without materialising repeated K/V, arbitrary softmax
// scale (1/sqrt(D) for GPT-2, query_pre_attn_scalar^-1/2 for Gemma), head dims 64/128/256.
//
// Layout: q/k/v are strided [B, S, H, D] views (D contiguous) so the packed QKV GEMM output is
// consumed in place (no permute/reshape copies, SURVEY §2.3 "transpose/permute"); O is written in
// [B, S, H, D] so the output projection reads it directly.  The forward also writes the row LSE
// (natural log) which the backward uses to recompute P without storing S x S.
//
// Tiling: a workgroup = 4 waves = 64 query rows (16 per wave) x one (batch, head).  K and V tiles
// of 64 keys are staged row-major in LDS with 16-B vector copies; S = Q K^T takes K by rows, and
// O += P V takes V through ds_read_b64_tr_b16 transposed reads (no transposed copy of V).
// Online softmax in base 2 with the scale folded into one multiplier.
#include "mfma.h"
#include "kernels.h"

namespace mft {

constexpr float kLog2e = 1.4426950408889634f;

struct AttnStrides {
  long sb, ss, sh;  // batch, seq, head strides (elements); D contiguous
};

template <int D>
__device__ __forceinline__ void stage_rows(bf16_t* lds, const bf16_t* src, AttnStrides st, int b, int h, int row0,
                                           int nrows_valid, int nrows) {
  // nrows x D tile -> lds[nrows][D]; rows >= nrows_valid are zero-filled.
  constexpr int CPR = D / 8;  // 16-B chunks per row
  const int total = nrows * CPR;
  for (int c = threadIdx.x; c < total; c += blockDim.x) {
    const int r = c / CPR, ch = c % CPR;
    u16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < nrows_valid) v = *reinterpret_cast<const u16x8_t*>(src + b * st.sb + (long)(row0 + r) * st.ss + h * st.sh + ch * 8);
    *reinterpret_cast<u16x8_t*>(lds + r * D + ch * 8) = v;
  }
}

__device__ __forceinline__ bool attn_allowed(int qi, int kj, int kv_len, int causal_off, int causal, int window) {
  if (kj >= kv_len) return false;
  if (causal && kj > qi + causal_off) return false;
  if (window > 0 && qi + causal_off - kj >= window) return false;
  return true;
}

template <int D>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                       const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                       float* __restrict__ lse, AttnStrides qs, AttnStrides ks,
                                                       AttnStrides vs, AttnStrides os, int H, int Hkv, int Sq, int Sk,
                                                       float scale, int causal, int window,
                                                       const int* __restrict__ kv_lens) {
  constexpr int BQ = 64, BK = 64, LDP = BK + 8;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* Ks = smem;                // [BK][D]
  bf16_t* Vs = Ks + BK * D;         // [BK][D]
  bf16_t* Ps = Vs + BK * D;         // [4][16][LDP]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * BQ;
  const int hk = h / (H / Hkv);
  const int kv_len = kv_lens ? min(kv_lens[b], Sk) : Sk;
  const int coff = Sk - Sq;  // bottom-right aligned causal mask
  const float c2 = scale * kLog2e;
  bf16_t* Pw = Ps + w * 16 * LDP;

  // Q fragments (A operand, rows = this wave's 16 queries) straight from global into registers.
  bf16x8_t qf[D / 32];
  {
    const int qr = q0 + 16 * w + (lane & 15);
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      if (qr < Sq)
        qf[s] = *reinterpret_cast<const bf16x8_t*>(q + b * qs.sb + (long)qr * qs.ss + h * qs.sh + s * 32 + 8 * (lane >> 4));
      else
        qf[s] = bf16x8_t{};
    }
  }
  float m[4], l[4];
  f32x4_t acc[D / 16];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m[i] = -INFINITY; l[i] = 0.f; }
#pragma unroll
  for (int n = 0; n < D / 16; ++n) acc[n] = zero4();

  int kend = kv_len;
  if (causal) kend = min(kend, q0 + BQ + coff);
  int kstart = 0;
  if (window > 0) kstart = max(0, (q0 + coff - window + 1) / BK * BK);

  for (int kb = kstart; kb < kend; kb += BK) {
    __syncthreads();
    const int nvalid = min(BK, kv_len - kb);
    stage_rows<D>(Ks, k, ks, b, hk, kb, nvalid, BK);
    stage_rows<D>(Vs, v, vs, b, hk, kb, nvalid, BK);
    __syncthreads();
    // S = Q K^T  (16 x 64 per wave)
    f32x4_t sacc[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      sacc[nb] = zero4();
#pragma unroll
      for (int s = 0; s < D / 32; ++s) sacc[nb] = mfma16(qf[s], frag_row(Ks, D, nb * 16, s * 32), sacc[nb]);
    }
    // mask + online softmax (rows 4*(lane>>4)+i, cols nb*16 + (lane&15))
    const bool need_mask = (kb + BK > kv_len) || (causal && kb + BK - 1 > q0 + 16 * w + coff) ||
                           (window > 0 && q0 + 16 * w + 15 + coff - kb >= window);
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qi = q0 + 16 * w + 4 * (lane >> 4) + i;
      float mx = -INFINITY;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        float sv = sacc[nb][i] * c2;
        if (need_mask && !attn_allowed(qi, kb + nb * 16 + (lane & 15), kv_len, coff, causal, window)) sv = -INFINITY;
        sacc[nb][i] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
      const float mnew = fmaxf(m[i], mx);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      alpha[i] = exp2f(m[i] - msafe);
      float rs = 0.f;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const float p = exp2f(sacc[nb][i] - msafe);
        sacc[nb][i] = p;
        rs += p;
      }
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) rs += __shfl_xor(rs, o2, 64);
      l[i] = l[i] * alpha[i] + rs;
      m[i] = mnew;
    }
#pragma unroll
    for (int n = 0; n < D / 16; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[n][i] *= alpha[i];
    // P (C layout) -> per-wave LDS scratch -> A operand
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) Pw[(4 * (lane >> 4) + i) * LDP + nb * 16 + (lane & 15)] = f2bf(sacc[nb][i]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    bf16x8_t pa0 = frag_row(Pw, LDP, 0, 0);
    bf16x8_t pa1 = frag_row(Pw, LDP, 0, 32);
#pragma unroll
    for (int n = 0; n < D / 16; ++n) {
      acc[n] = mfma16(pa0, frag_tr(Vs, D, 0, n * 16), acc[n]);
      acc[n] = mfma16(pa1, frag_tr(Vs, D, 32, n * 16), acc[n]);
    }
  }
  // epilogue
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qi = q0 + 16 * w + 4 * (lane >> 4) + i;
    const float inv = l[i] > 0.f ? 1.f / l[i] : 0.f;
    if (qi < Sq) {
      bf16_t* orow = o + b * os.sb + (long)qi * os.ss + h * os.sh;
#pragma unroll
      for (int n = 0; n < D / 16; ++n) orow[n * 16 + (lane & 15)] = f2bf(acc[n][i] * inv);
      if ((lane & 15) == 0)
        lse[((long)b * H + h) * Sq + qi] = l[i] > 0.f ? (m[i] + log2f(l[i])) / kLog2e : 1e30f;
    }
  }
}

// delta[b,h,i] = sum_d dO[b,i,h,d] * O[b,i,h,d]; D/8 consecutive lanes share one row so every row
// is read as contiguous 16-B pieces (a thread-per-row form strides the rows across lanes).
template <int D>
__global__ void attn_bwd_delta_kernel(const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
                                      float* __restrict__ delta, AttnStrides os, AttnStrides ds, int B, int H, int Sq) {
  constexpr int LPR = D / 8;  // lanes per row
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long idx = t / LPR;
  const int c = (int)(t % LPR) * 8;
  const bool ok = idx < (long)B * H * Sq;
  float s = 0.f;
  if (ok) {
    const int i = idx % Sq, h = (idx / Sq) % H, b = idx / ((long)Sq * H);
    float a[8], g[8];
    load8(o + b * os.sb + (long)i * os.ss + h * os.sh + c, a);
    load8(dout + b * ds.sb + (long)i * ds.ss + h * ds.sh + c, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] * g[j];
  }
#pragma unroll
  for (int off = 1; off < LPR; off <<= 1) s += __shfl_xor(s, off, 64);
  if (ok && c == 0) delta[idx] = s;
}

// Backward: one workgroup = 64 keys of one (batch, q-head); 4 waves x 16 keys.  dK/dV for the
// workgroup's keys live in registers across the sweep over query blocks; dQ is accumulated with
// fp32 atomics into a [B, Sq, H, D] buffer.  With GQA (H > Hkv) dK/dV are written per q-head into
// an expanded buffer and summed over the group afterwards (gqa_reduce), which keeps
// B*H*Sk/64 workgroups in flight (Gemma-3 has Hkv = 1).
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    float* __restrict__ dq_acc, bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, AttnStrides qs, AttnStrides ks,
    AttnStrides vs, AttnStrides dos, AttnStrides dks, AttnStrides dvs, int H, int Hkv, int Sq, int Sk, float scale,
    int causal, int window, const int* __restrict__ kv_lens, int dkv_per_qhead) {
  constexpr int BQ = 64, BK = 64, LDT = BQ + 8;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* Ks = smem;             // [BK][D]
  bf16_t* Vs = Ks + BK * D;      // [BK][D]
  bf16_t* Qs = Vs + BK * D;      // [BQ][D]
  bf16_t* dOs = Qs + BQ * D;     // [BQ][D]
  bf16_t* PT = dOs + BQ * D;     // [BK][LDT]  P^T
  bf16_t* DST = PT + BK * LDT;   // [BK][LDT]  dS^T * scale
  float* lse_s = reinterpret_cast<float*>(DST + BK * LDT);  // [BQ]
  float* del_s = lse_s + BQ;                                 // [BQ]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.z, h = blockIdx.y, kb = blockIdx.x * BK;
  const int hk = h / (H / Hkv);
  const int kv_len = kv_lens ? min(kv_lens[b], Sk) : Sk;
  const int coff = Sk - Sq;
  const float c2 = scale * kLog2e;

  const int nkv = max(0, min(BK, kv_len - kb));
  stage_rows<D>(Ks, k, ks, b, hk, kb, nkv, BK);
  stage_rows<D>(Vs, v, vs, b, hk, kb, nkv, BK);

  f32x4_t dKa[D / 16], dVa[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) { dKa[n] = zero4(); dVa[n] = zero4(); }

  // query range that can see this key block
  int qstart = 0, qend = Sq;
  if (causal) qstart = max(0, kb - coff) / BQ * BQ;
  if (window > 0) qend = min(Sq, kb + BK - 1 - coff + window);
  if (nkv <= 0) qend = qstart;  // fully padded key block: grads are zero

  for (int q0 = qstart; q0 < qend; q0 += BQ) {
    __syncthreads();
    const int nq = min(BQ, Sq - q0);
    stage_rows<D>(Qs, q, qs, b, h, q0, nq, BQ);
    stage_rows<D>(dOs, dout, dos, b, h, q0, nq, BQ);
    if (threadIdx.x < BQ) {
      const int qi = q0 + threadIdx.x;
      lse_s[threadIdx.x] = qi < Sq ? lse[((long)b * H + h) * Sq + qi] * kLog2e : 1e30f;
      del_s[threadIdx.x] = qi < Sq ? delta[((long)b * H + h) * Sq + qi] : 0.f;
    }
    __syncthreads();
    // S^T = K Q^T and dP^T = V dO^T : 16 keys (rows) x 64 queries (cols) per wave
    f32x4_t st[4], dpt[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      st[nb] = zero4();
      dpt[nb] = zero4();
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
        st[nb] = mfma16(frag_row(Ks, D, 16 * w, s * 32), frag_row(Qs, D, nb * 16, s * 32), st[nb]);
        dpt[nb] = mfma16(frag_row(Vs, D, 16 * w, s * 32), frag_row(dOs, D, nb * 16, s * 32), dpt[nb]);
      }
    }
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int qc = nb * 16 + (lane & 15);
      const int qi = q0 + qc;
      const float lq = lse_s[qc], dq = del_s[qc];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kr = 16 * w + 4 * (lane >> 4) + i;
        const bool ok = qi < Sq && attn_allowed(qi, kb + kr, kv_len, coff, causal, window);
        const float p = ok ? exp2f(st[nb][i] * c2 - lq) : 0.f;
        const float ds = p * (dpt[nb][i] - dq) * scale;
        PT[kr * LDT + qc] = f2bf(p);
        DST[kr * LDT + qc] = f2bf(ds);
      }
    }
    __syncthreads();
    // dV += P^T dO ; dK += dS^T Q   (A by rows from the scratch, B transposed from row-major tiles)
#pragma unroll
    for (int s = 0; s < BQ / 32; ++s) {
      const bf16x8_t pa = frag_row(PT, LDT, 16 * w, s * 32);
      const bf16x8_t da = frag_row(DST, LDT, 16 * w, s * 32);
#pragma unroll
      for (int n = 0; n < D / 16; ++n) {
        dVa[n] = mfma16(pa, frag_tr(dOs, D, s * 32, n * 16), dVa[n]);
        dKa[n] = mfma16(da, frag_tr(Qs, D, s * 32, n * 16), dKa[n]);
      }
    }
    // dQ[q][d] += dS[q][key] K[key][d] for this wave's 16 query rows, fp32 atomics
    {
      const bf16x8_t a0 = frag_tr(DST, LDT, 0, 16 * w);
      const bf16x8_t a1 = frag_tr(DST, LDT, 32, 16 * w);
#pragma unroll
      for (int n = 0; n < D / 16; ++n) {
        f32x4_t c = zero4();
        c = mfma16(a0, frag_tr(Ks, D, 0, n * 16), c);
        c = mfma16(a1, frag_tr(Ks, D, 32, n * 16), c);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qi = q0 + 16 * w + 4 * (lane >> 4) + i;
          if (qi < Sq) atomicAdd(dq_acc + (((long)b * Sq + qi) * H + h) * D + n * 16 + (lane & 15), c[i]);
        }
      }
    }
  }
  // write dK, dV (bf16) for valid keys
  const int hout = dkv_per_qhead ? h : hk;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kr = kb + 16 * w + 4 * (lane >> 4) + i;
    if (kr < Sk) {
      bf16_t* dkr = dk + b * dks.sb + (long)kr * dks.ss + hout * dks.sh;
      bf16_t* dvr = dv + b * dvs.sb + (long)kr * dvs.ss + hout * dvs.sh;
#pragma unroll
      for (int n = 0; n < D / 16; ++n) {
        dkr[n * 16 + (lane & 15)] = f2bf(dKa[n][i]);
        dvr[n * 16 + (lane & 15)] = f2bf(dVa[n][i]);
      }
    }
  }
}

// dq (bf16, strided) = dq_acc (fp32, contiguous [B,Sq,H,D])
__global__ void attn_dq_convert_kernel(const float* __restrict__ acc, bf16_t* __restrict__ dq, AttnStrides s, int B,
                                       int Sq, int H, int D) {
  const long idx8 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  const long total = (long)B * Sq * H * D;
  if (idx8 >= total) return;
  const int d = idx8 % D;
  const int h = (idx8 / D) % H;
  const int i = (idx8 / ((long)D * H)) % Sq;
  const int b = idx8 / ((long)D * H * Sq);
  const float4* a4 = reinterpret_cast<const float4*>(acc + idx8);
  float4 x = a4[0], y = a4[1];
  float f[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
  store8(dq + b * s.sb + (long)i * s.ss + h * s.sh + d, f);
}

// GQA: out[b,s,hk,:] = sum_g in[b,s,hk*G+g,:]   (in contiguous [B,S,H,D] bf16, out strided)
__global__ void gqa_reduce_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out, AttnStrides s, int B, int S,
                                  int H, int Hkv, int D) {
  const long idx8 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  const long total = (long)B * S * Hkv * D;
  if (idx8 >= total) return;
  const int G = H / Hkv;
  const int d = idx8 % D;
  const int hk = (idx8 / D) % Hkv;
  const int i = (idx8 / ((long)D * Hkv)) % S;
  const int b = idx8 / ((long)D * Hkv * S);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int g = 0; g < G; ++g) {
    float t[8];
    load8(in + (((long)b * S + i) * H + hk * G + g) * D + d, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += t[j];
  }
  store8(out + b * s.sb + (long)i * s.ss + hk * s.sh + d, acc);
}

// ============================================================================================
// Short-sequence path: Sq == Sk <= 128, D == 64, no sliding window (GPT-2 fine-tuning at seq 128).
// One workgroup = one (batch, head), 8 waves.  K and V (and for the backward Q, dO) are staged
// ONCE into LDS, so nothing is re-read across query/key blocks, the whole score row lives in
// registers (no online rescaling), the backward needs no dQ atomics or fp32 dQ workspace (dS^T is
// shared through LDS and dQ is formed in a second phase inside the same workgroup), and delta
// (rowsum dO*O) is computed while staging.  Outputs go through a per-wave LDS tile so every global
// store is a 16-B row piece.
// ============================================================================================
constexpr int kShortS = 128;

__host__ __device__ constexpr int short_ldp() { return kShortS + 8; }

// per-wave [16][D] C-layout tile (acc[n][i] = row 4(l>>4)+i, col n*16+(l&15)) -> 16 global rows
template <int D>
__device__ __forceinline__ void store_tile16(bf16_t* scratch, int ld, const f32x4_t* acc, const float* rs,
                                             bf16_t* dst, AttnStrides st, int b, int h, int row0, int nrows) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int n = 0; n < D / 16; ++n)
#pragma unroll
    for (int i = 0; i < 4; ++i) scratch[(4 * (lane >> 4) + i) * ld + n * 16 + (lane & 15)] = f2bf(acc[n][i] * rs[i]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  constexpr int CPR = D / 8;             // 16-B pieces per row
  for (int c = lane; c < 16 * CPR; c += 64) {
    const int r = c / CPR, ch = c % CPR;
    if (r < nrows)
      *reinterpret_cast<u16x8_t*>(dst + b * st.sb + (long)(row0 + r) * st.ss + h * st.sh + ch * 8) =
          *reinterpret_cast<const u16x8_t*>(scratch + r * ld + ch * 8);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int D>
__global__ __launch_bounds__(512) void attn_fwd_short_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                             const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                             float* __restrict__ lse, AttnStrides qs, AttnStrides ks,
                                                             AttnStrides vs, AttnStrides os, int H, int Hkv, int S,
                                                             float scale, int causal, const int* __restrict__ kv_lens) {
  constexpr int SM = kShortS, LDP = short_ldp(), NB = SM / 16, CPR = D / 8;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* Ks = smem;            // [SM][D]
  bf16_t* Vs = Ks + SM * D;     // [SM][D]
  bf16_t* Pw = Vs + SM * D + (threadIdx.x >> 6) * 16 * LDP;  // per-wave [16][LDP]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = blockIdx.x, b = blockIdx.y, hk = h / (H / Hkv);
  const int kv_len = kv_lens ? min(kv_lens[b], S) : S;
  const float c2 = scale * kLog2e;
  // issue every global load first (K, V pieces and this wave's Q fragments), then fill LDS
  constexpr int PER = SM * CPR / 512;
  u16x8_t kr[PER], vr[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = threadIdx.x + j * 512, r = c / CPR, ch = c % CPR;
    const bool ok = r < S;
    kr[j] = ok ? *reinterpret_cast<const u16x8_t*>(k + b * ks.sb + (long)r * ks.ss + hk * ks.sh + ch * 8) : u16x8_t{};
    vr[j] = ok ? *reinterpret_cast<const u16x8_t*>(v + b * vs.sb + (long)r * vs.ss + hk * vs.sh + ch * 8) : u16x8_t{};
  }
  bf16x8_t qf[D / 32];
  {
    const int qr = 16 * w + (lane & 15);
#pragma unroll
    for (int s = 0; s < D / 32; ++s)
      qf[s] = qr < S ? *reinterpret_cast<const bf16x8_t*>(q + b * qs.sb + (long)qr * qs.ss + h * qs.sh + s * 32 + 8 * (lane >> 4))
                     : bf16x8_t{};
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = threadIdx.x + j * 512, r = c / CPR, ch = c % CPR;
    *reinterpret_cast<u16x8_t*>(Ks + r * D + ch * 8) = kr[j];
    *reinterpret_cast<u16x8_t*>(Vs + r * D + ch * 8) = vr[j];
  }
  __syncthreads();
  if (16 * w >= S) return;  // no query rows for this wave (after the only barrier)
  const int nbmax = causal ? w + 1 : NB;  // key blocks of 16 visible to rows 16w..16w+15
  f32x4_t sacc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    sacc[nb] = zero4();
    if (nb < nbmax) {
#pragma unroll
      for (int s = 0; s < D / 32; ++s) sacc[nb] = mfma16(qf[s], frag_row(Ks, D, nb * 16, s * 32), sacc[nb]);
    }
  }
  float mrow[4], lrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qi = 16 * w + 4 * (lane >> 4) + i;
    float mx = -INFINITY;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int kj = nb * 16 + (lane & 15);
      const bool ok = nb < nbmax && kj < kv_len && (!causal || kj <= qi);
      const float sv = ok ? sacc[nb][i] * c2 : -INFINITY;
      sacc[nb][i] = sv;
      mx = fmaxf(mx, sv);
    }
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
    const float ms = mx == -INFINITY ? 0.f : mx;
    float rs = 0.f;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const float p = exp2f(sacc[nb][i] - ms);
      sacc[nb][i] = p;
      rs += p;
    }
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) rs += __shfl_xor(rs, o2, 64);
    mrow[i] = mx;
    lrow[i] = rs;
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) Pw[(4 * (lane >> 4) + i) * LDP + nb * 16 + (lane & 15)] = f2bf(sacc[nb][i]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  f32x4_t acc[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) acc[n] = zero4();
  const int ksmax = causal ? (16 * w + 15) / 32 + 1 : SM / 32;
#pragma unroll
  for (int kk = 0; kk < SM / 32; ++kk) {
    if (kk < ksmax) {
      const bf16x8_t pa = frag_row(Pw, LDP, 0, kk * 32);
#pragma unroll
      for (int n = 0; n < D / 16; ++n) acc[n] = mfma16(pa, frag_tr(Vs, D, kk * 32, n * 16), acc[n]);
    }
  }
  float inv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    inv[i] = lrow[i] > 0.f ? 1.f / lrow[i] : 0.f;
    const int qi = 16 * w + 4 * (lane >> 4) + i;
    if ((lane & 15) == 0 && qi < S)
      lse[((long)b * H + h) * S + qi] = lrow[i] > 0.f ? (mrow[i] + log2f(lrow[i])) / kLog2e : 1e30f;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  store_tile16<D>(Pw, LDP, acc, inv, o, os, b, h, 16 * w, min(16, S - 16 * w));
}

template <int D>
__global__ __launch_bounds__(512) void attn_bwd_short_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    bf16_t* __restrict__ dq, bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, AttnStrides qs, AttnStrides ks,
    AttnStrides vs, AttnStrides ost, AttnStrides dos, AttnStrides dqs, AttnStrides dks, AttnStrides dvs, int H, int Hkv,
    int S, float scale, int causal, const int* __restrict__ kv_lens, int dkv_per_qhead) {
  constexpr int SM = kShortS, LDT = short_ldp(), NB = SM / 16, CPR = D / 8;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* Ks = smem;              // [SM][D]
  bf16_t* Vs = Ks + SM * D;       // [SM][D]
  bf16_t* Qs = Vs + SM * D;       // [SM][D]
  bf16_t* dOs = Qs + SM * D;      // [SM][D]
  bf16_t* DST = dOs + SM * D;     // [SM keys][LDT]  dS^T * scale
  bf16_t* PTw = DST + SM * LDT + (threadIdx.x >> 6) * 16 * LDT;  // per-wave [16][LDT]
  float* lse_s = reinterpret_cast<float*>(DST + SM * LDT + 8 * 16 * LDT);  // [SM]
  float* del_s = lse_s + SM;                                             // [SM]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = blockIdx.x, b = blockIdx.y, hk = h / (H / Hkv);
  const int kv_len = kv_lens ? min(kv_lens[b], S) : S;
  const float c2 = scale * kLog2e;

  // ---- stage K, V, Q, dO; delta = rowsum(dO * O) from the same registers (CPR lanes per row)
  {
    constexpr int PER = SM * CPR / 512;
    u16x8_t kr[PER], vr[PER], qr[PER], dr[PER], orr[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = threadIdx.x + j * 512, r = c / CPR, ch = c % CPR;
      const bool ok = r < S;
      kr[j] = ok ? *reinterpret_cast<const u16x8_t*>(k + b * ks.sb + (long)r * ks.ss + hk * ks.sh + ch * 8) : u16x8_t{};
      vr[j] = ok ? *reinterpret_cast<const u16x8_t*>(v + b * vs.sb + (long)r * vs.ss + hk * vs.sh + ch * 8) : u16x8_t{};
      qr[j] = ok ? *reinterpret_cast<const u16x8_t*>(q + b * qs.sb + (long)r * qs.ss + h * qs.sh + ch * 8) : u16x8_t{};
      dr[j] = ok ? *reinterpret_cast<const u16x8_t*>(dout + b * dos.sb + (long)r * dos.ss + h * dos.sh + ch * 8) : u16x8_t{};
      orr[j] = ok ? *reinterpret_cast<const u16x8_t*>(o + b * ost.sb + (long)r * ost.ss + h * ost.sh + ch * 8) : u16x8_t{};
    }
    if (threadIdx.x < SM) lse_s[threadIdx.x] = threadIdx.x < S ? lse[((long)b * H + h) * S + threadIdx.x] * kLog2e : 1e30f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = threadIdx.x + j * 512, r = c / CPR, ch = c % CPR;
      *reinterpret_cast<u16x8_t*>(Ks + r * D + ch * 8) = kr[j];
      *reinterpret_cast<u16x8_t*>(Vs + r * D + ch * 8) = vr[j];
      *reinterpret_cast<u16x8_t*>(Qs + r * D + ch * 8) = qr[j];
      *reinterpret_cast<u16x8_t*>(dOs + r * D + ch * 8) = dr[j];
      float dsum = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum += bf2f(dr[j][e]) * bf2f(orr[j][e]);
#pragma unroll
      for (int off = 1; off < CPR; off <<= 1) dsum += __shfl_xor(dsum, off, 64);
      if (ch == 0) del_s[r] = dsum;
    }
  }
  __syncthreads();

  // ---- phase 1: wave w owns keys 16w..16w+15: P^T, dS^T rows, dV and dK
  f32x4_t dKa[D / 16], dVa[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) { dKa[n] = zero4(); dVa[n] = zero4(); }
  const int nbmin = causal ? w : 0;  // query blocks of 16 that can see these keys
  {
    f32x4_t st[NB], dpt[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      st[nb] = zero4();
      dpt[nb] = zero4();
      if (nb >= nbmin) {
#pragma unroll
        for (int s = 0; s < D / 32; ++s) {
          st[nb] = mfma16(frag_row(Ks, D, 16 * w, s * 32), frag_row(Qs, D, nb * 16, s * 32), st[nb]);
          dpt[nb] = mfma16(frag_row(Vs, D, 16 * w, s * 32), frag_row(dOs, D, nb * 16, s * 32), dpt[nb]);
        }
      }
    }
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int qi = nb * 16 + (lane & 15);
      const float lq = lse_s[qi], dq_ = del_s[qi];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kr = 16 * w + 4 * (lane >> 4) + i;
        const bool ok = nb >= nbmin && qi < S && kr < kv_len && (!causal || kr <= qi);
        const float p = ok ? exp2f(st[nb][i] * c2 - lq) : 0.f;
        const float ds = p * (dpt[nb][i] - dq_) * scale;
        PTw[(4 * (lane >> 4) + i) * LDT + qi] = f2bf(p);
        DST[kr * LDT + qi] = f2bf(ds);
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  {
    const int ksmin = causal ? (16 * w) / 32 : 0;
#pragma unroll
    for (int kk = 0; kk < SM / 32; ++kk) {
      if (kk >= ksmin) {
        const bf16x8_t pa = frag_row(PTw, LDT, 0, kk * 32);
        const bf16x8_t da = frag_row(DST, LDT, 16 * w, kk * 32);
#pragma unroll
        for (int n = 0; n < D / 16; ++n) {
          dVa[n] = mfma16(pa, frag_tr(dOs, D, kk * 32, n * 16), dVa[n]);
          dKa[n] = mfma16(da, frag_tr(Qs, D, kk * 32, n * 16), dKa[n]);
        }
      }
    }
  }
  __syncthreads();  // every wave's dS^T rows are in LDS

  // ---- phase 2: wave w owns queries 16w..16w+15: dQ = dS K
  f32x4_t dQa[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) dQa[n] = zero4();
  {
    const int ksmax = causal ? (16 * w + 15) / 32 + 1 : SM / 32;
#pragma unroll
    for (int kk = 0; kk < SM / 32; ++kk) {
      if (kk < ksmax) {
        const bf16x8_t a = frag_tr(DST, LDT, kk * 32, 16 * w);
#pragma unroll
        for (int n = 0; n < D / 16; ++n) dQa[n] = mfma16(a, frag_tr(Ks, D, kk * 32, n * 16), dQa[n]);
      }
    }
  }
  if (16 * w >= S) return;
  const float one[4] = {1.f, 1.f, 1.f, 1.f};
  const int nrows = min(16, S - 16 * w);
  const int hout = dkv_per_qhead ? h : hk;
  store_tile16<D>(PTw, LDT, dQa, one, dq, dqs, b, h, 16 * w, nrows);
  store_tile16<D>(PTw, LDT, dKa, one, dk, dks, b, hout, 16 * w, nrows);
  store_tile16<D>(PTw, LDT, dVa, one, dv, dvs, b, hout, 16 * w, nrows);
}

bool attn_short_path(int D, int Sq, int Sk, int window) {
  return D == 64 && Sq == Sk && Sq <= kShortS && window <= 0;
}

static AttnStrides mk(const long* st) { return AttnStrides{st[0], st[1], st[2]}; }

template <int D>
static void fwd_launch(const AttnArgs& a, hipStream_t stream) {
  if constexpr (D == 64) {
    if (attn_short_path(D, a.Sq, a.Sk, a.window)) {
      const size_t shm = sizeof(bf16_t) * (2 * kShortS * D + 8 * 16 * short_ldp());
      static bool attr = false;
      if (!attr) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_short_kernel<D>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
      }
      attn_fwd_short_kernel<D><<<dim3(a.H, a.B), 512, shm, stream>>>(a.q, a.k, a.v, a.o, a.lse, mk(a.q_st), mk(a.k_st),
                                                                      mk(a.v_st), mk(a.o_st), a.H, a.Hkv, a.Sq, a.scale,
                                                                      a.causal, a.kv_lens);
      return;
    }
  }
  constexpr int BQ = 64, BK = 64, LDP = BK + 8;
  const size_t shm = sizeof(bf16_t) * (2 * BK * D + 4 * 16 * LDP);
  dim3 grid(cdiv(a.Sq, BQ), a.H, a.B);
  attn_fwd_kernel<D><<<grid, 256, shm, stream>>>(a.q, a.k, a.v, a.o, a.lse, mk(a.q_st), mk(a.k_st), mk(a.v_st),
                                                 mk(a.o_st), a.H, a.Hkv, a.Sq, a.Sk, a.scale, a.causal, a.window,
                                                 a.kv_lens);
}

template <int D>
static void bwd_launch(const AttnBwdArgs& a, hipStream_t stream) {
  if constexpr (D == 64) {
    if (attn_short_path(D, a.Sq, a.Sk, a.window)) {
      const size_t shm = sizeof(bf16_t) * (4 * kShortS * D + 2 * kShortS * short_ldp()) + sizeof(float) * 2 * kShortS;
      static bool attr = false;
      if (!attr) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_short_kernel<D>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
      }
      const int per_qhead = a.H != a.Hkv;
      attn_bwd_short_kernel<D><<<dim3(a.H, a.B), 512, shm, stream>>>(
          a.q, a.k, a.v, a.o, a.dout, a.lse, a.dq, per_qhead ? a.dk_tmp : a.dk, per_qhead ? a.dv_tmp : a.dv,
          mk(a.q_st), mk(a.k_st), mk(a.v_st), mk(a.o_st), mk(a.do_st), mk(a.dq_st),
          per_qhead ? mk(a.tmp_st) : mk(a.dk_st), per_qhead ? mk(a.tmp_st) : mk(a.dv_st), a.H, a.Hkv, a.Sq, a.scale,
          a.causal, a.kv_lens, per_qhead);
      if (per_qhead) {
        const long nk8 = (long)a.B * a.Sk * a.Hkv * D / 8;
        gqa_reduce_kernel<<<cdiv(nk8, 256), 256, 0, stream>>>(a.dk_tmp, a.dk, mk(a.dk_st), a.B, a.Sk, a.H, a.Hkv, D);
        gqa_reduce_kernel<<<cdiv(nk8, 256), 256, 0, stream>>>(a.dv_tmp, a.dv, mk(a.dv_st), a.B, a.Sk, a.H, a.Hkv, D);
      }
      return;
    }
  }
  constexpr int BQ = 64, BK = 64, LDT = BQ + 8;
  {
    const long rows = (long)a.B * a.H * a.Sq;
    attn_bwd_delta_kernel<D><<<cdiv(rows * (D / 8), 256), 256, 0, stream>>>(a.o, a.dout, a.delta, mk(a.o_st),
                                                                            mk(a.do_st), a.B, a.H, a.Sq);
  }
  MFT_HIP_CHECK(hipMemsetAsync(a.dq_acc, 0, sizeof(float) * (size_t)a.B * a.Sq * a.H * D, stream));
  const size_t shm = sizeof(bf16_t) * (2 * BK * D + 2 * BQ * D + 2 * BK * LDT) + sizeof(float) * 2 * BQ;
  static bool attr_set = false;
  if (!attr_set) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_kernel<D>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  dim3 grid(cdiv(a.Sk, BK), a.H, a.B);
  const int per_qhead = a.H != a.Hkv;
  attn_bwd_kernel<D><<<grid, 256, shm, stream>>>(a.q, a.k, a.v, a.dout, a.lse, a.delta, a.dq_acc,
                                                 per_qhead ? a.dk_tmp : a.dk, per_qhead ? a.dv_tmp : a.dv, mk(a.q_st),
                                                 mk(a.k_st), mk(a.v_st), mk(a.do_st),
                                                 per_qhead ? mk(a.tmp_st) : mk(a.dk_st),
                                                 per_qhead ? mk(a.tmp_st) : mk(a.dv_st), a.H, a.Hkv, a.Sq, a.Sk,
                                                 a.scale, a.causal, a.window, a.kv_lens, per_qhead);
  const long nq8 = (long)a.B * a.Sq * a.H * D / 8;
  attn_dq_convert_kernel<<<cdiv(nq8, 256), 256, 0, stream>>>(a.dq_acc, a.dq, mk(a.dq_st), a.B, a.Sq, a.H, D);
  if (per_qhead) {
    const long nk8 = (long)a.B * a.Sk * a.Hkv * D / 8;
    gqa_reduce_kernel<<<cdiv(nk8, 256), 256, 0, stream>>>(a.dk_tmp, a.dk, mk(a.dk_st), a.B, a.Sk, a.H, a.Hkv, D);
    gqa_reduce_kernel<<<cdiv(nk8, 256), 256, 0, stream>>>(a.dv_tmp, a.dv, mk(a.dv_st), a.B, a.Sk, a.H, a.Hkv, D);
  }
}

void attn_fwd(const AttnArgs& a, hipStream_t s) {
  static bool init = false;
  if (!init) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    init = true;
  }
  switch (a.D) {
    case 64: fwd_launch<64>(a, s); break;
    case 128: fwd_launch<128>(a, s); break;
    case 256: fwd_launch<256>(a, s); break;
    default: fprintf(stderr, "attn_fwd: unsupported head dim %d\n", a.D); abort();
  }
}

void attn_bwd(const AttnBwdArgs& a, hipStream_t s) {
  switch (a.D) {
    case 64: bwd_launch<64>(a, s); break;
    case 128: bwd_launch<128>(a, s); break;
    case 256: bwd_launch<256>(a, s); break;
    default: fprintf(stderr, "attn_bwd: unsupported head dim %d\n", a.D); abort();
  }
}

}  // namespace mft
