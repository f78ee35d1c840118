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
#include <algorithm>
#include <cstdlib>

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
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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
      alpha[i] = fast_exp2(m[i] - msafe);
      float rs = 0.f;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const float p = fast_exp2(sacc[nb][i] - msafe);
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
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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
        const float p = ok ? fast_exp2(st[nb][i] * c2 - lq) : 0.f;
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

// ---- short-path LDS images ([rows][D] bf16, D = 64: 8 16-B chunks a row): chunk c of row r sits at
// c ^ sws(r), sws(r) = ((r >> 1) & 3) << 1 | ((r >> 3) & 1).  A ds_read_b128 row fragment (16 rows, one
// chunk) then covers 16 distinct 16-B bank groups, and each 32-lane half of a frag_tr_perm pair (rows
// 4g + q, 2 chunks x 2 halves) 32 distinct 8-B slots; the plain [rows][64] image put 58 % of the kernels'
// LDS cycles into bank conflicts (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, profiles/r5_attn64_lds.txt).
// Rows r and r + 16 share the swizzle (the second read of a pair is an immediate offset).
template <int D>
__device__ __forceinline__ int sws(int r) {
  if constexpr (D == 64) return (((r >> 1) & 3) << 1) | ((r >> 3) & 1);
  else return 0;
}
template <int D>
__device__ __forceinline__ int sw_off(int r, int ch) { return r * D + ((ch ^ sws<D>(r)) << 3); }
template <int D>
__device__ __forceinline__ bf16x8_t frag_row_s(const bf16_t* t, int r0, int c0) {
  const int l = threadIdx.x & 63;
  const int r = r0 + (l & 15), ch = (c0 >> 3) + (l >> 4);
  return *reinterpret_cast<const bf16x8_t*>(t + sw_off<D>(r, ch));
}
template <int D>
__device__ __forceinline__ bf16x8_t frag_tr_perm_s(const bf16_t* t, int r0, int c0) {  // frag_tr_perm (mfma.h)
  const int l = threadIdx.x & 63;
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int ra = r0 + 4 * g + q, col = c0 + 4 * p, ch = col >> 3, off = col & 7;
  s16x4_t lo = ds_tr16(t + sw_off<D>(ra, ch) + off);
  s16x4_t hi = ds_tr16(t + sw_off<D>(ra + 16, ch) + off);
  s16x8_t rr = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, rr);
}
template <int D>
__device__ __forceinline__ bf16x8_t frag_tr_s(const bf16_t* t, int r0, int c0) {  // frag_tr (mfma.h)
  const int l = threadIdx.x & 63;
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int ra = r0 + 8 * g + q, col = c0 + 4 * p, ch = col >> 3, off = col & 7;
  s16x4_t lo = ds_tr16(t + sw_off<D>(ra, ch) + off);
  s16x4_t hi = ds_tr16(t + sw_off<D>(ra + 4, ch) + off);
  s16x8_t rr = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, rr);
}

// ---- v2: P (fwd) / P^T, dS^T (bwd) stay in registers -------------------------------------------
// Scores are computed transposed (S^T = K Q^T: keys in C rows, queries in C columns), so two
// 16-key C blocks ARE the A operand of the next MFMA over keys (pack_c2a / frag_tr_perm, mfma.h):
// no LDS round trip for P, less LDS per workgroup -> several workgroups per CU overlap their loads.
// Forward LDS = K + V (32 KB) + a 2.3 KB output staging tile per wave.
template <int D>
__global__ __launch_bounds__(512) void attn_fwd_short2_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                              const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                              float* __restrict__ lse, AttnStrides qs, AttnStrides ks,
                                                              AttnStrides vs, AttnStrides os, int H, int Hkv, int S,
                                                              float scale, int causal, const int* __restrict__ kv_lens,
                                                              int o_pad) {
  constexpr int SM = kShortS, NB = SM / 16, CPR = D / 8, LDO = D + 8;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* Ks = smem;                                      // [SM][D]
  bf16_t* Vs = Ks + SM * D;                               // [SM][D]
  bf16_t* Ow = Vs + SM * D + (threadIdx.x >> 6) * 16 * LDO;  // per-wave [16][LDO] output staging
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  const int h = blockIdx.x, b = blockIdx.y, hk = h / (H / Hkv);
  const int kv_len = kv_lens ? min(kv_lens[b], S) : S;
  const float c2 = scale * kLog2e;
  if (h == 0 && o_pad > 0) {  // the o_pad zero columns after the H heads of every output row of batch b
    const int per = o_pad / 8;
    for (int c = threadIdx.x; c < S * per; c += 512)
      *reinterpret_cast<u16x8_t*>(o + b * os.sb + (long)(c / per) * os.ss + (long)H * D + (c % per) * 8) = u16x8_t{};
  }
  constexpr int PER = SM * CPR / 512;
  u16x8_t kr[PER], vr[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = threadIdx.x + j * 512, r = c / CPR, ch = c % CPR;
    const bool ok = r < S;
    kr[j] = ok ? *reinterpret_cast<const u16x8_t*>(k + b * ks.sb + (long)r * ks.ss + hk * ks.sh + ch * 8) : u16x8_t{};
    vr[j] = ok ? *reinterpret_cast<const u16x8_t*>(v + b * vs.sb + (long)r * vs.ss + hk * vs.sh + ch * 8) : u16x8_t{};
  }
  // this wave's 16 queries as the B operand of S^T = K Q^T (lane: Q[16w + (l&15)][8g + j + 32s])
  bf16x8_t qf[D / 32];
  {
    const int qr = 16 * w + (lane & 15);
#pragma unroll
    for (int s = 0; s < D / 32; ++s)
      qf[s] = qr < S ? *reinterpret_cast<const bf16x8_t*>(q + b * qs.sb + (long)qr * qs.ss + h * qs.sh + s * 32 + 8 * g)
                     : bf16x8_t{};
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = threadIdx.x + j * 512, r = c / CPR, ch = c % CPR;
    *reinterpret_cast<u16x8_t*>(Ks + sw_off<D>(r, ch)) = kr[j];
    *reinterpret_cast<u16x8_t*>(Vs + sw_off<D>(r, ch)) = vr[j];
  }
  __syncthreads();
  if (16 * w >= S) return;
  const int nbmax = causal ? w + 1 : NB;
  const int qi = 16 * w + (lane & 15);  // this lane's query (C column)
  f32x4_t st[NB];                        // st[kb][i] = S^T[key = 16 kb + 4g + i][qi]
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) {
    st[kb] = zero4();
    if (kb < nbmax) {
#pragma unroll
      for (int s = 0; s < D / 32; ++s) st[kb] = mfma16(frag_row_s<D>(Ks, kb * 16, s * 32), qf[s], st[kb]);
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kj = 16 * kb + 4 * g + i;
      const bool ok = kb < nbmax && kj < kv_len && (!causal || kj <= qi);
      const float sv = ok ? st[kb][i] * c2 : -INFINITY;
      st[kb][i] = sv;
      mx = fmaxf(mx, sv);
    }
  mx = fmaxf(mx, xor16_pl(mx));
  mx = fmaxf(mx, xor32_pl(mx));
  const float ms = mx == -INFINITY ? 0.f : mx;
  float rs = 0.f;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p = fast_exp2(st[kb][i] - ms);
      st[kb][i] = p;
      rs += p;
    }
  rs += xor16_pl(rs);
  rs += xor32_pl(rs);
  // O = P V over 32-key steps; P's A fragment comes straight from two S^T blocks
  f32x4_t acc[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) acc[n] = zero4();
#pragma unroll
  for (int kk = 0; kk < SM / 32; ++kk) {
    if (2 * kk < nbmax) {
      const bf16x8_t pa = pack_c2a(st[2 * kk], st[2 * kk + 1]);
#pragma unroll
      for (int n = 0; n < D / 16; ++n) acc[n] = mfma16(pa, frag_tr_perm_s<D>(Vs, kk * 32, n * 16), acc[n]);
    }
  }
  // acc rows are queries 4g+i: fetch their 1/l from the lane that owns that query column
  const float inv_own = rs > 0.f ? 1.f / rs : 0.f;
  if (g == 0 && qi < S)
    lse[((long)b * H + h) * S + qi] = rs > 0.f ? (mx + log2f(rs)) / kLog2e : 1e30f;
  float inv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) inv[i] = __shfl(inv_own, 4 * g + i, 64);
  store_tile16<D>(Ow, LDO, acc, inv, o, os, b, h, 16 * w, min(16, S - 16 * w));
}

// Backward v2.  Phase 1 (wave w owns keys 16w..16w+15): per pair of 16-query blocks, S = Q K^T and
// dP = dO V^T land in C layout with queries in rows and this wave's keys in columns -- exactly the
// A operand (m = key, k = query) of dV += P^T dO and dK += dS^T Q after pack_c2a, with the B rows
// permuted to match (frag_tr_perm).  dS is kept packed in registers; after a block barrier (V and
// dO dead) it is written to a swizzled [query][key] image that aliases them, and phase 2 (wave w
// owns queries 16w..) forms dQ = dS K.  LDS = K, V, Q, dO (64 KB) + lse/delta: two workgroups per CU,
// which needs 4 waves per SIMD, i.e. <= 128 VGPRs (the launch bound's second argument is waves per SIMD).
template <int D>
__global__ __launch_bounds__(512, 4) void attn_bwd_short2_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    bf16_t* __restrict__ dq, bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, AttnStrides qs, AttnStrides ks,
    AttnStrides vs, AttnStrides ost, AttnStrides dos, AttnStrides dqs, AttnStrides dks, AttnStrides dvs, int H, int Hkv,
    int S, float scale, int causal, const int* __restrict__ kv_lens, int dkv_per_qhead) {
  constexpr int SM = kShortS, CPR = D / 8;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* Ks = smem;           // [SM][D]
  bf16_t* Vs = Ks + SM * D;    // [SM][D]   } phase 2: dS image [SM q][SM keys], 16-B chunks
  bf16_t* dOs = Vs + SM * D;   // [SM][D]   }   swizzled chunk ^ (q & 15)
  bf16_t* Qs = dOs + SM * D;   // [SM][D]   (after phase 1: per-wave [16][D + 8] output staging)
  bf16_t* DS = Vs;
  float* lse_s = reinterpret_cast<float*>(Qs + SM * D);  // [SM]
  float* del_s = lse_s + SM;                             // [SM]
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, c16 = lane & 15;
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
      *reinterpret_cast<u16x8_t*>(Ks + sw_off<D>(r, ch)) = kr[j];
      *reinterpret_cast<u16x8_t*>(Vs + sw_off<D>(r, ch)) = vr[j];
      *reinterpret_cast<u16x8_t*>(Qs + sw_off<D>(r, ch)) = qr[j];
      *reinterpret_cast<u16x8_t*>(dOs + sw_off<D>(r, ch)) = dr[j];
      float dsum = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum += bf2f(dr[j][e]) * bf2f(orr[j][e]);
#pragma unroll
      for (int off = 1; off < CPR; off <<= 1) dsum += __shfl_xor(dsum, off, 64);
      if (ch == 0) del_s[r] = dsum;
    }
  }
  __syncthreads();

  // ---- phase 1: keys 16w..16w+15
  const int key = 16 * w + c16;  // this lane's key (C column)
  f32x4_t dKa[D / 16], dVa[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) { dKa[n] = zero4(); dVa[n] = zero4(); }
  uint32_t dsp[SM / 16][2];  // dS (bf16 pairs) per 16-query block, kept for the phase-2 image
#pragma unroll
  for (int kk = 0; kk < SM / 32; ++kk) {
    const bool live = !causal || 32 * kk + 31 >= 16 * w;  // some query of this step sees these keys
    f32x4_t sc[2], dp[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sc[t] = zero4();
      dp[t] = zero4();
      if (live) {
#pragma unroll
        for (int s2 = 0; s2 < D / 32; ++s2) {
          sc[t] = mfma16(frag_row_s<D>(Qs, 32 * kk + 16 * t, s2 * 32), frag_row_s<D>(Ks, 16 * w, s2 * 32), sc[t]);
          dp[t] = mfma16(frag_row_s<D>(dOs, 32 * kk + 16 * t, s2 * 32), frag_row_s<D>(Vs, 16 * w, s2 * 32), dp[t]);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qi = 32 * kk + 16 * t + 4 * g + i;
        const bool ok = live && qi < S && key < kv_len && (!causal || key <= qi);
        const float p = ok ? fast_exp2(sc[t][i] * c2 - lse_s[qi]) : 0.f;
        sc[t][i] = p;                                     // P
        dp[t][i] = p * (dp[t][i] - del_s[qi]) * scale;    // dS
      }
      dsp[2 * kk + t][0] = pack_bf2(dp[t][0], dp[t][1]);
      dsp[2 * kk + t][1] = pack_bf2(dp[t][2], dp[t][3]);
    }
    if (live) {
      const bf16x8_t pa = pack_c2a(sc[0], sc[1]);
      const bf16x8_t da = pack_c2a(dp[0], dp[1]);
#pragma unroll
      for (int n = 0; n < D / 16; ++n) {
        dVa[n] = mfma16(pa, frag_tr_perm_s<D>(dOs, 32 * kk, n * 16), dVa[n]);
        dKa[n] = mfma16(da, frag_tr_perm_s<D>(Qs, 32 * kk, n * 16), dKa[n]);
      }
    }
  }
  __syncthreads();  // V, dO (and Q) are dead from here on
  // dS image [q][key]: element (q, key) at q*SM + ((key/8 ^ (q&15)) * 8) + key%8.  Written as dwords (two
  // adjacent keys): a lane holds 4 queries of one key, so lane pairs (key, key + 1) swap halves by DPP --
  // the even lane writes queries 4g, 4g + 1, the odd lane 4g + 2, 4g + 3 (half the writes, no two lanes
  // sharing a dword)
  {
    const bool odd = key & 1;
    const int kp = key & ~1;
#pragma unroll
    for (int qb = 0; qb < SM / 16; ++qb) {
      const uint32_t p0 = dsp[qb][0], p1 = dsp[qb][1];  // queries (4g, 4g + 1), (4g + 2, 4g + 3)
      const uint32_t n0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p0, 0xB1, 0xF, 0xF, false);  // lane ^ 1
      const uint32_t n1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p1, 0xB1, 0xF, 0xF, false);
      const uint32_t wa = odd ? ((n1 & 0xFFFFu) | (p1 << 16)) : ((p0 & 0xFFFFu) | (n0 << 16));
      const uint32_t wb = odd ? ((n1 >> 16) | (p1 & 0xFFFF0000u)) : ((p0 >> 16) | (n0 & 0xFFFF0000u));
      const int qa = 16 * qb + 4 * g + (odd ? 2 : 0), qc = qa + 1;
      *reinterpret_cast<uint32_t*>(DS + qa * SM + (((kp >> 3) ^ (qa & 15)) << 3) + (kp & 7)) = wa;
      *reinterpret_cast<uint32_t*>(DS + qc * SM + (((kp >> 3) ^ (qc & 15)) << 3) + (kp & 7)) = wb;
    }
  }
  // dK, dV of this wave's keys (staging tile over the dead Q and lse / delta region, pitch D + 8: the four
  // 16-lane groups of the 2-byte staging writes on different banks -- at pitch D they all met, 4-way)
  const int hout = dkv_per_qhead ? h : hk;
  const float one[4] = {1.f, 1.f, 1.f, 1.f};
  constexpr int LDT = D + 8;
  bf16_t* T = Qs + w * 16 * LDT;
  if (16 * w < S) {
    store_tile16<D>(T, LDT, dKa, one, dk, dks, b, hout, 16 * w, min(16, S - 16 * w));
    store_tile16<D>(T, LDT, dVa, one, dv, dvs, b, hout, 16 * w, min(16, S - 16 * w));
  }
  __syncthreads();

  // ---- phase 2: queries 16w..16w+15: dQ = dS K
  f32x4_t dQa[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) dQa[n] = zero4();
  const int ksmax = causal ? (16 * w + 15) / 32 + 1 : SM / 32;
#pragma unroll
  for (int kk = 0; kk < SM / 32; ++kk) {
    if (kk < ksmax) {
      const int qr = 16 * w + c16, ch = 4 * kk + g;
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(DS + qr * SM + ((ch ^ (qr & 15)) << 3));
#pragma unroll
      for (int n = 0; n < D / 16; ++n) dQa[n] = mfma16(a, frag_tr_s<D>(Ks, kk * 32, n * 16), dQa[n]);
    }
  }
  if (16 * w < S) store_tile16<D>(T, LDT, dQa, one, dq, dqs, b, h, 16 * w, min(16, S - 16 * w));
}

// ============================================================================================
// Split path (every shape the short path does not take; Gemma-3: D = 256, GQA 4:1, S = 256..):
// scores are computed TRANSPOSED as in the short path, so P / dS become the A operand of the next
// MFMA straight from registers (pack_c2a + frag_tr_perm) -- no LDS round trip, no scalar LDS
// writes.  32-row K/V (or Q/dO) tiles are staged through LDS with rows padded to D + kSplitPad elements
// (conflict-free ds_read_b128 row fragments).
//   * forward: a workgroup owns 16*NW queries of one head (each wave 16, Q in registers as the B
//     operand of S^T = K Q^T); online softmax stats are per C column, reduced over the 4 lane groups.
//   * backward dK/dV: a workgroup owns 16*NW keys of one KV head and sweeps every query of EVERY
//     q-head of its GQA group, so dK/dV are summed over the group in registers (no expanded
//     per-q-head buffer, no reduction pass).
//   * backward dQ: a workgroup owns 16*NW queries and recomputes S and dP per key tile; dQ is
//     written once in bf16 (no fp32 atomics, workspace memset or conversion pass).
// ============================================================================================
constexpr int kSplitBK = 32;  // rows per staged tile
// LDS row pitch D + 16 elements (row stride = 8 banks mod 64): conflict-free for BOTH operand reads
// of these kernels -- ds_read_b128 row fragments (16-lane groups {0-3,12-15,20-27}, ...) and the
// ds_read_b64_tr_b16 pairs of frag_tr_perm (32-lane groups) -- where a D + 8 pitch left ~2 extra
// LDS cycles per instruction (SQ_LDS_BANK_CONFLICT, profiles/r1_attn_split_pmc.txt).  Measured at
// the Gemma-3 shape: conflict cycles -90 %, kernel time only -2..5 % -- the waves spend ~65 % of
// their cycles in SQ_WAIT_ANY (tile staging latency), not in LDS.
constexpr int kSplitPad = 16;
constexpr int kOutPad = 8;  // per-wave output staging rows (store_tile16): D + 8

// LDS writes / reads retired, then a raw s_barrier: unlike __syncthreads (whose fence implies
// vmcnt(0)) it lets global prefetches issued before it stay in flight
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Two 32-row tiles (rows >= nvalid zero-filled) held in registers between the global load and the
// LDS store, so the NEXT tile's loads are in flight while the current one is multiplied
// (double-buffered LDS, one barrier per step).  LDS rows are padded to D + kSplitPad elements.
template <int D, int NT>
struct Tile2 {
  static constexpr int CPR = D / 8, LD = D + kSplitPad, PER = (kSplitBK * CPR + NT - 1) / NT;
  u16x8_t r0[PER], r1[PER];
  __device__ __forceinline__ void load(const bf16_t* src0, const bf16_t* src1, AttnStrides s0, AttnStrides s1, int b,
                                       int h, int row0, int nvalid) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = threadIdx.x + j * NT, r = c / CPR, ch = c % CPR;
      const bool ok = c < kSplitBK * CPR && r < nvalid;
      r0[j] = ok ? *reinterpret_cast<const u16x8_t*>(src0 + b * s0.sb + (long)(row0 + r) * s0.ss + h * s0.sh + ch * 8)
                 : u16x8_t{};
      r1[j] = ok ? *reinterpret_cast<const u16x8_t*>(src1 + b * s1.sb + (long)(row0 + r) * s1.ss + h * s1.sh + ch * 8)
                 : u16x8_t{};
    }
  }
  __device__ __forceinline__ void store(bf16_t* lds0, bf16_t* lds1) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = threadIdx.x + j * NT, r = c / CPR, ch = c % CPR;
      if (c < kSplitBK * CPR) {
        *reinterpret_cast<u16x8_t*>(lds0 + r * LD + ch * 8) = r0[j];
        *reinterpret_cast<u16x8_t*>(lds1 + r * LD + ch * 8) = r1[j];
      }
    }
  }
};

// XCD-aware task order for the split kernels: the dispatcher deals workgroups round-robin over the
// 8 XCDs (each with its own L2); renumbered, the consecutive tasks of one batch row (the q-blocks /
// key blocks and heads that re-read the same K/V or Q/dO rows) run on ONE XCD and share its L2.
__device__ __forceinline__ void split_task(int& x, int& y, int& z) {
  const int nx = gridDim.x, ny = gridDim.y;
  const int n = nx * ny * gridDim.z;
  const int t = xcd_remap(blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), n);
  x = t % nx;
  y = (t / nx) % ny;
  z = t / (nx * ny);
}

// dynamic LDS of the split kernels: two {tile0, tile1} buffers (+ per-row floats), or the per-wave
// output staging of the epilogue, whichever is larger
template <int D, int NW>
constexpr size_t split_shm(int row_floats) {
  return std::max(sizeof(bf16_t) * 4 * kSplitBK * (D + kSplitPad) + sizeof(float) * 2 * row_floats * kSplitBK,
                  sizeof(bf16_t) * NW * 16 * (D + kSplitPad));
}

template <int D, int NW>
__global__ __launch_bounds__(64 * NW) void attn_fwd_split_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
    float* __restrict__ lse, AttnStrides qs, AttnStrides ks, AttnStrides vs, AttnStrides os, int H, int Hkv, int Sq,
    int Sk, float scale, int causal, int window, const int* __restrict__ kv_lens) {
  constexpr int NT = 64 * NW, BQ = 16 * NW, BK = kSplitBK, LD = D + kSplitPad;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];  // buffer j: K at smem + 2 j BK LD, V after it
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, c16 = lane & 15;
  int tx, h, b;
  split_task(tx, h, b);
  const int q0 = tx * BQ, hk = h / (H / Hkv);
  const int kv_len = kv_lens ? min(kv_lens[b], Sk) : Sk;
  const int coff = Sk - Sq;
  const float c2 = scale * kLog2e;
  const int wq_lo = q0 + 16 * w, wq_hi = wq_lo + 15;
  const int qi = wq_lo + c16;  // this lane's query (C column)
  int kend = kv_len;
  if (causal) kend = min(kend, q0 + BQ + coff);
  int kstart = 0;
  if (window > 0) kstart = max(0, q0 + coff - window + 1) / BK * BK;
  Tile2<D, NT> tl;
  if (kstart < kend) tl.load(k, v, ks, vs, b, hk, kstart, min(BK, kv_len - kstart));
  bf16x8_t qf[D / 32];  // B operand of S^T = K Q^T: Q[qi][32 s + 8 g + j]
#pragma unroll
  for (int s = 0; s < D / 32; ++s)
    qf[s] = qi < Sq ? *reinterpret_cast<const bf16x8_t*>(q + b * qs.sb + (long)qi * qs.ss + h * qs.sh + s * 32 + 8 * g)
                    : bf16x8_t{};
  if (kstart < kend) tl.store(smem, smem + BK * LD);
  f32x4_t acc[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) acc[n] = zero4();
  float m = -INFINITY, l = 0.f;  // running stats of query qi (identical in the 4 lane groups)
  for (int kb = kstart, j = 0; kb < kend; kb += BK, ++j) {
    const bool more = kb + BK < kend;
    if (more) tl.load(k, v, ks, vs, b, hk, kb + BK, min(BK, kv_len - kb - BK));
    lds_barrier();  // raw: the prefetch above stays in flight (no implied vmcnt(0))
    const bf16_t* Ks = smem + (j & 1) * 2 * BK * LD;
    const bf16_t* Vs = Ks + BK * LD;
    const bool live = wq_lo < Sq && (!causal || kb <= wq_hi + coff) &&
                      (window <= 0 || wq_lo + coff - (kb + BK - 1) < window);
    if (live) {           // wave-uniform
      f32x4_t st[2];      // st[t][i] = S[key kb + 16 t + 4 g + i][qi]
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        st[t] = zero4();
#pragma unroll
        for (int s = 0; s < D / 32; ++s) st[t] = mfma16(frag_row(Ks, LD, 16 * t, s * 32), qf[s], st[t]);
      }
      const bool need_mask = kb + BK > kv_len || (causal && kb + BK - 1 > wq_lo + coff) ||
                             (window > 0 && wq_hi + coff - kb >= window) || wq_hi >= Sq;
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float sv = st[t][i] * c2;
          if (need_mask && !(qi < Sq && attn_allowed(qi, kb + 16 * t + 4 * g + i, kv_len, coff, causal, window)))
            sv = -INFINITY;
          st[t][i] = sv;
          mx = fmaxf(mx, sv);
        }
      mx = fmaxf(mx, xor16_pl(mx));
      mx = fmaxf(mx, xor32_pl(mx));
      const float mnew = fmaxf(m, mx);
      const float msafe = mnew == -INFINITY ? 0.f : mnew;
      const float alpha = fast_exp2(m - msafe);
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = fast_exp2(st[t][i] - msafe);
          st[t][i] = p;
          rs += p;
        }
      rs += xor16_pl(rs);
      rs += xor32_pl(rs);
      l = l * alpha + rs;
      m = mnew;
      // acc rows are queries 4 g + i: their alpha lives in lane 4 g + i (C column = that query)
      float ar[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) ar[i] = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
      for (int n = 0; n < D / 16; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[n][i] *= ar[i];
      const bf16x8_t pa = pack_c2a(st[0], st[1]);
#pragma unroll
      for (int n = 0; n < D / 16; ++n) acc[n] = mfma16(pa, frag_tr_perm(Vs, LD, 0, n * 16), acc[n]);
    }
    if (more) {  // the other buffer was last read in step j - 1: every wave passed this step's barrier
      bf16_t* nb = smem + ((j + 1) & 1) * 2 * BK * LD;
      tl.store(nb, nb + BK * LD);
    }
  }
  const float inv_own = l > 0.f ? 1.f / l : 0.f;
  if (g == 0 && qi < Sq) lse[((long)b * H + h) * Sq + qi] = l > 0.f ? (m + log2f(l)) / kLog2e : 1e30f;
  float inv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) inv[i] = __shfl(inv_own, 4 * g + i, 64);
  __syncthreads();  // K/V tiles dead: reuse LDS as per-wave output staging
  if (wq_lo < Sq) store_tile16<D>(smem + w * 16 * LD, LD, acc, inv, o, os, b, h, wq_lo, min(16, Sq - wq_lo));
}

// ---- LDS-DMA ring variant of the split forward (D >= 128) -------------------------------------
// The register-staged pipeline above prefetches one tile ahead, which the measured kernels show is
// not enough (~65 % of wave cycles in SQ_WAIT_ANY, profiles/r1_attn_split_pmc.txt).  Here K/V tiles
// go global -> LDS by global_load_lds_dwordx4 (no VGPRs) into a 3-deep ring: tile j+2 streams in
// while tile j is multiplied.  LDS rows are unpadded (D elements) with the 16-B chunk index XORed
// by 2 (row & 7) on the SOURCE side (the DMA writes lane-linear), which keeps both the ds_read_b128
// row fragments and the ds_read_b64_tr_b16 pairs conflict-free (same bank algebra as the D + 16
// pitch).  Waits are counted (vmcnt) and barriers raw, so the DMA queue is never drained mid-loop.
constexpr int kRing = 3;

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ void dma4(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 4, 0, 0);
}
template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row & 7) << 1); }

// one 32-row tile, rows clamped into [0, rmax): LDS chunk c (lane-linear) <- global chunk swz(c)
template <int D, int NW>
__device__ __forceinline__ void dma_tile32(bf16_t* lds, const bf16_t* src, AttnStrides st, int b, int h, int row0,
                                           int rmax) {
  constexpr int CPR = D / 8, OPS = kSplitBK * CPR / 64;  // 1-KB DMA ops per tile
  static_assert(OPS % NW == 0, "every wave issues the same number of DMA ops");
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int k = 0; k < OPS / NW; ++k) {
    const int o = w + k * NW;
    const int c = o * 64 + lane, r = c / CPR, pos = c % CPR;
    const int gr = min(row0 + r, rmax - 1);
    dma16(src + b * st.sb + (long)gr * st.ss + h * st.sh + swz_chunk(r, pos) * 8, lds + o * 512);
  }
}

// lane holds T[r0 + (l&15)][c0 + 8 (l>>4) + j] of a swizzled [rows][D] image
template <int D>
__device__ __forceinline__ bf16x8_t frag_row_sw(const bf16_t* t, int r0, int c0) {
  const int l = threadIdx.x & 63;
  const int r = r0 + (l & 15), ch = (c0 >> 3) + (l >> 4);
  return *reinterpret_cast<const bf16x8_t*>(t + r * D + (swz_chunk(r, ch) << 3));
}
// frag_tr_perm (mfma.h) on a swizzled image
template <int D>
__device__ __forceinline__ bf16x8_t frag_tr_perm_sw(const bf16_t* t, int r0, int c0) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int ra = r0 + 4 * g + q, rb = ra + 16;
  const int col = c0 + 4 * p, ch = col >> 3, off = col & 7;
  s16x4_t lo = ds_tr16(t + ra * D + (swz_chunk(ra, ch) << 3) + off);
  s16x4_t hi = ds_tr16(t + rb * D + (swz_chunk(rb, ch) << 3) + off);
  s16x8_t rr = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, rr);
}

// ---- row-pair LDS image of a [32][256] bf16 tile (LDS-DMA target, D = 256) ----------------------
// One 1-KB LDS-DMA piece (a wave-instruction: 64 lanes x 16 B, lane-linear) holds two 512-B rows;
// pieces sit at a pitch of 1088 B (64 B pad).  Unlike the XOR swizzle this keeps every fragment
// read at ONE lane base + immediate offsets (the swizzled form needs a per-K-slice address
// register: at D = 256 those spilled and serialised the dK/dV loop, scratch reload -> ds_read ->
// MFMA).  Bank cost: 2-way on the ds_read_b128 row fragments and the ds_read_b64_tr_b16 pairs (the
// two rows of a piece share banks), which the kernels' LDS budget absorbs.
constexpr int kPairPitch = 544;  // elements per 2-row piece (1024 B data + 64 B pad)
constexpr int kPairTile = 16 * kPairPitch;
__device__ __forceinline__ int pr_row(int r) { return (r >> 1) * kPairPitch + (r & 1) * 256; }
// rows [row0, row0 + 32) of a [rows][256] operand (rows clamped into [0, rmax)) -> pair image
template <int NW>
__device__ __forceinline__ void dma_tile32_pr(bf16_t* lds, const bf16_t* src, AttnStrides st, int b, int h, int row0,
                                              int rmax) {
  static_assert(16 % NW == 0, "every wave issues the same number of DMA pieces");
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int k = 0; k < 16 / NW; ++k) {
    const int o = w + k * NW;
    const int gr = min(row0 + 2 * o + (lane >> 5), rmax - 1);
    dma16(src + b * st.sb + (long)gr * st.ss + h * st.sh + (lane & 31) * 8, lds + o * kPairPitch);
  }
}
// frag_row on the pair image (r0 even): lane holds T[r0 + (l&15)][c0 + 8 (l>>4) + j]
__device__ __forceinline__ bf16x8_t frag_row_pr(const bf16_t* t, int r0, int c0) {
  const int l = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8_t*>(t + (r0 >> 1) * kPairPitch + pr_row(l & 15) + c0 + 8 * (l >> 4));
}
// Swizzled pair image (the forward's K and V tiles): the odd row of each piece
// stores 16-B chunk c at slot c ^ 2 (the DMA writes lane-linear, so the swizzle is on the SOURCE
// column).  The two rows of a piece then no longer share banks: every 16-lane group of a
// ds_read_b128 row fragment hits 16 distinct 16-B slots (the plain pair image is 2-way: rows 2k and
// 2k + 1 sit 512 B apart, SQ_LDS_BANK_CONFLICT 11.5 M cycles on 5.1 M LDS instructions,
// profiles/r3_attn256_pmc.txt), and the read keeps one lane base + immediates: the XOR only touches
// bit 1 of the lane-group chunk index (chunk = 4 s2 + g).
template <int NW>
__device__ __forceinline__ void dma_tile32_prs(bf16_t* lds, const bf16_t* src, AttnStrides st, int b, int h, int row0,
                                               int rmax) {
  static_assert(16 % NW == 0, "every wave issues the same number of DMA pieces");
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = ((lane & 31) ^ ((lane >> 5) << 1)) * 8;
#pragma unroll
  for (int k = 0; k < 16 / NW; ++k) {
    const int o = w + k * NW;
    const int gr = min(row0 + 2 * o + (lane >> 5), rmax - 1);
    dma16(src + b * st.sb + (long)gr * st.ss + h * st.sh + col, lds + o * kPairPitch);
  }
}
// frag_row_pr on the swizzled pair image (r0 even: the lane's row parity is l & 1)
__device__ __forceinline__ bf16x8_t frag_row_prs(const bf16_t* t, int r0, int c0) {
  const int l = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8_t*>(t + (r0 >> 1) * kPairPitch + pr_row(l & 15) + c0 +
                                            8 * ((l >> 4) ^ ((l & 1) << 1)));
}
// frag_tr_pr on the swizzled pair image.  The transposed read's 16-B chunk is 2 n + (p >> 1) for c0 =
// 16 n, so the odd rows' XOR flips n's low bit: +16 elements for even n, -16 for odd n (n is an
// immediate of the unrolled loops -- two lane bases, no per-read address math).  Per 32-lane group
// the 8 rows then hit 8 distinct 32-B units (the plain image puts rows 2k, 2k + 1 on the same one).
__device__ __forceinline__ bf16x8_t frag_tr_prs(const bf16_t* t, int c0) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int sw = (q & 1) ? ((c0 & 16) ? -16 : 16) : 0;
  const bf16_t* a0 = t + pr_row(4 * g + q) + c0 + 4 * p + sw;
  s16x4_t lo = ds_tr16(a0);
  s16x4_t hi = ds_tr16(a0 + 8 * kPairPitch);  // row + 16 (same parity)
  s16x8_t rr = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, rr);
}
// Offset pair image (the dK/dV kernel's Q and dO tiles, read by rows AND transposed): the odd row of
// each piece starts 544 B (not 512 B) into it, i.e. 32 B further round the banks, so both read forms
// are conflict-free with ONE lane base (a row base + immediates): every 16-lane group of a
// ds_read_b128 row fragment covers 16 distinct 16-B slots (rows at 4 (r >> 1) + 2 (r & 1) slots), and
// each 32-lane group of a ds_read_b64_tr_b16 pair covers 8 distinct 32-B units (rows at 2 (r >> 1) +
// (r & 1)).  The price is two half-wave LDS-DMA instructions per piece (the even row's 32 lanes at the
// piece, the odd row's at piece + 32 B): the XOR-swizzled image needs a second lane base for the
// transposed reads, which spills this 256-VGPR kernel.
__device__ __forceinline__ int pr2_row(int r) { return (r >> 1) * kPairPitch + (r & 1) * 272; }
template <int NW>
__device__ __forceinline__ void dma_tile32_pr2(bf16_t* lds, const bf16_t* src, AttnStrides st, int b, int h, int row0,
                                               int rmax) {
  static_assert(16 % NW == 0, "every wave issues the same number of DMA pieces");
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int k = 0; k < 16 / NW; ++k) {
    const int o = w + k * NW;
    const int gr = min(row0 + 2 * o + (lane >> 5), rmax - 1);
    const bf16_t* sp = src + b * st.sb + (long)gr * st.ss + h * st.sh + (lane & 31) * 8;
    // Two half-wave instructions.  The empty asm after the second keeps the branches' tails different:
    // otherwise hipcc sinks both calls into ONE instruction with a per-lane select of the LDS base and
    // then takes lane 0's value for M0 -- the odd rows land at +512 B (measured: NaN dK).
    if (lane < 32) {
      dma16(sp, lds + o * kPairPitch);
    } else {
      dma16(sp, lds + o * kPairPitch + 16);  // lane 32 lands at 512 + 32 B
      asm volatile("" ::: "memory");
    }
  }
}
__device__ __forceinline__ bf16x8_t frag_row_pr2(const bf16_t* t, int r0, int c0) {
  const int l = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8_t*>(t + (r0 >> 1) * kPairPitch + pr2_row(l & 15) + c0 + 8 * (l >> 4));
}
__device__ __forceinline__ bf16x8_t frag_tr_pr2(const bf16_t* t, int c0) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const bf16_t* a0 = t + pr2_row(4 * g + q) + c0 + 4 * p;
  s16x4_t lo = ds_tr16(a0);
  s16x4_t hi = ds_tr16(a0 + 8 * kPairPitch);  // row + 16
  s16x8_t rr = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, rr);
}
// frag_tr_perm (mfma.h) on the pair image, rows 0..31
__device__ __forceinline__ bf16x8_t frag_tr_pr(const bf16_t* t, int c0) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const bf16_t* a0 = t + pr_row(4 * g + q) + c0 + 4 * p;
  s16x4_t lo = ds_tr16(a0);
  s16x4_t hi = ds_tr16(a0 + 8 * kPairPitch);  // row + 16
  s16x8_t rr = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, rr);
}


// RPW = query rows per wave (16 or 32).  At RPW = 32 every K fragment (ds_read_b128) and V^T
// fragment (ds_read_b64_tr_b16) read from LDS feeds TWO MFMAs -- one per 16-query half -- so the
// workgroup's LDS read bytes per FLOP halve (at D = 256 the 16-row form reads the whole 32 KB
// K+V stage per wave per 32-key tile: LDS-bandwidth bound), at ~2x the accumulator registers.
// RGF: ring depth of the D = 256 pair images (RGF - 1 tiles in flight; 4 x 34 KB holds the CU to one
// workgroup, 2 x 34 KB lets two co-reside)
// GQA: one workgroup per (query block, KV head, batch) -- the G = H / Hkv q-heads sharing the KV head
// split the waves (NW / G per head, RPW x NW / G query rows each), so every K / V tile lands in LDS
// once for all G heads (not once per q-head), and the workgroup's waves span G x fewer query rows,
// i.e. near-equal causal key ranges (a 128-row block idles its early-row waves on the late key tiles)
template <int D, int NW, int RPW = 16, bool SWZ = true, int RGF = 4, bool GQA = false>
__global__ __launch_bounds__(64 * NW) void attn_fwd_dma_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
    float* __restrict__ lse, AttnStrides qs, AttnStrides ks, AttnStrides vs, AttnStrides os, int H, int Hkv, int Sq,
    int Sk, float scale, int causal, int window, const int* __restrict__ kv_lens, int o_pad) {
  constexpr int R = RPW / 16;  // 16-query halves per wave
  constexpr bool kPair = D == 256;  // row-pair images (one address base per lane), else XOR swizzle
  // LDO: output staging pitch D + 8 (kOutPad): the four 16-lane groups of the 2-byte staging writes land
  // 16 banks apart (D + 16 put groups 0 / 2 and 1 / 3 on the same banks: the forward's last 2.1 M
  // conflict cycles, profiles/r4b_attn256_pmc.txt)
  constexpr int BK = kSplitBK, TILE = kPair ? kPairTile : BK * D, LDO = D + kOutPad;
  constexpr int OPW = 2 * (BK * D / 8 / 64) / NW;  // DMA ops per wave per ring stage (K + V)
  constexpr int RG = kPair ? RGF : kRing;  // ring depth: RG - 1 tiles in flight (RGF x 34 KB at D = 256)
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];  // ring stage s: K at smem + 2 s TILE, V after
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, c16 = lane & 15;
  int tx, hx, b;
  split_task(tx, hx, b);
  const int wph = GQA ? NW / (H / Hkv) : NW;  // waves per q-head
  const int bq = RPW * wph;                    // query rows per workgroup
  const int h = GQA ? hx * (H / Hkv) + w / wph : hx, hk = GQA ? hx : h / (H / Hkv);
  const int q0 = tx * bq;
  if (hx == 0 && o_pad > 0) {  // the widened output's zero columns of this block's rows (after the H heads)
    const int per = o_pad / 8, nr = min(bq, Sq - q0);
    for (int c = threadIdx.x; c < nr * per; c += 64 * NW)
      *reinterpret_cast<u16x8_t*>(o + b * os.sb + (long)(q0 + c / per) * os.ss + (long)H * D + (c % per) * 8) = u16x8_t{};
  }
  const int kv_len = kv_lens ? min(kv_lens[b], Sk) : Sk;
  const int coff = Sk - Sq;
  const float c2 = scale * kLog2e;
  const int wq_lo = q0 + RPW * (GQA ? w % wph : w), wq_hi = wq_lo + RPW - 1;
  int kend = kv_len;
  if (causal) kend = min(kend, q0 + bq + coff);
  int kstart = 0;
  if (window > 0) kstart = max(0, q0 + coff - window + 1) / BK * BK;
  const int nt = kend > kstart ? (kend - kstart + BK - 1) / BK : 0;  // WG-uniform
  bf16x8_t qf[R][D / 32];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int qi = wq_lo + 16 * r + c16;
#pragma unroll
    for (int s2 = 0; s2 < D / 32; ++s2)
      qf[r][s2] = qi < Sq ? *reinterpret_cast<const bf16x8_t*>(q + b * qs.sb + (long)qi * qs.ss + h * qs.sh + s2 * 32 + 8 * g)
                          : bf16x8_t{};
  }
  auto issue = [&](int j) {  // ring stage j % RG <- tile min(j, nt - 1) (tail re-reads keep counts uniform)
    const int kb = kstart + min(j, nt - 1) * BK;
    bf16_t* st = smem + (j % RG) * 2 * TILE;
    if constexpr (kPair) {
      if constexpr (SWZ) {  // swizzled pair images (conflict-free reads)
        dma_tile32_prs<NW>(st, k, ks, b, hk, kb, kv_len);
        dma_tile32_prs<NW>(st + TILE, v, vs, b, hk, kb, kv_len);
      } else {
        dma_tile32_pr<NW>(st, k, ks, b, hk, kb, kv_len);
        dma_tile32_pr<NW>(st + TILE, v, vs, b, hk, kb, kv_len);
      }
    } else {
      dma_tile32<D, NW>(st, k, ks, b, hk, kb, kv_len);
      dma_tile32<D, NW>(st + TILE, v, vs, b, hk, kb, kv_len);
    }
  };
  f32x4_t acc[R][D / 16];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int n = 0; n < D / 16; ++n) acc[r][n] = zero4();
  float m[R], l[R];
#pragma unroll
  for (int r = 0; r < R; ++r) m[r] = -INFINITY, l[r] = 0.f;
  if (nt > 0) {
#pragma unroll
    for (int j = 0; j < RG - 1; ++j) issue(j);
  }
  for (int j = 0; j < nt; ++j) {
    vmcnt_wait<OPW * (RG - 2)>();  // this wave's ops for stage j are done (later stages may still fly)
    lds_barrier();      // ... and every other wave's; stage (j + RG - 1) % RG was last read in step j - 1
    issue(j + RG - 1);
    const int kb = kstart + j * BK;
    const bf16_t* Ks = smem + (j % RG) * 2 * TILE;
    const bf16_t* Vs = Ks + TILE;
    const bool live = wq_lo < Sq && (!causal || kb <= wq_hi + coff) &&
                      (window <= 0 || wq_lo + coff - (kb + BK - 1) < window);
    if (live) {
      f32x4_t st[R][2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < R; ++r) st[r][t] = zero4();
#pragma unroll
        for (int s2 = 0; s2 < D / 32; ++s2) {
          const bf16x8_t kf = kPair ? (SWZ ? frag_row_prs(Ks, 16 * t, s2 * 32) : frag_row_pr(Ks, 16 * t, s2 * 32))
                                   : frag_row_sw<D>(Ks, 16 * t, s2 * 32);
#pragma unroll
          for (int r = 0; r < R; ++r) st[r][t] = mfma16(kf, qf[r][s2], st[r][t]);
        }
      }
      bf16x8_t pa[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int rlo = wq_lo + 16 * r, rhi = rlo + 15, qi = rlo + c16;
        const bool need_mask = kb + BK > kv_len || (causal && kb + BK - 1 > rlo + coff) ||
                               (window > 0 && rhi + coff - kb >= window) || rhi >= Sq;
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float sv = st[r][t][i] * c2;
            if (need_mask && !(qi < Sq && attn_allowed(qi, kb + 16 * t + 4 * g + i, kv_len, coff, causal, window)))
              sv = -INFINITY;
            st[r][t][i] = sv;
            mx = fmaxf(mx, sv);
          }
        mx = fmaxf(mx, xor16_pl(mx));
        mx = fmaxf(mx, xor32_pl(mx));
        const float mnew = fmaxf(m[r], mx);
        const float msafe = mnew == -INFINITY ? 0.f : mnew;
        const float alpha = fast_exp2(m[r] - msafe);
        float rs = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = fast_exp2(st[r][t][i] - msafe);
            st[r][t][i] = p;
            rs += p;
          }
        rs += xor16_pl(rs);
        rs += xor32_pl(rs);
        l[r] = l[r] * alpha + rs;
        m[r] = mnew;
        if (__any(alpha != 1.f)) {  // wave-uniform: skip the rescale when no running max moved
          float ar[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) ar[i] = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
          for (int n = 0; n < D / 16; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[r][n][i] *= ar[i];
        }
        pa[r] = pack_c2a(st[r][0], st[r][1]);
      }
#pragma unroll
      for (int n = 0; n < D / 16; ++n) {
        const bf16x8_t vf = kPair ? (SWZ ? frag_tr_prs(Vs, n * 16) : frag_tr_pr(Vs, n * 16)) : frag_tr_perm_sw<D>(Vs, 0, n * 16);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][n] = mfma16(pa[r], vf, acc[r][n]);
      }
    }
  }
  vmcnt_wait<0>();  // the tail's re-read DMA must land before the LDS is reused / the WG exits
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int rlo = wq_lo + 16 * r, qi = rlo + c16;
    const float inv_own = l[r] > 0.f ? 1.f / l[r] : 0.f;
    if (g == 0 && qi < Sq) lse[((long)b * H + h) * Sq + qi] = l[r] > 0.f ? (m[r] + log2f(l[r])) / kLog2e : 1e30f;
    float inv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) inv[i] = __shfl(inv_own, 4 * g + i, 64);
    if (rlo < Sq) store_tile16<D>(smem + w * 16 * LDO, LDO, acc[r], inv, o, os, b, h, rlo, min(16, Sq - rlo));
  }
}

// The (q-head, query tile) sweep is software-pipelined: the NEXT tile's Q / dO rows and row
// statistics are fetched while the current tile is multiplied, into the other half of a double-
// buffered LDS image -- one raw barrier per tile (the previous form staged every tile synchronously
// between two __syncthreads, whose implied vmcnt(0) exposed the whole global-load latency).
// D = 256: the tiles go global -> LDS by LDS-DMA (no VGPRs: the 16-key-per-wave dK/dV accumulators
// plus register staging spill at D = 256) into row-pair images (frag_row_pr / frag_tr_pr, one
// address base per lane); smaller D: register staging (Tile2) into rows padded to D + kSplitPad.
// The causal / window / padding mask is a select in front of the exp (exp2(-inf) = 0), not a
// branch around it: the branch split every step into divergent blocks the MFMAs could not cross.
// RGK: DMA ring slots at D = 256 (3: two tiles in flight, 102 KB -- one workgroup per CU; 2: one tile,
// 68 KB -- two co-resident workgroups)
template <int D, int NW, int RGK = 3>
__global__ __launch_bounds__(64 * NW, 2) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, AttnStrides qs, AttnStrides ks, AttnStrides vs, AttnStrides dos,
    AttnStrides dks, AttnStrides dvs, int H, int Hkv, int Sq, int Sk, float scale, int causal, int window,
    const int* __restrict__ kv_lens) {
  constexpr bool kDma = D == 256;
  constexpr int NT = 64 * NW, BKEY = 16 * NW, BQ = kSplitBK, LD = D + kSplitPad;
  constexpr int TILE = kDma ? kPairTile : BQ * LD;  // elements of one staged [BQ] x D tile
  // DMA: a 3-slot ring, two tiles in flight; register staging: 2 buffers
  // slots; DMA ops per wave per tile (two half-wave ops per offset-pair piece, + the row stats)
  constexpr int RG = kDma ? RGK : 2, OPT = 2 * 2 * (16 / NW) + 1;
  constexpr int PF = RG - 1;  // DMA: tiles of prefetch
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  // slot j: Q at smem + 2 j TILE, dO after it; row floats [j][lse | delta][BQ] after every slot
  float* const rowf = reinterpret_cast<float*>(smem + 2 * RG * TILE);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, c16 = lane & 15;
  int tx, hk, b;
  split_task(tx, hk, b);
  const int kb = tx * BKEY, G = H / Hkv;
  const int kv_len = kv_lens ? min(kv_lens[b], Sk) : Sk;
  const int coff = Sk - Sq;
  const float c2 = scale * kLog2e;
  const int wk_lo = kb + 16 * w, wk_hi = wk_lo + 15;
  const int key = wk_lo + c16;  // this lane's key (C column of S = Q K^T)
  int qstart = 0, qend = Sq;
  if (causal) qstart = max(0, kb - coff) / BQ * BQ;
  if (window > 0) qend = min(Sq, kb + BKEY - 1 - coff + window);
  if (kb >= kv_len) qend = qstart;  // fully padded key block: grads are zero
  const int nq = qend > qstart ? (qend - qstart + BQ - 1) / BQ : 0;
  const int total = G * nq;  // (q-head, query tile) steps, WG-uniform
  Tile2<D, NT> tl;
  float ls_r = 0.f, dl_r = 0.f;  // register staging: the prefetched tile's row statistics (threads < BQ)
  auto load = [&](int it, int j) {  // start fetching step it's tile into slot j
    const int h = hk * G + it / nq, q0 = qstart + (it % nq) * BQ;
    const long rs = ((long)b * H + h) * Sq;
    if constexpr (kDma) {
      dma_tile32_pr2<NW>(smem + 2 * j * TILE, q, qs, b, h, q0, Sq);  // rows past Sq: clamped, masked below
      dma_tile32_pr2<NW>(smem + (2 * j + 1) * TILE, dout, dos, b, h, q0, Sq);
      // row statistics by one 4-byte DMA per wave (every wave the same bytes: uniform vmcnt counts):
      // lanes 0-31 the tile's lse, lanes 32-63 its delta
      const int r = min(q0 + (lane & 31), Sq - 1);
      dma4((lane < 32 ? lse : delta) + rs + r, rowf + j * 2 * BQ);
    } else {
      tl.load(q, dout, qs, dos, b, h, q0, min(BQ, Sq - q0));
      if (threadIdx.x < BQ) {
        const int qi = q0 + threadIdx.x;
        ls_r = qi < Sq ? lse[rs + qi] : 1e30f;
        dl_r = qi < Sq ? delta[rs + qi] : 0.f;
      }
    }
  };
  auto land = [&](int j) {  // register staging: buffer j complete for every wave after the next barrier
    tl.store(smem + 2 * j * TILE, smem + (2 * j + 1) * TILE);
    if (threadIdx.x < BQ) {
      rowf[j * 2 * BQ + threadIdx.x] = ls_r;
      rowf[j * 2 * BQ + BQ + threadIdx.x] = dl_r;
    }
  };
  auto frow = [&](const bf16_t* t, int r0, int c0) {
    if constexpr (kDma) return frag_row_pr2(t, r0, c0);  // offset pair images (conflict-free)
    else return frag_row(t, LD, r0, c0);
  };
  auto ftr = [&](const bf16_t* t, int c0) {
    if constexpr (kDma) return frag_tr_pr2(t, c0);
    else return frag_tr_perm(t, LD, 0, c0);
  };
  if (total > 0) {
    load(0, 0);
    if constexpr (kDma) {
      if constexpr (PF > 1) load(min(1, total - 1), 1);  // past the end: the last tile again (uniform counts)
    }
  }
  bf16x8_t kf[D / 32], vf[D / 32];  // B operands: K[key][32 s + 8 g + j], V[key][...]
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    const bool ok = key < Sk;
    kf[s] = ok ? *reinterpret_cast<const bf16x8_t*>(k + b * ks.sb + (long)key * ks.ss + hk * ks.sh + s * 32 + 8 * g)
               : bf16x8_t{};
    vf[s] = ok ? *reinterpret_cast<const bf16x8_t*>(v + b * vs.sb + (long)key * vs.ss + hk * vs.sh + s * 32 + 8 * g)
               : bf16x8_t{};
  }
  if constexpr (!kDma) {
    if (total > 0) land(0);
  }
  f32x4_t dKa[D / 16], dVa[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) { dKa[n] = zero4(); dVa[n] = zero4(); }
  const bool wave_keys = wk_lo < kv_len;
  for (int it = 0; it < total; ++it) {
    const bool more = it + 1 < total;
    if constexpr (kDma) {
      vmcnt_wait<OPT * (PF - 1)>();  // this wave's pieces of step it's tile landed (later steps' may still fly)
      lds_barrier();                 // ... and every wave's; slot (it + PF) % RG, read in step it - 1, is free
      load(min(it + PF, total - 1), (it + PF) % RG);
    } else {
      // step it's buffer stored by every wave; the other buffer, read in step it - 1, is free.  Raw
      // barrier: the register prefetch below stays in flight across the next one.
      lds_barrier();
      if (more) load(it + 1, (it + 1) & 1);
    }
    const int j = it % RG, q0 = qstart + (it % nq) * BQ;
    const bf16_t* Qs = smem + 2 * j * TILE;
    const bf16_t* dOs = Qs + TILE;
    const float* ls = rowf + j * 2 * BQ;
    const float* dl = ls + BQ;
    const bool live = wave_keys && (!causal || q0 + BQ - 1 + coff >= wk_lo) &&
                      (window <= 0 || q0 + coff - wk_hi < window);
    if (live) {
      f32x4_t sc[2], dp[2];  // [t][i] = S / dP [query q0 + 16 t + 4 g + i][key]
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        sc[t] = zero4();
        dp[t] = zero4();
#pragma unroll
        for (int s = 0; s < D / 32; ++s) {
          sc[t] = mfma16(frow(Qs, 16 * t, s * 32), kf[s], sc[t]);
          dp[t] = mfma16(frow(dOs, 16 * t, s * 32), vf[s], dp[t]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qr = 16 * t + 4 * g + i, qi = q0 + qr;
          const bool ok = qi < Sq && attn_allowed(qi, key, kv_len, coff, causal, window);
          // unconditional reads, pinned (asm) so the compiler cannot sink them into a branch
          float lsq = ls[qr], dlq = dl[qr];
          asm volatile("" : "+v"(lsq), "+v"(dlq));
          float x = sc[t][i] * c2 - lsq * kLog2e;
          asm volatile("" : "+v"(x));
          const float p = fast_exp2(ok ? x : -INFINITY);
          sc[t][i] = p;
          dp[t][i] = p * (dp[t][i] - dlq) * scale;
        }
      }
      const bf16x8_t pa = pack_c2a(sc[0], sc[1]);  // A: m = key, k = query (permuted)
      const bf16x8_t da = pack_c2a(dp[0], dp[1]);
#pragma unroll
      for (int n = 0; n < D / 16; ++n) {
        dVa[n] = mfma16(pa, ftr(dOs, n * 16), dVa[n]);
        dKa[n] = mfma16(da, ftr(Qs, n * 16), dKa[n]);
      }
    }
    if constexpr (!kDma) {
      if (more) land((it + 1) & 1);
    }
  }
  vmcnt_wait<0>();  // the tail's re-read DMA must land before the LDS is reused
  __syncthreads();  // Q/dO tiles dead: reuse LDS as per-wave output staging
  const float one[4] = {1.f, 1.f, 1.f, 1.f};
  if (wk_lo < Sk) {
    bf16_t* T = smem + w * 16 * (D + kOutPad);
    store_tile16<D>(T, D + kOutPad, dKa, one, dk, dks, b, hk, wk_lo, min(16, Sk - wk_lo));
    store_tile16<D>(T, D + kOutPad, dVa, one, dv, dvs, b, hk, wk_lo, min(16, Sk - wk_lo));
  }
}

// D = 256: K / V tiles by LDS-DMA into row-pair images (no staging VGPRs, no per-element load
// predicates -- those became 8 divergent branches per step) prefetched one tile ahead; smaller D:
// register staging (Tile2) into padded rows.  The mask is a select in front of the exp.
// delta = rowsum(dO * O) of the wave's queries is computed here from the dO fragments the kernel
// holds anyway (+ one pass over the O row) and written out for the dK/dV kernel, which runs after
// this one -- no separate delta pass over O and dO.
// RGD: DMA ring slots (2: one tile of prefetch, 3: two); FOLD: compute delta here (else read it)
// GQA: workgroups per (query block, KV head, batch), the q-heads splitting the waves (as the forward)
template <int D, int NW, int RGD = 2, bool FOLD = true, bool GQA = false>
__global__ __launch_bounds__(64 * NW) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const bf16_t* __restrict__ o, const float* __restrict__ lse,
    float* __restrict__ delta, bf16_t* __restrict__ dq, AttnStrides qs, AttnStrides ks, AttnStrides vs,
    AttnStrides dos, AttnStrides oss, AttnStrides dqs, int H, int Hkv, int Sq, int Sk, float scale, int causal,
    int window, const int* __restrict__ kv_lens) {
  constexpr bool kDma = D == 256;
  constexpr int NT = 64 * NW, BK = kSplitBK, LD = D + kSplitPad;
  constexpr int TILE = kDma ? kPairTile : BK * LD;
  // DMA: a 3-slot ring, two tiles in flight (a step is only 48 MFMAs per wave: one tile of prefetch
  // leaves the load latency exposed); register staging: 2 buffers
  constexpr int RG = kDma ? RGD : 2, OPT = 2 * (16 / NW);  // ring slots; DMA ops per wave per tile
  constexpr int PF = RG - 1;                                // tiles of prefetch
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];  // slot j: K at smem + 2 j TILE, V after it
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, c16 = lane & 15;
  int tx, hx, b;
  split_task(tx, hx, b);
  const int wph = GQA ? NW / (H / Hkv) : NW;  // waves per q-head
  const int bq = 16 * wph;                     // query rows per workgroup
  const int h = GQA ? hx * (H / Hkv) + w / wph : hx, hk = GQA ? hx : h / (H / Hkv);
  const int q0 = tx * bq;
  const int kv_len = kv_lens ? min(kv_lens[b], Sk) : Sk;
  const int coff = Sk - Sq;
  const float c2 = scale * kLog2e;
  const int wq_lo = q0 + 16 * (GQA ? w % wph : w), wq_hi = wq_lo + 15;
  const int qi = wq_lo + c16;
  int kend = kv_len;
  if (causal) kend = min(kend, q0 + bq + coff);
  int kstart = 0;
  if (window > 0) kstart = max(0, q0 + coff - window + 1) / BK * BK;
  const int nt = kend > kstart ? (kend - kstart + BK - 1) / BK : 0;  // key tiles, WG-uniform
  Tile2<D, NT> tl;
  auto load = [&](int kb, int j) {  // start fetching key tile kb into slot j
    if constexpr (kDma) {
      dma_tile32_prs<NW>(smem + 2 * j * TILE, k, ks, b, hk, kb, kv_len);  // rows past kv_len: clamped, masked
      dma_tile32_prs<NW>(smem + (2 * j + 1) * TILE, v, vs, b, hk, kb, kv_len);
    } else {
      tl.load(k, v, ks, vs, b, hk, kb, min(BK, kv_len - kb));
    }
  };
  auto land = [&](int j) {
    if constexpr (kDma) vmcnt_wait<0>();
    else tl.store(smem + 2 * j * TILE, smem + (2 * j + 1) * TILE);
  };
  auto frow = [&](const bf16_t* t, int r0, int c0) {
    if constexpr (kDma) return frag_row_prs(t, r0, c0);  // swizzled pair images (conflict-free)
    else return frag_row(t, LD, r0, c0);
  };
  auto ftr = [&](const bf16_t* t, int c0) {
    if constexpr (kDma) return frag_tr_prs(t, c0);
    else return frag_tr_perm(t, LD, 0, c0);
  };
  if constexpr (kDma) {  // tiles 0 .. PF - 1 (past the end: the last tile again, keeping the counts uniform)
    if (nt > 0) {
#pragma unroll
      for (int t = 0; t < PF; ++t) load(kstart + min(t, nt - 1) * BK, t);
    }
  } else {
    if (nt > 0) load(kstart, 0);
  }
  bf16x8_t qf[D / 32], df[D / 32];  // B operands: Q[qi][32 s + 8 g + j], dO[qi][...]
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    const bool ok = qi < Sq;
    qf[s] = ok ? *reinterpret_cast<const bf16x8_t*>(q + b * qs.sb + (long)qi * qs.ss + h * qs.sh + s * 32 + 8 * g)
               : bf16x8_t{};
    df[s] = ok ? *reinterpret_cast<const bf16x8_t*>(dout + b * dos.sb + (long)qi * dos.ss + h * dos.sh + s * 32 + 8 * g)
               : bf16x8_t{};
  }
  const float lq = qi < Sq ? lse[((long)b * H + h) * Sq + qi] * kLog2e : 1e30f;
  float dlq = 0.f;  // delta of query qi: this lane's 64 of the D products, summed over the 4 lane groups
  if constexpr (!FOLD) {
    dlq = qi < Sq ? delta[((long)b * H + h) * Sq + qi] : 0.f;
  } else {
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    const bf16x8_t ov = qi < Sq ? *reinterpret_cast<const bf16x8_t*>(o + b * oss.sb + (long)qi * oss.ss + h * oss.sh +
                                                                     s * 32 + 8 * g)
                                : bf16x8_t{};
#pragma unroll
    for (int e = 0; e < 8; ++e) dlq += static_cast<float>(ov[e]) * static_cast<float>(df[s][e]);
  }
  dlq += xor16_pl(dlq);
  dlq += xor32_pl(dlq);
  if (g == 0 && qi < Sq) delta[((long)b * H + h) * Sq + qi] = dlq;
  }
  if constexpr (!kDma) {
    if (nt > 0) land(0);
  }
  f32x4_t dQa[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) dQa[n] = zero4();
  for (int j = 0; j < nt; ++j) {
    const int kb = kstart + j * BK;
    const bool more = j + 1 < nt;
    if constexpr (kDma) {
      vmcnt_wait<OPT * (PF - 1)>();  // this wave's pieces of tile j landed (later tiles may still fly)
      lds_barrier();                 // ... and every wave's; slot (j + PF) % RG, read in step j - 1, is free
      load(kstart + min(j + PF, nt - 1) * BK, (j + PF) % RG);
    } else {
      if (more) load(kb + BK, (j + 1) & 1);  // registers: in flight across the raw barrier
      lds_barrier();  // tile j stored by every wave; buffer (j + 1) & 1, read in step j - 1, is free
    }
    const bf16_t* Ks = smem + 2 * (j % RG) * TILE;
    const bf16_t* Vs = Ks + TILE;
    const bool live = wq_lo < Sq && (!causal || kb <= wq_hi + coff) &&
                      (window <= 0 || wq_lo + coff - (kb + BK - 1) < window);
    if (live) {
      f32x4_t st[2], dpt[2];  // [t][i] = S^T / dP^T [key kb + 16 t + 4 g + i][qi]
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        st[t] = zero4();
        dpt[t] = zero4();
#pragma unroll
        for (int s = 0; s < D / 32; ++s) {
          st[t] = mfma16(frow(Ks, 16 * t, s * 32), qf[s], st[t]);
          dpt[t] = mfma16(frow(Vs, 16 * t, s * 32), df[s], dpt[t]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = qi < Sq && attn_allowed(qi, kb + 16 * t + 4 * g + i, kv_len, coff, causal, window);
          float x = st[t][i] * c2 - lq;
          asm volatile("" : "+v"(x));  // a select, not a branch around the exp
          const float p = fast_exp2(ok ? x : -INFINITY);
          dpt[t][i] = p * (dpt[t][i] - dlq) * scale;
        }
      }
      const bf16x8_t da = pack_c2a(dpt[0], dpt[1]);  // A: m = query, k = key (permuted)
#pragma unroll
      for (int n = 0; n < D / 16; ++n) dQa[n] = mfma16(da, ftr(Ks, n * 16), dQa[n]);
    }
    if constexpr (!kDma) {
      if (more) land((j + 1) & 1);
    }
  }
  vmcnt_wait<0>();  // the tail's re-read DMA must land before the LDS is reused
  __syncthreads();
  const float one[4] = {1.f, 1.f, 1.f, 1.f};
  if (wq_lo < Sq) store_tile16<D>(smem + w * 16 * (D + kOutPad), D + kOutPad, dQa, one, dq, dqs, b, h, wq_lo, min(16, Sq - wq_lo));
}

static AttnStrides mk(const long* st) { return AttnStrides{st[0], st[1], st[2]}; }

bool attn_short_path(int D, int Sq, int Sk, int window) {
  return D == 64 && Sq == Sk && Sq <= kShortS && window <= 0;
}

static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}

// MFT_ATTN_V1=1 keeps the previous long-sequence kernels (fp32 dQ atomics, per-q-head GQA dK/dV)
// for A/B measurements.
int attn_bwd_path(int D, int Sq, int Sk, int window) {
  if (attn_short_path(D, Sq, Sk, window)) return 0;
  static const int v1 = env_int("MFT_ATTN_V1", 0);
  return v1 == 1 ? 1 : 2;
}

// waves per workgroup of the split kernels (4 or 8): MFT_ATTN_NW_{FWD,DKDV,DQ}
static int split_nw(const char* name, int dflt) {
  const int v = env_int(name, dflt);
  return v == 4 || v == 8 ? v : dflt;
}

template <int D, int NW>
static void fwd_split_launch(const AttnArgs& a, hipStream_t stream) {
  const size_t shm = split_shm<D, NW>(0);
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_split_kernel<D, NW>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  attn_fwd_split_kernel<D, NW><<<dim3(cdiv(a.Sq, 16 * NW), a.H, a.B), 64 * NW, shm, stream>>>(
      a.q, a.k, a.v, a.o, a.lse, mk(a.q_st), mk(a.k_st), mk(a.v_st), mk(a.o_st), a.H, a.Hkv, a.Sq, a.Sk, a.scale,
      a.causal, a.window, a.kv_lens);
}

template <int D, int NW, int RPW, bool SWZ, int RGF = 4, bool GQA = false>
static void fwd_dma_launch_rpw(const AttnArgs& a, hipStream_t stream) {
  const size_t shm = std::max(D == 256 ? sizeof(bf16_t) * RGF * 2 * kPairTile : sizeof(bf16_t) * kRing * 2 * kSplitBK * D,
                              sizeof(bf16_t) * NW * 16 * (D + kSplitPad));
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_dma_kernel<D, NW, RPW, SWZ, RGF, GQA>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int G = a.H / a.Hkv;
  if (GQA && (a.H % a.Hkv || G < 2 || NW % G)) {
    fprintf(stderr, "mft::attn_fwd: GQA workgroups need H / Hkv to divide %d waves (H=%d Hkv=%d)\n", NW, a.H, a.Hkv);
    abort();
  }
  const dim3 grid = GQA ? dim3(cdiv(a.Sq, RPW * (NW / G)), a.Hkv, a.B) : dim3(cdiv(a.Sq, RPW * NW), a.H, a.B);
  attn_fwd_dma_kernel<D, NW, RPW, SWZ, RGF, GQA><<<grid, 64 * NW, shm, stream>>>(
      a.q, a.k, a.v, a.o, a.lse, mk(a.q_st), mk(a.k_st), mk(a.v_st), mk(a.o_st), a.H, a.Hkv, a.Sq, a.Sk, a.scale,
      a.causal, a.window, a.kv_lens, a.o_pad);
}

// MFT_ATTN_RPW=16|32: query rows per wave of the DMA forward (A/B).  32 rows need the 512-register
// budget of one wave per SIMD (4 waves: 128 queries per workgroup, as 8 x 16).
template <int D>
static void fwd_dma_launch(const AttnArgs& a, hipStream_t stream) {
  static const int rpw = env_int("MFT_ATTN_RPW", 16);
  // MFT_ATTN_SWZ=0: the plain (2-way bank-conflicted) K / V pair images, for A/B
  static const int swz = env_int("MFT_ATTN_SWZ", 1);
  // GQA-packed workgroups (all q-heads of a KV head) with a 2-slot ring (two workgroups per CU) where
  // H / Hkv divides the waves: 138 us vs 167 us per-q-head at the Gemma-3 bench shape (B 256, S 256, H 4,
  // Hkv 1; profiles/r5_attn_gqa_fwd.txt).  A/B knobs: MFT_ATTN_GQA=0|1, MFT_ATTN_FWD_RING=2|3|4 (D = 256
  // ring depth; 0 = 2 packed, 4 per-q-head), MFT_ATTN_NW_FWD=4|8
  static const int gqa = env_int("MFT_ATTN_GQA", 1);
  static const int ring_env = env_int("MFT_ATTN_FWD_RING", 0);
  static const int nw = split_nw("MFT_ATTN_NW_FWD", 8);
  const int G = a.H / a.Hkv;
  if (D == 256 && rpw == 16 && swz && gqa && a.H % a.Hkv == 0 && G >= 2 && nw % G == 0) {
    const int ring = ring_env ? ring_env : 2;
    if (nw == 4) {
      if (ring == 2) return fwd_dma_launch_rpw<D, 4, 16, true, 2, true>(a, stream);
      return fwd_dma_launch_rpw<D, 4, 16, true, 4, true>(a, stream);
    }
    if (ring == 2) return fwd_dma_launch_rpw<D, 8, 16, true, 2, true>(a, stream);
    return fwd_dma_launch_rpw<D, 8, 16, true, 4, true>(a, stream);
  }
  const int ring = ring_env ? ring_env : 4;
  if (D == 256 && rpw == 16 && swz && (ring != 4 || nw != 8)) {
    if (nw == 4) {
      if (ring == 2) return fwd_dma_launch_rpw<D, 4, 16, true, 2>(a, stream);
      if (ring == 3) return fwd_dma_launch_rpw<D, 4, 16, true, 3>(a, stream);
      return fwd_dma_launch_rpw<D, 4, 16, true, 4>(a, stream);
    }
    if (ring == 2) return fwd_dma_launch_rpw<D, 8, 16, true, 2>(a, stream);
    if (ring == 3) return fwd_dma_launch_rpw<D, 8, 16, true, 3>(a, stream);
  }
  if (rpw == 32) fwd_dma_launch_rpw<D, 4, 32, true>(a, stream);
  else if (swz) fwd_dma_launch_rpw<D, 8, 16, true>(a, stream);
  else fwd_dma_launch_rpw<D, 8, 16, false>(a, stream);
}

template <int D, int NW, int RGK = 3>
static void dkdv_split_launch(const AttnBwdArgs& a, hipStream_t stream) {
  constexpr int LD = D + kSplitPad;
  // two {Q, dO} tile buffers (row-pair images for the D = 256 LDS-DMA form) + their row statistics, or the
  // epilogue's per-wave output staging
  const size_t shm = std::max(D == 256 ? sizeof(bf16_t) * 2 * RGK * kPairTile + sizeof(float) * 2 * RGK * kSplitBK
                                        : sizeof(bf16_t) * 4 * kSplitBK * LD + sizeof(float) * 4 * kSplitBK,
                              sizeof(bf16_t) * NW * 16 * LD);
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_dkdv_kernel<D, NW, RGK>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  attn_bwd_dkdv_kernel<D, NW, RGK><<<dim3(cdiv(a.Sk, 16 * NW), a.Hkv, a.B), 64 * NW, shm, stream>>>(
      a.q, a.k, a.v, a.dout, a.lse, a.delta, a.dk, a.dv, mk(a.q_st), mk(a.k_st), mk(a.v_st), mk(a.do_st),
      mk(a.dk_st), mk(a.dv_st), a.H, a.Hkv, a.Sq, a.Sk, a.scale, a.causal, a.window, a.kv_lens);
}

template <int D, int NW, int RGD, bool FOLD, bool GQA = false>
static void dq_split_launch_v(const AttnBwdArgs& a, hipStream_t stream) {
  const size_t shm = D == 256 ? std::max(sizeof(bf16_t) * RGD * 2 * kPairTile, sizeof(bf16_t) * NW * 16 * (D + kSplitPad))
                              : split_shm<D, NW>(0);
  static bool attr = false;
  if (!attr) {
    MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_dq_kernel<D, NW, RGD, FOLD, GQA>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int G = a.H / a.Hkv;
  if (GQA && (a.H % a.Hkv || G < 2 || NW % G)) {
    fprintf(stderr, "mft::attn_bwd: GQA dQ workgroups need H / Hkv to divide %d waves (H=%d Hkv=%d)\n", NW, a.H, a.Hkv);
    abort();
  }
  const dim3 grid = GQA ? dim3(cdiv(a.Sq, 16 * (NW / G)), a.Hkv, a.B) : dim3(cdiv(a.Sq, 16 * NW), a.H, a.B);
  attn_bwd_dq_kernel<D, NW, RGD, FOLD, GQA><<<grid, 64 * NW, shm, stream>>>(
      a.q, a.k, a.v, a.dout, a.o, a.lse, a.delta, a.dq, mk(a.q_st), mk(a.k_st), mk(a.v_st), mk(a.do_st), mk(a.o_st),
      mk(a.dq_st), a.H, a.Hkv, a.Sq, a.Sk, a.scale, a.causal, a.window, a.kv_lens);
}
// D = 256 A/B knobs: MFT_ATTN_DQ_RING=2|3 (DMA ring slots), MFT_ATTN_DELTA_FOLD=1|0 (delta in the dQ
// kernel, or by the separate pass).  Measured at B 256 S 256 H 4 Hkv 1 (profiles/r3_attn256_bwd_ab.txt):
// dQ 240 us with 2 slots + fold vs 252 (3 slots), and 207 + 45 (delta pass) unfolded
static bool delta_fold(int D) {
  static const int f = env_int("MFT_ATTN_DELTA_FOLD", 1);
  return D != 256 || f != 0;
}
// GQA-packed dQ workgroups (all q-heads of a KV head; MFT_ATTN_GQA_DQ=0 per-q-head, A/B): dQ + dK/dV
// 408 us vs 455 us at the Gemma-3 bench shape (profiles/r5_attn_gqa_fwd.txt)
static bool dq_gqa() {
  static const int v = env_int("MFT_ATTN_GQA_DQ", 1);
  return v != 0;
}
template <int D, int NW>
static void dq_split_launch(const AttnBwdArgs& a, hipStream_t stream) {
  if constexpr (D == 256) {
    static const int ring = env_int("MFT_ATTN_DQ_RING", 2);
    const bool fold = delta_fold(D);
    const int G = a.H / a.Hkv;
    if (dq_gqa() && ring == 2 && fold && a.H % a.Hkv == 0 && G >= 2 && NW % G == 0)
      return dq_split_launch_v<D, NW, 2, true, true>(a, stream);
    if (ring == 2) {
      if (fold) dq_split_launch_v<D, NW, 2, true>(a, stream);
      else dq_split_launch_v<D, NW, 2, false>(a, stream);
    } else {
      if (fold) dq_split_launch_v<D, NW, 3, true>(a, stream);
      else dq_split_launch_v<D, NW, 3, false>(a, stream);
    }
  } else {
    dq_split_launch_v<D, NW, 2, true>(a, stream);
  }
}


template <int D>
// returns whether the launched kernel wrote the o_pad zero columns itself (short and DMA paths)
static bool fwd_launch(const AttnArgs& a, hipStream_t stream) {
  if constexpr (D == 64) {
    if (attn_short_path(D, a.Sq, a.Sk, a.window)) {
      const size_t shm = sizeof(bf16_t) * (2 * kShortS * D + 8 * 16 * (D + 8));
      static bool attr = false;
      if (!attr) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_short2_kernel<D>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
      }
      attn_fwd_short2_kernel<D><<<dim3(a.H, a.B), 512, shm, stream>>>(a.q, a.k, a.v, a.o, a.lse, mk(a.q_st), mk(a.k_st),
                                                                       mk(a.v_st), mk(a.o_st), a.H, a.Hkv, a.Sq, a.scale,
                                                                       a.causal, a.kv_lens, a.o_pad);
      return true;
    }
  }
  if (attn_bwd_path(D, a.Sq, a.Sk, a.window) == 2) {
    if constexpr (D >= 128) {
      static const int dma = env_int("MFT_ATTN_DMA", 1);
      if (dma) {
        fwd_dma_launch<D>(a, stream);
        return true;
      }
    }
    if (split_nw("MFT_ATTN_NW_FWD", 8) == 8) fwd_split_launch<D, 8>(a, stream);
    else fwd_split_launch<D, 4>(a, stream);
    return false;
  }
  constexpr int BQ = 64, BK = 64, LDP = BK + 8;
  const size_t shm = sizeof(bf16_t) * (2 * BK * D + 4 * 16 * LDP);
  dim3 grid(cdiv(a.Sq, BQ), a.H, a.B);
  attn_fwd_kernel<D><<<grid, 256, shm, stream>>>(a.q, a.k, a.v, a.o, a.lse, mk(a.q_st), mk(a.k_st), mk(a.v_st),
                                                 mk(a.o_st), a.H, a.Hkv, a.Sq, a.Sk, a.scale, a.causal, a.window,
                                                 a.kv_lens);
  return false;
}

template <int D>
static void bwd_launch(const AttnBwdArgs& a, hipStream_t stream) {
  if constexpr (D == 64) {
    if (attn_short_path(D, a.Sq, a.Sk, a.window)) {
      // K, V, dO + max(Q + lse / delta, the per-wave output staging at pitch D + 8 that overlays them)
      const size_t shm = sizeof(bf16_t) * 3 * kShortS * D +
                         std::max(sizeof(bf16_t) * kShortS * D + sizeof(float) * 2 * kShortS, sizeof(bf16_t) * 8 * 16 * (D + 8));
      static bool attr = false;
      if (!attr) {
        MFT_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_short2_kernel<D>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
      }
      const int per_qhead = a.H != a.Hkv;
      attn_bwd_short2_kernel<D><<<dim3(a.H, a.B), 512, shm, stream>>>(
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
  if (attn_bwd_path(D, a.Sq, a.Sk, a.window) == 2) {
    if (!delta_fold(D)) {
      const long rows = (long)a.B * a.H * a.Sq;
      attn_bwd_delta_kernel<D><<<cdiv(rows * (D / 8), 256), 256, 0, stream>>>(a.o, a.dout, a.delta, mk(a.o_st),
                                                                              mk(a.do_st), a.B, a.H, a.Sq);
    }
    // dQ first: it writes delta (rowsum dO * O), which the dK/dV kernel reads
    // GQA-packed dQ (D = 256, H / Hkv | 4): 4 waves, i.e. 16 query rows of every q-head per workgroup
    const int G = a.H / a.Hkv;
    const bool packed = D == 256 && a.H % a.Hkv == 0 && G >= 2 && 4 % G == 0 && dq_gqa();
    if (split_nw("MFT_ATTN_NW_DQ", packed ? 4 : 8) == 8) dq_split_launch<D, 8>(a, stream);
    else dq_split_launch<D, 4>(a, stream);
    // D = 256: 8 waves (its 3-slot DMA ring holds one workgroup per CU; 4 waves would leave one per SIMD)
    // D = 256: a 2-slot ring, two workgroups per CU (399 us dQ + dK/dV vs 411 us with 3 slots at the Gemma-3
    // bench shape, profiles/r5_attn_gqa_fwd.txt; MFT_ATTN_DKDV_RING=3 for A/B)
    static const int dkdv_ring = env_int("MFT_ATTN_DKDV_RING", 2);
    if (D == 256 && dkdv_ring == 2) {
      if (split_nw("MFT_ATTN_NW_DKDV", 8) == 8) dkdv_split_launch<D, 8, 2>(a, stream);
      else dkdv_split_launch<D, 4, 2>(a, stream);
    } else if (split_nw("MFT_ATTN_NW_DKDV", D == 256 ? 8 : 4) == 8) dkdv_split_launch<D, 8>(a, stream);
    else dkdv_split_launch<D, 4>(a, stream);
    return;
  }
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
  if (a.o_pad % 8 || (a.o_pad > 0 && a.o_st[0] != (long)a.Sq * a.o_st[1])) {
    fprintf(stderr, "attn_fwd: o_pad %d needs a multiple of 8 and batch-contiguous output rows\n", a.o_pad);
    abort();
  }
  bool padded = false;
  switch (a.D) {
    case 64: padded = fwd_launch<64>(a, s); break;
    case 128: padded = fwd_launch<128>(a, s); break;
    case 256: padded = fwd_launch<256>(a, s); break;
    default: fprintf(stderr, "attn_fwd: unsupported head dim %d\n", a.D); abort();
  }
  if (a.o_pad > 0 && !padded) zero_cols(a.o, a.o_st[1], (long)a.B * a.Sq, a.H * a.D, a.o_pad, s);
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
