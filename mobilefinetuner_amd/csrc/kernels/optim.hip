// Fused optimizer kernels: global grad-norm (two-stage, deterministic), non-finite check, and a
// single-launch AdamW over the flat fp32 parameter/grad/moment buffers.
// Replaces Adam::step (optim/adam.cpp:25-90, per-element loops per tensor with coupled L2 decay,
// SURVEY §8 Q8) and the three copies of clip_grad_norm (gpt2_lora_finetune/main.cpp:491-516,
// optim/gemma_trainer.cpp:84-102, optim/trainer.cpp:66-92).
// Everything that depends on step-time values (lr, step count, grad-norm, skip flag) is read from
// device memory, so a captured hipGraph of the whole train step replays without host sync.
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace mft {

int sumsq_blocks(long n) {
  long b = (n / 4 + 255) / 256;
  if (b < 1) b = 1;
  return (int)(b < 1024 ? b : 1024);
}

__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* __restrict__ x, long n, float* __restrict__ part) {
  __shared__ float red[16];
  float s = 0.f;
  const long n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = x4[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0)
    for (long i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) s += x[i] * x[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void sumsq_final_kernel(const float* __restrict__ part, int nb, float* __restrict__ out, int accumulate) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + s : s;
}

void sumsq(const float* x, long n, float* partial, float* out, int accumulate, hipStream_t st) {
  const int nb = sumsq_blocks(n);
  sumsq_partial_kernel<<<nb, 256, 0, st>>>(x, n, partial);
  sumsq_final_kernel<<<1, 256, 0, st>>>(partial, nb, out, accumulate);
}

__global__ void nonfinite_kernel(const float* __restrict__ x, long n, int* __restrict__ flag) {
  int bad = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

void nonfinite_check(const float* x, long n, int* flag, hipStream_t st) {
  long g = (n + 255) / 256;
  nonfinite_kernel<<<(int)(g < 1024 ? (g > 0 ? g : 1) : 1024), 256, 0, st>>>(x, n, flag);
}

// A step is skipped when any grad is non-finite (the flag, all-reduced over ranks by the ZeRO
// optimizers so every rank skips together) or when the global grad norm itself is non-finite.
__device__ __forceinline__ bool adamw_skip(const int* nonfinite, const float* sumsq) {
  return (nonfinite && *nonfinite) || (sumsq && !isfinite(*sumsq));
}

// bf16 moments (MB): stochastic rounding with a counter hash of (step, GLOBAL element index: the
// launch's sr_offset + local index, so chunked / sharded launches draw independent noise) -- round-to-nearest
// would freeze v under beta2 = 0.999 (a 0.1% change is below half a bf16 ulp) and bias m; SR keeps
// both unbiased.  The fp32 master weights and the update itself stay fp32.
__device__ __forceinline__ uint32_t sr_hash(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352DU;
  x ^= x >> 15;
  x *= 0x846CA68BU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint16_t f2bf_sr(float f, uint32_t r) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7F800000U) == 0x7F800000U) return (uint16_t)(u >> 16);  // inf / nan
  return (uint16_t)((u + (r & 0xFFFFU)) >> 16);
}

template <bool MB>
__device__ __forceinline__ float ld_mom(const void* p, long i) {
  if constexpr (MB) return bf2f(reinterpret_cast<const uint16_t*>(p)[i]);
  else return reinterpret_cast<const float*>(p)[i];
}
template <bool MB>
__device__ __forceinline__ void st_mom(void* p, long i, float x, uint32_t r) {
  if constexpr (MB) reinterpret_cast<uint16_t*>(p)[i] = f2bf_sr(x, r);
  else reinterpret_cast<float*>(p)[i] = x;
}

template <bool MB>
using Mom4 = typename std::conditional<MB, uint2, float4>::type;

// U > 1: each thread keeps U float4 groups in flight (all loads first, then the updates) -- the
// host-moment launches that run beside the compute kernels on a few CUs are bound by PCIe latency,
// so their memory-level parallelism has to come from each wave (engine/zero3.cpp)
template <bool MB, int U>
__global__ __launch_bounds__(256) void adamw_kernel(AdamWArgs a) {
  if (a.enable && *a.enable == 0) return;         // delayed optimizer: no gradients pending
  if (adamw_skip(a.nonfinite, a.sumsq)) return;  // skip-step on NaN/Inf grads (fault tolerance)
  const float lr = *a.lr_ptr;
  const float t = *a.step_ptr + 1.f;  // *step_ptr counts APPLIED steps; adamw_commit advances it
  const float bc1 = 1.f - powf(a.beta1, t);
  const float bc2 = 1.f - powf(a.beta2, t);
  float clip = 1.f;
  if (a.sumsq) {
    const float norm = sqrtf(*a.sumsq);
    if (norm > a.max_norm) clip = a.max_norm / (norm + 1e-6f);
  }
  const float step_size = lr / bc1;
  const float rbc2 = 1.f / sqrtf(bc2);
  const float decay = a.l2_coupled ? 1.f : 1.f - lr * a.weight_decay;
  const long n4 = a.n / 4;
  const uint32_t seed = sr_hash((uint32_t)t * 0x9E3779B9U);
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += stride * U) {
    float4 P[U], G[U];
    Mom4<MB> M[U], V[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i < n4) {
        P[u] = reinterpret_cast<const float4*>(a.p)[i];
        G[u] = reinterpret_cast<const float4*>(a.g)[i];
        M[u] = reinterpret_cast<const Mom4<MB>*>(a.m)[i];
        V[u] = reinterpret_cast<const Mom4<MB>*>(a.v)[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i >= n4) break;
      float pp[4] = {P[u].x, P[u].y, P[u].z, P[u].w}, gg[4] = {G[u].x, G[u].y, G[u].z, G[u].w}, mm[4], vv[4];
      if constexpr (MB) {
        const uint2 mb = M[u], vb = V[u];
        mm[0] = __uint_as_float(mb.x << 16); mm[1] = __uint_as_float(mb.x & 0xFFFF0000U);
        mm[2] = __uint_as_float(mb.y << 16); mm[3] = __uint_as_float(mb.y & 0xFFFF0000U);
        vv[0] = __uint_as_float(vb.x << 16); vv[1] = __uint_as_float(vb.x & 0xFFFF0000U);
        vv[2] = __uint_as_float(vb.y << 16); vv[3] = __uint_as_float(vb.y & 0xFFFF0000U);
      } else {
        const float4 m = M[u], v = V[u];
        mm[0] = m.x; mm[1] = m.y; mm[2] = m.z; mm[3] = m.w;
        vv[0] = v.x; vv[1] = v.y; vv[2] = v.z; vv[3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float gj = gg[j] * clip;
        if (a.l2_coupled) gj += a.weight_decay * pp[j];
        mm[j] = a.beta1 * mm[j] + (1.f - a.beta1) * gj;
        vv[j] = a.beta2 * vv[j] + (1.f - a.beta2) * gj * gj;
        float denom = sqrtf(vv[j]) * rbc2 + a.eps;
        if (!MB && a.vmax) {  // AMSGrad, the reference's rule (optim/adam.cpp:75-80): the running max of
          // the BIAS-CORRECTED second moment, v_hat = max(v_hat, v / bc2), used as is in the denominator
          const float vd = fmaxf(a.vmax[4 * i + j], vv[j] * (rbc2 * rbc2));
          a.vmax[4 * i + j] = vd;
          denom = sqrtf(vd) + a.eps;
        }
        pp[j] = pp[j] * decay - step_size * mm[j] / denom;
      }
      reinterpret_cast<float4*>(a.p)[i] = make_float4(pp[0], pp[1], pp[2], pp[3]);
      if constexpr (MB) {
        const uint32_t r = sr_hash(seed ^ (uint32_t)(a.sr_offset / 4 + i)), r2 = sr_hash(r);
        uint2 mb, vb;
        mb.x = (uint32_t)f2bf_sr(mm[0], r) | ((uint32_t)f2bf_sr(mm[1], r >> 16) << 16);
        mb.y = (uint32_t)f2bf_sr(mm[2], r2) | ((uint32_t)f2bf_sr(mm[3], r2 >> 16) << 16);
        const uint32_t r3 = sr_hash(r2), r4 = sr_hash(r3);
        vb.x = (uint32_t)f2bf_sr(vv[0], r3) | ((uint32_t)f2bf_sr(vv[1], r3 >> 16) << 16);
        vb.y = (uint32_t)f2bf_sr(vv[2], r4) | ((uint32_t)f2bf_sr(vv[3], r4 >> 16) << 16);
        reinterpret_cast<uint2*>(a.m)[i] = mb;
        reinterpret_cast<uint2*>(a.v)[i] = vb;
      } else {
        reinterpret_cast<float4*>(a.m)[i] = make_float4(mm[0], mm[1], mm[2], mm[3]);
        reinterpret_cast<float4*>(a.v)[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
      }
      if (a.shadow) {
        uint2 sh;
        sh.x = pack_bf2(pp[0], pp[1]);
        sh.y = pack_bf2(pp[2], pp[3]);
        reinterpret_cast<uint2*>(a.shadow)[i] = sh;
      }
    }
  }
  if (blockIdx.x == 0) {
    for (long i = n4 * 4 + threadIdx.x; i < a.n; i += blockDim.x) {
      float gj = a.g[i] * clip;
      float pj = a.p[i];
      if (a.l2_coupled) gj += a.weight_decay * pj;
      const float mj = a.beta1 * ld_mom<MB>(a.m, i) + (1.f - a.beta1) * gj;
      const float vj = a.beta2 * ld_mom<MB>(a.v, i) + (1.f - a.beta2) * gj * gj;
      float denom = sqrtf(vj) * rbc2 + a.eps;
      if (!MB && a.vmax) {  // AMSGrad (reference rule, as above)
        const float vd = fmaxf(a.vmax[i], vj * (rbc2 * rbc2));
        a.vmax[i] = vd;
        denom = sqrtf(vd) + a.eps;
      }
      pj = pj * decay - step_size * mj / denom;
      a.p[i] = pj;
      const uint32_t r = sr_hash(seed ^ 0x5bd1e995U ^ (uint32_t)(a.sr_offset + i));
      st_mom<MB>(a.m, i, mj, r);
      st_mom<MB>(a.v, i, vj, r >> 16);
      if (a.shadow) a.shadow[i] = f2bf(pj);
    }
  }
}

// step += 1 only when the update was applied (a skipped step must not advance bias correction);
// flag_out (optional) records whether the step was skipped -- with clipping on, a non-finite grad
// makes the global norm^2 non-finite, so that one reduction replaces the separate scan of the grads
__global__ void adamw_commit_kernel(float* step, const int* nonfinite, const float* sumsq, int* flag_out, int* enable,
                                    int clear_enable) {
  if (threadIdx.x == 0) {
    if (enable && *enable == 0) return;  // nothing was pending: nothing applied, nothing to record
    const bool skip = adamw_skip(nonfinite, sumsq);
    if (!skip) step[0] += 1.f;
    if (flag_out) flag_out[0] = skip ? 1 : 0;
    if (enable && clear_enable) *enable = 0;
  }
}

void adamw_commit(float* step, const int* nonfinite, const float* sumsq, hipStream_t st, int* flag_out, int* enable,
                  int clear_enable) {
  adamw_commit_kernel<<<1, 64, 0, st>>>(step, nonfinite, sumsq, flag_out, enable, clear_enable);
}

void adamw_step(const AdamWArgs& a, hipStream_t st) {
  if (a.vmax && a.moments_bf16) {
    fprintf(stderr, "mft::adamw_step: AMSGrad needs fp32 moments\n");
    abort();
  }
  long g = (a.n / 4 + 255) / 256;
  if (g < 1) g = 1;
  const long cap = a.max_grid > 0 ? a.max_grid : 2048;
  const int grid = (int)(g < cap ? g : cap);
  static const int unroll = [] {  // MFT_OPT_UNROLL=4|8: float4 groups in flight in a bounded launch
    const char* e = std::getenv("MFT_OPT_UNROLL");
    return e && std::atoi(e) == 8 ? 8 : 4;
  }();
  if (a.max_grid > 0 && unroll == 8) {
    if (a.moments_bf16) adamw_kernel<true, 8><<<grid, 256, 0, st>>>(a);
    else adamw_kernel<false, 8><<<grid, 256, 0, st>>>(a);
  } else if (a.max_grid > 0) {  // a bounded launch beside other kernels: more loads in flight per thread
    if (a.moments_bf16) adamw_kernel<true, 4><<<grid, 256, 0, st>>>(a);
    else adamw_kernel<false, 4><<<grid, 256, 0, st>>>(a);
  } else {
    if (a.moments_bf16) adamw_kernel<true, 1><<<grid, 256, 0, st>>>(a);
    else adamw_kernel<false, 1><<<grid, 256, 0, st>>>(a);
  }
}

}  // namespace mft
