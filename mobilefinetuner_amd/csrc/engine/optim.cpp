// libmft engine: flat params + fused AdamW + schedules (see optim.h).
#include "engine/optim.h"

#include <algorithm>
#include <cmath>

#include "engine/autograd.h"
#include "engine/ops.h"
#include "kernels.h"

namespace mft {
namespace eng {

namespace {
constexpr int64_t kAlign = 64;  // every param starts 16-B aligned in fp32 and bf16 views
int64_t round_up(int64_t n, int64_t a) { return (n + a - 1) / a * a; }
}  // namespace

FlatParams::FlatParams(std::vector<std::pair<std::string, Param*>> ps) : params(std::move(ps)) {
  NoGradGuard ng;
  int64_t off = 0;
  for (auto& kv : params) {
    offsets.push_back(off);
    off += round_up(kv.second->leaf.numel(), kAlign);
  }
  numel = round_up(std::max<int64_t>(off, kAlign), kAlign);
  master = zeros({numel}, DType::F32);
  grad = zeros({numel}, DType::F32);
  shadow = zeros({numel}, DType::BF16);
  for (size_t i = 0; i < params.size(); ++i) {
    Param& p = *params[i].second;
    const int64_t n = p.leaf.numel(), o = offsets[i];
    const bool fp32_compute = p.c.dtype() == DType::F32;
    Tensor mv = master.slice(0, o, o + n).view(p.leaf.shape());
    mv.copy_(p.leaf.detach());
    Tensor leaf = mv.alias();
    leaf.requires_grad_(true);
    leaf.set_grad(grad.slice(0, o, o + n).view(p.leaf.shape()));
    p.leaf = leaf;
    p.c = fp32_compute ? leaf.alias() : shadow.slice(0, o, o + n).view(leaf.shape());
    p.wt = Tensor();
  }
  refresh_shadow();
}

void FlatParams::zero_grad() { grad.zero_(); }

void FlatParams::refresh_shadow() { ::mft::cast_f32_bf16(master.data<float>(), (::mft::bf16_t*)shadow.data_ptr(), numel, current_stream()); }

AdamW::AdamW(FlatParams& flat, const AdamWConfig& cfg) : flat_(flat), cfg_(cfg) {
  NoGradGuard ng;
  m = zeros({flat.numel}, DType::F32);
  v = zeros({flat.numel}, DType::F32);
  lr_dev = full({1}, cfg.lr, DType::F32);
  step_dev = zeros({1}, DType::F32);
  sumsq_dev = zeros({1}, DType::F32);
  nonfinite_dev = zeros({1}, DType::I32);
  skipped_dev = zeros({1}, DType::I32);
}

void AdamW::set_lr(float lr) {
  cfg_.lr = lr;
  lr_dev.fill_(lr);  // the value travels as a kernel argument: no host-buffer race, no sync
}

void AdamW::step() {
  hipStream_t s = current_stream();
  const bool clip = cfg_.max_grad_norm > 0.f;
  if (clip) {
    Tensor part = empty({(int64_t)::mft::sumsq_blocks(flat_.numel)}, DType::F32);
    ::mft::sumsq(flat_.grad.data<float>(), flat_.numel, part.data<float>(), sumsq_dev.data<float>(), 0, s);
  }
  if (cfg_.skip_nonfinite) {
    nonfinite_dev.zero_();
    ::mft::nonfinite_check(flat_.grad.data<float>(), flat_.numel, nonfinite_dev.data<int>(), s);
  }
  ::mft::AdamWArgs a{};
  a.p = flat_.master.data<float>();
  a.g = flat_.grad.data<float>();
  a.m = m.data<float>();
  a.v = v.data<float>();
  a.n = flat_.numel;
  a.lr_ptr = lr_dev.data<float>();
  a.beta1 = cfg_.beta1;
  a.beta2 = cfg_.beta2;
  a.eps = cfg_.eps;
  a.weight_decay = cfg_.weight_decay;
  a.step_ptr = step_dev.data<float>();
  a.sumsq = clip ? sumsq_dev.data<float>() : nullptr;
  a.max_norm = cfg_.max_grad_norm;
  a.l2_coupled = cfg_.l2_coupled;
  a.shadow = (::mft::bf16_t*)flat_.shadow.data_ptr();
  a.nonfinite = cfg_.skip_nonfinite ? nonfinite_dev.data<int>() : nullptr;
  ::mft::adamw_step(a, s);
  ::mft::adamw_commit(step_dev.data<float>(), a.nonfinite, a.sumsq, s);
  if (cfg_.skip_nonfinite) {
    // skipped += nonfinite (int32 counters)
    k::Desc d = desc(skipped_dev), x = desc(nonfinite_dev);
    k::binary(d, d, x, k::B_ADD, 1.f, s);
  }
}

float AdamW::grad_norm() const { return std::sqrt(std::max(0.f, (float)sumsq_dev.item())); }
bool AdamW::skipped_last() const { return nonfinite_dev.to_vector_f32()[0] != 0.f; }
int64_t AdamW::applied_steps() const { return (int64_t)step_dev.item(); }

void AdamW::load_state(const Tensor& m_h, const Tensor& v_h, int64_t steps) {
  m.copy_(m_h);
  v.copy_(v_h);
  step_dev.fill_((double)steps);
}

float gpt2_cli_lr(int64_t step, float base, int64_t warmup, int64_t total, float min_ratio) {
  if (warmup > 0 && step < warmup) return base * (float)(step + 1) / (float)warmup;
  if (total <= warmup) return base;
  double p = (double)(step - warmup) / (double)std::max<int64_t>(1, total - warmup);
  p = std::min(std::max(p, 0.0), 1.0);
  const double c = 0.5 * (1.0 + std::cos(M_PI * p));
  return (float)(base * (min_ratio + (1.0 - min_ratio) * c));
}

float gemma_lr(int64_t step, float base, float ratio, int64_t total, bool cosine) {
  const int64_t warmup = ratio > 0 ? (int64_t)std::ceil(ratio * total) : 0;
  if (warmup > 0 && step <= warmup) return base * (float)step / (float)warmup;
  if (total <= warmup) return base;
  double p = (double)(step - warmup) / (double)std::max<int64_t>(1, total - warmup);
  p = std::min(std::max(p, 0.0), 1.0);
  return (float)(cosine ? base * 0.5 * (1.0 + std::cos(M_PI * p)) : base * (1.0 - p));
}

float trainer_lr(int64_t step, float base, int64_t warmup, int64_t total, bool cosine) {
  if (warmup > 0 && step < warmup) return base * (float)step / (float)warmup;
  double p = (double)(step - warmup) / (double)std::max<int64_t>(1, total - warmup);
  p = std::min(std::max(p, 0.0), 1.0);
  return (float)(cosine ? base * 0.5 * (1.0 + std::cos(M_PI * p)) : base * (1.0 - p));
}

}  // namespace eng
}  // namespace mft
