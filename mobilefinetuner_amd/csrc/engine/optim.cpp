// libmft engine: flat params + fused AdamW + schedules (see optim.h).
#include "engine/optim.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cstring>
#include <filesystem>

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

FlatParams::FlatParams(std::vector<std::pair<std::string, Param*>> ps, std::vector<int64_t> offs, int64_t total)
    : params(std::move(ps)) {
  NoGradGuard ng;
  if (!offs.empty()) {
    MFT_CHECK(offs.size() == params.size(), "FlatParams: one offset per parameter");
    offsets = std::move(offs);
    numel = total;
    for (size_t i = 0; i < params.size(); ++i)
      MFT_CHECK(offsets[i] % kAlign == 0 && offsets[i] + params[i].second->leaf.numel() <= numel,
                "FlatParams: bad planned offset for ", params[i].first);
  } else {
    int64_t off = 0;
    for (auto& kv : params) {
      offsets.push_back(off);
      off += round_up(kv.second->leaf.numel(), kAlign);
    }
    numel = round_up(std::max<int64_t>(off, kAlign), kAlign);
  }
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

FlatParams FlatParams::buffers(int64_t n) {
  FlatParams f({});
  f.numel = round_up(std::max<int64_t>(n, kAlign), kAlign);
  f.master = zeros({f.numel}, DType::F32);
  f.grad = zeros({f.numel}, DType::F32);
  f.shadow = zeros({f.numel}, DType::BF16);
  return f;
}

void FlatParams::zero_grad() { grad.zero_(); }

void FlatParams::refresh_shadow() { ::mft::cast_f32_bf16(master.data<float>(), (::mft::bf16_t*)shadow.data_ptr(), numel, current_stream()); }

AdamW::AdamW(FlatParams& flat, const AdamWConfig& cfg) : flat_(flat), cfg_(cfg) {
  NoGradGuard ng;
  m = zeros({flat.numel}, DType::F32);
  v = zeros({flat.numel}, DType::F32);
  if (cfg.amsgrad) vmax = zeros({flat.numel}, DType::F32);
  lr_dev = full({1}, cfg.lr, DType::F32);
  step_dev = zeros({1}, DType::F32);
  sumsq_dev = zeros({1}, DType::F32);
  nonfinite_dev = zeros({1}, DType::I32);
  skipped_dev = zeros({1}, DType::I32);
  segs_ = {OptSegment{0, flat.numel, 0}};
  state_numel_ = flat.numel;
}

void AdamW::shard(const std::vector<OptSegment>& segs, Communicator* comm, bool host_moments, bool host_fp32) {
  NoGradGuard ng;
  segs_ = segs;
  comm_ = comm;
  host_moments_ = host_moments;
  state_numel_ = 0;
  for (auto& s : segs_) {
    MFT_CHECK(s.off % 4 == 0 && s.len % 4 == 0 && s.off + s.len <= flat_.numel, "AdamW::shard: bad segment");
    state_numel_ = std::max(state_numel_, s.state_off + s.len);
  }
  const int64_t n = std::max<int64_t>(state_numel_, 4);
  MFT_CHECK(!(host_moments && cfg_.amsgrad), "AdamW: AMSGrad keeps fp32 moments on the device (no --offload host)");
  if (host_moments) {  // pinned host DRAM, read / written in place by the kernel (bf16 SR-rounded, or fp32)
    const DType md = host_fp32 ? DType::F32 : DType::BF16;
    m = zeros({n}, md, Device::cpu(true));
    v = zeros({n}, md, Device::cpu(true));
  } else {
    m = zeros({n}, DType::F32);
    v = zeros({n}, DType::F32);
  }
  if (cfg_.amsgrad) vmax = zeros({n}, DType::F32);
}

void AdamW::set_lr(float lr) {
  cfg_.lr = lr;
  lr_dev.fill_(lr);  // the value travels as a kernel argument: no host-buffer race, no sync
}

void AdamW::prepare() {
  hipStream_t s = current_stream();
  const bool clip = cfg_.max_grad_norm > 0.f;
  float* g0 = flat_.grad.data<float>();
  if (clip) {
    int64_t mx = 0;
    for (auto& sg : segs_) mx = std::max<int64_t>(mx, ::mft::sumsq_blocks(sg.len));
    if (!part_.defined() || part_.numel() < mx) part_ = empty({std::max<int64_t>(mx, 1)}, DType::F32);
    int n = 0;  // partitioned segments: summed over the ranks; replicated ones: added once, after
    for (const auto& sg : segs_)
      if (!sg.replicated) ::mft::sumsq(g0 + sg.off, sg.len, part_.data<float>(), sumsq_dev.data<float>(), n++ > 0, s);
    if (n == 0) sumsq_dev.zero_();
    if (comm_) comm_->all_reduce(sumsq_dev.data_ptr(), 1, CommType::F32, CommOp::Sum, s);  // global norm^2
    for (const auto& sg : segs_)
      if (sg.replicated) ::mft::sumsq(g0 + sg.off, sg.len, part_.data<float>(), sumsq_dev.data<float>(), 1, s);
  }
  // non-finite grads: with clipping the (all-reduced) norm^2 is non-finite exactly then, so no
  // separate pass over the grads is needed (adamw_commit records the flag); without, one scan
  if (cfg_.skip_nonfinite && !clip) {
    nonfinite_dev.zero_();
    for (auto& sg : segs_) ::mft::nonfinite_check(g0 + sg.off, sg.len, nonfinite_dev.data<int>(), s);
    if (comm_) comm_->all_reduce(nonfinite_dev.data_ptr(), 1, CommType::I32, CommOp::Max, s);  // skip together
  }
}

::mft::AdamWArgs AdamW::args() const {
  const bool clip = cfg_.max_grad_norm > 0.f;
  ::mft::AdamWArgs a{};
  a.lr_ptr = lr_dev.data<float>();
  a.beta1 = cfg_.beta1;
  a.beta2 = cfg_.beta2;
  a.eps = cfg_.eps;
  a.weight_decay = cfg_.weight_decay;
  a.step_ptr = step_dev.data<float>();
  a.sumsq = clip ? sumsq_dev.data<float>() : nullptr;
  a.max_norm = cfg_.max_grad_norm;
  a.l2_coupled = cfg_.l2_coupled;
  a.nonfinite = (cfg_.skip_nonfinite && !clip) ? nonfinite_dev.data<int>() : nullptr;
  return a;
}

void AdamW::step() {
  hipStream_t s = current_stream();
  prepare();
  ::mft::AdamWArgs a = args();
  if (disk_.active) return step_disk(a, s);
  float* g0 = flat_.grad.data<float>();
  a.moments_bf16 = m.dtype() == DType::BF16;
  const size_t ms = m.dtype() == DType::BF16 ? 2 : 4;
  for (auto& sg : segs_) {
    a.p = flat_.master.data<float>() + sg.off;
    a.g = g0 + sg.off;
    a.m = reinterpret_cast<float*>(static_cast<char*>(m.data_ptr()) + sg.state_off * ms);
    a.v = reinterpret_cast<float*>(static_cast<char*>(v.data_ptr()) + sg.state_off * ms);
    a.vmax = vmax.defined() ? vmax.data<float>() + sg.state_off : nullptr;
    a.n = sg.len;
    a.shadow = (::mft::bf16_t*)flat_.shadow.data_ptr() + sg.off;
    a.sr_offset = sg.off;
    ::mft::adamw_step(a, s);
  }
  ::mft::adamw_commit(step_dev.data<float>(), a.nonfinite, a.sumsq, s,
                      cfg_.skip_nonfinite ? nonfinite_dev.data<int>() : nullptr);
  if (cfg_.skip_nonfinite) {
    // skipped += nonfinite (int32 counters)
    k::Desc d = desc(skipped_dev), x = desc(nonfinite_dev);
    k::binary(d, d, x, k::B_ADD, 1.f, s);
  }
}

// ---------------------------------------------------------------- moments on disk (--offload disk)
void AdamW::to_disk(const std::string& dir, int rank, bool fp32) {
  MFT_CHECK(!disk_.active, "AdamW::to_disk: already on disk");
  MFT_CHECK(!host_moments_ && !vmax.defined(), "AdamW::to_disk: not with host moments or AMSGrad");
  NoGradGuard ng;
  std::error_code ec;
  std::filesystem::create_directories(dir, ec);
  const int64_t n = std::max<int64_t>(state_numel_, 4);
  disk_.elem = fp32 ? 4 : 2;
  disk_.bytes = (size_t)n * disk_.elem;
  const char* names[2] = {"m", "v"};
  for (int i = 0; i < 2; ++i) {
    const std::string path = dir + "/adamw_" + names[i] + ".rank" + std::to_string(rank) + ".bin";
    const int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
    MFT_CHECK(fd >= 0, "AdamW::to_disk: cannot create ", path);
    MFT_CHECK(::ftruncate(fd, (off_t)disk_.bytes) == 0, "AdamW::to_disk: cannot size ", path);  // zeros
    void* p = ::mmap(nullptr, disk_.bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    MFT_CHECK(p != MAP_FAILED, "AdamW::to_disk: cannot map ", path);
    disk_.map[i] = p;
  }
  const DType md = fp32 ? DType::F32 : DType::BF16;
  m = from_blob(disk_.map[0], {n}, md, Device::cpu());
  v = from_blob(disk_.map[1], {n}, md, Device::cpu());
  static const int64_t env_chunk = std::getenv("MFT_DISK_CHUNK") ? std::atoll(std::getenv("MFT_DISK_CHUNK")) : 0;
  disk_.chunk = std::min<int64_t>(n, env_chunk > 0 ? (env_chunk + 3) / 4 * 4 : (int64_t)16 << 20);
  for (int i = 0; i < 2; ++i) {
    disk_.dev[i] = empty({disk_.chunk}, md);
    disk_.pin[i] = empty({disk_.chunk}, md, Device::cpu(true));
  }
  disk_.active = true;
}

void AdamW::step_disk(::mft::AdamWArgs a, hipStream_t s) {
  float* g0 = flat_.grad.data<float>();
  a.moments_bf16 = disk_.elem == 2;
  char* mp[2] = {static_cast<char*>(disk_.map[0]), static_cast<char*>(disk_.map[1])};
  for (auto& sg : segs_) {
    for (int64_t o = 0; o < sg.len; o += disk_.chunk) {
      const int64_t len = std::min(disk_.chunk, sg.len - o);
      const size_t off = (size_t)(sg.state_off + o) * disk_.elem, nb = (size_t)len * disk_.elem;
      for (int i = 0; i < 2; ++i) {  // mapping -> pinned -> device (the page cache faults the file in)
        std::memcpy(disk_.pin[i].data_ptr(), mp[i] + off, nb);
        HIP_OK(hipMemcpyAsync(disk_.dev[i].data_ptr(), disk_.pin[i].data_ptr(), nb, hipMemcpyHostToDevice, s));
      }
      a.p = flat_.master.data<float>() + sg.off + o;
      a.g = g0 + sg.off + o;
      a.m = static_cast<float*>(disk_.dev[0].data_ptr());
      a.v = static_cast<float*>(disk_.dev[1].data_ptr());
      a.vmax = nullptr;
      a.n = len;
      a.shadow = (::mft::bf16_t*)flat_.shadow.data_ptr() + sg.off + o;
      a.sr_offset = sg.off + o;
      ::mft::adamw_step(a, s);
      for (int i = 0; i < 2; ++i)
        HIP_OK(hipMemcpyAsync(disk_.pin[i].data_ptr(), disk_.dev[i].data_ptr(), nb, hipMemcpyDeviceToHost, s));
      HIP_OK(hipStreamSynchronize(s));
      for (int i = 0; i < 2; ++i) std::memcpy(mp[i] + off, disk_.pin[i].data_ptr(), nb);  // dirty pages -> file
    }
  }
  ::mft::adamw_commit(step_dev.data<float>(), a.nonfinite, a.sumsq, s, cfg_.skip_nonfinite ? nonfinite_dev.data<int>() : nullptr);
  if (cfg_.skip_nonfinite) {
    k::Desc d = desc(skipped_dev), x = desc(nonfinite_dev);
    k::binary(d, d, x, k::B_ADD, 1.f, s);
  }
}

AdamW::~AdamW() {
  if (!disk_.active) return;
  m = Tensor();
  v = Tensor();
  for (void* p : disk_.map)
    if (p) ::munmap(p, disk_.bytes);
}

// ---------------------------------------------------------------- delayed (streamed) updates
void AdamW::prepare_delayed() {
  if (!pending_dev.defined()) {
    pending_dev = zeros({1}, DType::I32);
    lr_step_dev = zeros({1}, DType::F32);
  }
  prepare();
  lr_step_dev.copy_(lr_dev);  // this step's lr travels with its gradients
  pending_dev.fill_(1.0);
}

void AdamW::apply_delayed(int64_t off, int64_t len, void* m_dev, void* v_dev, bool moments_bf16, hipStream_t s,
                          int max_grid) {
  MFT_CHECK(pending_dev.defined() && !vmax.defined(), "AdamW::apply_delayed: prepare_delayed first (no AMSGrad)");
  ::mft::AdamWArgs a = args();
  a.lr_ptr = lr_step_dev.data<float>();
  a.enable = pending_dev.data<int>();
  a.p = flat_.master.data<float>() + off;
  a.g = flat_.grad.data<float>() + off;
  a.m = static_cast<float*>(m_dev);
  a.v = static_cast<float*>(v_dev);
  a.moments_bf16 = moments_bf16;
  a.n = len;
  a.shadow = (::mft::bf16_t*)flat_.shadow.data_ptr() + off;
  a.sr_offset = off;
  a.max_grid = max_grid;
  ::mft::adamw_step(a, s);
}

void AdamW::commit_delayed(hipStream_t s) {
  if (!pending_dev.defined()) return;
  ::mft::AdamWArgs a = args();
  ::mft::adamw_commit(step_dev.data<float>(), a.nonfinite, a.sumsq, s, nullptr, pending_dev.data<int>(), 1);
}

float AdamW::grad_norm() const { return std::sqrt(std::max(0.f, (float)sumsq_dev.item())); }
bool AdamW::skipped_last() const { return nonfinite_dev.to_vector_f32()[0] != 0.f; }
int64_t AdamW::applied_steps() const { return (int64_t)step_dev.item(); }

void AdamW::load_vmax(const Tensor& h) {
  MFT_CHECK(vmax.defined() && h.numel() == vmax.numel(), "AdamW::load_vmax: AMSGrad state mismatch");
  vmax.copy_(h.to(DType::F32));
}

void AdamW::load_state(const Tensor& m_h, const Tensor& v_h, int64_t steps) {
  MFT_CHECK(m_h.numel() == m.numel() && v_h.numel() == v.numel(), "AdamW::load_state: state has ", m_h.numel(),
            " elements, the optimizer ", m.numel());
  m.copy_(m_h.to(m.dtype()));
  v.copy_(v_h.to(v.dtype()));
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
