// libmft engine: bucketed / overlapped data parallelism and ZeRO-1/2 (see dist.h).
#include "engine/dist.h"

#include <cstdio>

#include <algorithm>
#include <sstream>

#include "engine/autograd.h"
#include "kernels.h"

namespace mft {
namespace eng {

namespace {
constexpr int64_t kAlign = 64;
int64_t round_up(int64_t n, int64_t a) { return (n + a - 1) / a * a; }
}  // namespace

FlatPlan plan_flat(const std::vector<std::pair<std::string, Param*>>& params, int world, int64_t bucket_bytes) {
  MFT_CHECK(world >= 1, "plan_flat: world ", world);
  const int n = (int)params.size();
  FlatPlan p;
  p.offsets.assign(n, 0);
  p.bucket_of.assign(n, 0);
  // Parameters that COMPUTE in fp32 (the norm weights) read the fp32 master itself (FlatParams), so
  // under ZeRO-1/2 a rank that does not own their chunk would never see their update: they go into
  // one trailing REPLICATED bucket (all-reduced, updated in full on every rank; it is small).
  std::vector<int> part, rep;
  for (int i = 0; i < n; ++i) (params[i].second->c.dtype() == DType::F32 ? rep : part).push_back(i);
  // buckets of consecutive partitioned parameters, formed in backward order (last parameter first);
  // each is a list of parameter indices in forward order
  std::vector<std::vector<int>> groups;
  {
    std::vector<int> cur;
    int64_t bytes = 0;
    for (int j = (int)part.size() - 1; j >= 0; --j) {
      cur.insert(cur.begin(), part[j]);
      bytes += params[part[j]].second->leaf.numel() * 4;
      if (bytes >= bucket_bytes || j == 0) {
        groups.push_back(cur);
        cur.clear();
        bytes = 0;
      }
    }
    if (groups.empty() && rep.empty()) groups.push_back({});
  }
  const int np = (int)groups.size();
  if (!rep.empty()) groups.push_back(rep);  // launched last: its grads are final only at the end
  // offsets in forward order (partitioned buckets: the launch order reversed, then the replicated
  // one); every bucket padded to world x 64 elements
  const int64_t quantum = kAlign * world;
  int64_t off = 0;
  std::vector<std::pair<int64_t, int64_t>> fwd(groups.size());
  std::vector<int> layout;
  for (int k = np - 1; k >= 0; --k) layout.push_back(k);
  if ((int)groups.size() > np) layout.push_back(np);
  for (int k : layout) {
    const int64_t lo = off;
    for (int i : groups[k]) {
      p.offsets[i] = off;
      p.bucket_of[i] = k;
      off += round_up(params[i].second->leaf.numel(), kAlign);
    }
    off = lo + std::max(round_up(off - lo, quantum), quantum);
    fwd[k] = {lo, off};
  }
  p.numel = off;
  p.buckets = fwd;  // index k = launch order (k = 0 holds the last parameters of the forward)
  p.replicated.assign(groups.size(), 0);
  if ((int)groups.size() > np) p.replicated[np] = 1;
  return p;
}

DataParallel::DataParallel(FlatParams& flat, const FlatPlan& plan, Communicator& comm, AdamW& opt,
                           const DistConfig& cfg)
    : flat_(flat), plan_(plan), comm_(comm), opt_(opt), cfg_(cfg) {
  MFT_CHECK(flat.numel == plan.numel && flat.offsets == plan.offsets, "DataParallel: FlatParams not built from the plan");
  MFT_CHECK(cfg.zero_stage >= 0 && cfg.zero_stage <= 2, "DataParallel: ZeRO stage ", cfg.zero_stage,
            " (stage 3 partitions the parameters: engine/zero3.h)");
  MFT_CHECK(!cfg.host_moments || cfg.zero_stage >= 1 || comm.world() == 1,
            "DataParallel: host-offloaded moments need a partitioned optimizer (--zero_stage >= 1)");
  const int nb = (int)plan_.buckets.size();
  HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  ready_ev_.resize(nb);
  for (auto& e : ready_ev_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&join_ev_, hipEventDisableTiming));
  total_.assign(nb, 0);
  for (int b : plan_.bucket_of) total_[b]++;
  pending_ = total_;
  done_.assign(nb, 0);
  for (size_t i = 0; i < flat_.params.size(); ++i) {
    const int pi = (int)i;
    add_ready_hook(flat_.params[i].second->leaf, [this, pi](TensorImpl*) { on_ready(pi); });
  }
  if (cfg_.bf16_reduce) comm_buf_ = zeros({plan_.numel}, DType::BF16);
  if (cfg_.zero_stage >= 1 || cfg_.host_moments) {
    const int r = comm_.rank();
    std::vector<OptSegment> segs;
    int64_t st = 0;
    // ascending offsets: the owned chunks, moments packed in the same order
    std::vector<int> order(nb);
    for (int b = 0; b < nb; ++b) order[b] = b;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return plan_.buckets[a].first < plan_.buckets[b].first; });
    for (int b : order) {
      if (plan_.replicated[b]) {  // every rank updates (and keeps moments for) the whole bucket
        const int64_t len = plan_.buckets[b].second - plan_.buckets[b].first;
        segs.push_back({plan_.buckets[b].first, len, st, true});
        st += len;
        continue;
      }
      const int64_t cs = chunk(b);
      segs.push_back({plan_.buckets[b].first + r * cs, cs, st});
      st += cs;
    }
    opt_.shard(segs, &comm_, cfg_.host_moments, cfg_.host_fp32);
  }
}

DataParallel::~DataParallel() {
  if (stream_) (void)hipStreamSynchronize(stream_);
  for (auto& e : ready_ev_) (void)hipEventDestroy(e);
  if (join_ev_) (void)hipEventDestroy(join_ev_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

std::string DataParallel::describe() const {
  std::ostringstream os;
  os << (cfg_.zero_stage == 0 ? "DDP" : cfg_.zero_stage == 1 ? "ZeRO-1" : "ZeRO-2") << " over " << comm_.world()
     << " rank(s) [" << comm_.backend() << "], " << plan_.buckets.size() << " bucket(s) of <= "
     << cfg_.bucket_bytes / 1048576 << " MB fp32, " << (cfg_.bf16_reduce ? "bf16" : "fp32") << " reduction, "
     << (cfg_.overlap ? "overlapped with the backward" : "after the backward");
  if (cfg_.host_moments) os << ", AdamW moments in pinned host DRAM (" << (cfg_.host_fp32 ? "fp32" : "bf16") << ")";
  return os.str();
}

void DataParallel::begin_micro(int i, int n) {
  if (i == 0) {
    pending_ = total_;
    std::fill(done_.begin(), done_.end(), 0);
    hooked_ = 0;
  }
  last_micro_ = i == n - 1;
}

void DataParallel::on_ready(int pi) {
  if (!last_micro_ || !cfg_.overlap) return;
  const int b = plan_.bucket_of[pi];
  if (--pending_[b] == 0) {
    if (!done_[b]) ++hooked_;
    launch(b);
  }
}

void DataParallel::launch(int b) {
  if (done_[b]) return;
  done_[b] = 1;
  ++launched;
  hipStream_t cs = current_stream();
  // the bucket's gradients were produced by kernels already enqueued on the compute stream
  HIP_OK(hipEventRecord(ready_ev_[b], cs));
  HIP_OK(hipStreamWaitEvent(stream_, ready_ev_[b], 0));
  const int64_t lo = plan_.buckets[b].first, n = plan_.buckets[b].second - lo, c = chunk(b);
  const int r = comm_.rank();
  float* g = flat_.grad.data<float>() + lo;
  const bool scatter = cfg_.zero_stage == 2 && !plan_.replicated[b];
  if (!cfg_.bf16_reduce) {
    if (scatter) comm_.reduce_scatter(g, g + r * c, c, CommType::F32, CommOp::Sum, stream_);
    else comm_.all_reduce(g, n, CommType::F32, CommOp::Sum, stream_);
    return;
  }
  ::mft::bf16_t* h = (::mft::bf16_t*)comm_buf_.data_ptr() + lo;
  ::mft::cast_f32_bf16(g, h, n, stream_);
  if (scatter) {
    comm_.reduce_scatter(h, h + r * c, c, CommType::BF16, CommOp::Sum, stream_);
    ::mft::cast_bf16_f32(h + r * c, g + r * c, c, stream_);
  } else {
    comm_.all_reduce(h, n, CommType::BF16, CommOp::Sum, stream_);
    ::mft::cast_bf16_f32(h, g, n, stream_);
  }
}

void DataParallel::finish() {
  if (!reported_) {  // overlap evidence (tests): how many reductions the backward itself started
    reported_ = true;
    std::printf("[dp] first step: %d of %zu bucket reduction(s) launched from the backward's grad-ready hooks\n",
                hooked_, plan_.buckets.size());
  }
  for (int b = 0; b < (int)plan_.buckets.size(); ++b) launch(b);
  HIP_OK(hipEventRecord(join_ev_, stream_));
  HIP_OK(hipStreamWaitEvent(current_stream(), join_ev_, 0));
}

void DataParallel::after_optimizer() {
  if (cfg_.zero_stage == 0) return;
  const int r = comm_.rank();
  ::mft::bf16_t* sh = (::mft::bf16_t*)flat_.shadow.data_ptr();
  for (int b = 0; b < (int)plan_.buckets.size(); ++b) {
    if (plan_.replicated[b]) continue;  // updated in full on every rank
    const int64_t lo = plan_.buckets[b].first, c = chunk(b);
    comm_.all_gather(sh + lo + r * c, sh + lo, c, CommType::BF16, current_stream());
  }
}

void DataParallel::gather_master() {
  if (cfg_.zero_stage == 0) return;
  const int r = comm_.rank();
  float* m = flat_.master.data<float>();
  for (int b = 0; b < (int)plan_.buckets.size(); ++b) {
    if (plan_.replicated[b]) continue;
    const int64_t lo = plan_.buckets[b].first, c = chunk(b);
    comm_.all_gather(m + lo + r * c, m + lo, c, CommType::F32, current_stream());
  }
  flat_.refresh_shadow();
}

}  // namespace eng
}  // namespace mft
