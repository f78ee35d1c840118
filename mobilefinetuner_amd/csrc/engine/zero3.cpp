// libmft engine: ZeRO-3 parameter partitioning (see zero3.h).
#include "engine/zero3.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <sstream>

#include "engine/autograd.h"
#include "engine/ops.h"
#include "engine/tensor_kernels.h"
#include "kernels.h"

namespace mft {
namespace eng {

namespace {
constexpr int64_t kAlign = 64;
int64_t round_up(int64_t n, int64_t a) { return (n + a - 1) / a * a; }
Tensor value_of(Param& p) { return p.trainable() ? p.leaf.detach() : p.c; }
}  // namespace

Zero3Layout plan_zero3(const std::vector<NamedParams>& units, const NamedParams& rep, int world) {
  MFT_CHECK(world >= 1, "plan_zero3: world ", world);
  Zero3Layout L;
  int64_t local = 0;
  for (size_t u = 0; u < units.size(); ++u) {
    Zero3Layout::UnitLayout un;
    int64_t off = 0;
    for (auto& kv : units[u]) {
      MFT_CHECK(kv.second->c.dtype() == DType::BF16, "Zero3: unit parameter ", kv.first, " must compute in bf16");
      un.off.push_back(off);
      off += round_up(kv.second->c.numel(), kAlign);
    }
    un.n = round_up(std::max<int64_t>(off, kAlign), kAlign * world);
    un.s = un.n / world;
    un.local = local;
    local += un.s;
    un.slot = u == 0 ? 0 : 1 + (int)((u - 1) % 2);
    if (u > 0) L.max_block = std::max(L.max_block, un.n);
    L.units.push_back(std::move(un));
  }
  L.rep_off = local;
  for (auto& kv : rep) {
    MFT_CHECK(kv.second->c.dtype() == DType::F32, "Zero3: replicated parameter ", kv.first, " must compute in fp32");
    L.rep_at.push_back(local);
    local += round_up(kv.second->c.numel(), kAlign);
  }
  L.rep_n = local - L.rep_off;
  L.numel = local;
  return L;
}

Zero3::Zero3(const std::vector<NamedParams>& units, const NamedParams& rep, Communicator& comm)
    : comm_(comm), rep_(rep), flat_(FlatParams::buffers(kAlign)) {
  NoGradGuard ng;
  MFT_CHECK(units.size() >= 2, "Zero3: an outer unit and at least one block");
  const int W = comm_.world(), r = comm_.rank();
  hipStream_t cs = current_stream();
  // layout: each unit's partition, then the replicated parameters
  const Zero3Layout lay = plan_zero3(units, rep_, W);
  for (size_t u = 0; u < units.size(); ++u) {
    Unit un;
    un.params = units[u];
    un.off = lay.units[u].off;
    un.n = lay.units[u].n;
    un.s = lay.units[u].s;
    un.local = lay.units[u].local;
    un.slot = lay.units[u].slot;
    un.total = (int)un.params.size();
    units_.push_back(std::move(un));
  }
  const int64_t local = lay.numel, max_block = lay.max_block;
  const std::vector<int64_t>& rep_at = lay.rep_at;
  rep_off_ = lay.rep_off;
  rep_n_ = lay.rep_n;
  flat_ = FlatParams::buffers(std::max<int64_t>(local, kAlign));
  slot_ = {zeros({units_[0].n}, DType::BF16), zeros({max_block}, DType::BF16), zeros({max_block}, DType::BF16)};
  gwork_ = {zeros({units_[0].n}, DType::F32), zeros({max_block}, DType::F32), zeros({max_block}, DType::F32)};
  holder_.assign(3, -1);
  int64_t max_param = kAlign, max_s = kAlign;
  for (auto& un : units_) {
    max_s = std::max(max_s, un.s);
    for (auto& kv : un.params) max_param = std::max(max_param, kv.second->c.numel());
  }
  dummy_ = zeros({max_param}, DType::F32);
  tmp_ = zeros({max_s}, DType::F32);
  // partitions: every unit's full fp32 value from rank 0, this rank keeps its slice
  for (auto& un : units_) {
    Tensor full = zeros({un.n}, DType::F32);
    for (size_t j = 0; j < un.params.size(); ++j) {
      Param& p = *un.params[j].second;
      const int64_t m = p.c.numel();
      full.slice(0, un.off[j], un.off[j] + m).copy_(value_of(p).contiguous().view({m}));
    }
    comm_.broadcast(full.data_ptr(), (size_t)un.n * 4, 0, cs);
    flat_.master.slice(0, un.local, un.local + un.s).copy_(full.slice(0, (int64_t)r * un.s, (int64_t)(r + 1) * un.s));
    for (size_t j = 0; j < un.params.size(); ++j) {
      Param& p = *un.params[j].second;
      const Shape shp = p.c.shape();
      const int64_t m = p.c.numel(), o = un.off[j];
      p.c = slot_[un.slot].slice(0, o, o + m).view(shp);
      Tensor leaf = dummy_.slice(0, 0, m).view(shp).alias();  // placeholder: never read
      leaf.requires_grad_(true);
      leaf.set_grad(gwork_[un.slot].slice(0, o, o + m).view(shp));
      p.leaf = leaf;
      p.wt = Tensor();
      p.streamed = true;
    }
  }
  for (size_t j = 0; j < rep_.size(); ++j) {
    Param& p = *rep_[j].second;
    const Shape shp = p.c.shape();
    const int64_t m = p.c.numel(), o = rep_at[j];
    Tensor mv = flat_.master.slice(0, o, o + m).view(shp);
    mv.copy_(value_of(p));
    Tensor leaf = mv.alias();
    leaf.requires_grad_(true);
    leaf.set_grad(flat_.grad.slice(0, o, o + m).view(shp));
    p.leaf = leaf;
    p.c = leaf.alias();
    p.wt = Tensor();
  }
  if (rep_n_ > 0) comm_.broadcast(flat_.master.data<float>() + rep_off_, (size_t)rep_n_ * 4, 0, cs);
  flat_.refresh_shadow();
  HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  ready_.resize(units_.size());
  for (auto& e : ready_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  rs_done_.resize(3);
  rs_live_.assign(3, 0);
  for (auto& e : rs_done_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&order_, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&join_, hipEventDisableTiming));
  for (size_t u = 0; u < units_.size(); ++u)
    for (auto& kv : units_[u].params) {
      const int uu = (int)u;
      add_ready_hook(kv.second->leaf, [this, uu](TensorImpl*) { on_ready(uu); });
    }
  synchronize();
}

Zero3::~Zero3() {
  if (cstream_) {
    (void)hipStreamSynchronize(cstream_);
    (void)hipStreamDestroy(cstream_);
    for (auto e : h2d_ev_) (void)hipEventDestroy(e);
    (void)hipEventDestroy(cjoin_ev_);
  }
  if (ostream_) {
    ::mft::gemm4_reserve_cus(0);
    (void)hipStreamSynchronize(ostream_);
    (void)hipStreamDestroy(ostream_);
  }
  for (auto& e : upd_ev_) (void)hipEventDestroy(e);
  if (fork_ev_) (void)hipEventDestroy(fork_ev_);
  if (ojoin_ev_) (void)hipEventDestroy(ojoin_ev_);
  if (stream_) (void)hipStreamSynchronize(stream_);
  for (auto& e : ready_) (void)hipEventDestroy(e);
  for (auto& e : rs_done_) (void)hipEventDestroy(e);
  if (order_) (void)hipEventDestroy(order_);
  if (join_) (void)hipEventDestroy(join_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

std::string Zero3::describe() const {
  std::ostringstream os;
  int64_t n = 0;
  for (auto& u : units_) n += u.n;
  os << "ZeRO-3 over " << comm_.world() << " rank(s) [" << comm_.backend() << "]: " << units_.size()
     << " units (" << n / 1000000 << "M params partitioned, " << rep_n_ / 1000 << "K replicated), blocks gathered into "
     << "2 slots with one-block prefetch, per-block gradient reduce-scatter";
  return os.str();
}

void Zero3::shard_optimizer(AdamW& opt, bool host_moments, bool host_fp32, bool streamed) {
  std::vector<OptSegment> segs{OptSegment{0, rep_off_, 0, false}};
  if (rep_n_ > 0) segs.push_back(OptSegment{rep_off_, rep_n_, rep_off_, true});
  opt.shard(segs, &comm_, host_moments, host_fp32);
  if (!(host_moments && streamed)) return;
  MFT_CHECK(!opt.config().amsgrad, "Zero3: the host-streamed optimizer has no AMSGrad state");
  sopt_ = &opt;
  sfp32_ = host_fp32;
  const int nupd = 1 + (int)units_.size();
  supd_.assign(nupd, 0);
  upd_ev_.resize(nupd);
  for (auto& e : upd_ev_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&fork_ev_, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&ojoin_ev_, hipEventDisableTiming));
  // the updates run beside the forward's kernels: a low-priority stream and a bounded grid (the
  // kernel waits on PCIe, not on the CU)
  const char* pr = std::getenv("MFT_Z3_OPT_PRIO");
  const char* stg = std::getenv("MFT_Z3_STAGED");
  if (!(stg && stg[0] == '0')) {
    // (staged: no optimizer stream)
  } else if (!(pr && pr[0] == '0')) {
    int least = 0, greatest = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_OK(hipStreamCreateWithPriority(&ostream_, hipStreamNonBlocking, least));
  } else {
    HIP_OK(hipStreamCreateWithFlags(&ostream_, hipStreamNonBlocking));
  }
  const char* gr = std::getenv("MFT_Z3_OPT_GRID");
  opt_grid_ = gr ? std::atoi(gr) : 32;  // profiles/r4_offload_modes.txt: 32 best of 16-2048
  const char* st = std::getenv("MFT_Z3_STAGED");
  staged_ = !(st && st[0] == '0');
  if (staged_) {
    // device slots for the moments of S updates (default: half of them), refilled by SDMA copies on one
    // copy stream: update i reads / writes slot i % S on the communication stream, then the copy stream
    // writes the slot back and prefetches the slot's next user (i + S, or next step's i % S) -- the
    // PCIe traffic runs from the forward through the backward instead of inside the forward
    const char* se = std::getenv("MFT_Z3_SLOTS");
    nslot_ = se && *se ? std::atoi(se) : (nupd + 1) / 2 + 1;
    nslot_ = std::max(1, std::min(nslot_, nupd));
    int64_t mx = 0;
    for (int i = 0; i < nupd; ++i) mx = std::max(mx, upd_len(i));
    slot_elems_ = (mx + 63) / 64 * 64;
    const int64_t es = sfp32_ ? 4 : 2;
    slot_mv_ = empty({(int64_t)nslot_ * 2 * slot_elems_ * es / 2}, DType::BF16);
    HIP_OK(hipStreamCreateWithFlags(&cstream_, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&cjoin_ev_, hipEventDisableTiming));
    h2d_ev_.resize(nupd);
    for (auto& e : h2d_ev_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    h2d_pending_.assign(nupd, 0);
    for (int i = 0; i < nslot_; ++i) slot_copy(i, true);  // the first S updates' moments
    HIP_OK(hipStreamSynchronize(cstream_));
    return;
  }
  // in place: the updates' workgroups hold their CUs for milliseconds (PCIe-bound): the persistent GEMMs
  // keep that many CUs out of their grids instead of queueing a statically assigned workgroup behind one
  // (MFT_Z3_RESERVE=0: off, A/B; profiles/r5_offload_reserve.txt)
  const char* rv = std::getenv("MFT_Z3_RESERVE");
  ::mft::gemm4_reserve_cus(rv && rv[0] == '0' ? 0 : opt_grid_);
}

void* Zero3::slot_ptr(int i, int which) {
  const int64_t es = sfp32_ ? 4 : 2;
  return static_cast<char*>(slot_mv_.data_ptr()) + ((int64_t)(i % nslot_) * 2 + which) * slot_elems_ * es;
}

void Zero3::slot_copy(int i, bool h2d) {
  const int64_t n = upd_len(i);
  if (n <= 0) return;
  const size_t es = sfp32_ ? 4 : 2, off = (size_t)upd_off(i) * es;
  char* hm = static_cast<char*>(sopt_->m.data_ptr()) + off;
  char* hv = static_cast<char*>(sopt_->v.data_ptr()) + off;
  if (h2d) {
    HIP_OK(hipMemcpyAsync(slot_ptr(i, 0), hm, (size_t)n * es, hipMemcpyHostToDevice, cstream_));
    HIP_OK(hipMemcpyAsync(slot_ptr(i, 1), hv, (size_t)n * es, hipMemcpyHostToDevice, cstream_));
  } else {
    HIP_OK(hipMemcpyAsync(hm, slot_ptr(i, 0), (size_t)n * es, hipMemcpyDeviceToHost, cstream_));
    HIP_OK(hipMemcpyAsync(hv, slot_ptr(i, 1), (size_t)n * es, hipMemcpyDeviceToHost, cstream_));
  }
}

// ---------------------------------------------------------------- host-streamed optimizer
// MFT_Z3_TRACE=1: one stderr line per streamed-optimizer call (locating a failure without a debugger)
static bool z3_trace() {
  static const bool on = [] {
    const char* e = std::getenv("MFT_Z3_TRACE");
    return e && e[0] == '1';
  }();
  return on;
}
#define Z3_TRACE(...)                            \
  do {                                           \
    if (z3_trace()) {                            \
      std::fprintf(stderr, "[z3] " __VA_ARGS__); \
      std::fflush(stderr);                       \
    }                                            \
  } while (0)

void Zero3::opt_fork() {
  if (forked_) return;
  forked_ = true;
  HIP_OK(hipEventRecord(fork_ev_, current_stream()));
  HIP_OK(hipStreamWaitEvent(staged_ ? stream_ : ostream_, fork_ev_, 0));
}

void Zero3::join_opt_stream() {
  if (staged_) {  // copy stream -> communication stream -> current stream (never a side-stream ring)
    HIP_OK(hipEventRecord(cjoin_ev_, cstream_));
    HIP_OK(hipStreamWaitEvent(stream_, cjoin_ev_, 0));
    HIP_OK(hipEventRecord(ojoin_ev_, stream_));
  } else {
    HIP_OK(hipEventRecord(ojoin_ev_, ostream_));
  }
  HIP_OK(hipStreamWaitEvent(current_stream(), ojoin_ev_, 0));
}

void Zero3::opt_update(int i) {
  if (supd_[i]) return;
  supd_[i] = 1;
  Z3_TRACE("update %d\n", i);
  opt_fork();
  if (staged_) {
    // on the communication stream, which all-gathers the updated partition next.  Its slot was filled
    // either this step (an event of this step) or in the previous one (joined at that step's finish)
    const int nupd = (int)supd_.size();
    if (h2d_pending_[i]) HIP_OK(hipStreamWaitEvent(stream_, h2d_ev_[i], 0));
    h2d_pending_[i] = 0;
    const int64_t n = upd_len(i);
    if (n > 0)
      sopt_->apply_delayed(upd_off(i), n, slot_ptr(i, 0), slot_ptr(i, 1), !sfp32_, stream_, 0);
    HIP_OK(hipEventRecord(upd_ev_[i], stream_));
    HIP_OK(hipStreamWaitEvent(cstream_, upd_ev_[i], 0));
    slot_copy(i, false);                                          // write the moments back ...
    const int next = i + nslot_ < nupd ? i + nslot_ : i % nslot_;  // ... and prefetch the slot's next user
    if (next != i) {
      slot_copy(next, true);
      if (next > i) {
        HIP_OK(hipEventRecord(h2d_ev_[next], cstream_));
        h2d_pending_[next] = 1;
      }
    }
    bool all = true;
    for (int c : supd_) all = all && c;
    if (all) sopt_->commit_delayed(stream_);
    return;
  }
  const int64_t n = upd_len(i);
  if (n > 0) {  // the moments of the partition, in place in pinned host DRAM
    const size_t es = sfp32_ ? 4 : 2, off = (size_t)upd_off(i) * es;
    sopt_->apply_delayed(upd_off(i), n, static_cast<char*>(sopt_->m.data_ptr()) + off,
                         static_cast<char*>(sopt_->v.data_ptr()) + off, !sfp32_, ostream_, opt_grid_);
  }
  HIP_OK(hipEventRecord(upd_ev_[i], ostream_));
  bool all = true;
  for (int c : supd_) all = all && c;
  if (all) sopt_->commit_delayed(ostream_);  // after every update of the step (same stream)
}

void Zero3::prepare_optimizer() {
  // end of the step's backward (finish() joined every collective): the gradients, their norm and
  // the lr wait in place; the next forward applies them unit by unit
  Z3_TRACE("prepare\n");
  sopt_->prepare_delayed();
  primed_ = true;
  std::fill(supd_.begin(), supd_.end(), 0);
  forked_ = false;
}

void Zero3::flush_optimizer() {
  // issued whether or not the host believes an update is pending: in graph mode the replays (never
  // host code) leave the device flag ahead of any host-side bookkeeping, and the kernels and the
  // commit are gated on that device flag (a no-op when nothing is pending) -- ADVICE r4
  if (!sopt_ || !primed_) return;
  for (int i = 0; i < (int)supd_.size(); ++i) opt_update(i);
  join_opt_stream();
  synchronize();
  forked_ = false;
  std::fill(supd_.begin(), supd_.end(), 0);
  holder_.assign(holder_.size(), -1);  // every partition changed
}

void Zero3::optimizer_state_loaded() {
  if (!staged_) return;
  // the step starts with slot k holding update k's moments
  HIP_OK(hipDeviceSynchronize());
  for (int i = 0; i < nslot_; ++i) slot_copy(i, true);
  HIP_OK(hipStreamSynchronize(cstream_));
  std::fill(h2d_pending_.begin(), h2d_pending_.end(), 0);
}

void Zero3::gather(int u) {
  Unit& un = units_[u];
  HIP_OK(hipEventRecord(order_, current_stream()));  // the slot's previous user has been enqueued
  HIP_OK(hipStreamWaitEvent(stream_, order_, 0));
  if (sopt_ && primed_ && grad_enabled()) {  // the previous step's update of this partition first (gated on device)
    opt_update(1 + u);
    // (staged: the update ran on this same stream, already in order.  A stream waiting on an event it
    // recorded itself is a self-edge in a captured graph: hipStreamEndCapture then recursed without end
    // -- a stack-overflow segfault, or a hang with an unlimited stack; profiles/r6_z3_capture_trace.txt)
    if (!staged_) HIP_OK(hipStreamWaitEvent(stream_, upd_ev_[1 + u], 0));
  }
  const ::mft::bf16_t* src = (const ::mft::bf16_t*)flat_.shadow.data_ptr() + un.local;
  comm_.all_gather(src, slot_[un.slot].data_ptr(), (size_t)un.s, CommType::BF16, stream_);
  HIP_OK(hipEventRecord(ready_[u], stream_));
  holder_[un.slot] = u;
  ++gathers;
}

void Zero3::reduce_scatter(int u) {
  Unit& un = units_[u];
  if (un.reduced) return;
  un.reduced = true;
  HIP_OK(hipEventRecord(order_, current_stream()));  // every gradient kernel of the unit enqueued
  HIP_OK(hipStreamWaitEvent(stream_, order_, 0));
  Tensor dst = flat_.grad.slice(0, un.local, un.local + un.s);
  if (first_micro_) {  // the partition's first contribution of the step: written in place
    comm_.reduce_scatter(gwork_[un.slot].data_ptr(), dst.data_ptr(), (size_t)un.s, CommType::F32, CommOp::Sum, stream_);
  } else {  // later micro-batches accumulate
    comm_.reduce_scatter(gwork_[un.slot].data_ptr(), tmp_.data_ptr(), (size_t)un.s, CommType::F32, CommOp::Sum, stream_);
    Tensor src = tmp_.slice(0, 0, un.s);
    k::axpy(desc(dst), desc(src), 1.f, 1, stream_);
  }
  HIP_OK(hipEventRecord(rs_done_[un.slot], stream_));
  rs_live_[un.slot] = 1;
  ++reduce_scatters;
}

void Zero3::zero_work(int s) {
  // after the slot's last reduce-scatter (this step's) has read it; events of earlier steps are
  // never waited on, so a hipGraph capture only depends on work it recorded itself
  if (rs_live_[s]) HIP_OK(hipStreamWaitEvent(current_stream(), rs_done_[s], 0));
  gwork_[s].zero_();
}

void Zero3::after_optimizer() { holder_.assign(holder_.size(), -1); }  // every partition changed

void Zero3::on_ready(int u) {
  if (--units_[u].pending == 0) reduce_scatter(u);
}

float Zero3::grad_prescale() const { return 1.f / (float)comm_.world(); }

void Zero3::zero_grad(FlatParams& flat) {
  // streamed optimizer: the replicated parameters' pending update reads their gradients -- it runs
  // before they are cleared, with the first units' moment prefetches behind it
  if (sopt_ && primed_) {  // (device-gated: a no-op when a flush already applied it)
    opt_update(0);
    HIP_OK(hipStreamWaitEvent(current_stream(), upd_ev_[0], 0));
  }
  // the partitions are overwritten by the first micro-batch's reduce-scatters; only the replicated
  // gradients accumulate from zero
  if (rep_n_ > 0) flat.grad.slice(0, rep_off_, rep_off_ + rep_n_).zero_();
}

void Zero3::begin_micro(int i, int n) {
  (void)n;
  if (i > 0)  // (a unit no hook completed in the previous micro-batch: reduce it before its slot is reused)
    for (size_t u = 0; u < units_.size(); ++u) reduce_scatter((int)u);
  first_micro_ = i == 0;
  if (i == 0) {  // nothing carries over from the previous step (its finish() joined every collective)
    holder_.assign(holder_.size(), -1);
    rs_live_.assign(rs_live_.size(), 0);
  }
  for (auto& un : units_) {
    un.pending = un.total;
    un.reduced = false;
  }
}

void Zero3::begin_forward() {
  if (holder_[0] != 0) gather(0);
  HIP_OK(hipStreamWaitEvent(current_stream(), ready_[0], 0));
  if (grad_enabled()) {  // the tied embedding's gradient starts in the LM-head CE of this forward
    zero_work(0);
  }
}

void Zero3::ensure(int block, int next) {
  const int u = 1 + block;
  if (holder_[units_[u].slot] != u) gather(u);
  HIP_OK(hipStreamWaitEvent(current_stream(), ready_[u], 0));
  const int nu = 1 + next;
  if (next >= 0 && nu < (int)units_.size() && units_[nu].slot != units_[u].slot && holder_[units_[nu].slot] != nu)
    gather(nu);
}

std::pair<Tensor, Tensor> Zero3::gate(const Tensor& x, const Tensor& h, int block) {
  Tensor xo = x.alias(), ho = h.alias();
  if (any_needs_grad({x, h})) {
    Zero3* self = this;
    auto n = lambda_node("Zero3GateBackward", [self, block](std::vector<Tensor>& grads) {
      self->ensure(block, block - 1);  // the block's weights back before its backward reads them
      self->zero_work(self->units_[1 + block].slot);
      return std::vector<Tensor>{grads[0], grads[1]};
    });
    connect(n, {x, h}, {xo, ho});
  }
  return {xo, ho};
}

void Zero3::finish() {
  Z3_TRACE("finish (primed %d)\n", (int)primed_);
  if (sopt_ && primed_) {
    // every pending update issued (a unit the forward did not gather) and the optimizer stream
    // joined back: a captured step ends with every stream it forked
    for (int i = 0; i < (int)supd_.size(); ++i) opt_update(i);
    join_opt_stream();
  }
  for (size_t u = 0; u < units_.size(); ++u) reduce_scatter((int)u);  // units no hook completed
  if (rep_n_ > 0) {
    HIP_OK(hipEventRecord(order_, current_stream()));
    HIP_OK(hipStreamWaitEvent(stream_, order_, 0));
    comm_.all_reduce(flat_.grad.data<float>() + rep_off_, (size_t)rep_n_, CommType::F32, CommOp::Sum, stream_);
  }
  HIP_OK(hipEventRecord(join_, stream_));
  HIP_OK(hipStreamWaitEvent(current_stream(), join_, 0));
  Z3_TRACE("finish done\n");
}

void Zero3::materialize() {
  NoGradGuard ng;
  synchronize();
  for (auto& un : units_) {
    Tensor full = zeros({un.n}, DType::F32);
    comm_.all_gather(flat_.master.data<float>() + un.local, full.data_ptr(), (size_t)un.s, CommType::F32,
                     current_stream());
    for (size_t j = 0; j < un.params.size(); ++j) {
      Param& p = *un.params[j].second;
      const Shape shp = p.c.shape();
      const int64_t m = p.c.numel(), o = un.off[j];
      Tensor v = full.slice(0, o, o + m).view(shp).clone();
      p.c = v.to(DType::BF16);
      v.requires_grad_(true);  // trainable(): writers read the fp32 value
      p.leaf = v;
      p.streamed = false;
    }
  }
  synchronize();
}

}  // namespace eng
}  // namespace mft
