// libmft engine: frozen-weight streaming (see weight_stream.h).
#include "engine/weight_stream.h"

#include <algorithm>

#include "engine/autograd.h"

namespace mft {
namespace eng {

WeightStreamer::WeightStreamer(const std::vector<std::vector<Param*>>& groups, size_t budget_bytes) {
  MFT_CHECK(!groups.empty(), "weight streaming: no blocks");
  NoGradGuard ng;
  int64_t max_elems = 0;
  for (auto& ps : groups) {
    Group gr;
    for (Param* p : ps) {
      MFT_CHECK(!p->trainable() && p->c.dtype() == DType::BF16, "weight streaming: frozen bf16 weights only");
      gr.ps.push_back(p);
      gr.off.push_back(gr.elems);
      gr.elems += (p->c.numel() + 63) / 64 * 64;  // 128-B aligned views
    }
    max_elems = std::max(max_elems, gr.elems);
    groups_.push_back(std::move(gr));
  }
  slot_bytes_ = (size_t)max_elems * 2;
  const int n = (int)groups_.size();
  const int k = std::max(2, std::min(n, (int)(budget_bytes / std::max<size_t>(1, slot_bytes_))));
  for (int s = 0; s < k; ++s) slot_.push_back(zeros({max_elems}, DType::BF16));
  holder_.assign(k, -1);
  // host copies (one pinned buffer per block), then every Param becomes a view of its slot
  for (int g = 0; g < n; ++g) {
    Group& gr = groups_[g];
    gr.host = empty({gr.elems}, DType::BF16, Device::cpu(true));
    host_bytes_ += (size_t)gr.elems * 2;
    for (size_t j = 0; j < gr.ps.size(); ++j) {
      Param* p = gr.ps[j];
      const int64_t m = p->c.numel();
      gr.host.slice(0, gr.off[j], gr.off[j] + m).copy_(p->c.contiguous().view({m}));
      Tensor v = slot_[g % k].slice(0, gr.off[j], gr.off[j] + m).view(p->c.shape());
      p->c = v;
      p->leaf = v;
      p->wt = Tensor();
      p->streamed = true;
    }
  }
  synchronize();
  ready_.resize(n);
  for (auto& e : ready_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&order_, hipEventDisableTiming));
  HIP_OK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
}

WeightStreamer::~WeightStreamer() {
  if (copy_) (void)hipStreamSynchronize(copy_);
  for (auto& e : ready_) (void)hipEventDestroy(e);
  if (order_) (void)hipEventDestroy(order_);
  if (copy_) (void)hipStreamDestroy(copy_);
}

void WeightStreamer::issue(int g) {
  const int s = g % (int)slot_.size();
  // the copy starts after every kernel enqueued so far on the compute stream (the slot's previous
  // block included), then the block's bytes move as one H2D copy
  HIP_OK(hipEventRecord(order_, current_stream()));
  HIP_OK(hipStreamWaitEvent(copy_, order_, 0));
  const Group& gr = groups_[g];
  HIP_OK(hipMemcpyAsync(slot_[s].data_ptr(), gr.host.data_ptr(), (size_t)gr.elems * 2, hipMemcpyHostToDevice, copy_));
  HIP_OK(hipEventRecord(ready_[g], copy_));
  holder_[s] = g;
  ++copies;
}

void WeightStreamer::ensure(int g, int next) {
  const int k = (int)slot_.size();
  // a hipGraph capture must not depend on copies issued before it: at capture start nothing counts
  // as resident, so the recorded schedule loads every block it uses (and ends in the same slot
  // state every replay leaves behind, which later eager calls build on)
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_OK(hipStreamIsCapturing(current_stream(), &cs));
  const bool cap = cs == hipStreamCaptureStatusActive;
  if (cap && !capturing_) holder_.assign(holder_.size(), -1);
  capturing_ = cap;
  if (holder_[g % k] != g) issue(g);
  HIP_OK(hipStreamWaitEvent(current_stream(), ready_[g], 0));
  if (next >= 0 && next < (int)groups_.size() && next % k != g % k && holder_[next % k] != next) issue(next);
}

std::pair<Tensor, Tensor> WeightStreamer::gate(const Tensor& x, const Tensor& h, int g) {
  Tensor xo = x.alias(), ho = h.alias();
  if (any_needs_grad({x, h})) {
    WeightStreamer* self = this;
    auto n = lambda_node("WeightStreamGateBackward", [self, g](std::vector<Tensor>& grads) {
      self->ensure(g, g - 1);  // block g back in its slot before its backward reads the weights
      return std::vector<Tensor>{grads[0], grads[1]};
    });
    connect(n, {x, h}, {xo, ho});
  }
  return {xo, ho};
}

}  // namespace eng
}  // namespace mft
