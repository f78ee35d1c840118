// libmft engine: frozen-weight streaming (see weight_stream.h).
#include "engine/weight_stream.h"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>

#include "engine/autograd.h"
#include "engine/ops.h"
#include "engine/tensor_kernels.h"

namespace mft {
namespace eng {

WeightStreamer::WeightStreamer(const std::vector<std::vector<Param*>>& groups, size_t budget_bytes, const DiskTier& disk)
    : disk_(disk) {
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
  // host copies (one pinned buffer per block) or block files, then every Param becomes a view of its slot
  const bool on_disk = !disk_.dir.empty();
  if (on_disk) {
    std::filesystem::create_directories(disk_.dir);
    const size_t stage_bytes = slot_bytes_;  // (fp16 blocks take the same bytes as bf16)
    for (int i = 0; i < 2; ++i) stage_host_.push_back(empty({(int64_t)stage_bytes}, DType::U8, Device::cpu(true)));
    host_bytes_ = 2 * stage_bytes;
    if (disk_.fp16) stage_dev_ = empty({max_elems}, DType::F16);
  }
  for (int g = 0; g < n; ++g) {
    Group& gr = groups_[g];
    Tensor hostv = empty({gr.elems}, DType::BF16, on_disk ? Device::cpu() : Device::cpu(true));
    hostv.zero_();
    for (size_t j = 0; j < gr.ps.size(); ++j) {
      Param* p = gr.ps[j];
      const int64_t m = p->c.numel();
      hostv.slice(0, gr.off[j], gr.off[j] + m).copy_(p->c.contiguous().view({m}));
    }
    if (on_disk) {
      Tensor out = hostv;
      if (disk_.fp16) {
        // bf16 -> fp16 is exact only inside fp16's NORMAL range (|x| in [6.1e-5, 65504] or 0):
        // a block stays fp16 on disk only if every value survives the round trip, else bf16 (the
        // same 2 bytes per value, lossless)
        Tensor h = empty({gr.elems}, DType::F16, Device::cpu());
        h.copy_(hostv);
        Tensor back = empty({gr.elems}, DType::BF16, Device::cpu());
        back.copy_(h);
        gr.fp16 = std::memcmp(back.data_ptr(), hostv.data_ptr(), hostv.nbytes()) == 0;
        if (gr.fp16) out = h;
        else ++bf16_fallbacks;
      }
      gr.path = disk_.dir + "/block_" + std::to_string(g) + ".bin";
      std::FILE* f = std::fopen(gr.path.c_str(), "wb");
      MFT_CHECK(f, "weight streaming: cannot write ", gr.path);
      const size_t wrote = std::fwrite(out.data_ptr(), 1, out.nbytes(), f);
      std::fclose(f);
      MFT_CHECK(wrote == out.nbytes(), "weight streaming: short write to ", gr.path);
      gr.bytes = out.nbytes();
      disk_bytes_ += gr.bytes;
      gr.fd = ::open(gr.path.c_str(), O_RDONLY);
      MFT_CHECK(gr.fd >= 0, "weight streaming: cannot open ", gr.path);
      gr.stage = stage_host_[g % 2].data_ptr();
    } else {
      gr.host = hostv;
      host_bytes_ += (size_t)gr.elems * 2;
    }
    for (size_t j = 0; j < gr.ps.size(); ++j) {
      Param* p = gr.ps[j];
      const int64_t m = p->c.numel();
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
  for (auto& gr : groups_)
    if (gr.fd >= 0) ::close(gr.fd);
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
  Group& gr = groups_[g];
  if (disk_.dir.empty()) {
    HIP_OK(hipMemcpyAsync(slot_[s].data_ptr(), gr.host.data_ptr(), (size_t)gr.elems * 2, hipMemcpyHostToDevice, copy_));
  } else {
    // disk -> pinned staging (host node, ordered after the staging buffer's previous H2D on this
    // stream) -> HBM (+ fp16 -> bf16 on the device)
    HIP_OK(hipLaunchHostFunc(copy_, &WeightStreamer::read_group, &gr));
    if (!gr.fp16) {
      HIP_OK(hipMemcpyAsync(slot_[s].data_ptr(), gr.stage, gr.bytes, hipMemcpyHostToDevice, copy_));
    } else {
      HIP_OK(hipMemcpyAsync(stage_dev_.data_ptr(), gr.stage, gr.bytes, hipMemcpyHostToDevice, copy_));
      Tensor dst = slot_[s].slice(0, 0, gr.elems), src = stage_dev_.slice(0, 0, gr.elems);
      k::copy(desc(dst), desc(src), copy_);
    }
  }
  HIP_OK(hipEventRecord(ready_[g], copy_));
  holder_[s] = g;
  ++copies;
}

void WeightStreamer::read_group(void* group) {
  // runs on a HIP callback thread: file IO only (no HIP calls); a failed read is fatal
  Group* gr = static_cast<Group*>(group);
  size_t done = 0;
  while (done < gr->bytes) {
    const ssize_t r = ::pread(gr->fd, static_cast<char*>(gr->stage) + done, gr->bytes - done, (off_t)done);
    if (r <= 0) {
      std::fprintf(stderr, "[mft] weight streaming: read of %s failed at byte %zu of %zu\n", gr->path.c_str(), done,
                   gr->bytes);
      std::fflush(stderr);
      std::_Exit(4);
    }
    done += (size_t)r;
  }
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
