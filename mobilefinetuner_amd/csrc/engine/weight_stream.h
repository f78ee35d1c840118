// libmft engine: frozen-weight streaming for `--shard_enable` (host-DRAM weight tier).
//
// Reference: ParameterSharder (operators/opt_ops/sharding/parameter_sharder.h:36-93, .cpp:86-276):
// register_parameter drops the RAM copy to disk, require(name) reloads it under a byte budget with
// LRU eviction, called from the model forward per block (graph/gpt2_model.cpp:536-554).
//
// MI355X design (native engine): each transformer block's frozen bf16 weights are ONE contiguous
// pinned host buffer; K device slots (K = budget / largest block, at least 2) hold the blocks in
// use, block i always in slot i % K, so every Param of a streamed block is a fixed view into its
// slot and the whole schedule is static -- it records into the trainer's hipGraph like any other
// work.  ensure(i, next) makes block i resident (one H2D copy on a dedicated copy stream, ordered
// after every kernel that used the slot before through an event recorded on the compute stream)
// and prefetches `next` into its own slot while block i computes.  The forward walks the blocks up,
// a gate node at each block boundary re-loads the block on the way back down in the backward.
// Embeddings, norms and trainable (LoRA) parameters stay resident.
//
// Disk tier (--shard_dir D [--shard_fp16_disk 0|1]; the reference's offload files,
// parameter_sharder.cpp:21-76,205-276): every block's bytes go to D/block_<i>.bin -- as fp16 when
// asked AND every value of the block survives bf16 -> fp16 -> bf16 exactly (fp16's normal range);
// otherwise that block is written as bf16 (the same 2 bytes, lossless) -- and no host copy
// stays resident.  A load is then a HOST NODE on the copy stream (pread of the file into one of two
// pinned staging buffers) followed by the H2D copy (+ an fp16 -> bf16 cast kernel on the device),
// so the disk -> DRAM -> HBM pipeline is still one static schedule that a hipGraph records.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "engine/nn.h"

namespace mft {
namespace eng {

// Per-block residency of a model's weights, driven by the model forward (GPT2::hidden): the
// host-DRAM weight stream below (--shard_enable, frozen weights) and the ZeRO-3 partitioner
// (engine/zero3.h, trainable weights gathered from their rank partitions).
class BlockProvider {
 public:
  virtual ~BlockProvider() = default;
  // start of a forward: the non-block weights (embeddings) resident
  virtual void begin_forward() {}
  // block g resident before the current stream's next kernel; prefetch block `next` (-1: none)
  virtual void ensure(int g, int next) = 0;
  // identity on (x, h), the block's outputs; its backward runs before block g's backward does
  virtual std::pair<Tensor, Tensor> gate(const Tensor& x, const Tensor& h, int g) = 0;
};

struct DiskTier {
  std::string dir;    // empty: host-DRAM tier only
  bool fp16 = true;   // store fp16 on disk (reference --shard_fp16_disk, default 1)
};

class WeightStreamer : public BlockProvider {
 public:
  // groups[i]: the frozen bf16 Params of block i (re-bound to slot views; their device copies freed)
  WeightStreamer(const std::vector<std::vector<Param*>>& groups, size_t budget_bytes, const DiskTier& disk = {});
  ~WeightStreamer();
  WeightStreamer(const WeightStreamer&) = delete;
  WeightStreamer& operator=(const WeightStreamer&) = delete;
  // block g resident before the current stream's next kernel; prefetch block `next` (-1: none)
  void ensure(int g, int next) override;
  // identity on (x, h) whose backward calls ensure(g, g - 1) before block g's backward runs
  std::pair<Tensor, Tensor> gate(const Tensor& x, const Tensor& h, int g) override;
  int slots() const { return (int)slot_.size(); }
  size_t device_bytes() const { return slot_bytes_ * slot_.size(); }
  size_t host_bytes() const { return host_bytes_; }    // resident pinned bytes (staging only with a disk tier)
  size_t disk_bytes() const { return disk_bytes_; }
  bool on_disk() const { return !disk_.dir.empty(); }
  int64_t copies = 0;  // H2D group copies issued (a graph replay repeats its recorded ones)
  int64_t bf16_fallbacks = 0;  // --shard_fp16_disk blocks kept bf16 (values outside fp16's exact range)

 private:
  void issue(int g);
  struct Group {
    std::vector<Param*> ps;
    std::vector<int64_t> off;  // element offsets inside the slot
    Tensor host;               // pinned bf16 [elems] (host tier)
    int64_t elems = 0;
    // disk tier: the host node's arguments (stable addresses for hipLaunchHostFunc)
    int fd = -1;
    void* stage = nullptr;
    size_t bytes = 0;
    std::string path;
    bool fp16 = false;  // this block's file holds fp16 (exact round trip), else bf16
  };
  static void read_group(void* group);  // host node: pread the block's file into its staging buffer
  std::vector<Group> groups_;
  std::vector<Tensor> slot_;
  std::vector<int> holder_;  // group whose copy was last issued into each slot (-1: none)
  std::vector<hipEvent_t> ready_;
  hipEvent_t order_ = nullptr;
  hipStream_t copy_ = nullptr;
  size_t slot_bytes_ = 0, host_bytes_ = 0, disk_bytes_ = 0;
  bool capturing_ = false;
  DiskTier disk_;
  std::vector<Tensor> stage_host_;  // two pinned staging buffers (disk tier)
  Tensor stage_dev_;                // fp16 landing buffer before the cast (fp16 on disk)
};

}  // namespace eng
}  // namespace mft
