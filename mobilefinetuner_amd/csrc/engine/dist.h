// libmft engine: data parallelism over the Communicator -- bucketed gradient reduction overlapped
// with the backward, ZeRO-1 / ZeRO-2 partitioning of the optimizer, host-offloaded moments.
//
// Reference: there is no distributed code in the reference; its "ZeRO-inspired"
// ParameterSharder (operators/opt_ops/sharding/parameter_sharder.cpp:94-276) is a single-device
// RAM <-> disk LRU.  BASELINE.json asks for a real cross-GPU partition with RCCL reduce-scatter /
// all-gather over xGMI plus a host-DRAM tier; this file is that for the native engine (ZeRO-3 --
// the parameters themselves partitioned -- is engine/zero3.h).
//
// Layout.  plan_flat() orders the trainable parameters into BUCKETS in backward order (the last
// parameters of the forward are ready first) of about `bucket_bytes` of fp32 gradient each, and
// pads every bucket to a multiple of world x 64 elements, so bucket b = [lo, hi) splits into
// `world` equal, 256-B aligned chunks.  Rank r owns chunk r of every bucket: its ZeRO partition.
// Parameters that compute in fp32 (norm weights: their compute tensor IS the fp32 master) form one
// extra REPLICATED bucket, launched last: always all-reduced and updated in full on every rank, so
// no rank computes with a stale copy of a chunk it does not own.
//
// Step.  The autograd tape's grad-ready hooks (engine/autograd.h) count the parameters of each
// bucket during the LAST micro-batch's backward; when a bucket is complete, an event on the compute
// stream orders a collective on a dedicated communication stream:
//   stage 0 / 1  all-reduce (sum; the loss seed carries 1 / world) of the bucket (fp32, or bf16)
//   stage 2      reduce-scatter (sum) into the owned chunk (half the bytes of an all-reduce)
// so the reduction of early buckets overlaps the backward of the remaining layers.  finish() joins
// the communication stream back.  The optimizer then updates either everything (stage 0) or only
// the owned chunks (stages 1 / 2: AdamW::shard, moments for 1/world of the parameters, optionally
// in pinned host DRAM), and after_optimizer() all-gathers the updated bf16 compute shadows.
// Every piece is stream-ordered (events, no host syncs), so the whole step -- forward, backward,
// bucket collectives, optimizer, all-gather -- records into ONE hipGraph (RCCL kernels, or the
// loopback backend's host nodes).
#pragma once
#include <string>
#include <utility>
#include <vector>

#include "engine/comm.h"
#include "engine/optim.h"

namespace mft {
namespace eng {

// What the Trainer drives around each step: the data-parallel reducer (DataParallel, ZeRO-0/1/2)
// or the ZeRO-3 partitioner (engine/zero3.h).
class GradReducer {
 public:
  virtual ~GradReducer() = default;
  // host bookkeeping of a step (also inside a graph capture): micro-batch i of n starts
  virtual void begin_micro(int i, int n) = 0;
  // after the last backward: the reductions no hook launched, comm stream joined back
  virtual void finish() = 0;
  // after the optimizer step (ZeRO-1/2: all-gather the updated bf16 shadows)
  virtual void after_optimizer() {}
  // full fp32 masters on every rank before a checkpoint (ZeRO-1/2)
  virtual void gather_master() {}
  // a reducer that runs the optimizer itself (ZeRO-3's host-streamed AdamW, engine/zero3.h): the
  // trainer calls prepare_optimizer() after the backward instead of AdamW::step(); the update is
  // applied per unit during the NEXT forward, and flush_optimizer() applies a pending update at once
  // (before evaluation, checkpoints, exports and at the end of training)
  virtual bool owns_optimizer() const { return false; }
  virtual void prepare_optimizer() {}
  virtual void flush_optimizer() {}
  // the optimizer's (host) moments were overwritten (checkpoint load): drop any device copies of them
  virtual void optimizer_state_loaded() {}
  // false: the step must run eagerly (its stream pattern cannot be captured into a hipGraph)
  virtual bool graph_capturable() const { return true; }
  // ZeRO-3: each rank's flat holds only its partitions (no initial broadcast, per-rank masters)
  virtual bool params_sharded() const { return false; }
  // factor folded into the loss seed (and the fused LM-head weight grad): a reducer that SUMS
  // returns 1 / world so the reduced gradient is the average
  virtual float grad_prescale() const { return 1.f; }
  // clear the gradients a step accumulates into (a reducer whose first reduction overwrites its
  // destination clears less)
  virtual void zero_grad(FlatParams& flat) { flat.zero_grad(); }
  virtual std::string describe() const = 0;
};

struct DistConfig {
  int zero_stage = 0;                // 0 DDP, 1 partitioned optimizer, 2 + reduce-scattered grads
  int64_t bucket_bytes = 25 << 20;   // fp32 gradient bytes per bucket (MFT_BUCKET_MB)
  bool bf16_reduce = false;          // reduce gradients in bf16 (half the bytes on the links)
  bool overlap = true;               // launch buckets from the grad-ready hooks during backward
  bool host_moments = false;         // stage >= 1: AdamW moments in pinned host DRAM
  bool host_fp32 = false;            // ... as fp32 (default bf16, stochastically rounded)
  std::string disk_dir;              // --offload disk: AdamW moments in files under this directory
                                     // (AdamW::to_disk; stages 0-2, eager step)
  bool host_stream = true;           // ZeRO-3: each unit's update applied in place (moments read and
                                     // written over PCIe) during the next forward on a side stream;
                                     // false: one update of everything after the backward
};

struct FlatPlan {
  std::vector<int64_t> offsets;                      // per parameter (forward order)
  int64_t numel = 0;
  std::vector<std::pair<int64_t, int64_t>> buckets;  // [lo, hi) in backward (launch) order
  std::vector<int> bucket_of;                        // per parameter
  std::vector<char> replicated;                      // per bucket: the fp32-compute parameters' bucket
};

// Bucketed, padded flat layout for `world` ranks (world 1: still bucketed, chunking trivial).
FlatPlan plan_flat(const std::vector<std::pair<std::string, Param*>>& params, int world, int64_t bucket_bytes);

class DataParallel : public GradReducer {
 public:
  DataParallel(FlatParams& flat, const FlatPlan& plan, Communicator& comm, AdamW& opt, const DistConfig& cfg);
  ~DataParallel();
  DataParallel(const DataParallel&) = delete;
  DataParallel& operator=(const DataParallel&) = delete;

  void begin_micro(int i, int n) override;
  // after the last backward: launch the buckets no hook completed, join the comm stream
  void finish() override;
  // stage >= 1 after the optimizer step: all-gather the updated bf16 shadow chunks
  void after_optimizer() override;
  // stage >= 1: the full fp32 master on every rank (checkpoints / exports), then every shadow
  void gather_master() override;
  // the loss seed carries 1 / world, the buckets are SUMMED (RCCL's Avg is inexact at some lengths:
  // comm.h)
  float grad_prescale() const override { return 1.f / (float)comm_.world(); }
  int stage() const { return cfg_.zero_stage; }
  const FlatPlan& plan() const { return plan_; }
  std::string describe() const override;
  int64_t launched = 0;  // bucket collectives issued (host count; graph replays repeat theirs)

 private:
  void on_ready(int param_index);
  void launch(int b);
  int64_t chunk(int b) const { return (plan_.buckets[b].second - plan_.buckets[b].first) / comm_.world(); }
  FlatParams& flat_;
  FlatPlan plan_;
  Communicator& comm_;
  AdamW& opt_;
  DistConfig cfg_;
  hipStream_t stream_ = nullptr;  // communication stream
  std::vector<hipEvent_t> ready_ev_;
  hipEvent_t join_ev_ = nullptr;
  std::vector<int> pending_, total_;
  std::vector<char> done_;
  bool last_micro_ = true;
  int hooked_ = 0;          // buckets of this step launched from a grad-ready hook (inside the backward)
  bool reported_ = false;   // the first step's overlap line printed
  Tensor comm_buf_;  // bf16 reduce staging [numel]
};

}  // namespace eng
}  // namespace mft
