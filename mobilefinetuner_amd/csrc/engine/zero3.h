// libmft engine: ZeRO-3 -- the trainable parameters themselves partitioned over the ranks.
//
// Reference: the reference's ParameterSharder (operators/opt_ops/sharding/parameter_sharder.cpp:
// 94-276) keeps a byte budget of weights resident and reloads the rest from disk per block
// (require(), called from the model forward, graph/gpt2_model.cpp:536-554).  BASELINE.json config 5
// asks for that capability as a real cross-GPU partition: GPT-2 XL full fine-tuning with ZeRO-style
// parameter sharding + host-DRAM offload over RCCL.  Same design as the Python package's
// parallel/zero3.py, native:
//
//   * units: unit 0 = the weights used outside the blocks (token / position embeddings = the tied
//     LM head), unit 1 + i = transformer block i's projection weights and biases.  fp32-compute
//     parameters (LayerNorm scales / shifts) are small and stay REPLICATED (all-reduced gradients).
//   * every rank keeps 1 / world of each unit: fp32 master, AdamW moments (optionally bf16 in
//     pinned host DRAM), gradient and bf16 shadow -- the local FlatParams buffers are just these
//     partitions plus the replicated parameters;
//   * compute copies: a unit is ALL-GATHERED (bf16 shadow partitions -> the full unit) into a
//     device slot right before the model needs it: unit 0 into its own slot for the whole micro-
//     batch, block i into slot i % 2, block i + 1 prefetched into the other slot on the
//     communication stream while block i computes; in the backward the gate at block i's output
//     re-gathers it (prefetching i - 1).  The Params' compute views point into the slots.
//   * gradients: block i's kernels accumulate into an fp32 work slot (i % 2) that is zeroed at the
//     gate; when the last of the unit's parameters is final (the tape's grad-ready hooks) the slot
//     is REDUCE-SCATTERED (sum; the loss seed carries 1 / world) straight into this rank's
//     partition of the gradient in the first micro-batch, through a landing buffer + add in later
//     ones -- so the partitions are never zeroed.  Replicated gradients are all-reduced in finish().
// Every cross-stream dependency is an event, so the whole step (gathers, reduce-scatters, the
// partitioned optimizer) records into the trainer's hipGraph like any other work.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <string>
#include <utility>
#include <vector>

#include "engine/comm.h"
#include "engine/dist.h"
#include "engine/optim.h"
#include "engine/weight_stream.h"

namespace mft {
namespace eng {

using NamedParams = std::vector<std::pair<std::string, Param*>>;

// The local flat layout of a rank (pure function of the parameter sizes and the world size; the
// host self-test checks it without a GPU): unit u is padded to n = world x s elements (s a
// multiple of 64), each parameter at off[j] inside it; this rank's partition of unit u sits at
// `local` in the flat, then the replicated parameters at rep_at[j] in [rep_off, rep_off + rep_n).
struct Zero3Layout {
  struct UnitLayout {
    std::vector<int64_t> off;
    int64_t n = 0, s = 0, local = 0;
    int slot = 0;  // 0: the outer unit's slot; blocks alternate 1, 2
  };
  std::vector<UnitLayout> units;
  std::vector<int64_t> rep_at;
  int64_t rep_off = 0, rep_n = 0, numel = 0, max_block = 0;
};
Zero3Layout plan_zero3(const std::vector<NamedParams>& units, const NamedParams& rep, int world);

class Zero3 : public GradReducer, public BlockProvider {
 public:
  // units[0]: the outer unit; units[1 + i]: block i; rep: replicated fp32-compute parameters.
  // Parameter values are taken from rank 0 (broadcast) and partitioned.
  Zero3(const std::vector<NamedParams>& units, const NamedParams& rep, Communicator& comm);
  ~Zero3() override;
  Zero3(const Zero3&) = delete;
  Zero3& operator=(const Zero3&) = delete;

  FlatParams& flat() { return flat_; }  // this rank's partitions + the replicated parameters
  // the partitioned AdamW (moments for the local flat; host_moments: in pinned host DRAM, bf16 or
  // fp32).  streamed (with host_moments): the update moves out of the step's critical path -- each
  // unit's partition is updated right before the next forward gathers it, by the fused AdamW on its
  // own stream reading and writing that unit's moments in place over PCIe (both directions at once),
  // under the forward's compute; the unit's all-gather waits only for its own update.  The step's
  // gradients, norm and lr wait in place from the end of one backward to the next forward
  // (AdamW::prepare_delayed).
  void shard_optimizer(AdamW& opt, bool host_moments, bool host_fp32 = false, bool streamed = false);

  // GradReducer
  void begin_micro(int i, int n) override;
  void finish() override;
  void after_optimizer() override;
  bool owns_optimizer() const override { return sopt_ != nullptr; }
  void prepare_optimizer() override;
  void flush_optimizer() override;
  void optimizer_state_loaded() override;
  // The staged step captures since round 6 (it crashed hipStreamEndCapture before: gather() made the
  // communication stream wait on an event it had recorded itself -- a self-edge in the captured graph;
  // profiles/r6_z3_capture_trace.txt), but it runs eagerly by default: as graph memcpy nodes its SDMA
  // moment copies measured 57 K against 80 K tok/s eager (gpt2-xl).  MFT_Z3_CAPTURE=1 captures it.
  bool graph_capturable() const override {
    static const bool on = std::getenv("MFT_Z3_CAPTURE") && std::getenv("MFT_Z3_CAPTURE")[0] == '1';
    return on || !(sopt_ && staged_);
  }
  int staged_slots() const { return sopt_ && staged_ ? nslot_ : 0; }  // 0: in place (or no host moments)
  bool params_sharded() const override { return true; }
  float grad_prescale() const override;
  void zero_grad(FlatParams& flat) override;
  std::string describe() const override;
  // BlockProvider
  void begin_forward() override;
  void ensure(int block, int next) override;
  std::pair<Tensor, Tensor> gate(const Tensor& x, const Tensor& h, int block) override;

  // after training: every partitioned Param gets its full fp32 value back (a fresh leaf) and a
  // matching bf16 compute copy, so checkpoint writers see whole tensors (collective: all ranks)
  void materialize();
  int64_t gathers = 0, reduce_scatters = 0;  // collectives issued (host count)

 private:
  struct Unit {
    NamedParams params;
    std::vector<int64_t> off;  // element offsets inside the unit
    int64_t n = 0, s = 0;      // padded unit size, partition size (n = world * s)
    int64_t local = 0;         // partition offset in the local flat
    int slot = 0;              // gather / gradient slot
    int pending = 0, total = 0;
    bool reduced = false;
  };
  bool first_micro_ = true;
  void gather(int u);
  void reduce_scatter(int u);
  void on_ready(int u);
  void zero_work(int slot);
  Communicator& comm_;
  std::vector<Unit> units_;
  NamedParams rep_;
  int64_t rep_off_ = 0, rep_n_ = 0;
  FlatParams flat_;
  std::vector<Tensor> slot_, gwork_;  // bf16 gathered units, fp32 gradient work buffers
  std::vector<int> holder_;           // unit whose gather was last issued into each slot
  std::vector<hipEvent_t> ready_, rs_done_;
  std::vector<char> rs_live_;  // rs_done_[slot] recorded in the current step
  hipEvent_t order_ = nullptr, join_ = nullptr;
  hipStream_t stream_ = nullptr;  // communication stream
  Tensor dummy_, tmp_;            // placeholder leaf storage, reduce-scatter landing buffer
  // ---- host-streamed optimizer (shard_optimizer(..., streamed = true))
  // update index i: 0 = the replicated parameters, 1 + u = unit u (forward order)
  int64_t upd_off(int i) const { return i == 0 ? rep_off_ : units_[i - 1].local; }
  int64_t upd_len(int i) const { return i == 0 ? rep_n_ : units_[i - 1].s; }
  void opt_fork();             // the optimizer stream joins the current stream's work
  void opt_update(int i);      // AdamW on update i, moments in place in host DRAM
  void join_opt_stream();      // the current stream waits for the optimizer stream
  AdamW* sopt_ = nullptr;
  // primed_: an update has been prepared at least once (the device flag exists); the updates are then
  // issued at every gather / zero_grad / finish / flush and gated on the device flag -- never on host
  // state, which a hipGraph replay does not advance
  bool sfp32_ = false, primed_ = false, forked_ = false;
  std::vector<int> supd_;             // per update: issued this step
  std::vector<hipEvent_t> upd_ev_;    // per update: applied
  hipEvent_t fork_ev_ = nullptr, ojoin_ev_ = nullptr;
  // ONE side stream: a staged variant (H2D copy -> update -> D2H copy on three streams, the slot's
  // next H2D behind its D2H) forms a dependency ring over three side streams, which crashes
  // hipStreamEndCapture on this ROCm (scripts/probes/r4_capture_probe.hip, profiles/r4_capture_probe.txt),
  // and with the copies folded onto one stream its two PCIe directions serialise (slower than in place:
  // profiles/r4_offload_modes.txt).
  hipStream_t ostream_ = nullptr;
  int opt_grid_ = 0;  // workgroups per update (MFT_Z3_OPT_GRID)
  // staged (default; MFT_Z3_STAGED=0: in place): the moments of update i live in device slot i % S during
  // the step; update i runs on the communication stream (device-resident, full grid), the one copy stream
  // writes the slot back and prefetches its next user -- streams: copy <-> communication ping-pong only
  bool staged_ = false;
  int nslot_ = 0;
  int64_t slot_elems_ = 0;
  Tensor slot_mv_;                   // [S][m | v][slot_elems_] (bf16 or fp32 moments)
  hipStream_t cstream_ = nullptr;    // SDMA copies, both directions
  hipEvent_t cjoin_ev_ = nullptr;
  std::vector<hipEvent_t> h2d_ev_;   // per update: its slot filled (recorded this step)
  std::vector<char> h2d_pending_;    // h2d_ev_[i] recorded this step and not yet waited on
  void* slot_ptr(int i, int which);  // which: 0 = m, 1 = v
  void slot_copy(int i, bool h2d);
};

}  // namespace eng
}  // namespace mft
