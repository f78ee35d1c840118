// libmft engine: flat parameter storage, fused AdamW with global-norm clipping, LR schedules.
//
// Reference: Adam (operators/finetune_ops/optim/adam.h:23-104, adam.cpp:25-140: bias-corrected,
// coupled L2 decay, per-tensor state map), the clip_grad_norm copies (gpt2_lora_finetune/main.cpp:
// 491-516) and the three LR schedules (main.cpp:470-488, gemma_trainer.cpp:63-82,
// trainer.cpp:44-64).  MI355X design (same as the Python package's utils/params.py + optim/adamw.py):
// every trainable parameter lives in ONE fp32 master buffer with ONE fp32 grad buffer and ONE bf16
// compute shadow; one sumsq reduction, one non-finite check and one fused AdamW launch per step,
// lr / step / norm^2 in device memory so the whole optimizer step replays inside a hipGraph.
#pragma once
#include <string>
#include <utility>
#include <vector>

#include "engine/comm.h"
#include "engine/nn.h"
#include "kernels.h"

namespace mft {
namespace eng {

class FlatParams {
 public:
  // re-homes every param: leaf -> view of `master` (requires grad, .grad = view of `grad`),
  // compute view -> view of `shadow` (bf16) unless the param computes in fp32.  `offsets` / `numel`
  // (optional): a layout planned by the data-parallel reducer (bucket padding, engine/dist.h);
  // default: params packed in order, each 64-element aligned.
  explicit FlatParams(std::vector<std::pair<std::string, Param*>> params, std::vector<int64_t> offsets = {},
                      int64_t numel = 0);
  // bare buffers of `numel` elements that their owner lays out itself (ZeRO-3 partitions)
  static FlatParams buffers(int64_t numel);
  Tensor master, grad, shadow;
  int64_t numel = 0;
  std::vector<std::pair<std::string, Param*>> params;
  std::vector<int64_t> offsets;
  void zero_grad();
  void refresh_shadow();
};

// one contiguous range of the flat buffers this rank updates; its moments live at state_off
struct OptSegment {
  int64_t off = 0, len = 0, state_off = 0;
  bool replicated = false;  // identical on every rank: its norm^2 counts once, outside the all-reduce
};

struct AdamWConfig {
  float lr = 1e-4f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, weight_decay = 0.f;
  float max_grad_norm = 1.f;  // <= 0: no clipping
  bool l2_coupled = false;    // reference Adam (L2 added to the gradient)
  bool skip_nonfinite = true;
  bool amsgrad = false;       // AMSGrad, reference rule (optim/adam.cpp:52,75-80): v_hat = max(v_hat, v / bc2)
};

class AdamW {
 public:
  AdamW(FlatParams& flat, const AdamWConfig& cfg);
  void set_lr(float lr);  // host -> device scalar (outside graph capture)
  void step();            // device-only work: capturable (prepare + every segment + commit)
  // the gradient statistics of step(): global norm^2 (all-reduced) / non-finite flag
  void prepare();
  // Delayed, streamed updates (ZeRO-3 + host moments, engine/zero3.h): prepare_delayed() after the
  // backward records the step's statistics and lr and marks the gradients pending;
  // apply_delayed() then updates one flat range [off, off + len) with moments staged on the device
  // (gated on the pending flag); commit_delayed() advances the step count and clears the flag.
  void prepare_delayed();
  void apply_delayed(int64_t off, int64_t len, void* m_dev, void* v_dev, bool moments_bf16, hipStream_t s,
                     int max_grid = 0);
  void commit_delayed(hipStream_t s);
  Tensor pending_dev, lr_step_dev;  // delayed mode: gradients pending (int32), their lr
  float grad_norm() const;  // host sync
  bool skipped_last() const;
  int64_t applied_steps() const;
  Tensor m, v, lr_dev, step_dev, sumsq_dev, nonfinite_dev, skipped_dev;
  Tensor vmax;  // AMSGrad running max of v (undefined when off)
  const AdamWConfig& config() const { return cfg_; }
  void load_vmax(const Tensor& h);  // AMSGrad running max (checkpoint resume)
  void load_state(const Tensor& m_h, const Tensor& v_h, int64_t steps);
  // ZeRO-1/2 (engine/dist.h): update only `segs` -- this rank's partition of the flat buffers --
  // with moments of sum(len) elements; host_moments: bf16 moments in pinned host DRAM that the
  // kernel reads and writes in place over PCIe (the host-offload tier of the optimizer state).
  // The grad-norm^2 and the non-finite flag are all-reduced over `comm`, so every rank clips and
  // skips identically.
  void shard(const std::vector<OptSegment>& segs, Communicator* comm, bool host_moments, bool host_fp32 = false);
  const std::vector<OptSegment>& segments() const { return segs_; }
  bool sharded() const { return comm_ != nullptr; }
  bool moments_on_host() const { return host_moments_; }
  int64_t state_numel() const { return state_numel_; }
  // --offload disk: the moments (this rank's state_numel() of each) live in file-backed memory --
  // MAP_SHARED mappings of <dir>/adamw_{m,v}.rank<r>.bin, so the page cache keeps what fits and the
  // kernel writes the rest back to the file -- and step() streams them through two device chunk buffers
  // (mapping -> pinned staging -> device -> fused AdamW -> back), chunk by chunk.  Host copies run inside
  // the step, so it is not graph-capturable (the trainer runs it eagerly).  Call after shard().
  // (SURVEY §5.6's `--offload none|host|disk`; the reference's own disk tier holds frozen weights only,
  // opt_ops/sharding/parameter_sharder.cpp:94-276 -- here engine/weight_stream.h's --shard_dir.)
  void to_disk(const std::string& dir, int rank, bool fp32);
  bool moments_on_disk() const { return disk_.active; }
  ~AdamW();
  AdamW(const AdamW&) = delete;
  AdamW& operator=(const AdamW&) = delete;

 private:
  struct DiskMoments {
    bool active = false;
    void* map[2] = {nullptr, nullptr};  // m, v mappings
    size_t bytes = 0, elem = 4;
    int64_t chunk = 0;
    Tensor dev[2], pin[2];  // device chunk buffers, pinned staging
  };
  DiskMoments disk_;
  void step_disk(::mft::AdamWArgs a, hipStream_t s);
  FlatParams& flat_;
  AdamWConfig cfg_;
  std::vector<OptSegment> segs_;  // default: one segment = the whole flat buffer
  Communicator* comm_ = nullptr;
  bool host_moments_ = false;
  int64_t state_numel_ = 0;
  Tensor part_;  // sumsq partials
  ::mft::AdamWArgs args() const;  // hyper-parameters, lr / step / norm / skip pointers
};

// (a) GPT-2 CLIs: linear warmup (step+1)/W, then cosine to min_ratio of lr (0-indexed step)
float gpt2_cli_lr(int64_t step, float base, int64_t warmup, int64_t total, float min_ratio = 0.1f);
// (b) Gemma trainer: warmup = ceil(ratio * total), 1-indexed, then linear (or cosine) to 0
float gemma_lr(int64_t step, float base, float warmup_ratio, int64_t total, bool cosine = false);
// (c) LoRATrainer: linear / cosine after warmup
float trainer_lr(int64_t step, float base, int64_t warmup, int64_t total, bool cosine = false);

}  // namespace eng
}  // namespace mft
