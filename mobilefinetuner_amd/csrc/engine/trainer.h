// libmft engine: the training loop (micro-batch accumulation, hipGraph-captured step, eval, logs).
//
// Reference call stack: gpt2_lora_finetune/main.cpp:561-684 -- per step `accum`
// micro-batches of forward -> lm_cross_entropy -> loss/accum -> backward, clip_and_get_grad_norm,
// lr schedule, Adam::step, zero_grad, force_cleanup; eval every eval_interval (JSONL), periodic
// LoRA checkpoints, power-monitor sleep.  MI355X design: the whole step (zero-grad, every
// micro-batch forward+backward, clip, AdamW) is captured ONCE into a hipGraph after two eager
// warm-up steps (relaxed capture mode, private allocator pool) and replayed with the next batch
// copied into the graph's static input buffers; the loss stays on the device and is read only when
// a log line is due.  Data parallelism (engine/comm.h communicator + engine/dist.h reducer): every
// rank starts from rank 0's weights (broadcast), reads its own data shard, and the gradient buckets
// are reduced on a communication stream as the backward completes them (grad-ready hooks), ZeRO-1/2
// partitioning the optimizer; the bucket collectives, the optimizer and the shadow all-gather are
// recorded into the same hipGraph as the forward / backward (MFT_GRAPH_COMM=0: run them eagerly
// after each replay instead).  Logged losses and eval sums are reduced over the ranks and only
// rank 0 prints and saves.
#pragma once
#include <chrono>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "engine/comm.h"
#include "engine/dist.h"
#include "engine/lm.h"
#include "engine/optim.h"
#include "runtime/dataset.h"
#include "runtime/power_monitor.h"

namespace mft {
namespace eng {

struct TrainConfig {
  int epochs = 0;
  int64_t steps = 0;
  int batch = 1, accum = 1, seq = 128;
  int warmup = 0;
  float lr = 1e-4f;  // base learning rate of the schedule
  int log_interval = 1, eval_interval = 0, eval_batches = 50, eval_batch_size = 2, save_every = 0;
  float ema_beta = 0.9f;
  // console line format: "gpt2" = the reference GPT-2 CLI's "[Train] epoch .. | step s/S (global g/G)
  // | lr | loss | ppl | grad_norm | tokens", "gemma" = the reference Gemma trainer's "[Step n] Loss=.."
  std::string log_style = "gpt2";
  bool use_graph = true;
  std::string eval_out, metrics_out;
  std::string state_dir;  // full training-state checkpoint written at every save point and at the end
  // failure injection (--inject_fault step:rank): rank `fault_rank` throws before
  // running step `fault_step` (1-indexed); the CLI exits non-zero and the launcher stops the job
  int64_t fault_step = 0;
  int fault_rank = 0;
  int pm_interval = 0;
  // --profile_steps a:b: steps a..b (1-indexed, inclusive) run inside one
  // "mft.profile" roctx range with the profiler resumed (rocprofv3 --selected-regions collects only
  // them) and each step's device time printed ([profile] lines, hipEvents); 0 = off
  int64_t profile_from = 0, profile_to = 0;
  // --compat_grad_overwrite: the reference overwrites .grad at every backward, so of
  // an accumulated step only the last micro-batch's gradient (scaled by 1/accum) survives
  bool compat_grad_overwrite = false;
  // learning rate of 0-indexed update `it` of `total`; unset: the GPT-2 CLI schedule (gpt2_cli_lr)
  std::function<float(int64_t it, int64_t total)> lr_fn;
  // called on the host before each optimizer step for every micro-batch, with the running 1-based
  // micro-step count and the batch's token ids [B, S] (e.g. the Gemma CLI's --dump_embedding)
  std::function<void(int64_t micro_step, const int64_t* ids, int B, int S)> micro_hook;
};

class Trainer {
 public:
  // comm != null requires dp (the reducer of that communicator)
  Trainer(LanguageModel& model, FlatParams& flat, AdamW& opt, TokenDataset& train, TokenDataset* valid, const TrainConfig& cfg,
          PowerMonitor* pm = nullptr, Communicator* comm = nullptr, GradReducer* dp = nullptr);
  ~Trainer();
  int64_t total_steps() const { return total_steps_; }
  int64_t steps_per_epoch() const { return steps_per_epoch_; }
  // one optimizer step on `accum` micro-batches (host int64 [B, S] ids / targets); returns the
  // device loss (mean over micro-batches)
  Tensor step(const std::vector<std::pair<const int64_t*, const int64_t*>>& micro);
  // ZeRO-1/2: the full fp32 masters on every rank before a checkpoint writer reads them
  // (collective; train() calls it before periodic save_fn exports and once at the end)
  void gather_for_export();
  // a reducer-owned delayed optimizer (ZeRO-3 host-streamed AdamW): apply the pending update now
  void flush_optimizer();
  void train(const std::function<void(int64_t)>& save_fn);
  // Benchmark (bench.py's native engine): `warmup` untimed optimizer steps (the first two eager,
  // then the hipGraph capture), then `steps` timed steps bracketed on both sides by a device
  // synchronize and, with a communicator, a cross-rank barrier.  Returns the MAX over ranks of the
  // timed wall seconds; *final_loss = the last step's (rank-mean) loss.
  double bench(int warmup, int steps, float* final_loss);
  // the step actually replays a captured hipGraph (false: eager -- --no_graph or an uncapturable reducer)
  bool graph_replayed() const { return exec_ != nullptr; }
  // the step will be captured (after the warm-up steps): the config's use_graph less what the trainer ruled out
  bool uses_graph() const { return cfg_.use_graph; }
  std::pair<double, double> evaluate(int max_batches, int batch_size);  // (nll, ppl)
  // Full training state (same directory layout as the Python CLIs' --state_dir):
  // trainable.safetensors (fp32 master) + optimizer.safetensors (AdamW m, v) from rank 0 -- data
  // parallelism keeps them identical on every rank -- and trainer_state.rank<r>.json per rank
  // {global_step, applied optimizer steps, tokens, EMA, data epoch / cursor / shuffle RNG, LoRA-
  // dropout counter}.  load_state returns false when `dir` holds no state; train() then continues
  // from global_step with the same LR schedule position, batches and dropout masks.
  void save_state(const std::string& dir);
  bool load_state(const std::string& dir);
  double ema_loss = 0.0;
  bool ema_init = false;
  int64_t global_step = 0, total_tokens = 0;
  std::vector<float> losses;  // per-step mean loss (read at log points)
  double step_ms = 0.0;

 private:
  void eager_step();
  void fwd_bwd();
  void reduce_grads();   // dp: the buckets no hook launched + join the comm stream
  void optimizer();      // AdamW (+ ZeRO shadow all-gather)
  void capture();
  void sync_ema();       // host mirror (ema_loss / ema_init) of the device EMA, rank-mean
  bool lead() const { return !comm_ || comm_->rank() == 0; }
  LanguageModel& model_;
  FlatParams& flat_;
  AdamW& opt_;
  TokenDataset& train_;
  TokenDataset* valid_;
  TrainConfig cfg_;
  int64_t micro_steps_ = 0;  // micro-batches drawn by train() (TrainConfig::micro_hook)
  std::chrono::steady_clock::time_point pm_t0_;  // end of the last energy-scheduler sleep
  PowerMonitor* pm_;
  Communicator* comm_;
  GradReducer* dp_;
  bool graph_comm_ = true;  // collectives + optimizer inside the captured step
  int64_t total_steps_ = 0, steps_per_epoch_ = 1;
  // static device inputs (the graph reads these) + loss accumulator
  std::vector<Tensor> ids_, labels_;
  Tensor loss_acc_, one_, ema_dev_;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  hipStream_t stream_ = nullptr;
  int warm_ = 0;
  int pool_ = 0;
};

}  // namespace eng
}  // namespace mft
