// libmft engine: training loop (see trainer.h).
#include "engine/trainer.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <stdexcept>
#include <thread>

#include <filesystem>

#include "engine/allocator.h"
#include "engine/autograd.h"
#include "engine/ops.h"
#include "engine/tensor_kernels.h"
#include "engine/trace.h"
#include "runtime/json.h"
#include "runtime/safetensors.h"

namespace mft {
namespace eng {

Trainer::Trainer(LanguageModel& model, FlatParams& flat, AdamW& opt, TokenDataset& train, TokenDataset* valid,
                 const TrainConfig& cfg, PowerMonitor* pm, Communicator* comm, GradReducer* dp)
    : model_(model), flat_(flat), opt_(opt), train_(train), valid_(valid), cfg_(cfg), pm_(pm), comm_(comm), dp_(dp) {
  stream_ = current_stream();
  MFT_CHECK(!comm_ || dp_, "Trainer: a communicator needs its DataParallel reducer");
  const char* gc = std::getenv("MFT_GRAPH_COMM");
  graph_comm_ = !(gc && gc[0] == '0');
  if (!graph_comm_ && dp_ && dp_->owns_optimizer()) {
    // the streamed ZeRO-3 optimizer forks its stream inside fwd_bwd() and joins it in finish(): a
    // capture of fwd_bwd() alone would end with an unjoined stream
    std::fprintf(stderr, "[trainer] MFT_GRAPH_COMM=0 ignored: the host-streamed ZeRO-3 optimizer runs inside the graph\n");
    graph_comm_ = true;
  }
  if (cfg_.use_graph && dp_ && !dp_->graph_capturable()) {
    // the staged host-moment ZeRO-3 optimizer: eager by default, faster than its captured form
    // (engine/zero3.h graph_capturable(); MFT_Z3_CAPTURE=1 captures it)
    std::printf("[trainer] step runs eagerly (no hipGraph): staged host-moment optimizer (faster eager; MFT_Z3_CAPTURE=1)\n");
    cfg_.use_graph = false;
  }
  if (cfg_.use_graph && opt_.moments_on_disk()) {  // host copies from the file mappings inside the step
    std::printf("[trainer] step runs eagerly (no hipGraph): AdamW moments on disk\n");
    cfg_.use_graph = false;
  }
  if (cfg_.use_graph && !model_.capturable()) {
    // the composite path (--dtype fp32 / --attn_impl naive) reads host values inside the step
    std::printf("[trainer] step runs eagerly (no hipGraph): %s composite path\n",
                compute_dtype() == DType::F32 ? "--dtype fp32" : "--attn_impl naive");
    cfg_.use_graph = false;
  }
  MFT_CHECK(!(cfg_.compat_grad_overwrite && cfg.accum > 1 && dp_ && dp_->params_sharded()),
            "--compat_grad_overwrite with ZeRO-3 is not supported");
  if (comm_ && !(dp_ && dp_->params_sharded())) {  // every rank starts from rank 0's trainable weights
    comm_->broadcast(flat_.master.data_ptr(), (size_t)flat_.numel * sizeof(float), 0, stream_);
    flat_.refresh_shadow();
  }
  const int64_t micro = cfg.batch, accum = std::max(1, cfg.accum);
  const int64_t n_local = (int64_t)train.num_local();
  steps_per_epoch_ = std::max<int64_t>(1, (n_local + micro * accum - 1) / (micro * accum));
  total_steps_ = cfg.steps;
  if (cfg.epochs > 0) total_steps_ = steps_per_epoch_ * cfg.epochs;
  for (int i = 0; i < accum; ++i) {
    ids_.push_back(zeros({micro, cfg.seq}, DType::I64));
    labels_.push_back(full({micro, cfg.seq}, -100.0, DType::I64));
  }
  loss_acc_ = zeros({1}, DType::F32);
  one_ = ones({1}, DType::I64);
  ema_dev_ = zeros({2}, DType::F32);
}

Trainer::~Trainer() {
  if (exec_) (void)hipGraphExecDestroy(exec_);
  if (graph_) (void)hipGraphDestroy(graph_);
}

void Trainer::eager_step() {
  fwd_bwd();
  reduce_grads();
  optimizer();
}

void Trainer::reduce_grads() {
  if (dp_) dp_->finish();
}

void Trainer::optimizer() {
  if (dp_ && dp_->owns_optimizer()) {  // ZeRO-3 host-streamed AdamW: applied during the next forward
    dp_->prepare_optimizer();
    return;
  }
  opt_.step();
  if (dp_) dp_->after_optimizer();
}

void Trainer::flush_optimizer() {
  if (dp_ && dp_->owns_optimizer()) dp_->flush_optimizer();
}

void Trainer::fwd_bwd() {
  const float inv = 1.f / (float)ids_.size();
  const float gs = inv * (dp_ ? dp_->grad_prescale() : 1.f);  // backward seed
  if (dp_) dp_->zero_grad(flat_);
  else flat_.zero_grad();
  loss_acc_.zero_();
  {
    // fresh LoRA-dropout masks every step (device counter, advanced inside the graph too)
    k::Desc c = desc(model_.dropout_ctr);
    k::binary(c, c, desc(one_), k::B_ADD, 1.f, current_stream());
  }
  for (size_t i = 0; i < ids_.size(); ++i) {
    if (dp_) dp_->begin_micro((int)i, (int)ids_.size());  // the last micro-batch's hooks launch buckets
    if (cfg_.compat_grad_overwrite && i > 0) {  // reference .grad overwrite: earlier micro-batches drop out
      if (dp_) dp_->zero_grad(flat_);
      else flat_.zero_grad();
    }
    Tensor loss = model_.loss(ids_[i], labels_[i], gs);
    Tensor scaled = mul_scalar(loss, gs);
    backward({scaled});
    lora_prep_step_end();  // the LoRA weight-prep batch covered this forward + backward only
    add_(loss_acc_, loss.detach(), inv);
  }
}

void Trainer::capture() {
  TraceRange range("mft.capture");
  auto& al = CachingAllocator::get(Device::current_hip_device());
  pool_ = al.new_pool();
  CachingAllocator::set_current_pool(pool_);
  HIP_OK(hipStreamBeginCapture(stream_, hipStreamCaptureModeRelaxed));
  // the whole step, collectives included (the reducer's comm stream forks from and joins back
  // into the capture stream through events); MFT_GRAPH_COMM=0 leaves the collectives and the
  // optimizer out of the graph (then run eagerly after each replay, buckets not overlapped)
  if (graph_comm_) eager_step();
  else fwd_bwd();
  if (std::getenv("MFT_Z3_TRACE")) std::fprintf(stderr, "[trainer] ending capture\n");
  const auto tc0 = std::chrono::steady_clock::now();
  HIP_OK(hipStreamEndCapture(stream_, &graph_));
  CachingAllocator::set_current_pool(0);
  if (std::getenv("MFT_Z3_TRACE")) {
    size_t nn = 0;
    (void)hipGraphGetNodes(graph_, nullptr, &nn);
    std::fprintf(stderr, "[trainer] captured %zu nodes in %.1f ms; instantiating\n", nn,
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc0).count());
  }
  HIP_OK(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0));
  if (std::getenv("MFT_Z3_TRACE")) std::fprintf(stderr, "[trainer] instantiated\n");
}

Tensor Trainer::step(const std::vector<std::pair<const int64_t*, const int64_t*>>& micro) {
  TraceRange range("mft.step");
  MFT_CHECK(micro.size() == ids_.size(), "trainer: expected ", ids_.size(), " micro-batches");
  for (size_t i = 0; i < micro.size(); ++i) {
    Tensor hi = from_blob(const_cast<int64_t*>(micro[i].first), ids_[i].shape(), DType::I64, Device::cpu());
    Tensor hl = from_blob(const_cast<int64_t*>(micro[i].second), labels_[i].shape(), DType::I64, Device::cpu());
    ids_[i].copy_(hi);
    labels_[i].copy_(hl);
  }
  if (!cfg_.use_graph) {
    eager_step();
  } else if (!exec_) {
    if (warm_ < 2) {
      ++warm_;
      eager_step();
    } else {
      capture();
      HIP_OK(hipGraphLaunch(exec_, stream_));
      if (!graph_comm_) {
        reduce_grads();
        optimizer();
      }
    }
  } else {
    HIP_OK(hipGraphLaunch(exec_, stream_));
    if (!graph_comm_) {
      reduce_grads();
      optimizer();
    }
  }
  if (comm_) comm_->heartbeat();
  return loss_acc_;
}

std::pair<double, double> Trainer::evaluate(int max_batches, int batch_size) {
  TraceRange range("mft.eval");
  if (!valid_) return {0.0, 0.0};
  Communicator::QuietScope quiet(comm_);  // rank-local work between collectives: not a hang
  flush_optimizer();                      // the weights of every step so far
  NoGradGuard ng;
  valid_->reset_cursor();
  const int S = cfg_.seq;
  std::vector<int64_t> ids((size_t)batch_size * S), tg((size_t)batch_size * S);
  std::vector<float> mk((size_t)batch_size * S);
  double nll = 0.0, cnt = 0.0;
  int done = 0;
  const bool tr = model_.training;
  model_.training = false;
  while (max_batches <= 0 || done < max_batches) {
    const int got = valid_->next_batch(batch_size, false, ids.data(), tg.data(), mk.data(), nullptr);
    if (got == 0) break;
    Tensor di = from_host(ids.data(), {batch_size, S}, DType::I64);
    Tensor dl = from_host(tg.data(), {batch_size, S}, DType::I64);
    auto r = model_.nll(di, dl);
    nll += r.first.item();
    cnt += r.second.item();
    ++done;
  }
  model_.training = tr;
  if (comm_) {  // token-weighted over every rank's shard
    float h2[2] = {(float)nll, (float)cnt};
    Tensor d = from_host(h2, {2}, DType::F32);
    comm_->all_reduce_sum(static_cast<float*>(d.data_ptr()), 2, current_stream());
    Tensor back = d.to(Device::cpu());
    nll = static_cast<const float*>(back.data_ptr())[0];
    cnt = static_cast<const float*>(back.data_ptr())[1];
  }
  const double m = nll / std::max(1.0, cnt);
  return {m, std::exp(std::min(m, 50.0))};
}

double Trainer::bench(int warmup, int steps, float* final_loss) {
  const int B = cfg_.batch, S = cfg_.seq, A = (int)ids_.size();
  std::vector<std::vector<int64_t>> hid(A, std::vector<int64_t>((size_t)B * S)),
      htg(A, std::vector<int64_t>((size_t)B * S));
  std::vector<float> mk((size_t)B * S);
  Tensor loss;
  auto one = [&](int64_t it) {
    opt_.set_lr(cfg_.lr_fn ? cfg_.lr_fn(it, warmup + steps) : cfg_.lr);
    std::vector<std::pair<const int64_t*, const int64_t*>> micro;
    for (int a = 0; a < A; ++a) {
      train_.next_batch(B, true, hid[a].data(), htg[a].data(), mk.data(), nullptr);
      micro.push_back({hid[a].data(), htg[a].data()});
    }
    loss = step(micro);
    ++global_step;
    total_tokens += (int64_t)A * B * S;
  };
  for (int i = 0; i < warmup; ++i) one(i);
  auto fence = [&]() {
    synchronize();
    if (comm_) comm_->barrier(stream_);
    synchronize();
  };
  // MFT_BENCH_MARKS=1 (bench.py): rank 0 brackets the timed region on stdout, so the parent can
  // integrate the GPU's power over exactly these steps (energy per token)
  static const bool marks = std::getenv("MFT_BENCH_MARKS") && std::getenv("MFT_BENCH_MARKS")[0] == '1';
  const bool lead = !comm_ || comm_->rank() == 0;
  fence();
  if (marks && lead) {  // + this GPU's PCI address: the parent maps it to its sysfs hwmon node
    char bus[64] = "";
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) bus[0] = 0;
    std::printf("MFT_BENCH_T0 %s\n", bus);
    std::fflush(stdout);
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < steps; ++i) one(warmup + i);
  fence();
  double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (marks && lead) {
    std::printf("MFT_BENCH_T1\n");
    std::fflush(stdout);
  }
  float l = (float)loss.item();
  if (comm_) {  // slowest rank's clock; rank-mean loss
    float h2[2] = {(float)dt, l};
    Tensor d = from_host(h2, {2}, DType::F32);
    comm_->all_reduce_max(static_cast<float*>(d.data_ptr()), 1, stream_);
    comm_->all_reduce_avg(static_cast<float*>(d.data_ptr()) + 1, 1, stream_);
    const std::vector<float> back = d.to_vector_f32();
    dt = back[0];
    l = back[1];
  }
  if (final_loss) *final_loss = l;
  return dt;
}

void Trainer::sync_ema() {
  const std::vector<float> h = ema_dev_.to_vector_f32();  // {ema, initialised}
  float e[2] = {h[0] * h[1], h[1]};
  if (comm_) {  // every rank joins (rank-invariant): the mean over the initialised ranks
    Tensor d = from_host(e, {2}, DType::F32);
    comm_->all_reduce_sum(static_cast<float*>(d.data_ptr()), 2, current_stream());
    const std::vector<float> b = d.to_vector_f32();
    e[0] = b[0], e[1] = b[1];
  }
  if (e[1] > 0.f) {
    ema_loss = e[0] / e[1];
    ema_init = true;
  }
}

void Trainer::train(const std::function<void(int64_t)>& save_fn) {
  if (total_steps_ <= 0) {
    std::printf("[Train] nothing to do (steps=0)\n");
    return;
  }
  const int B = cfg_.batch, S = cfg_.seq, A = (int)ids_.size();
  std::vector<std::vector<int64_t>> hid(A, std::vector<int64_t>((size_t)B * S)),
      htg(A, std::vector<int64_t>((size_t)B * S));
  std::vector<float> mk((size_t)B * S);
  std::ofstream metrics;
  if (!cfg_.metrics_out.empty()) {
    metrics.open(cfg_.metrics_out, std::ios::app);
    metrics.precision(9);
  }
  auto t_last = std::chrono::steady_clock::now();
  pm_t0_ = t_last;
  int64_t tok_since = 0, steps_since = 0;
  const bool prof = cfg_.profile_to > 0 && cfg_.profile_to >= cfg_.profile_from;
  bool prof_open = false;  // (a resumed run may start inside the window: open it at its first step)
  hipEvent_t pe0 = nullptr, pe1 = nullptr;
  if (prof) {
    profiler_pause();
    HIP_OK(hipEventCreate(&pe0));
    HIP_OK(hipEventCreate(&pe1));
  }
  for (int64_t it = global_step; it < total_steps_; ++it) {  // global_step > 0 after load_state
    if (cfg_.fault_step > 0 && it + 1 == cfg_.fault_step && (comm_ ? comm_->rank() : 0) == cfg_.fault_rank)
      throw std::runtime_error("injected fault at step " + std::to_string(it + 1) + " on rank " +
                               std::to_string(cfg_.fault_rank) + " (--inject_fault)");
    const float lr = cfg_.lr_fn ? cfg_.lr_fn(it, total_steps_) : gpt2_cli_lr(it, cfg_.lr, cfg_.warmup, total_steps_);
    opt_.set_lr(lr);
    std::vector<std::pair<const int64_t*, const int64_t*>> micro;
    int64_t tokens = 0;
    for (int a = 0; a < A; ++a) {
      train_.next_batch(B, true, hid[a].data(), htg[a].data(), mk.data(), nullptr);
      for (float m : mk) tokens += m > 0.f;
      micro.push_back({hid[a].data(), htg[a].data()});
      ++micro_steps_;
      if (cfg_.micro_hook) cfg_.micro_hook(micro_steps_, hid[a].data(), B, S);
    }
    const bool in_prof = prof && it + 1 >= cfg_.profile_from && it + 1 <= cfg_.profile_to;
    if (in_prof && !prof_open) {
      synchronize();
      profiler_resume();
      roctxRangePushA("mft.profile");
      prof_open = true;
    }
    if (in_prof) HIP_OK(hipEventRecord(pe0, stream_));
    Tensor loss = step(micro);
    if (in_prof) {
      HIP_OK(hipEventRecord(pe1, stream_));
      HIP_OK(hipEventSynchronize(pe1));
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, pe0, pe1));
      std::printf("[profile] step %lld: %.3f ms device\n", (long long)(it + 1), ms);
      if (it + 1 == cfg_.profile_to || it + 1 == total_steps_) {
        roctxRangePop();
        profiler_pause();
        prof_open = false;
      }
    }
    ++global_step;
    total_tokens += tokens;
    tok_since += tokens;
    ++steps_since;
    // training-loss EMA every step, on device (a non-finite loss is skipped); read at log / save
    k::ema_update(ema_dev_.data<float>(), loss.data<float>(), std::max(0.f, std::min(0.9999f, cfg_.ema_beta)), stream_);
    const bool log_now = cfg_.log_interval > 0 && (global_step % cfg_.log_interval == 0 || it + 1 == total_steps_);
    if (log_now) {
      if (comm_) {  // mean over ranks (a copy: the graph keeps accumulating into loss_acc_)
        Tensor lc = loss.clone();
        comm_->all_reduce_avg(static_cast<float*>(lc.data_ptr()), 1, current_stream());
        loss = lc;
      }
      const float l = (float)loss.item();  // syncs the stream
      sync_ema();
      const auto now = std::chrono::steady_clock::now();
      const double dt = std::chrono::duration<double>(now - t_last).count();
      t_last = now;
      step_ms = dt * 1e3 / std::max<int64_t>(1, steps_since);
      const double tps = tok_since / std::max(dt, 1e-9);
      tok_since = 0;
      steps_since = 0;
      losses.push_back(l);
      const float gn = opt_.grad_norm();
      const int nr = comm_ ? comm_->world() : 1;
      const double ppl = std::exp(std::min<double>(l, 50.0));
      if (lead()) {
        if (cfg_.log_style == "gemma") {
          // reference optim/gemma_trainer.cpp:193-197
          std::printf("[Step %lld] Loss=%.4f PPL=%.2f LR=%.6g GradNorm=%.4f EMA=%.4f tok/s=%.0f step_ms=%.2f\n",
                      (long long)global_step, l, ppl, lr, gn, ema_loss, tps * nr, step_ms);
        } else {
          // reference gpt2_lora_finetune/main.cpp:627-635 (+ throughput fields at the end)
          std::printf("[Train] epoch %lld/%d | step %lld/%lld (global %lld/%lld) | lr %.6f | loss %.4f | ppl %.2f | "
                      "grad_norm %.3f | tokens %lld | tok/s %.0f | step_ms %.2f\n",
                      (long long)(it / steps_per_epoch_ + 1), cfg_.epochs, (long long)(it % steps_per_epoch_ + 1),
                      (long long)steps_per_epoch_, (long long)global_step, (long long)total_steps_, lr, l, ppl, gn,
                      (long long)(tokens * nr), tps * nr, step_ms);
        }
      }
      std::fflush(stdout);
      if (metrics.is_open() && lead()) {
        metrics << "{\"step\": " << global_step << ", \"loss\": " << l << ", \"lr\": " << lr << ", \"grad_norm\": " << gn
                << ", \"ema_loss\": " << ema_loss << ", \"tokens_per_s\": " << tps * nr << ", \"step_ms\": " << step_ms
                << "}\n";
        metrics.flush();
      }
    }
    if (cfg_.eval_interval > 0 && global_step % cfg_.eval_interval == 0 && valid_) {
      auto ev = evaluate(cfg_.eval_batches, cfg_.eval_batch_size);
      sync_ema();
      const long long epoch = it / steps_per_epoch_ + 1;
      if (lead())  // reference gpt2_lora_finetune/main.cpp:645-664
        std::printf("\n[Eval] epoch %lld | step %lld | valid_ppl %.2f | ema_loss %.4f | total_tokens %lld | valid_nll %.4f\n\n",
                    epoch, (long long)global_step, ev.second, ema_loss, (long long)(total_tokens * (comm_ ? comm_->world() : 1)),
                    ev.first);
      if (!cfg_.eval_out.empty() && lead()) {
        std::ofstream eo(cfg_.eval_out, std::ios::app);
        eo.precision(9);
        eo << "{\"step\":" << global_step << ",\"epoch\":" << epoch << ",\"valid_ppl\":" << ev.second
           << ",\"ema_loss\":" << ema_loss << ",\"total_tokens\":" << total_tokens * (comm_ ? comm_->world() : 1)
           << ",\"valid_nll\":" << ev.first << "}\n";
      }
    }
    if (cfg_.save_every > 0 && global_step % cfg_.save_every == 0) {
      if (!cfg_.state_dir.empty()) save_state(cfg_.state_dir);  // every rank (per-rank data state; gathers)
      else if (save_fn) gather_for_export();                    // collective: whole masters on every rank
      if (save_fn && lead()) save_fn(global_step);
      if (comm_) comm_->heartbeat();
    }
    if (pm_) {
      // the energy scheduler sleeps between whole steps: drain the GPU queue first (an async host
      // would otherwise sleep while the GPU keeps running), so the busy time it sees is the step's
      synchronize();
      const auto t_busy = std::chrono::steady_clock::now();
      pm_->note_step_ms((float)std::chrono::duration<double, std::milli>(t_busy - pm_t0_).count());
      const int ms = pm_->suggest_sleep_ms(global_step);
      if (ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(ms));
      pm_t0_ = std::chrono::steady_clock::now();
    }
  }
  synchronize();
  if (pe0) (void)hipEventDestroy(pe0);
  if (pe1) (void)hipEventDestroy(pe1);
  // the final exports (LoRA / HF writers read the fp32 masters) need every rank's ZeRO-1/2 chunks
  if (!cfg_.state_dir.empty()) save_state(cfg_.state_dir);
  else gather_for_export();
}

void Trainer::gather_for_export() {
  if (!dp_) return;
  flush_optimizer();
  synchronize();
  dp_->gather_master();  // ZeRO-1/2: all-gather the master chunks (a no-op otherwise); collective
  synchronize();
  if (comm_) comm_->heartbeat();
}

// ------------------------------------------------------------------ full-state checkpoint
void Trainer::save_state(const std::string& dir) {
  TraceRange range("mft.save_state");
  Communicator::QuietScope quiet(comm_);
  // Written into <dir>.tmp, then swapped in by rank 0 (<dir> -> <dir>.old, <dir>.tmp -> <dir>), so a
  // crash mid-save never leaves a torn checkpoint: load_state falls back to <dir>.old.
  namespace fs = std::filesystem;
  synchronize();
  const int r = comm_ ? comm_->rank() : 0;
  flush_optimizer();
  if (dp_) dp_->gather_master();  // ZeRO: every rank's master chunks (collective)
  sync_ema();
  synchronize();
  const std::string tmp = dir + ".tmp", old = dir + ".old";
  if (r == 0) {
    fs::remove_all(tmp);
    fs::create_directories(tmp);
  }
  if (comm_) comm_->barrier(stream_);
  const bool per_rank = dp_ && dp_->params_sharded();  // ZeRO-3: every rank's own partitions
  if (r == 0 || per_rank) {
    const Tensor mh = flat_.master.to(Device::cpu());
    const size_t nb = (size_t)flat_.numel * sizeof(float);
    safetensors_save(tmp + (per_rank ? "/trainable.rank" + std::to_string(r) + ".safetensors" : "/trainable.safetensors"),
                     {{"master", "F32", {flat_.numel}, mh.data_ptr(), nb}},
                     {{"format", per_rank ? "mft-zero3-partition" : "mft-flat"}}, false, true);
  }
  // AdamW moments: the whole flat (replicated, rank 0 writes it) or each rank's ZeRO partition
  if (r == 0 || opt_.sharded()) {
    Tensor m1 = empty({opt_.m.numel()}, DType::F32, Device::cpu()), m2 = empty({opt_.v.numel()}, DType::F32, Device::cpu());
    m1.copy_(opt_.m.is_hip() ? opt_.m.to(Device::cpu()) : opt_.m);
    m2.copy_(opt_.v.is_hip() ? opt_.v.to(Device::cpu()) : opt_.v);
    const std::string fn = opt_.sharded() ? "/optimizer.rank" + std::to_string(r) + ".safetensors" : "/optimizer.safetensors";
    const size_t sb = (size_t)m1.numel() * sizeof(float);
    std::vector<TensorBlob> outs{{"m", "F32", {m1.numel()}, m1.data_ptr(), sb}, {"v", "F32", {m2.numel()}, m2.data_ptr(), sb}};
    Tensor m3;
    if (opt_.vmax.defined()) {  // AMSGrad running max
      m3 = opt_.vmax.to(Device::cpu());
      outs.push_back({"vmax", "F32", {m3.numel()}, m3.data_ptr(), (size_t)m3.numel() * sizeof(float)});
    }
    // opt_state_version 2: 'vmax' is the running max of the bias-corrected v / bc2 (reference
    // optim/adam.cpp:75-80); version 1 files (no key) held the running max of the raw v
    safetensors_save(tmp + fn, outs,
                     {{"format", opt_.sharded() ? "mft-zero-partition" : "mft-flat"}, {"opt_state_version", "2"}}, false,
                     true);
  }
  std::ofstream f(tmp + "/trainer_state.rank" + std::to_string(r) + ".json");
  f.precision(17);
  f << "{\"global_step\": " << global_step << ", \"opt_step\": " << opt_.applied_steps()
    << ", \"total_tokens\": " << total_tokens << ", \"ema_loss\": " << ema_loss
    << ", \"ema_init\": " << (ema_init ? 1 : 0) << ", \"total_steps\": " << total_steps_
    << ", \"numel\": " << flat_.numel << ", \"dropout_ctr\": " << (int64_t)model_.dropout_ctr.item()
    << ", \"data\": {\"epoch\": " << train_.epoch() << ", \"cursor\": " << train_.cursor() << ", \"rng\": "
    << json::escape(train_.rng_state()) << "}}\n";
  f.close();
  MFT_CHECK(!f.fail(), "save_state: cannot write ", tmp);
  if (comm_) comm_->barrier(stream_);
  if (r == 0) {
    fs::remove_all(old);
    if (fs::exists(dir)) fs::rename(dir, old);
    fs::rename(tmp, dir);
    fs::remove_all(old);
  }
  if (comm_) comm_->barrier(stream_);
}

bool Trainer::load_state(const std::string& dir0) {
  Communicator::QuietScope quiet(comm_);
  const int r = comm_ ? comm_->rank() : 0;
  // a crash between save_state's two renames leaves only <dir>.old
  const std::string dir = std::filesystem::exists(dir0) || !std::filesystem::exists(dir0 + ".old") ? dir0 : dir0 + ".old";
  std::string sp = dir + "/trainer_state.rank" + std::to_string(r) + ".json";
  if (!std::filesystem::exists(sp)) sp = dir + "/trainer_state.rank0.json";
  if (!std::filesystem::exists(sp)) return false;
  std::ifstream f(sp);
  const std::string txt((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  const json::Value st = json::parse(txt);
  MFT_CHECK(st["numel"].as_int() == flat_.numel, "load_state: ", dir, " holds ", st["numel"].as_int(),
            " trainable values, the model has ", flat_.numel);
  const bool per_rank = dp_ && dp_->params_sharded();
  SafeTensorsFile tw(dir + (per_rank ? "/trainable.rank" + std::to_string(r) + ".safetensors" : "/trainable.safetensors"));
  SafeTensorsFile to(dir + (opt_.sharded() ? "/optimizer.rank" + std::to_string(r) + ".safetensors" : "/optimizer.safetensors"));
  auto host_view = [&](SafeTensorsFile& sf, const char* k, int64_t n) {
    MFT_CHECK(sf.has(k) && sf.info(k).dtype == "F32" && sf.info(k).end - sf.info(k).begin == (uint64_t)n * 4,
              "load_state: bad tensor ", k, " in ", sf.path(), " (a different ZeRO stage / world size?)");
    return from_blob(const_cast<void*>(sf.data(k)), {n}, DType::F32, Device::cpu());
  };
  flat_.master.copy_(host_view(tw, "master", flat_.numel));
  opt_.load_state(host_view(to, "m", opt_.m.numel()), host_view(to, "v", opt_.v.numel()), st["opt_step"].as_int());
  if (dp_) dp_->optimizer_state_loaded();
  if (opt_.vmax.defined()) {
    const auto mv = to.metadata().find("opt_state_version");
    const bool vmax_v2 = mv != to.metadata().end() && std::atoi(mv->second.c_str()) >= 2;
    if (to.has("vmax") && vmax_v2) {
      opt_.load_vmax(host_view(to, "vmax", opt_.vmax.numel()));
    } else {  // a checkpoint written without AMSGrad, or by a build whose 'vmax' was the max of the raw v
      // (ADVICE r5): start the running max at the loaded v / bc2 (the first step then matches plain
      // Adam), never at zero beside restored moments
      if (to.has("vmax"))
        std::fprintf(stderr, "[warn] load_state: 'vmax' of an older optimizer-state version (raw-v max); rebuilt from v / bc2\n");
      else
        std::fprintf(stderr, "[warn] load_state: --amsgrad but the checkpoint has no 'vmax'; initialised from v / bc2\n");
      const int64_t steps = st["opt_step"].as_int(), n = opt_.vmax.numel();
      const double bc2 = 1.0 - std::pow((double)opt_.config().beta2, (double)std::max<int64_t>(steps, 1));
      Tensor vh = host_view(to, "v", n);
      std::vector<float> vm((size_t)n);
      const float* src = static_cast<const float*>(vh.data_ptr());
      for (int64_t i = 0; i < n; ++i) vm[(size_t)i] = (float)(src[i] / bc2);
      opt_.load_vmax(from_blob(vm.data(), {n}, DType::F32, Device::cpu()));
      synchronize();
    }
  }
  synchronize();  // the mmaps go away with the files
  flat_.refresh_shadow();
  global_step = st["global_step"].as_int();
  total_tokens = st["total_tokens"].as_int();
  ema_loss = st["ema_loss"].as_double();
  ema_init = st["ema_init"].as_int() != 0;
  {
    const float e[2] = {(float)ema_loss, ema_init ? 1.f : 0.f};
    ema_dev_.copy_(from_blob(const_cast<float*>(e), {2}, DType::F32, Device::cpu()));
  }
  model_.dropout_ctr.fill_((double)st["dropout_ctr"].as_int());
  const json::Value& d = st["data"];
  train_.restore(d["epoch"].as_int(), (size_t)d["cursor"].as_int(), d["rng"].as_string());
  synchronize();
  return true;
}

}  // namespace eng
}  // namespace mft
