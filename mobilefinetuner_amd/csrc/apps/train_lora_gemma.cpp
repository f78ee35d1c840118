// Native CLI `train_lora_gemma` on the libmft engine: LoRA fine-tuning of Gemma-3 (270M / 1B) with
// the C++ tensor / caching allocator / autograd tape and a hipGraph-captured step (no Python, no
// torch).
//
// Reference: operators/finetune_ops/optim/train_lora_gemma.cpp:352-975 (CliOptions, unknown flags
// reported and ignored, targets presets, GemmaLoRATrainer loop optim/gemma_trainer.cpp:18-233 with
// warmup = ceil(ratio * updates), 1-indexed, then linear / cosine to 0; LoRA saved as
// <output_dir>/gemma_lora.safetensors).  Flag names and defaults are the Python CLI's
// (cli/train_lora_gemma.py, which follows the reference); extras:
//   --model P --random_init --synthetic_data [--synthetic_tokens N] --resume_from F (initial
//   adapter) --no_graph --compat_l2_adam --metrics_out F --deterministic --interleaved_rope
//   --shard_enable --shard_budget_mb N: frozen layer weights streamed from pinned host memory
// The alignment-dump harness (--align_*) and the embedding dump stay in the Python CLI.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "apps/app_common.h"
#include "engine/allocator.h"
#include "engine/comm.h"
#include "engine/gemm.h"
#include "engine/gemma3.h"
#include "engine/optim.h"
#include "engine/trainer.h"
#include "runtime/dataset.h"
#include "runtime/tokenizer.h"

using namespace mft;
using namespace mft::eng;
using mft::apps::Args;
using mft::apps::file_exists;

namespace {

const char* kProg = "train_lora_gemma";

const std::set<std::string> kBool = {"random_init", "synthetic_data", "no_graph", "compat_l2_adam", "deterministic",
                                     "interleaved_rope", "pm_disable_batt", "pm_disable_temp", "pm_gpu_telemetry",
                                     "shard_enable", "bf16_grads", "no_overlap", "help"};
const std::set<std::string> kValued = {
    "model_dir", "data_dir", "pretokenized_path", "pretokenized_meta", "output_dir", "targets", "lora_targets",
    "epochs", "max_steps", "seq_len", "batch", "grad_accum", "lr", "learning_rate", "rank", "lora_r", "alpha",
    "lora_alpha", "lora_dropout", "warmup_ratio", "max_grad_norm", "weight_decay", "loss_reduction", "lr_schedule",
    "data_fraction", "log_interval", "eval_steps", "eval_batches", "save_every", "seed", "model", "synthetic_tokens",
    "resume_from", "state_dir", "inject_fault", "metrics_out", "eval_out", "pm_interval", "pm_batt_thresh", "pm_temp_thresh", "pm_fb_high",
    "pm_fb_low", "pm_ft_high", "pm_ft_low", "pm_manual_batt", "pm_manual_temp", "pm_schedule", "device",
    "shard_budget_mb", "shard_dir", "shard_fp16_disk", "bench_steps", "bench_warmup", "zero_stage", "offload", "bucket_mb"};

// first present of several alias flags
std::string pick(const Args& a, std::initializer_list<const char*> keys, const std::string& d) {
  for (const char* k : keys)
    if (a.kv.count(k)) return a.kv.at(k);
  return d;
}

std::string checkpoint_path(const std::string& stem, int64_t step) {
  const size_t dot = stem.rfind('.');
  return (dot == std::string::npos ? stem : stem.substr(0, dot)) + "_step" + std::to_string(step) + ".safetensors";
}

void usage() {
  std::printf(
      "%s -- native MI355X engine (libmft)\n"
      "  --model_dir D --data_dir D | --pretokenized_path F [--pretokenized_meta M] --output_dir D\n"
      "  --targets full|attn|light --lora_targets q,k,v,o,gate,up,down --epochs N --max_steps N --seq_len S\n"
      "  --batch B --grad_accum A --lr LR --rank R --alpha A --lora_dropout P --warmup_ratio R --max_grad_norm C\n"
      "  --weight_decay W --lr_schedule linear|cosine|constant --data_fraction F --log_interval N --eval_steps N\n"
      "  --eval_batches N --save_every N --seed S --pm_* (energy)\n"
      "  extras: --model P --random_init --synthetic_data --synthetic_tokens N --resume_from F --no_graph\n"
      "          --compat_l2_adam --metrics_out F --deterministic --interleaved_rope\n"
      "          --zero_stage 0|1|2 --offload host|none --bucket_mb N --bf16_grads --no_overlap\n"
      "          --state_dir D (full training state: written at --save_every and at the end, resumed if present)\n"
      "          --inject_fault STEP:RANK (failure test: that rank throws before that step)\n"
      "          --bench_steps K [--bench_warmup W] (bench.py: time K steps after W, print one MFT_BENCH line)\n",
      kProg);
}

int run(int argc, char** argv) {
  Args a = mft::apps::parse_args(argc, argv, kBool, kValued, /*lenient=*/true);
  if (a.b("help")) {
    usage();
    return 0;
  }
  if (!a.unknown.empty()) {
    std::printf("[%s] ignoring unknown arguments:", kProg);
    for (auto& u : a.unknown) std::printf(" %s", u.c_str());
    std::printf("\n");
  }
  if (a.get("loss_reduction", "mean") != "mean")
    throw std::runtime_error("--loss_reduction sum: the native engine trains on the mean token loss");
  if (a.b("deterministic")) set_deterministic(true);
  const DistConfig dcfg = mft::apps::dist_config_from(a);
  if (dcfg.zero_stage == 3)  // the adapters are the only trainable tensors: nothing for ZeRO-3 to partition
    throw std::runtime_error("--zero_stage 3 partitions full fine-tuning weights; LoRA uses stages 0-2");
  std::unique_ptr<Communicator> comm = mft::apps::comm_from(dcfg);
  if (!comm) HIP_OK(hipSetDevice(0));
  if (comm && comm->rank() != 0) std::setvbuf(stdout, nullptr, _IOFBF, 1 << 16);
  hipStream_t stream;
  HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  set_current_stream(stream);
  const bool lead = !comm || comm->rank() == 0;
  const uint64_t seed = (uint64_t)a.l("seed", 42);

  std::printf("\n========== Gemma-3 LoRA Finetune (MI355X native engine) ==========\n");
  if (comm)
    std::printf("  data parallel: rank %d of %d (%s, device %d)\n", comm->rank(), comm->world(), comm->backend(),
                comm->device());
  const std::string mdir = a.get("model_dir");
  const bool random_init = a.b("random_init") || mdir.empty();
  Gemma3Config cfg = (!mdir.empty() && file_exists(mdir + "/config.json")) ? Gemma3Config::from_json(mdir + "/config.json")
                                                                         : Gemma3Config::preset(a.get("model", "gemma3-270m"));
  std::printf("  Gemma-3 config: layers=%d hidden=%d heads=%d/%d head_dim=%d vocab=%d\n", cfg.n_layer, cfg.hidden,
              cfg.n_head, cfg.n_kv, cfg.head_dim, cfg.vocab_size);
  auto model = std::make_unique<Gemma3>(cfg);
  model->interleaved_rope = a.b("interleaved_rope");
  if (random_init) {
    model->init_random(1234);
    std::printf("  random-initialised weights\n");
  } else {
    model->load_hf(mdir);
    std::printf("  Gemma weights loaded from %s\n", mdir.c_str());
  }

  const std::string resume = a.get("resume_from");
  if (!resume.empty()) {
    model->load_lora(resume);
    std::printf("  adapter loaded from %s (rank=%d)\n", resume.c_str(), model->lora_spec().rank);
  } else {
    GemmaLoraSpec spec;
    spec.rank = std::stoi(pick(a, {"rank", "lora_r"}, "8"));
    spec.alpha = std::stof(pick(a, {"alpha", "lora_alpha"}, "32"));
    spec.dropout = a.f("lora_dropout", 0.1f);
    spec.targets = GemmaLoraSpec::parse_targets(a.kv.count("lora_targets") ? a.get("lora_targets") : a.get("targets", "full"));
    spec.seed = 42;
    model->inject_lora(spec);
    std::string t;
    for (auto& x : spec.targets) t += (t.empty() ? "" : ",") + x;
    std::printf("  LoRA rank=%d alpha=%g dropout=%g targets=%s\n", spec.rank, spec.alpha, spec.dropout, t.c_str());
  }
  if (a.b("shard_enable")) {
    // --shard_budget_mb: device bytes for the streamed layer weights (the reference CLI raised its
    // budget to the largest parameter, train_lora_gemma.cpp:431-441; here the tied embedding stays
    // resident and every slot holds one whole layer)
    const size_t budget = (size_t)a.l("shard_budget_mb", 512) << 20;
    model->enable_weight_streaming(budget);
    const WeightStreamer* ws = model->streamer();
    std::printf("  weight streaming ON: %d device slots (%.1f MB) for %.1f MB of frozen layer weights in pinned host memory\n",
                ws->slots(), ws->device_bytes() / 1048576.0, ws->host_bytes() / 1048576.0);
  }
  mft::apps::DistSetup ds;
  ds.make_flat(model->trainable(), comm.get(), dcfg);
  FlatParams& flat = *ds.flat;
  std::printf("  trainable params: %lld (padded)  |  total: %zu\n", (long long)flat.numel, model->num_parameters());

  DataConfig dc;
  dc.seq_len = a.i("seq_len", 256);
  dc.eos_id = cfg.eos_id;
  dc.pad_id = cfg.pad_id;
  dc.seed = seed;
  dc.data_fraction = a.f("data_fraction", 1.f);
  if (comm) {
    dc.rank = comm->rank();
    dc.world = comm->world();
  }
  DataConfig vc = dc;
  vc.drop_last = false;
  vc.shuffle = false;
  TokenDataset train(dc), valid(vc);
  const bool have_valid = mft::apps::load_token_splits(a, dc, cfg.vocab_size, train, valid, [&]() -> mft::apps::Encoder {
    std::shared_ptr<SentencePieceBPE> tok = SentencePieceBPE::from_tokenizer_json(mdir + "/tokenizer.json");
    return [tok](const std::string& s) { return tok->encode(s, false); };
  });
  std::printf("  Train %zu seqs, valid %zu seqs (seq_len=%d)\n", train.num_sequences(),
              have_valid ? valid.num_sequences() : (size_t)0, dc.seq_len);

  AdamWConfig oc;
  oc.lr = std::stof(pick(a, {"lr", "learning_rate"}, "2e-4"));
  oc.weight_decay = a.f("weight_decay", 0.f);
  oc.max_grad_norm = a.f("max_grad_norm", 1.f);
  oc.l2_coupled = a.b("compat_l2_adam");
  AdamW opt(flat, oc);
  ds.make_dp(comm.get(), opt, dcfg);
  TrainConfig tc;
  tc.epochs = a.i("epochs", 1);
  tc.steps = a.l("max_steps", -1);
  if (tc.steps > 0) tc.epochs = 0;  // --max_steps caps the run (reference: max_steps > 0 wins)
  tc.batch = a.i("batch", 4);
  tc.accum = a.i("grad_accum", 1);
  tc.seq = dc.seq_len;
  tc.lr = oc.lr;
  tc.log_interval = a.i("log_interval", 1);
  tc.eval_interval = a.i("eval_steps", 0);
  tc.eval_batches = a.i("eval_batches", 50);
  tc.eval_batch_size = tc.batch;
  tc.save_every = a.i("save_every", 0);
  tc.use_graph = !a.b("no_graph");
  tc.metrics_out = a.get("metrics_out");
  tc.state_dir = a.get("state_dir");
  if (!a.get("inject_fault").empty()) {  // step:rank
    const std::string f = a.get("inject_fault");
    const size_t c = f.find(':');
    tc.fault_step = std::stoll(f.substr(0, c));
    tc.fault_rank = c == std::string::npos ? 0 : std::stoi(f.substr(c + 1));
  }
  tc.eval_out = a.get("eval_out");
  tc.log_style = "gemma";
  const std::string sched = a.get("lr_schedule", "linear");
  const float ratio = a.f("warmup_ratio", 0.03f), base = oc.lr;
  if (sched == "constant") tc.lr_fn = [base](int64_t, int64_t) { return base; };
  else tc.lr_fn = [base, ratio, sched](int64_t it, int64_t total) { return gemma_lr(it + 1, base, ratio, total, sched == "cosine"); };
  std::unique_ptr<PowerMonitor> pm = mft::apps::power_monitor_from(a);
  Trainer trainer(*model, flat, opt, train, have_valid ? &valid : nullptr, tc, pm.get(), comm.get(), ds.reducer());
  if (!tc.state_dir.empty() && trainer.load_state(tc.state_dir))
    std::printf("  resumed full training state from %s at step %lld / %lld\n", tc.state_dir.c_str(),
                (long long)trainer.global_step, (long long)trainer.total_steps());
  if (a.i("bench_steps", 0) > 0) {
    mft::apps::bench_report(trainer, flat, a, comm ? comm->world() : 1, lead, a.get("model", "gemma3-270m"),
                            model->num_parameters(), tc.batch, tc.seq, tc.accum);
    return 0;
  }
  const std::string out_dir = a.get("output_dir", "runs/gemma_lora");
  const std::string out = out_dir + "/gemma_lora.safetensors";
  if (lead) {
    const std::string mk = "mkdir -p '" + out_dir + "'";
    if (std::system(mk.c_str()) != 0) throw std::runtime_error("cannot create " + out_dir);
  }
  auto save = [&](int64_t step) {
    const std::string p = checkpoint_path(out, step);
    model->save_lora(p);
    std::printf("\n[Checkpoint] Saved %s\n\n", p.c_str());
  };
  std::printf("[Plan] steps/epoch=%lld total=%lld (micro=%d x accum=%d, %s)\n", (long long)trainer.steps_per_epoch(),
              (long long)trainer.total_steps(), tc.batch, tc.accum, tc.use_graph ? "hipGraph-captured step" : "eager");
  const auto t0 = std::chrono::steady_clock::now();
  trainer.train(save);
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (lead) {
    model->save_lora(out);
    std::printf("  Saved LoRA to %s\n", out.c_str());
  }
  if (have_valid) {
    auto ev = trainer.evaluate(tc.eval_batches, tc.eval_batch_size);
    if (lead) std::printf("[Eval] valid_loss=%.4f valid_ppl=%.2f\n", ev.first, ev.second);
  }
  const AllocStats st = CachingAllocator::get(0).stats();
  std::printf("\nTraining complete: %lld steps, %lld tokens, %.2f s (%.0f tokens/s), final EMA loss %.4f, "
              "HBM peak allocated %.2f GB\n",
              (long long)trainer.global_step, (long long)trainer.total_tokens, secs, trainer.total_tokens / secs,
              trainer.ema_loss, st.peak_allocated / 1e9);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  try {
    return run(argc, argv);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s: error: %s\n", kProg, e.what());
    return 1;
  }
}
