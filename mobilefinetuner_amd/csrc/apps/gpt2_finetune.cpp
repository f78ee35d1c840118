// Native CLIs `gpt2_lora_finetune` and `gpt2_full_finetune` on the libmft engine (C++ tensor,
// caching allocator, autograd tape, hipGraph-captured step; no Python, no torch).
//
// Reference: gpt2_lora_finetune/main.cpp:32-710 (CmdArgs :32-78, parse :114-171, LoRA on the fused
// c_attn + attn.c_proj :382-399, resume :361-381, train loop :561-684, periodic `<stem>_stepN`
// checkpoints :180-187) and gpt2_full_finetune/main.cpp:25-583 (all params trainable, full
// HF-keyed safetensors output).  Flag names and defaults are the reference's; extras:
//   --model P --random_init         random-init weights of preset P (no checkpoint needed)
//   --synthetic_data [--synthetic_tokens N]   counter-hash token stream (no dataset needed)
//   --pretokenized_path F [--pretokenized_meta M]   int32 token stream + meta.json
//   --lora_targets AttnQKV,AttnProj[,MlpFcIn,MlpFcOut] --split_qkv
//   --no_graph --compat_l2_adam --amsgrad --metrics_out F --deterministic
//   + the common block of apps/app_common.h: --dtype bf16|fp32 --attn_impl flash|naive --profile_steps a:b
//     --compat_grad_overwrite --compat_reference
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "apps/app_common.h"
#include "engine/allocator.h"
#include "engine/comm.h"
#include "engine/gemm.h"
#include "engine/gpt2.h"
#include "engine/optim.h"
#include "engine/trainer.h"
#include "runtime/dataset.h"
#include "runtime/power_monitor.h"
#include "runtime/tokenizer.h"

using namespace mft;
using namespace mft::eng;
using mft::apps::Args;
using mft::apps::file_exists;
using mft::apps::parse_args;
using mft::apps::split_file;

#ifdef MFT_FULL_FT
static const char* kProg = "gpt2_full_finetune";
#else
static const char* kProg = "gpt2_lora_finetune";
#endif

namespace {

const std::set<std::string> kBool = {"split_qkv", "random_init", "synthetic_data", "no_graph", "compat_l2_adam", "amsgrad",
                                     "activation_checkpointing", "shard_enable", "pm_disable_batt", "pm_disable_temp", "pm_gpu_telemetry",
                                     "deterministic", "bf16_grads", "no_overlap", "help"};
const std::set<std::string> kValued = {
    "data_dir", "pretrained_dir", "lora_out", "resume_from", "state_dir", "inject_fault", "eval_out", "output_path", "epochs", "steps",
    "batch_size", "grad_accum_steps", "seq_len", "rank", "alpha", "lr", "weight_decay", "warmup_steps",
    "clip_grad_norm", "lora_dropout", "data_fraction", "log_interval", "eval_interval", "eval_batches",
    "eval_batch_size", "save_every", "ema_beta", "seed", "pm_interval", "pm_batt_thresh", "pm_temp_thresh",
    "pm_fb_high", "pm_fb_low", "pm_ft_high", "pm_ft_low", "pm_manual_batt", "pm_manual_temp", "pm_schedule", "pm_power_cap",
    "shard_dir", "shard_budget_mb", "shard_fp16_disk", "model", "synthetic_tokens", "pretokenized_path",
    "pretokenized_meta", "lora_targets", "metrics_out", "device", "bench_steps", "bench_warmup", "zero_stage", "offload", "offload_moments", "offload_mode", "offload_dir", "bucket_mb", "dump_grads"};

Args parse(int argc, char** argv) { return parse_args(argc, argv, kBool, kValued); }

std::string checkpoint_path(const std::string& stem, int64_t step) {
  const size_t dot = stem.rfind('.');
  const size_t slash = stem.rfind('/');
  std::string root = stem, ext = ".safetensors";
  if (dot != std::string::npos && (slash == std::string::npos || dot > slash)) {
    root = stem.substr(0, dot);
    ext = stem.substr(dot);
  }
  return root + "_step" + std::to_string(step) + ext;
}

std::vector<std::string> split_csv(const std::string& s) {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, ','))
    if (!item.empty()) out.push_back(item);
  return out;
}

std::string norm_target(std::string t) {
  std::string l = t;
  for (auto& c : l) c = (char)std::tolower(c);
  if (l == "attnqkv" || l == "attn_qkv" || l == "c_attn" || l == "qkv") return "AttnQKV";
  if (l == "attnproj" || l == "attn_proj" || l == "proj") return "AttnProj";
  if (l == "mlpfcin" || l == "mlp_fc_in" || l == "c_fc" || l == "fc_in") return "MlpFcIn";
  if (l == "mlpfcout" || l == "mlp_fc_out" || l == "fc_out") return "MlpFcOut";
  throw std::runtime_error("unknown GPT-2 LoRA target '" + t + "'");
}

void usage() {
  std::printf(
      "%s -- native MI355X engine (libmft)\n"
      "  --data_dir D --pretrained_dir P [--lora_out F] [--resume_from F] [--eval_out F] [--output_path F]\n"
      "  --epochs N --steps N --batch_size B --grad_accum_steps A --seq_len S --rank R --alpha A --lr LR\n"
      "  --weight_decay W --warmup_steps W --clip_grad_norm C --lora_dropout P --data_fraction F --log_interval N\n"
      "  --eval_interval N --eval_batches N --eval_batch_size B --save_every N --ema_beta B --seed S\n"
      "  --pm_interval --pm_batt_thresh --pm_temp_thresh --pm_fb_high --pm_fb_low --pm_ft_high --pm_ft_low\n"
      "  --pm_manual_batt --pm_manual_temp --pm_disable_batt --pm_disable_temp --pm_schedule --pm_gpu_telemetry --pm_power_cap W\n"
      "  extras: --model P --random_init --synthetic_data --synthetic_tokens N --pretokenized_path F\n"
      "          --pretokenized_meta F --lora_targets T --split_qkv --no_graph --compat_l2_adam --amsgrad --metrics_out F\n"
      "          --state_dir D (full training state: written at --save_every and at the end, resumed if present)\n"
      "          --inject_fault STEP:RANK (failure test: that rank throws before that step)\n"
      "          --deterministic\n"
      "  multi-GPU / memory: --zero_stage 0|1|2|3 --offload host|disk|none [--offload_dir D] --offload_moments bf16|fp32\n"
      "          --offload_mode stream|zerocopy --bucket_mb N --bf16_grads --no_overlap\n"
      "  common: --dtype bf16|fp32 --attn_impl flash|naive --profile_steps A:B --compat_grad_overwrite --compat_reference\n",
      kProg);
}

int run(int argc, char** argv) {
  Args a = parse(argc, argv);
  if (a.b("help")) {
    usage();
    return 0;
  }
#ifdef MFT_FULL_FT
  const bool full = true;
#else
  const bool full = false;
#endif
  if (a.b("shard_enable") && full)
    throw std::runtime_error("--shard_enable streams FROZEN weights; in full fine-tuning every weight trains "
                             "(use --zero_stage 3 [--offload host]: weights partitioned over the ranks, moments in host DRAM)");
  if (a.b("deterministic")) set_deterministic(true);
  // data parallelism: one process per GPU (RANK / WORLD_SIZE / LOCAL_RANK, e.g. under
  // `python -m mobilefinetuner_amd.launch --nproc N`), native RCCL communicator; the communicator
  // selects the device LOCAL_RANK.  MFT_DP_FORCE_COMM=1 builds a 1-rank one on a single GPU.
  const DistConfig dcfg = mft::apps::dist_config_from(a);
  std::unique_ptr<Communicator> comm = mft::apps::comm_from(dcfg);
  if (!comm) HIP_OK(hipSetDevice(0));
  if (comm && comm->rank() != 0) std::setvbuf(stdout, nullptr, _IOFBF, 1 << 16);  // rank 0 reports
  // one non-blocking stream for everything (graph capture target)
  hipStream_t stream;
  HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  set_current_stream(stream);
  mft::apps::install_crash_report();  // again: the HIP runtime's initialisation may replace handlers

  mft::apps::apply_dtype_flag(a);
  const int seq_len = a.i("seq_len", 128);
  const uint64_t seed = (uint64_t)a.l("seed", 42);
  std::printf("\n========== %s (MI355X native engine) ==========\n", kProg);
  if (comm)
    std::printf("  data parallel: rank %d of %d (%s, device %d)\n", comm->rank(), comm->world(), comm->backend(),
                comm->device());

  std::printf("\n[1/6] Loading model...\n");
  const std::string pdir = a.get("pretrained_dir");
  GPT2Config cfg;
  const bool random_init = a.b("random_init") || pdir.empty();
  if (!random_init && file_exists(pdir + "/config.json")) cfg = GPT2Config::from_json(pdir + "/config.json");
  else cfg = GPT2Config::preset(a.get("model", "gpt2"));
  auto model = std::make_unique<GPT2>(cfg);
  model->grad_checkpoint = a.b("activation_checkpointing");  // recompute blocks in the backward
  mft::apps::apply_model_flags(a, *model);
  if (random_init) {
    model->init_random(1234);
    std::printf("  random-init %s (%d layers, C=%d, H=%d)\n", a.get("model", "gpt2").c_str(), cfg.n_layer,
                cfg.n_embd, cfg.n_head);
  } else {
    model->load_hf(pdir);
    std::printf("  loaded %s/model.safetensors\n", pdir.c_str());
  }
  int seq = seq_len;
  if (seq > cfg.n_positions) {
    std::printf("  seq_len(%d) exceeds n_positions(%d), clamped\n", seq, cfg.n_positions);
    seq = cfg.n_positions;
  }

  std::printf("\n[2/6] %s...\n", full ? "Full fine-tuning: every parameter trainable" : "LoRA adapters");
  const std::string resume = a.get("resume_from");
  if (full) {
    model->set_full_finetune();
  } else if (!resume.empty() && file_exists(resume)) {
    model->load_lora(resume);
    std::printf("  resumed adapter from %s (rank=%d)\n", resume.c_str(), model->lora_spec().rank);
  } else {
    LoraSpec spec;
    spec.rank = a.i("rank", 8);
    spec.alpha = a.f("alpha", 16.f);
    spec.dropout = a.f("lora_dropout", 0.f);
    spec.split_qkv = a.b("split_qkv");
    spec.targets.clear();
    for (auto& t : split_csv(a.get("lora_targets", "AttnQKV,AttnProj"))) spec.targets.push_back(norm_target(t));
    model->inject_lora(spec);
    std::printf("  injected adapters (rank=%d, alpha=%g, targets=%s)\n", spec.rank, spec.alpha,
                a.get("lora_targets", "AttnQKV,AttnProj").c_str());
  }
  if (a.b("shard_enable")) {
    // reference ParameterSharder flags: --shard_budget_mb (device bytes for streamed weights);
    // --shard_dir D [--shard_fp16_disk 0|1]: block files on disk (fp16 by default) instead of
    // resident pinned host copies
    const size_t budget = (size_t)a.l("shard_budget_mb", 512) << 20;
    model->enable_weight_streaming(budget, mft::apps::disk_tier_from(a));
    mft::apps::print_streaming(model->streamer(), "block");
  }
  mft::apps::DistSetup ds;
  if (dcfg.zero_stage == 3) {  // parameters partitioned over the ranks, gathered per block
    if (!full) throw std::runtime_error("--zero_stage 3 partitions full fine-tuning weights (gpt2_full_finetune)");
    std::vector<eng::NamedParams> units;
    eng::NamedParams rep;
    model->zero3_layout(units, rep);
    ds.make_zero3(units, rep, *comm);
    model->set_block_provider(ds.z3.get());
  } else {
    ds.make_flat(model->trainable(), comm.get(), dcfg);
  }
  FlatParams& flat = *ds.flat;
  std::printf("  trainable params: %lld (padded)  |  total: %zu\n", (long long)flat.numel, model->num_parameters());

  std::printf("\n[3/6] Loading dataset...\n");
  DataConfig dc;
  dc.seq_len = seq;
  if (comm) {  // this rank's shard of every epoch's shuffled order
    dc.rank = comm->rank();
    dc.world = comm->world();
  }
  dc.eos_id = 50256;
  dc.seed = seed;
  dc.data_fraction = a.f("data_fraction", 1.f);
  DataConfig vc = dc;
  vc.drop_last = false;
  vc.shuffle = false;
  TokenDataset train(dc), valid(vc);
  const bool have_valid = mft::apps::load_token_splits(a, dc, cfg.vocab_size, train, valid, [&]() -> mft::apps::Encoder {
    std::shared_ptr<ByteLevelBPE> tok = ByteLevelBPE::from_files(pdir + "/vocab.json", pdir + "/merges.txt");
    return [tok](const std::string& s) { return tok->encode(s); };
  });
  std::printf("  train: %zu sequences | valid: %zu sequences\n", train.num_sequences(),
              have_valid ? valid.num_sequences() : (size_t)0);

  if (!a.get("dump_grads").empty()) {  // parity tests: one fwd+bwd, gradients in the checkpoint layout
    MFT_CHECK(!comm && !ds.z3, "--dump_grads runs on one process without ZeRO-3");
    const float lv = mft::apps::grads_into_masters(*model, flat, train, a.i("batch_size", 1), seq);
    if (full) model->save_hf(a.get("dump_grads"));
    else model->save_lora(a.get("dump_grads"));
    std::printf("MFT_DUMP loss=%.8f path=%s\n", lv, a.get("dump_grads").c_str());
    return 0;
  }
  AdamWConfig oc;
  oc.lr = a.f("lr", full ? 5e-5f : 1e-4f);
  oc.weight_decay = a.f("weight_decay", full ? 0.01f : 0.f);
  oc.max_grad_norm = a.f("clip_grad_norm", 1.f);
  oc.l2_coupled = a.b("compat_l2_adam") || a.b("compat_reference");
  oc.amsgrad = a.b("amsgrad");
  AdamW opt(flat, oc);
  ds.make_dp(comm.get(), opt, dcfg);
  TrainConfig tc;
  tc.epochs = a.i("epochs", 0);
  tc.steps = a.l("steps", 0);
  tc.batch = a.i("batch_size", 1);
  tc.accum = a.i("grad_accum_steps", 1);
  tc.seq = seq;
  tc.lr = oc.lr;
  tc.warmup = a.i("warmup_steps", 0);
  tc.log_interval = a.i("log_interval", 1);
  tc.eval_interval = a.i("eval_interval", 0);
  tc.eval_batches = a.i("eval_batches", 50);
  tc.eval_batch_size = a.i("eval_batch_size", 2);
  tc.save_every = a.i("save_every", 0);
  tc.ema_beta = a.f("ema_beta", 0.9f);
  tc.use_graph = !a.b("no_graph");
  tc.eval_out = a.get("eval_out");
  tc.metrics_out = a.get("metrics_out");
  tc.state_dir = a.get("state_dir");
  mft::apps::apply_train_flags(a, tc);
  if (!a.get("inject_fault").empty()) {  // step:rank
    const std::string f = a.get("inject_fault");
    const size_t c = f.find(':');
    tc.fault_step = std::stoll(f.substr(0, c));
    tc.fault_rank = c == std::string::npos ? 0 : std::stoi(f.substr(c + 1));
  }
  std::unique_ptr<PowerMonitor> pm = mft::apps::power_monitor_from(a);
  Trainer trainer(*model, flat, opt, train, have_valid ? &valid : nullptr, tc, pm.get(), comm.get(), ds.reducer());
  if (!tc.state_dir.empty() && trainer.load_state(tc.state_dir))
    std::printf("  resumed full training state from %s at step %lld / %lld\n", tc.state_dir.c_str(),
                (long long)trainer.global_step, (long long)trainer.total_steps());
  if (a.i("bench_steps", 0) > 0) {
    mft::apps::bench_report(trainer, flat, a, comm ? comm->world() : 1, !comm || comm->rank() == 0, a.get("model", "gpt2"),
                            model->num_parameters(), tc.batch, tc.seq, tc.accum);
    return 0;
  }
  const std::string lora_out = a.get("lora_out"), out_path = a.get("output_path");
  auto save = [&](int64_t step) {
    if (!full && !lora_out.empty()) {
      const std::string p = checkpoint_path(lora_out, step);
      model->save_lora(p);
      std::printf("\n[Checkpoint] Saved %s\n\n", p.c_str());
    }
  };
  std::printf("\n[Training plan]\n  epochs         : %d\n  steps_per_epoch: %lld\n  total_steps    : %lld\n"
              "  effective_batch: %d (micro=%d x accum=%d)\n",
              tc.epochs, (long long)trainer.steps_per_epoch(), (long long)trainer.total_steps(), tc.batch * tc.accum,
              tc.batch, tc.accum);
  std::printf("\n[4/6] Optimizer: fused AdamW (%s)\n", oc.l2_coupled ? "coupled L2, reference" : "decoupled");
  std::printf("\n[5/6] Starting training (%s)...\n========================================\n",
              trainer.uses_graph() ? "hipGraph-captured step" : "eager");
  const auto t0 = std::chrono::steady_clock::now();
  trainer.train(save);
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const bool lead = !comm || comm->rank() == 0;
  std::printf("\n[6/6] Saving...\n");
  if (!full && !lora_out.empty() && lead) {
    model->save_lora(lora_out);
    std::printf("  LoRA saved to: %s\n", lora_out.c_str());
  }
  if (full && !out_path.empty() && ds.z3) ds.z3->materialize();  // collective: whole tensors again
  if (full && !out_path.empty() && lead) {
    model->save_hf(out_path);
    std::printf("  model saved to: %s\n", out_path.c_str());
  }
  const AllocStats st = CachingAllocator::get(Device::current_hip_device()).stats();
  std::printf("\n========================================\nTraining complete!\n  Total steps: %lld\n"
              "  Total tokens: %lld\n  Wall time: %.2f s (%.0f tokens/s)\n  Final EMA loss: %.4f\n"
              "  HBM: peak allocated %.2f GB, reserved %.2f GB\n========================================\n",
              (long long)trainer.global_step, (long long)trainer.total_tokens, secs, trainer.total_tokens / secs,
              trainer.ema_loss, st.peak_allocated / 1e9, st.peak_reserved / 1e9);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  mft::apps::install_crash_report();
  try {
    return run(argc, argv);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s: error: %s\n", kProg, e.what());
    return 1;
  }
}
