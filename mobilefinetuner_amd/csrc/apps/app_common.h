// Shared plumbing of the native CLIs (csrc/apps): reference-style "--flag value" / "--flag=value"
// parsing against per-program flag sets, file helpers, the token-data sources every training /
// eval CLI accepts (pretokenized stream, synthetic stream, raw WikiText-2 text) and the
// power-monitor flags.
#pragma once
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <sys/stat.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "engine/allocator.h"
#include "engine/autograd.h"
#include "engine/comm.h"
#include "engine/dist.h"
#include "engine/gemm.h"
#include "engine/lm.h"
#include "engine/optim.h"
#include "engine/trainer.h"
#include "engine/weight_stream.h"
#include "engine/zero3.h"
#include "runtime/dataset.h"
#include "runtime/power_monitor.h"

namespace mft {
namespace apps {

// Fatal-signal report (SIGSEGV / SIGBUS / SIGFPE / SIGILL / SIGABRT): the native backtrace of the
// faulting thread on stderr, then the default action (core / exit status unchanged) -- how a crash
// inside a runtime call (e.g. a profiler hooking hipGraphLaunch) is located without a debugger.
inline void crash_report(int sig) {
  void* frames[64];
  const int n = ::backtrace(frames, 64);
  char head[96];
  const int k = std::snprintf(head, sizeof(head), "\n[mft] fatal signal %d; native backtrace (%d frames):\n", sig, n);
  if (k > 0) (void)!::write(2, head, (size_t)k);
  ::backtrace_symbols_fd(frames, n, 2);
  ::signal(sig, SIG_DFL);
  ::raise(sig);
}
inline void install_crash_report() {
  struct sigaction sa {};
  sa.sa_handler = crash_report;
  sigemptyset(&sa.sa_mask);
  for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT}) ::sigaction(sig, &sa, nullptr);
}

using eng::DistConfig;

struct Args {
  std::map<std::string, std::string> kv;
  std::set<std::string> flags;
  std::vector<std::string> unknown;  // lenient parsing: flags outside the program's sets
  std::string get(const std::string& k, const std::string& d = "") const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
  int i(const std::string& k, int d) const { return kv.count(k) ? std::stoi(kv.at(k)) : d; }
  int64_t l(const std::string& k, int64_t d) const { return kv.count(k) ? std::stoll(kv.at(k)) : d; }
  float f(const std::string& k, float d) const { return kv.count(k) ? std::stof(kv.at(k)) : d; }
  bool b(const std::string& k) const { return flags.count(k) || (kv.count(k) && kv.at(k) != "0" && kv.at(k) != "false"); }
};

// The common flag block every native CLI accepts on top of its reference flags:
//   --dtype bf16|fp32        compute precision (fp32: the reference's precision, the composite path of
//                            every op on fp32 tensors -- eager, for parity checks; bf16: the fused kernels)
//   --attn_impl flash|naive  flash-attention kernels, or the materialized masked softmax (reference
//                            graph/gpt2_model.cpp:679-711 standard path)
//   --profile_steps a:b      steps a..b inside one roctx range, profiler resumed only there
//                            (rocprofv3 --selected-regions), per-step device times printed
//   --compat_grad_overwrite  reference .grad overwrite across micro-batches
//   --compat_reference       every reference-quirk switch: coupled L2 Adam (Q8), .grad overwrite (Q1),
//                            interleaved RoPE pairs (Q9, Gemma)
inline const std::set<std::string>& common_bool_flags() {
  static const std::set<std::string> s = {"compat_grad_overwrite", "compat_reference"};
  return s;
}
inline const std::set<std::string>& common_valued_flags() {
  static const std::set<std::string> s = {"dtype", "attn_impl", "profile_steps"};
  return s;
}

// kBool flags may appear bare; kValued flags take a value; anything else is an error (lenient: it
// is recorded in Args::unknown and skipped with its value, like the reference Gemma CLI parser).  The
// common flag block above is accepted by every program.
inline Args parse_args(int argc, char** argv, const std::set<std::string>& kBool0, const std::set<std::string>& kValued0,
                       bool lenient = false) {
  std::set<std::string> kBool = kBool0, kValued = kValued0;
  kBool.insert(common_bool_flags().begin(), common_bool_flags().end());
  kValued.insert(common_valued_flags().begin(), common_valued_flags().end());
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    if (s.rfind("--", 0) != 0) throw std::runtime_error("unexpected argument '" + s + "'");
    s = s.substr(2);
    std::string key = s, val;
    bool has_val = false;
    const size_t eq = s.find('=');
    if (eq != std::string::npos) {
      key = s.substr(0, eq);
      val = s.substr(eq + 1);
      has_val = true;
    }
    if (kBool.count(key)) {
      if (!has_val && i + 1 < argc) {  // "--flag 0" / "--flag true" (the reference's get_val form)
        const std::string nx = argv[i + 1];
        if (nx == "0" || nx == "1" || nx == "true" || nx == "false" || nx == "True" || nx == "False") {
          val = nx;
          has_val = true;
          ++i;
        }
      }
      if (has_val) a.kv[key] = val;
      else a.flags.insert(key);
      continue;
    }
    if (!kValued.count(key)) {
      if (!lenient) throw std::runtime_error("unknown flag --" + key + " (see --help)");
      a.unknown.push_back("--" + key);
      if (!has_val && i + 1 < argc && std::string(argv[i + 1]).rfind("--", 0) != 0) ++i;
      continue;
    }
    if (!has_val) {
      if (i + 1 >= argc) throw std::runtime_error("flag --" + key + " needs a value");
      val = argv[++i];
    }
    a.kv[key] = val;
  }
  return a;
}

// --dtype: before any model is built (weights are allocated in the compute dtype)
inline void apply_dtype_flag(const Args& a) {
  const std::string d = a.get("dtype", "bf16");
  if (d == "fp32" || d == "float32" || d == "f32") {
    eng::set_compute_dtype(eng::DType::F32);
    std::printf("  --dtype fp32: reference-precision composite path (fp32 weights / activations, eager)\n");
  } else if (d != "bf16" && d != "bfloat16") {
    throw std::runtime_error("--dtype " + d + ": bf16 or fp32");
  }
}
inline void apply_model_flags(const Args& a, eng::LanguageModel& m) {
  const std::string ai = a.get("attn_impl", "flash");
  if (ai != "flash" && ai != "naive") throw std::runtime_error("--attn_impl " + ai + ": flash or naive");
  m.attn_naive = ai == "naive";
}
inline void apply_train_flags(const Args& a, eng::TrainConfig& tc) {
  const std::string ps = a.get("profile_steps");
  if (!ps.empty()) {  // a:b (1-indexed, inclusive); "a" alone = that one step
    const size_t c = ps.find(':');
    tc.profile_from = std::stoll(ps.substr(0, c));
    tc.profile_to = c == std::string::npos ? tc.profile_from : std::stoll(ps.substr(c + 1));
    if (tc.profile_from < 1 || tc.profile_to < tc.profile_from) throw std::runtime_error("--profile_steps a:b with 1 <= a <= b");
  }
  tc.compat_grad_overwrite = a.b("compat_grad_overwrite") || a.b("compat_reference");
}

inline bool file_exists(const std::string& p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

inline std::string split_file(const std::string& dir, const char* const* names) {
  for (int i = 0; names[i]; ++i) {
    const std::string p = dir + "/" + names[i];
    if (file_exists(p)) return p;
  }
  return "";
}

// counter-hash token stream (no dataset needed): --synthetic_data [--synthetic_tokens N]
inline std::vector<int32_t> synthetic_tokens(int64_t count, uint64_t seed, int vocab) {
  std::vector<int32_t> v(count);
  uint64_t z = seed;
  for (int64_t i = 0; i < count; ++i) {
    z += 0x9E3779B97F4A7C15ull;
    uint64_t x = z;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    v[i] = (int32_t)((x ^ (x >> 31)) % (uint64_t)vocab);
  }
  return v;
}

using Encoder = std::function<std::vector<int>(const std::string&)>;

// Fill train / valid from --pretokenized_path (+ --pretokenized_meta), --synthetic_data, or the raw
// text of --data_dir encoded by make_encoder() (built only on that path).  Returns whether a
// validation split exists.  The pretokenized meta's eos / pad ids override dc's.
inline bool load_token_splits(const Args& a, DataConfig& dc, int vocab, TokenDataset& train, TokenDataset& valid,
                              const std::function<Encoder()>& make_encoder) {
  const int seq = dc.seq_len;
  const std::string ddir = a.get("data_dir"), pt = a.get("pretokenized_path");
  if (!pt.empty()) {
    std::string meta = a.get("pretokenized_meta");
    if (meta.empty()) meta = pt.substr(0, pt.rfind('/') + 1) + "meta.json";
    PretokMeta m = read_pretok_meta(meta);
    train.set_tokens(read_pretok_split(pt, m, 0, dc.data_fraction, seq));
    std::printf("  pretokenized stream %s\n", pt.c_str());
    if (m.len[1] <= 0) return false;
    valid.set_tokens(read_pretok_split(pt, m, 1, 1.f, seq));
    return true;
  }
  if (a.b("synthetic_data") || ddir.empty()) {
    const int64_t n = a.l("synthetic_tokens", 2000000);
    train.set_tokens(synthetic_tokens(n, dc.seed, vocab));
    valid.set_tokens(synthetic_tokens(std::max<int64_t>(n / 20, 4 * seq), dc.seed + 1, vocab));
    std::printf("  (synthetic token data, %lld tokens)\n", (long long)n);
    return true;
  }
  const char* tr_names[] = {"wiki.train.raw", "wiki.train.tokens", "train.txt", nullptr};
  const char* va_names[] = {"wiki.valid.raw", "wiki.valid.tokens", "valid.txt", "validation.txt", nullptr};
  Encoder enc = make_encoder();
  const int threads = std::max(1u, std::thread::hardware_concurrency());
  const std::string ftr = split_file(ddir, tr_names), fva = split_file(ddir, va_names);
  if (ftr.empty()) throw std::runtime_error("no train split under " + ddir);
  train.set_tokens(pack_lines(read_lines(ftr, true), enc, dc.eos_id, true, dc.data_fraction, seq, threads));
  if (fva.empty()) return false;
  valid.set_tokens(pack_lines(read_lines(fva, true), enc, dc.eos_id, true, 1.f, seq, threads));
  return true;
}

// Data-parallel / ZeRO flags shared by the training CLIs:
//   --zero_stage 0|1|2|3 optimizer partition (1) + reduce-scattered gradients (2) + partitioned
//                        parameters (3, full fine-tuning: engine/zero3.h); > 0 also on one process
//                        (a 1-rank communicator: the partitioned code path runs)
//   --offload host|disk|none  AdamW moments in pinned host DRAM, or (disk, --offload_dir D, default
//                        ./mft_offload; ZeRO stages 0-2) in files under D streamed through device chunks
//                        each step (--offload_moments bf16 (stochastically
//                        rounded, default) | fp32); ZeRO-3: --offload_mode stream (default: each
//                        unit updated during the next forward, on its own stream, under the
//                        compute) | zerocopy (one update after the backward); both read / write the
//                        moments in place over PCIe
//   --bucket_mb N        fp32 gradient bytes per reduction bucket (default 25)
//   --bf16_grads         reduce gradients in bf16      --no_overlap   reduce after the backward
// MFT_DP_FORCE_COMM=1: a 1-rank communicator even without ZeRO (profiling the reducer on one GPU).
inline DistConfig dist_config_from(const Args& a) {
  DistConfig d;
  d.zero_stage = a.i("zero_stage", 0);
  d.bucket_bytes = (int64_t)(a.f("bucket_mb", 25.f) * 1048576.0);
  d.bf16_reduce = a.b("bf16_grads");
  d.overlap = !a.b("no_overlap");
  const std::string off = a.get("offload", "none");
  if (off != "none" && off != "host" && off != "disk") throw std::runtime_error("--offload host|disk|none (got '" + off + "')");
  d.host_moments = off == "host";
  if (off == "disk") d.disk_dir = a.get("offload_dir", "mft_offload");
  const std::string om = a.get("offload_moments", "bf16");
  if (om != "bf16" && om != "fp32") throw std::runtime_error("--offload_moments bf16|fp32 (got '" + om + "')");
  d.host_fp32 = om == "fp32";
  const std::string mode = a.get("offload_mode", "stream");
  if (mode != "stream" && mode != "zerocopy") throw std::runtime_error("--offload_mode stream|zerocopy (got '" + mode + "')");
  d.host_stream = mode == "stream";
  if (d.zero_stage < 0 || d.zero_stage > 3) throw std::runtime_error("--zero_stage 0|1|2|3 in the native engine");
  return d;
}

inline std::unique_ptr<eng::Communicator> comm_from(const DistConfig& d) {
  const char* fc = std::getenv("MFT_DP_FORCE_COMM");
  auto c = eng::Communicator::from_env((fc && fc[0] == '1') || d.zero_stage > 0);
  // ranks must not pick kernels by timing on their own: hipBLASLt takes its heuristic's first algorithm
  // (the gemm8 / hipBLASLt routing itself is a fixed table)
  return c;
}

// the flat trainable buffers, bucket-planned when a communicator exists, plus its reducer; or,
// with --zero_stage 3, the parameter partitioner whose flat holds only this rank's partitions
struct DistSetup {
  std::unique_ptr<eng::FlatParams> own;
  eng::FlatParams* flat = nullptr;
  eng::FlatPlan plan;
  std::unique_ptr<eng::DataParallel> dp;
  std::unique_ptr<eng::Zero3> z3;
  void make_flat(std::vector<std::pair<std::string, eng::Param*>> params, eng::Communicator* comm, const DistConfig& d) {
    if (comm) {
      plan = eng::plan_flat(params, comm->world(), d.bucket_bytes);
      own = std::make_unique<eng::FlatParams>(std::move(params), plan.offsets, plan.numel);
    } else {
      own = std::make_unique<eng::FlatParams>(std::move(params));
    }
    flat = own.get();
  }
  void make_zero3(const std::vector<eng::NamedParams>& units, const eng::NamedParams& rep, eng::Communicator& comm) {
    z3 = std::make_unique<eng::Zero3>(units, rep, comm);
    flat = &z3->flat();
  }
  // after the optimizer exists (the reducer shards it)
  void make_dp(eng::Communicator* comm, eng::AdamW& opt, const DistConfig& d) {
    if (z3 && !d.disk_dir.empty()) throw std::runtime_error("--offload disk: ZeRO stages 0-2 (ZeRO-3 takes --offload host)");
    if (z3) {
      z3->shard_optimizer(opt, d.host_moments, d.host_fp32, d.host_stream);
      std::printf("  %s%s%s%s\n", z3->describe().c_str(),
                  !d.host_moments ? "" : d.host_fp32 ? "; AdamW moments in pinned host DRAM (fp32)" : "; AdamW moments in pinned host DRAM (bf16)",
                  !d.host_moments ? "" : !d.host_stream ? ", read in place over PCIe after the backward"
                  : z3->staged_slots() > 0 ? ", staged through device slots by SDMA copies (each written back after its "
                                             "unit's update in the next forward and prefetched for the slot's next unit)"
                                           : ", read in place over PCIe, each unit updated during the next forward on its own stream",
                  z3->staged_slots() > 0 ? (" [" + std::to_string(z3->staged_slots()) + " slots]").c_str() : "");
    } else if (comm) {
      dp = std::make_unique<eng::DataParallel>(*flat, plan, *comm, opt, d);
      std::printf("  data parallel: %s\n", dp->describe().c_str());
    } else if (d.host_moments) {
      opt.shard({eng::OptSegment{0, flat->numel, 0}}, nullptr, true, d.host_fp32);
      std::printf("  AdamW moments in pinned host DRAM (%s)\n", d.host_fp32 ? "fp32" : "bf16");
    }
    if (!d.disk_dir.empty()) {  // after the reducer planned this rank's optimizer segments
      opt.to_disk(d.disk_dir, comm ? comm->rank() : 0, d.host_fp32);
      std::printf("  AdamW moments on disk (%s, %s/adamw_{m,v}.rank%d.bin), streamed through device chunks each step\n",
                  d.host_fp32 ? "fp32" : "bf16", d.disk_dir.c_str(), comm ? comm->rank() : 0);
    }
  }
  eng::GradReducer* reducer() { return z3 ? static_cast<eng::GradReducer*>(z3.get()) : dp.get(); }
};

// bench.py's native engine (--bench_steps K [--bench_warmup W]): time K full training steps after W
// untimed ones (Trainer::bench) and print ONE machine-readable line on rank 0:
//   MFT_BENCH {"seconds": .., "steps": K, "warmup": W, "world": N, "batch": B, "seq": S, "accum": A, ...}
// bench.py turns it into the driver's JSON record.
template <class TrainerT, class FlatT>
inline void bench_report(TrainerT& trainer, const FlatT& flat, const Args& a, int world, bool lead, const std::string& model,
                         size_t n_params, int batch, int seq, int accum) {
  const int steps = a.i("bench_steps", 0), warmup = a.i("bench_warmup", 3);
  float loss = 0.f;
  const double secs = trainer.bench(warmup, steps, &loss);
  long long n_train = 0;  // (ZeRO-3: this rank's partitions)
  for (auto& kv : flat.params) n_train += (long long)kv.second->leaf.numel();
  if (flat.params.empty()) n_train = (long long)flat.numel;
  if (!lead) return;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const eng::AllocStats ms = eng::CachingAllocator::get(dev).stats();  // HBM high-water mark of this rank
  std::printf("MFT_BENCH {\"seconds\": %.9f, \"steps\": %d, \"warmup\": %d, \"world\": %d, \"batch\": %d, "
              "\"seq\": %d, \"accum\": %d, \"final_loss\": %.6f, \"model\": \"%s\", \"n_params\": %zu, "
              "\"n_trainable\": %lld, \"peak_allocated_gb\": %.3f, \"peak_reserved_gb\": %.3f, \"hipgraph\": %s}\n",
              secs, steps, warmup, world, batch, seq, accum, loss, model.c_str(), n_params, n_train,
              ms.peak_allocated / 1e9, ms.peak_reserved / 1e9, trainer.graph_replayed() ? "true" : "false");
  std::fflush(stdout);
}

// --dump_grads PATH (parity tests): ONE forward + backward of the first B chunks of the train split
// (chunk order 0..B-1, no shuffle, no optimizer step); the gradients then REPLACE the trainable
// fp32 masters so the model's own checkpoint writer (LoRA or HF layout) stores them under the
// usual keys.  Returns the (mean) loss.
template <class ModelT>
inline float grads_into_masters(ModelT& model, eng::FlatParams& flat, TokenDataset& train, int B, int S) {
  std::vector<size_t> idx((size_t)B);
  for (int i = 0; i < B; ++i) idx[i] = (size_t)i % std::max<size_t>(1, train.num_sequences());
  std::vector<int64_t> hid((size_t)B * S), htg((size_t)B * S);
  std::vector<float> mk((size_t)B * S);
  train.get_batch(idx.data(), B, hid.data(), htg.data(), mk.data(), nullptr);
  eng::Tensor ids = eng::from_host(hid.data(), {B, S}, eng::DType::I64);
  eng::Tensor tg = eng::from_host(htg.data(), {B, S}, eng::DType::I64);
  flat.zero_grad();
  eng::Tensor loss = model.loss(ids, tg, 1.f);
  eng::backward({loss});
  const float lv = (float)loss.item();
  flat.master.copy_(flat.grad);
  eng::synchronize();
  return lv;
}

// --shard_dir D [--shard_fp16_disk 0|1]: the streamed weights' disk tier (weight_stream.h)
inline eng::DiskTier disk_tier_from(const Args& a) {
  eng::DiskTier d;
  d.dir = a.get("shard_dir");
  d.fp16 = !a.kv.count("shard_fp16_disk") || (a.kv.at("shard_fp16_disk") != "0" && a.kv.at("shard_fp16_disk") != "false");
  return d;
}

inline void print_streaming(const eng::WeightStreamer* ws, const char* what) {
  if (ws->on_disk())
    std::printf("  weight streaming ON: %d device slots (%.1f MB) for %.1f MB of frozen %s weights on disk (%s), "
                "%.1f MB pinned staging; %lld block(s) kept bf16 (not exactly representable in fp16)\n", ws->slots(),
                ws->device_bytes() / 1048576.0, ws->disk_bytes() / 1048576.0, what, "block files",
                ws->host_bytes() / 1048576.0, (long long)ws->bf16_fallbacks);
  else
    std::printf("  weight streaming ON: %d device slots (%.1f MB) for %.1f MB of frozen %s weights in pinned host memory\n",
                ws->slots(), ws->device_bytes() / 1048576.0, ws->host_bytes() / 1048576.0, what);
}

// NumPy .npy v1.0 writer for the alignment dumps (the reference's save_npy, train_lora_gemma.cpp:
// 137-178): descr "<f4" / "<i4", C order, header padded to a 64-byte boundary.  Parent directories
// are created.
inline void save_npy(const std::string& path, const void* data, const std::vector<int64_t>& shape, const char* descr,
                     size_t elem_bytes) {
  std::filesystem::path fp(path);
  if (fp.has_parent_path()) std::filesystem::create_directories(fp.parent_path());
  std::string sh = "(";
  size_t n = 1;
  for (size_t i = 0; i < shape.size(); ++i) {
    sh += std::to_string(shape[i]) + (shape.size() == 1 ? "," : (i + 1 < shape.size() ? ", " : ""));
    n *= (size_t)shape[i];
  }
  sh += ")";
  std::string hdr = std::string("{'descr': '") + descr + "', 'fortran_order': False, 'shape': " + sh + ", }";
  const size_t base = 10;  // magic (6) + version (2) + header length (2)
  hdr.append((64 - (base + hdr.size() + 1) % 64) % 64, ' ');
  hdr += '\n';
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot write " + path);
  const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
  f.write((const char*)magic, 8);
  const uint16_t hl = (uint16_t)hdr.size();
  const unsigned char hlb[2] = {(unsigned char)(hl & 0xff), (unsigned char)(hl >> 8)};
  f.write((const char*)hlb, 2);
  f.write(hdr.data(), (std::streamsize)hdr.size());
  f.write((const char*)data, (std::streamsize)(n * elem_bytes));
  if (!f) throw std::runtime_error("short write " + path);
}
inline void save_npy_f32(const std::string& path, const std::vector<float>& v, const std::vector<int64_t>& shape) {
  save_npy(path, v.data(), shape, "<f4", 4);
}

// --pm_* flags (reference energy options) -> PowerMonitor, or null when off.  The telemetry is this
// rank's own GPU (the HIP device's PCI address -> its DRM card's hwmon), never "card 0".
// --pm_power_cap W: software power cap (sleep per step so the socket power averages <= W; implies
// GPU telemetry and, without --pm_interval, a check every step).
inline std::unique_ptr<PowerMonitor> power_monitor_from(const Args& a) {
  const float cap = a.f("pm_power_cap", 0.f);
  if (a.i("pm_interval", 0) <= 0 && a.get("pm_schedule").empty() && cap <= 0.f) return nullptr;
  PowerConfig pc;
  pc.check_interval_steps = a.i("pm_interval", 0);
  pc.battery_threshold = a.f("pm_batt_thresh", 20.f);
  pc.temp_threshold = a.f("pm_temp_thresh", 42.f);
  pc.freq_b_high = a.f("pm_fb_high", 2.f);
  pc.freq_b_low = a.f("pm_fb_low", 0.5f);
  pc.freq_t_high = a.f("pm_ft_high", 2.f);
  pc.freq_t_low = a.f("pm_ft_low", 0.5f);
  pc.enable_battery = !a.b("pm_disable_batt");
  pc.enable_temp = !a.b("pm_disable_temp");
  pc.use_gpu_telemetry = a.b("pm_gpu_telemetry") || cap > 0.f;
  pc.power_cap_w = cap;
  if (cap > 0.f && pc.check_interval_steps <= 0) pc.check_interval_steps = 1;
  {
    int dev = 0;
    char bus[64] = {0};
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetPCIBusId(bus, sizeof(bus), dev) == hipSuccess) pc.pci_bus = bus;
  }
  auto pm = std::make_unique<PowerMonitor>(pc);
  pm->set_manual_readings(a.f("pm_manual_batt", 100.f), a.f("pm_manual_temp", 30.f));
  if (!a.get("pm_schedule").empty()) pm->set_step_schedule(PowerMonitor::parse_schedule(a.get("pm_schedule")));
  return pm;
}

}  // namespace apps
}  // namespace mft
