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
//   adapter) --no_graph --compat_l2_adam --amsgrad --metrics_out F --deterministic --interleaved_rope
//   --shard_enable --shard_budget_mb N: frozen layer weights streamed from pinned host memory
// Alignment harness (--align_dump_dir D, reference train_lora_gemma.cpp:609-922): one fixed batch,
// LoRA dropout off; dumps input_ids / labels / per-token NLL / loss_scalar, the MLP output of each
// --align_layers layer, the LoRA gradients of those layers (--align_dump_grads, default on) and,
// with --align_do_step (default on), the adapters after one AdamW step (wd 0); --align_numeric_attn
// adds central finite-difference checks of the largest attention-LoRA gradients
// (--align_numeric_targets q,k,v,o; --align_numeric_eps; --align_numeric_count) and
// --align_pt_weights_dir overrides the initial adapters from a PyTorch dump.  File names follow the
// reference: grads/base_model_model_model_layers_<i>_self_attn_q_proj_lora_A_default_weight.npy
// (A as [in, r], B as [r, out]).  --loss_reduction sum|sum_debug: summed token NLL, unnormalised
// gradient (core/lm_loss.cpp:184-192).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <set>
#include <string>
#include <vector>

#include "apps/app_common.h"
#include "engine/allocator.h"
#include "engine/autograd.h"
#include "engine/nn.h"
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

const std::set<std::string> kBool = {"random_init", "synthetic_data", "no_graph", "compat_l2_adam", "amsgrad", "deterministic",
                                     "interleaved_rope", "pm_disable_batt", "pm_disable_temp", "pm_gpu_telemetry",
                                     "activation_checkpointing", "shard_enable", "bf16_grads", "no_overlap", "help", "align_dump_grads",
                                     "align_do_step", "align_disable_debug", "align_no_retain_grad", "align_numeric_attn"};
const std::set<std::string> kValued = {
    "model_dir", "data_dir", "pretokenized_path", "pretokenized_meta", "output_dir", "targets", "lora_targets",
    "epochs", "max_steps", "seq_len", "batch", "grad_accum", "lr", "learning_rate", "rank", "lora_r", "alpha",
    "lora_alpha", "lora_dropout", "warmup_ratio", "max_grad_norm", "weight_decay", "loss_reduction", "lr_schedule",
    "data_fraction", "log_interval", "eval_steps", "eval_batches", "save_every", "seed", "model", "synthetic_tokens",
    "resume_from", "state_dir", "inject_fault", "metrics_out", "eval_out", "pm_interval", "pm_batt_thresh", "pm_temp_thresh", "pm_fb_high",
    "pm_fb_low", "pm_ft_high", "pm_ft_low", "pm_manual_batt", "pm_manual_temp", "pm_schedule", "pm_power_cap", "device",
    "shard_budget_mb", "shard_dir", "shard_fp16_disk", "bench_steps", "bench_warmup", "zero_stage", "offload", "offload_moments", "offload_mode", "offload_dir", "bucket_mb",
    "align_dump_dir", "align_layers", "align_pt_weights_dir", "align_numeric_eps", "align_numeric_count",
    "align_numeric_targets", "dump_grads", "dump_embedding", "dump_embedding_step", "dump_embedding_dir",
    "preview_tokens"};

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
      "  --eval_batches N --save_every N --seed S --pm_* (energy; --pm_power_cap W)\n"
      "  --dump_embedding 1 --dump_embedding_step N --dump_embedding_dir D --preview_tokens N\n"
      "  extras: --model P --random_init --synthetic_data --synthetic_tokens N --resume_from F --no_graph\n"
      "          --compat_l2_adam --amsgrad --metrics_out F --deterministic --interleaved_rope\n"
      "          --zero_stage 0|1|2 --offload host|disk|none [--offload_dir D] --bucket_mb N --bf16_grads --no_overlap\n"
      "          --state_dir D (full training state: written at --save_every and at the end, resumed if present)\n"
      "          --inject_fault STEP:RANK (failure test: that rank throws before that step)\n"
      "          --bench_steps K [--bench_warmup W] (bench.py: time K steps after W, print one MFT_BENCH line)\n"
      "  common: --dtype bf16|fp32 --attn_impl flash|naive --profile_steps A:B --compat_grad_overwrite --compat_reference\n",
      kProg);
}

// ---------------------------------------------------------------- alignment harness
bool flag_on(const Args& a, const char* k, bool d) {
  if (!a.kv.count(k)) return a.flags.count(k) ? true : d;
  const std::string v = a.kv.at(k);
  return !(v == "0" || v == "false" || v == "False");
}

// "layer.3.attn.q" -> "layers_3_self_attn_q_proj" (the PEFT module path, '.' -> '_')
std::string peft_stem(const std::string& name) {
  const size_t d1 = name.find('.', 6);
  const std::string li = name.substr(6, d1 - 6), part = name.substr(d1 + 1);
  static const std::map<std::string, std::string> m = {
      {"attn.q", "self_attn_q_proj"}, {"attn.k", "self_attn_k_proj"}, {"attn.v", "self_attn_v_proj"},
      {"attn.proj", "self_attn_o_proj"}, {"mlp.gate", "mlp_gate_proj"}, {"mlp.up", "mlp_up_proj"},
      {"mlp.down", "mlp_down_proj"}};
  auto it = m.find(part);
  return "layers_" + li + "_" + (it == m.end() ? part : it->second);
}

// "<stem>_lora_A_default_weight" for a trainable "layer.i.<part>.lora_A"
std::string ref_key(const std::string& name) {
  const bool isA = name.substr(name.size() - 7) == ".lora_A";
  return "base_model_model_model_" + peft_stem(name.substr(0, name.size() - 7)) + (isA ? "_lora_A" : "_lora_B") +
         "_default_weight";
}

int layer_of(const std::string& name) { return std::stoi(name.substr(6, name.find('.', 6) - 6)); }

// a LoRA tensor in the reference's layout: A [r, in] -> [in, r], B [r, out] as is
void dump_lora_tensor(const std::string& path, const std::string& name, const Tensor& t) {
  const bool isA = name.substr(name.size() - 7) == ".lora_A";
  Tensor src = isA ? t.t() : t;
  Tensor h = empty(src.shape(), DType::F32, Device::cpu());
  h.copy_(src);
  mft::apps::save_npy(path, h.data_ptr(), h.shape(), "<f4", 4);
}

// minimal float32 .npy reader (C order, v1/v2 header)
bool load_npy_f32(const std::string& path, std::vector<int64_t>& shape, std::vector<float>& data) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  char magic[8];
  f.read(magic, 8);
  if (!f || std::memcmp(magic, "\x93NUMPY", 6) != 0) return false;
  uint32_t hl = 0;
  if (magic[6] == 1) {
    unsigned char b[2];
    f.read((char*)b, 2);
    hl = b[0] | (b[1] << 8);
  } else {
    unsigned char b[4];
    f.read((char*)b, 4);
    hl = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
  }
  std::string hdr(hl, ' ');
  f.read(&hdr[0], hl);
  if (hdr.find("'<f4'") == std::string::npos || hdr.find("'fortran_order': True") != std::string::npos) return false;
  const size_t l = hdr.find('(', hdr.find("'shape'")), r = hdr.find(')', l);
  shape.clear();
  std::stringstream ss(hdr.substr(l + 1, r - l - 1));
  std::string tok;
  size_t n = 1;
  while (std::getline(ss, tok, ','))
    if (tok.find_first_of("0123456789") != std::string::npos) {
      shape.push_back(std::stoll(tok));
      n *= (size_t)shape.back();
    }
  data.resize(n);
  f.read((char*)data.data(), (std::streamsize)(n * 4));
  return (bool)f;
}

int alignment_mode(const Args& a, Gemma3& model, FlatParams& flat, TokenDataset& train, AdamWConfig oc, int S) {
  const std::string d = a.get("align_dump_dir");
  std::filesystem::create_directories(d);
  std::vector<int> layers;
  {
    std::stringstream ss(a.get("align_layers", "0,1,17"));
    std::string t;
    while (std::getline(ss, t, ','))
      if (!t.empty() && std::stoi(t) < model.cfg().n_layer) layers.push_back(std::stoi(t));
  }
  std::string ls;
  for (int l : layers) ls += (ls.empty() ? "" : ",") + std::to_string(l);
  std::printf("[Align] align_layers=%s\n", ls.c_str());
  auto in_layers = [&](const std::string& name) {
    return std::find(layers.begin(), layers.end(), layer_of(name)) != layers.end();
  };
  // optional: initial adapters from a PyTorch dump (either orientation)
  const std::string ptw = a.get("align_pt_weights_dir");
  if (!ptw.empty()) {
    NoGradGuard ng;
    int loaded = 0;
    for (auto& kv : flat.params) {
      const std::string fn = ptw + "/weights_after_step/" + ref_key(kv.first) + ".npy";
      std::vector<int64_t> shp;
      std::vector<float> v;
      if (!std::filesystem::exists(fn) || !load_npy_f32(fn, shp, v)) continue;
      Tensor leaf = kv.second->leaf;
      Tensor h = from_blob(v.data(), shp, DType::F32, Device::cpu());
      if (shp.size() == 2 && shp[0] == leaf.size(1) && shp[1] == leaf.size(0) && shp[0] != shp[1]) h = h.t();
      MFT_CHECK(h.numel() == leaf.numel() && h.size(0) == leaf.size(0), "align_pt_weights_dir: ", fn, " has shape ",
                shape_str(shp), ", the adapter is ", leaf.str());
      Tensor c = empty(leaf.shape(), DType::F32, Device::cpu());
      c.copy_(h);
      leaf.copy_(c);
      ++loaded;
    }
    flat.refresh_shadow();
    synchronize();
    std::printf("[Align] %d adapter tensors loaded from %s\n", loaded, ptw.c_str());
  }
  // the fixed batch: the first chunks of the train split
  const int B = std::max(1, std::min<int>(a.i("batch", 4), (int)train.num_sequences()));
  std::vector<size_t> idx(B);
  for (int i = 0; i < B; ++i) idx[i] = (size_t)i;
  std::vector<int64_t> hid((size_t)B * S), htg((size_t)B * S);
  std::vector<float> mk((size_t)B * S);
  train.get_batch(idx.data(), B, hid.data(), htg.data(), mk.data(), nullptr);
  {
    std::vector<int32_t> i32(hid.begin(), hid.end()), t32(htg.begin(), htg.end());
    mft::apps::save_npy(d + "/input_ids.npy", i32.data(), {B, S}, "<i4", 4);
    mft::apps::save_npy(d + "/labels.npy", t32.data(), {B, S}, "<i4", 4);  // next-token targets, -100 ignored
    mft::apps::save_npy(d + "/attention_mask.npy", mk.data(), {B, S}, "<f4", 4);
  }
  Tensor ids = from_host(hid.data(), {B, S}, DType::I64), tg = from_host(htg.data(), {B, S}, DType::I64);
  model.training = true;
  model.capture_layers = layers;
  Tensor loss = model.loss(ids, tg, 1.f);
  model.capture_layers.clear();
  const float lv = (float)loss.item();
  mft::apps::save_npy_f32(d + "/loss_scalar.npy", {lv}, {1});
  for (auto& kv : model.captured)
    mft::apps::save_npy_f32(d + "/layer" + std::to_string(kv.first) + "_mlp_out.npy", kv.second.to_vector_f32(),
                            {B, S, model.cfg().hidden});
  {
    NoGradGuard ng;
    Tensor h = model.hidden(ids);
    Tensor rows = lm_head_token_nll(h, model.output_embedding(), tg, model.vocab(), model.ce_chunk);
    mft::apps::save_npy_f32(d + "/per_token_nll.npy", rows.to_vector_f32(), {B, S});
  }
  std::printf("[Align] loss=%.6f (%s)\n", lv, model.loss_sum ? "sum" : "mean");
  const bool dump_grads = flag_on(a, "align_dump_grads", true), do_step = flag_on(a, "align_do_step", true);
  if (dump_grads || do_step || flag_on(a, "align_numeric_attn", false)) {
    flat.zero_grad();
    backward({loss});
    synchronize();
  }
  if (dump_grads) {
    int n = 0;
    for (auto& kv : flat.params)
      if (in_layers(kv.first)) {
        dump_lora_tensor(d + "/grads/" + ref_key(kv.first) + ".npy", kv.first, kv.second->leaf.grad());
        ++n;
      }
    std::printf("[Align] %d LoRA gradients dumped\n", n);
  }
  if (flag_on(a, "align_numeric_attn", false)) {
    // central differences on the largest-|grad| element of each attention adapter in the layers
    const float eps = a.f("align_numeric_eps", 1e-3f);
    const int count = a.i("align_numeric_count", 4);
    std::vector<std::string> tgs;
    {
      std::stringstream ss(a.get("align_numeric_targets", "q,v"));
      std::string t;
      while (std::getline(ss, t, ','))
        if (!t.empty()) tgs.push_back(".attn." + std::string(t == "o" ? "proj" : t) + ".lora_");
    }
    model.training = false;  // (dropout is off anyway; deterministic forward)
    std::vector<float> ana, num;
    int checked = 0;
    for (auto& kv : flat.params) {
      if (checked >= count || !in_layers(kv.first)) continue;
      bool hit = false;
      for (auto& t : tgs) hit = hit || kv.first.find(t) != std::string::npos;
      if (!hit) continue;
      Tensor leaf = kv.second->leaf;
      const std::vector<float> g = leaf.grad().to_vector_f32(), w = leaf.to_vector_f32();
      size_t i = 0;
      for (size_t j = 1; j < g.size(); ++j)
        if (std::fabs(g[j]) > std::fabs(g[i])) i = j;
      auto loss_at = [&](float val) {
        NoGradGuard ng;
        float hv = val;
        leaf.view({-1}).slice(0, (int64_t)i, (int64_t)i + 1).copy_(from_blob(&hv, {1}, DType::F32, Device::cpu()));
        flat.refresh_shadow();
        return model.loss(ids, tg, 1.f).item();
      };
      const double lp = loss_at(w[i] + eps), lm = loss_at(w[i] - eps);
      loss_at(w[i]);
      const double nd = (lp - lm) / (2.0 * eps);
      std::printf("[Align] %s[%zu] analytic=%.6e numeric=%.6e rel=%.3e\n", kv.first.c_str(), i, g[i], nd,
                  std::fabs(g[i] - nd) / std::max(std::fabs(nd), 1e-12));
      ana.push_back(g[i]);
      num.push_back((float)nd);
      ++checked;
    }
    mft::apps::save_npy_f32(d + "/numeric/lora_numeric_grad.npy", num, {(int64_t)num.size()});
    mft::apps::save_npy_f32(d + "/numeric/lora_analytic_grad.npy", ana, {(int64_t)ana.size()});
    model.training = true;
  }
  if (do_step) {
    oc.weight_decay = 0.f;  // reference: single AdamW step, wd 0
    AdamW opt(flat, oc);
    opt.set_lr(oc.lr);
    opt.step();
    synchronize();
    int n = 0;
    for (auto& kv : flat.params)
      if (in_layers(kv.first)) {
        dump_lora_tensor(d + "/weights_after_step/" + ref_key(kv.first) + ".npy", kv.first, kv.second->leaf.detach());
        ++n;
      }
    std::printf("[Align] one AdamW step (grad_norm=%.6f), %d adapter tensors dumped\n", opt.grad_norm(), n);
  }
  std::printf("[AlignDump] wrote activations and loss to %s\n", d.c_str());
  return 0;
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
  const std::string red = a.get("loss_reduction", "mean");
  if (red != "mean" && red != "sum" && red != "sum_debug")
    throw std::runtime_error("--loss_reduction mean|sum|sum_debug (got '" + red + "')");
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
  mft::apps::install_crash_report();  // again: the HIP runtime's initialisation may replace handlers
  const bool lead = !comm || comm->rank() == 0;
  const uint64_t seed = (uint64_t)a.l("seed", 42);

  std::printf("\n========== Gemma-3 LoRA Finetune (MI355X native engine) ==========\n");
  if (comm)
    std::printf("  data parallel: rank %d of %d (%s, device %d)\n", comm->rank(), comm->world(), comm->backend(),
                comm->device());
  mft::apps::apply_dtype_flag(a);
  const std::string mdir = a.get("model_dir");
  const bool random_init = a.b("random_init") || mdir.empty();
  Gemma3Config cfg = (!mdir.empty() && file_exists(mdir + "/config.json")) ? Gemma3Config::from_json(mdir + "/config.json")
                                                                         : Gemma3Config::preset(a.get("model", "gemma3-270m"));
  std::printf("  Gemma-3 config: layers=%d hidden=%d heads=%d/%d head_dim=%d vocab=%d\n", cfg.n_layer, cfg.hidden,
              cfg.n_head, cfg.n_kv, cfg.head_dim, cfg.vocab_size);
  auto model = std::make_unique<Gemma3>(cfg);
  model->interleaved_rope = a.b("interleaved_rope") || a.b("compat_reference");
  mft::apps::apply_model_flags(a, *model);
  model->grad_checkpoint = a.b("activation_checkpointing");  // recompute blocks in the backward
  model->loss_sum = red != "mean";
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
    spec.dropout = a.get("align_dump_dir").empty() ? a.f("lora_dropout", 0.1f) : 0.f;  // alignment: no dropout
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
    model->enable_weight_streaming(budget, mft::apps::disk_tier_from(a));
    mft::apps::print_streaming(model->streamer(), "layer");
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
  oc.l2_coupled = a.b("compat_l2_adam") || a.b("compat_reference");
  oc.amsgrad = a.b("amsgrad");
  if (!a.get("dump_grads").empty()) {  // parity tests: one fwd+bwd, gradients in the adapter layout
    MFT_CHECK(!comm, "--dump_grads runs on one process");
    const float lv = mft::apps::grads_into_masters(*model, flat, train, a.i("batch", 4), dc.seq_len);
    model->save_lora(a.get("dump_grads"));
    std::printf("MFT_DUMP loss=%.8f path=%s\n", lv, a.get("dump_grads").c_str());
    return 0;
  }
  if (!a.get("align_dump_dir").empty()) {
    if (comm) throw std::runtime_error("--align_dump_dir runs on one process");
    return alignment_mode(a, *model, flat, train, oc, dc.seq_len);
  }
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
  mft::apps::apply_train_flags(a, tc);
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
  // --preview_tokens N: the first N training tokens (reference train_lora_gemma.cpp:924-932)
  if (a.i("preview_tokens", 0) > 0 && lead) {
    const auto& tk = train.tokens();
    const size_t n = std::min(tk.size(), (size_t)a.i("preview_tokens", 0));
    std::printf("First %zu train tokens: [", n);
    for (size_t i = 0; i < n; ++i) std::printf("%s%d", i ? ", " : "", tk[i]);
    std::printf("]\n");
  }
  // --dump_embedding 1 [--dump_embedding_step N --dump_embedding_dir D]: the scaled token embeddings
  // of the N-th training micro-batch -- statistics, a preview of the first tokens' values and the raw
  // fp32 tensor as D/embedding_stepN.bin (reference gemma_trainer.cpp:104-109,
  // gemma_model.cpp:875-940).  The embedding of a frozen table is a pure function of the batch's
  // ids, so it is recomputed eagerly for that batch (the captured training step is not touched).
  const std::string de = a.get("dump_embedding", "0");
  if ((de == "1" || de == "true" || de == "True") && lead) {
    const int target = std::max(1, a.i("dump_embedding_step", 1));
    const std::string ddir = a.get("dump_embedding_dir", "./debug");
    Gemma3* gm = model.get();
    tc.micro_hook = [gm, target, ddir](int64_t micro, const int64_t* ids, int B, int S) {
      if (micro != target) return;
      Tensor di = from_host(ids, {B, S}, DType::I64);
      Tensor e = gm->embed_tokens(di).to(DType::F32).to(Device::cpu());
      const float* d = e.data<float>();
      const int H = (int)e.size(-1);
      const int64_t n = (int64_t)B * S * H;
      double sum = 0.0, sq = 0.0;
      float mn = std::numeric_limits<float>::max(), mx = std::numeric_limits<float>::lowest();
      for (int64_t i = 0; i < n; ++i) {
        sum += d[i];
        sq += (double)d[i] * d[i];
        mn = std::min(mn, d[i]);
        mx = std::max(mx, d[i]);
      }
      const double mean = sum / (double)std::max<int64_t>(n, 1);
      const double sd = std::sqrt(std::max(0.0, sq / (double)std::max<int64_t>(n, 1) - mean * mean));
      std::printf("[EmbeddingDump] step %d shape=[%d,%d,%d] mean=%.6f std=%.6f min=%.6f max=%.6f\n", target, B, S, H,
                  mean, sd, mn, mx);
      for (int t = 0; t < std::min(S, 4); ++t) {
        std::printf("  hidden[0,%d,0:%d] = [", t, std::min(H, 8));
        for (int k = 0; k < std::min(H, 8); ++k) std::printf("%s%.4g", k ? ", " : "", d[(int64_t)t * H + k]);
        std::printf("]\n");
      }
      std::filesystem::create_directories(ddir);
      const std::string fn = ddir + "/embedding_step" + std::to_string(target) + ".bin";
      std::ofstream out(fn, std::ios::binary);
      out.write(reinterpret_cast<const char*>(d), (std::streamsize)(n * sizeof(float)));
      if (out) std::printf("  [EmbeddingDump] wrote raw tensor to %s\n", fn.c_str());
      else std::fprintf(stderr, "  [EmbeddingDump] failed to write %s\n", fn.c_str());
      std::fflush(stdout);
    };
  }
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
              (long long)trainer.total_steps(), tc.batch, tc.accum, trainer.uses_graph() ? "hipGraph-captured step" : "eager");
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
  const AllocStats st = CachingAllocator::get(Device::current_hip_device()).stats();
  std::printf("\nTraining complete: %lld steps, %lld tokens, %.2f s (%.0f tokens/s), final EMA loss %.4f, "
              "HBM peak allocated %.2f GB\n",
              (long long)trainer.global_step, (long long)trainer.total_tokens, secs, trainer.total_tokens / secs,
              trainer.ema_loss, st.peak_allocated / 1e9);
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
