// libmft engine: GPT-2 model (see gpt2.h).
#include "engine/gpt2.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <regex>
#include <sstream>
#include <tuple>

#include "engine/autograd.h"
#include "engine/ops.h"
#include "kernels.h"
#include "runtime/json.h"
#include "runtime/safetensors.h"

namespace mft {
namespace eng {

GPT2Config GPT2Config::preset(const std::string& n0) {
  std::string n = n0;
  for (auto& c : n) c = (c == '_') ? '-' : (char)std::tolower(c);
  GPT2Config c;
  if (n == "gpt2" || n == "gpt2-small" || n == "gpt2-124m") return c;
  if (n == "gpt2-medium") {
    c.n_embd = 1024, c.n_layer = 24, c.n_head = 16;
  } else if (n == "gpt2-large") {
    c.n_embd = 1280, c.n_layer = 36, c.n_head = 20;
  } else if (n == "gpt2-xl") {
    c.n_embd = 1600, c.n_layer = 48, c.n_head = 25;
  } else if (n == "gpt2-tiny") {
    c.n_embd = 128, c.n_layer = 2, c.n_head = 2, c.vocab_size = 1000, c.n_positions = 256;
  } else {
    MFT_CHECK(false, "unknown GPT-2 preset '", n0, "'");
  }
  return c;
}

GPT2Config GPT2Config::from_json(const std::string& path) {
  std::ifstream f(path);
  MFT_CHECK(f.good(), "cannot open ", path);
  std::stringstream ss;
  ss << f.rdbuf();
  json::Value v = json::parse(ss.str());
  GPT2Config c;
  auto gi = [&](const char* k, int d) { return v.get(k) ? (int)v[k].as_int() : d; };
  c.vocab_size = gi("vocab_size", c.vocab_size);
  c.n_positions = v.get("n_positions") ? gi("n_positions", c.n_positions) : gi("n_ctx", c.n_positions);
  c.n_embd = gi("n_embd", c.n_embd);
  c.n_layer = gi("n_layer", c.n_layer);
  c.n_head = gi("n_head", c.n_head);
  if (v.get("layer_norm_epsilon")) c.eps = (float)v["layer_norm_epsilon"].as_double();
  if (v.get("initializer_range")) c.init_range = (float)v["initializer_range"].as_double();
  return c;
}

bool LoraSpec::has(const std::string& t) const { return std::find(targets.begin(), targets.end(), t) != targets.end(); }

namespace {
Param frozen(Tensor t) {
  Param p;
  p.leaf = t;
  p.c = t;
  return p;
}
}  // namespace

GPT2::GPT2(const GPT2Config& cfg) : cfg_(cfg) { alloc(); }

void GPT2::alloc() {
  const int C = cfg_.n_embd;
  NoGradGuard ng;
  const DType wd = compute_dtype();  // bf16, or fp32 for --dtype fp32 (LayerNorm parameters are fp32 either way)
  wte_ = frozen(zeros({cfg_.vocab_padded(), C}, wd));
  wpe_ = frozen(zeros({cfg_.n_positions, C}, wd));
  lnf_w_ = frozen(ones({C}, DType::F32));
  lnf_b_ = frozen(zeros({C}, DType::F32));
  blocks_.resize(cfg_.n_layer);
  for (auto& b : blocks_) {
    b.ln1_w = frozen(ones({C}, DType::F32));
    b.ln1_b = frozen(zeros({C}, DType::F32));
    b.ln2_w = frozen(ones({C}, DType::F32));
    b.ln2_b = frozen(zeros({C}, DType::F32));
    b.attn_w = frozen(zeros({3 * C, C}, wd));
    b.attn_b = frozen(zeros({3 * C}, wd));
    b.proj_w = frozen(zeros({C, C}, wd));
    b.proj_b = frozen(zeros({C}, wd));
    b.fc_w = frozen(zeros({4 * C, C}, wd));
    b.fc_b = frozen(zeros({4 * C}, wd));
    b.mproj_w = frozen(zeros({C, 4 * C}, wd));
    b.mproj_b = frozen(zeros({C}, wd));
  }
  dropout_ctr = zeros({1}, DType::I64);
  ce_chunk = default_ce_chunk(cfg_.vocab_padded());
}

void GPT2::init_random(uint64_t seed) {
  NoGradGuard ng;
  const float std0 = cfg_.init_range, std_proj = cfg_.init_range / std::sqrt(2.f * cfg_.n_layer);
  uint64_t s = seed * 1000003ull + 17;
  auto nrm = [&](Param& p, float sd) { p.c.copy_(randn(p.c.shape(), ++s, sd, DType::F32)); };
  nrm(wte_, std0);
  wte_.c.slice(0, cfg_.vocab_size, cfg_.vocab_padded()).zero_();
  nrm(wpe_, 0.01f);
  for (auto& b : blocks_) {
    nrm(b.attn_w, std0);
    nrm(b.fc_w, std0);
    nrm(b.proj_w, std_proj);
    nrm(b.mproj_w, std_proj);
  }
}

// ------------------------------------------------------------------ HF checkpoint IO
namespace {
DType st_dtype(const std::string& d) {
  if (d == "F32") return DType::F32;
  if (d == "BF16") return DType::BF16;
  if (d == "F16") return DType::F16;
  MFT_CHECK(false, "safetensors: unsupported dtype ", d);
  return DType::F32;
}
}  // namespace

void GPT2::load_hf(const std::string& dir) {
  NoGradGuard ng;
  std::string path = dir;
  if (path.size() < 12 || path.substr(path.size() - 12) != ".safetensors") path = dir + "/model.safetensors";
  SafeTensorsFile f(path);
  auto find = [&](const std::string& k) -> const TensorInfo* {
    if (f.has(k)) return &f.info(k);
    if (f.has("transformer." + k)) return &f.info("transformer." + k);
    return nullptr;
  };
  auto load = [&](Param& p, const std::string& key, bool conv1d) {
    const TensorInfo* ti = find(key);
    MFT_CHECK(ti, "checkpoint ", path, " has no tensor '", key, "'");
    Tensor host = from_blob(const_cast<void*>(f.data(ti->name)), ti->shape, st_dtype(ti->dtype), Device::cpu());
    Tensor src = conv1d ? host.t() : host;  // HF Conv1D [in, out] -> [out, in]
    Tensor dst = p.c;
    if (key == "wte.weight") dst = p.c.slice(0, 0, ti->shape[0]);
    MFT_CHECK(shape_numel(src.shape()) == dst.numel(), "checkpoint tensor '", key, "' ", shape_str(ti->shape),
              " does not fit ", dst.str());
    Tensor staged = empty(src.shape(), DType::F32, Device::cpu());
    staged.copy_(src);  // host transpose + cast
    dst.copy_(staged.view(dst.shape()));
  };
  load(wte_, "wte.weight", false);
  load(wpe_, "wpe.weight", false);
  load(lnf_w_, "ln_f.weight", false);
  load(lnf_b_, "ln_f.bias", false);
  for (int i = 0; i < cfg_.n_layer; ++i) {
    auto& b = blocks_[i];
    const std::string p = "h." + std::to_string(i) + ".";
    load(b.ln1_w, p + "ln_1.weight", false);
    load(b.ln1_b, p + "ln_1.bias", false);
    load(b.attn_w, p + "attn.c_attn.weight", true);
    load(b.attn_b, p + "attn.c_attn.bias", false);
    load(b.proj_w, p + "attn.c_proj.weight", true);
    load(b.proj_b, p + "attn.c_proj.bias", false);
    load(b.ln2_w, p + "ln_2.weight", false);
    load(b.ln2_b, p + "ln_2.bias", false);
    load(b.fc_w, p + "mlp.c_fc.weight", true);
    load(b.fc_b, p + "mlp.c_fc.bias", false);
    load(b.mproj_w, p + "mlp.c_proj.weight", true);
    load(b.mproj_b, p + "mlp.c_proj.bias", false);
  }
  synchronize();
}

std::vector<std::pair<std::string, Param*>> GPT2::all_params() {
  std::vector<std::pair<std::string, Param*>> v{{"wte.weight", &wte_}, {"wpe.weight", &wpe_}};
  for (int i = 0; i < cfg_.n_layer; ++i) {
    auto& b = blocks_[i];
    const std::string p = "h." + std::to_string(i) + ".";
    v.push_back({p + "ln_1.weight", &b.ln1_w});
    v.push_back({p + "ln_1.bias", &b.ln1_b});
    v.push_back({p + "attn.c_attn.weight", &b.attn_w});
    v.push_back({p + "attn.c_attn.bias", &b.attn_b});
    v.push_back({p + "attn.c_proj.weight", &b.proj_w});
    v.push_back({p + "attn.c_proj.bias", &b.proj_b});
    v.push_back({p + "ln_2.weight", &b.ln2_w});
    v.push_back({p + "ln_2.bias", &b.ln2_b});
    v.push_back({p + "mlp.c_fc.weight", &b.fc_w});
    v.push_back({p + "mlp.c_fc.bias", &b.fc_b});
    v.push_back({p + "mlp.c_proj.weight", &b.mproj_w});
    v.push_back({p + "mlp.c_proj.bias", &b.mproj_b});
  }
  v.push_back({"ln_f.weight", &lnf_w_});
  v.push_back({"ln_f.bias", &lnf_b_});
  return v;
}

void GPT2::save_hf(const std::string& path) {
  std::vector<Tensor> keep;
  std::vector<TensorBlob> blobs;
  for (auto& kv : all_params()) {
    const std::string& k = kv.first;
    Tensor src = kv.second->trainable() ? kv.second->leaf.detach() : kv.second->c;
    if (k == "wte.weight") src = src.slice(0, 0, cfg_.vocab_size);
    const bool conv1d = k.find("attn.c_attn.weight") != std::string::npos ||
                        k.find("attn.c_proj.weight") != std::string::npos ||
                        k.find("mlp.c_fc.weight") != std::string::npos || k.find("mlp.c_proj.weight") != std::string::npos;
    Tensor h = empty(conv1d ? Shape{src.size(1), src.size(0)} : src.shape(), DType::F32, Device::cpu());
    h.copy_(conv1d ? src.t() : src);
    keep.push_back(h);
    blobs.push_back({k, "F32", h.shape(), h.data_ptr(), h.nbytes()});
  }
  safetensors_save(path, blobs, {{"format", "pt"}}, true, true);
}

// ------------------------------------------------------------------ parameters
void GPT2::make_trainable(Param& p) {
  if (p.trainable()) return;
  NoGradGuard ng;
  Tensor master = p.c.to(DType::F32);
  if (master.impl() == p.c.impl()) master = p.c.clone();
  master.requires_grad_(true);
  p.leaf = master;
  if (p.c.dtype() == DType::F32) p.c = master;  // fp32-compute (norm) weights read the master
  p.wt = Tensor();
}

void GPT2::set_full_finetune() {
  full_ = true;
  for (auto& kv : all_params()) make_trainable(*kv.second);
}

void GPT2::zero3_layout(std::vector<std::vector<std::pair<std::string, Param*>>>& units,
                        std::vector<std::pair<std::string, Param*>>& rep) {
  MFT_CHECK(full_, "zero3_layout: ZeRO-3 partitions full fine-tuning weights");
  units.assign(1 + cfg_.n_layer, {});
  rep.clear();
  for (auto& kv : all_params()) {
    const std::string& k = kv.first;
    if (kv.second->c.dtype() == DType::F32) {
      rep.push_back(kv);
      continue;
    }
    int u = 0;
    if (k.compare(0, 2, "h.") == 0) u = 1 + std::stoi(k.substr(2, k.find('.', 2) - 2));
    units[u].push_back(kv);
  }
}

std::vector<std::pair<std::string, Param*>> GPT2::trainable() {
  std::vector<std::pair<std::string, Param*>> v;
  if (full_) {
    for (auto& kv : all_params())
      if (kv.second->trainable()) v.push_back(kv);
  }
  for (int i = 0; i < cfg_.n_layer; ++i) {
    auto& b = blocks_[i];
    auto add = [&](std::vector<LoraAdapter>& ads, std::vector<std::string>& names) {
      for (size_t j = 0; j < ads.size(); ++j) {
        v.push_back({names[j] + ".lora_A", &ads[j].A});
        v.push_back({names[j] + ".lora_B", &ads[j].B});
      }
    };
    add(b.lqkv, b.names_qkv);
    add(b.lproj, b.names_proj);
    add(b.lfc, b.names_fc);
    add(b.lfcout, b.names_fcout);
  }
  return v;
}

size_t GPT2::num_parameters() const {
  size_t n = 0;
  auto self = const_cast<GPT2*>(this);
  for (auto& kv : self->all_params()) n += kv.second->c.numel();
  return n - (size_t)(cfg_.vocab_padded() - cfg_.vocab_size) * cfg_.n_embd;
}

// ------------------------------------------------------------------ LoRA
void GPT2::inject_lora(const LoraSpec& spec) {
  spec_ = spec;
  lora_ = true;
  const int C = cfg_.n_embd;
  std::vector<int> layers = spec.layers;
  if (layers.empty())
    for (int i = 0; i < cfg_.n_layer; ++i) layers.push_back(i);
  for (int i : layers) {
    auto& b = blocks_[i];
    const std::string pre = "layer." + std::to_string(i) + ".";
    auto add = [&](std::vector<LoraAdapter>& ads, std::vector<std::string>& names, int col0, int n, int in,
                   const std::string& nm) {
      // reference init (graph/lora_injector.cpp:70-85): A[in, r] ~ U(+-sqrt(6/(in+r))), seed 42+in+out
      const float bound = std::sqrt(6.f / (float)(in + spec.rank));
      Tensor A = rand_uniform({in, spec.rank}, spec.seed + in + n, -bound, bound, DType::F32).t();
      ads.push_back(make_adapter(col0, n, spec.rank, A, spec.dropout, pre + nm));
      names.push_back(pre + nm);
    };
    if (spec.has("AttnQKV")) {
      if (spec.split_qkv) {
        add(b.lqkv, b.names_qkv, 0, C, C, "attn.q");
        add(b.lqkv, b.names_qkv, C, C, C, "attn.k");
        add(b.lqkv, b.names_qkv, 2 * C, C, C, "attn.v");
      } else {
        add(b.lqkv, b.names_qkv, 0, 3 * C, C, "attn.qkv");
      }
    }
    if (spec.has("AttnProj")) add(b.lproj, b.names_proj, 0, C, C, "attn.proj");
    if (spec.has("MlpFcIn")) add(b.lfc, b.names_fc, 0, 4 * C, C, "mlp.fc_in");
    if (spec.has("MlpFcOut")) add(b.lfcout, b.names_fcout, 0, C, 4 * C, "mlp.fc_out");
  }
}

void GPT2::load_lora(const std::string& path) {
  SafeTensorsFile f(path);
  const auto& meta = f.metadata();
  LoraSpec spec;
  auto mget = [&](const char* k) -> std::string {
    auto it = meta.find(k);
    return it == meta.end() ? "" : it->second;
  };
  std::map<std::string, const TensorInfo*> A, B;
  std::regex re(R"(layer\.(\d+)\.(attn\.qkv|attn\.q|attn\.k|attn\.v|attn\.proj|mlp\.fc_in|mlp\.fc_out)\.lora_(A|B))");
  std::vector<int> layers;
  for (auto& ti : f.tensors()) {
    std::smatch m;
    if (!std::regex_match(ti.name, m, re)) continue;
    const std::string stem = "layer." + m[1].str() + "." + m[2].str();
    (m[3].str() == "A" ? A : B)[stem] = &ti;
    const int li = std::stoi(m[1].str());
    if (std::find(layers.begin(), layers.end(), li) == layers.end()) layers.push_back(li);
  }
  MFT_CHECK(!A.empty(), "no LoRA tensors in ", path);
  spec.rank = mget("rank").empty() ? (int)std::min(A.begin()->second->shape[0], A.begin()->second->shape[1])
                                   : std::stoi(mget("rank"));
  spec.alpha = mget("alpha").empty() ? 2.f * spec.rank : std::stof(mget("alpha"));
  spec.dropout = mget("dropout").empty() ? 0.f : std::stof(mget("dropout"));
  spec.split_qkv = mget("split_qkv") == "true";
  spec.targets.clear();
  {  // metadata order wins (spec_from_metadata); else the canonical target order
    const std::string t = mget("targets");
    if (!t.empty() && t.find("attn.") == std::string::npos) {
      std::stringstream ss(t);
      std::string item;
      while (std::getline(ss, item, ','))
        if (!item.empty()) spec.targets.push_back(item);
    }
  }
  for (const char* canon : {"attn.qkv", "attn.q", "attn.proj", "mlp.fc_in", "mlp.fc_out"}) {
    const std::string part = canon;
    bool present = false;
    for (auto& kv : A) present = present || kv.first.substr(kv.first.find('.', 6) + 1) == part;
    if (!present) continue;
    std::string t = part == "attn.proj" ? "AttnProj" : part == "mlp.fc_in" ? "MlpFcIn" : part == "mlp.fc_out" ? "MlpFcOut" : "AttnQKV";
    if (part == "attn.q") spec.split_qkv = true;
    if (!spec.has(t)) spec.targets.push_back(t);
  }
  for (auto& kv : A) {
    const std::string part = kv.first.substr(kv.first.find('.', 6) + 1);
    std::string t = part == "attn.proj" ? "AttnProj" : part == "mlp.fc_in" ? "MlpFcIn" : part == "mlp.fc_out" ? "MlpFcOut" : "AttnQKV";
    if (part == "attn.q") spec.split_qkv = true;
    if (!spec.has(t)) spec.targets.push_back(t);
  }
  std::sort(layers.begin(), layers.end());
  spec.layers = layers;
  for (auto& b : blocks_) {
    b.lqkv.clear(), b.lproj.clear(), b.lfc.clear(), b.lfcout.clear();
    b.names_qkv.clear(), b.names_proj.clear(), b.names_fc.clear(), b.names_fcout.clear();
    b.waug_qkv = Tensor(), b.waug_proj = Tensor();
  }
  inject_lora(spec);
  // overwrite the fresh adapters with the checkpoint's values: A [in, r] -> [r, in], B [r, out]
  NoGradGuard ng;
  for (auto& kv : trainable()) {
    const std::string& name = kv.first;
    const bool isA = name.size() > 7 && name.substr(name.size() - 7) == ".lora_A";
    const std::string stem = name.substr(0, name.size() - 7);
    auto& mp = isA ? A : B;
    auto it = mp.find(stem);
    MFT_CHECK(it != mp.end(), "LoRA checkpoint lacks ", name);
    const TensorInfo* ti = it->second;
    Tensor host = from_blob(const_cast<void*>(f.data(ti->name)), ti->shape, st_dtype(ti->dtype), Device::cpu());
    Tensor src = isA ? host.t() : host;
    Tensor staged = empty(src.shape(), DType::F32, Device::cpu());
    staged.copy_(src);
    Param* p = kv.second;
    MFT_CHECK(staged.numel() == p->leaf.numel(), "LoRA tensor ", name, " shape mismatch");
    p->leaf.copy_(staged.view(p->leaf.shape()));
    p->c.copy_(p->leaf);
  }
}

void GPT2::save_lora(const std::string& path) {
  std::vector<Tensor> keep;
  std::vector<TensorBlob> blobs;
  for (auto& kv : trainable()) {
    const std::string& name = kv.first;
    if (name.find(".lora_") == std::string::npos) continue;
    const bool isA = name.substr(name.size() - 7) == ".lora_A";
    Tensor src = kv.second->leaf.detach();
    if (isA) src = src.t();  // [r, in] -> reference [in, r]
    Tensor h = empty(src.shape(), DType::F32, Device::cpu());
    h.copy_(src);
    keep.push_back(h);
    blobs.push_back({name, "F32", h.shape(), h.data_ptr(), h.nbytes()});
  }
  auto fmt = [](double x) {
    std::ostringstream os;
    os << x;
    return os.str();
  };
  std::string targets;
  for (size_t i = 0; i < spec_.targets.size(); ++i) targets += (i ? "," : "") + spec_.targets[i];
  safetensors_save(path, blobs,
                   {{"rank", std::to_string(spec_.rank)},
                    {"alpha", fmt(spec_.alpha)},
                    {"dropout", fmt(spec_.dropout)},
                    {"split_qkv", spec_.split_qkv ? "true" : "false"},
                    {"targets", targets}},
                   true, false);
}

void GPT2::merge_lora(float sign) {
  NoGradGuard ng;
  MFT_CHECK(!streamer_, "merge_lora: streamed weights are re-loaded from the host tier (merge before enable_weight_streaming)");
  lora_enabled = sign < 0;
  auto merge = [&](Param& w, std::vector<LoraAdapter>& ads) {
    for (auto& a : ads) {
      Tensor A = a.A.leaf.detach().contiguous(), B = a.B.leaf.detach().contiguous();
      Tensor rows = w.c.slice(0, a.col0, a.col0 + a.ncols);
      ::mft::lora_merge(rows.data_ptr(), w.c.dtype() == DType::BF16 ? 1 : 0, 1, w.c.size(1), A.data<float>(), B.data<float>(), (int)A.size(1), a.ncols,
                        a.rank, sign * spec_.scale(), current_stream());
    }
    w.wt = Tensor();
  };
  for (auto& b : blocks_) {
    merge(b.attn_w, b.lqkv);
    merge(b.proj_w, b.lproj);
    merge(b.fc_w, b.lfc);
    merge(b.mproj_w, b.lfcout);
    b.waug_qkv = Tensor();
    b.waug_proj = Tensor();
  }
}

void GPT2::enable_weight_streaming(size_t budget_bytes, const DiskTier& disk) {
  std::vector<std::vector<Param*>> groups;
  for (auto& b : blocks_) {
    std::vector<Param*> g;
    for (Param* p : {&b.attn_w, &b.attn_b, &b.proj_w, &b.proj_b, &b.fc_w, &b.fc_b, &b.mproj_w, &b.mproj_b})
      if (!p->trainable()) g.push_back(p);
    groups.push_back(g);
    b.waug_qkv = Tensor(), b.waug_proj = Tensor();
  }
  streamer_ = std::make_unique<WeightStreamer>(groups, budget_bytes, disk);
}

// ------------------------------------------------------------------ forward
std::pair<Tensor, Tensor> GPT2::block(int i, const Tensor& x0, const Tensor& h, int64_t B, int64_t S) {
  const int C = cfg_.n_embd, H = cfg_.n_head, D = cfg_.head_dim();
  const float scale = spec_.scale();
  // streamed weights: no resident augmented-K copy [W | s B^T], the adapters run beside the GEMM
  const bool st = streamer_ != nullptr;
  auto aug = [&](std::vector<LoraAdapter>& ads) { return (ads.empty() || st) ? 0 : lora_aug_cols(C, ads); };
  auto& b = blocks_[i];
  Tensor x = x0;
  // attention (u = ln_1(x) A^T of the qkv adapter(s) was written by the LayerNorm that produced h)
  const bool u_ready = !st && !active(b.lqkv).empty() && lora_fused_a(active(b.lqkv), training).defined();
  Tensor qkv = active(b.lqkv).empty() ? linear_p(h, b.attn_w, &b.attn_b)
               : st ? lora_linear(h, b.attn_w, &b.attn_b, active(b.lqkv), scale, training, dropout_ctr)
                    : lora_linear_aug(h, C, b.attn_w, &b.attn_b, active(b.lqkv), scale, b.waug_qkv, training, dropout_ctr,
                                      u_ready);
  Tensor o;
  if (attn_naive) {  // --attn_impl naive: materialized masked softmax on the q / k / v views of qkv
    Tensor q5 = qkv.view({B, S, 3, H, D});
    o = attention_ref(q5.select(2, 0), q5.select(2, 1), q5.select(2, 2), 1.f / std::sqrt((float)D), true, 0);
    o = pad_cols(o.view({B * S, C}), std::max(C, aug(active(b.lproj))));
  } else {
    o = attention_packed(qkv.view({B, S, 3, H, D}), 1.f / std::sqrt((float)D), true, 0, aug(active(b.lproj)));
  }
  o = o.view({B * S, o.size(-1)});
  // The residual adds ride in the producing GEMMs' epilogues where the producer supports it (augmented-K
  // LoRA projection, the fused GELU MLP): s = x + proj(o) comes out of the projection, and the norm that
  // follows reads s alone -- one [M, C] read and one write fewer per add than norm(x + delta)
  const bool fuse_proj = !active(b.lproj).empty() && !st;
  Tensor a = active(b.lproj).empty() ? linear_p(o, b.proj_w, &b.proj_b)
             : st ? lora_linear(o, b.proj_w, &b.proj_b, active(b.lproj), scale, training, dropout_ctr)
                  : lora_linear_aug(o, C, b.proj_w, &b.proj_b, active(b.lproj), scale, b.waug_proj, training, dropout_ctr,
                                    false, x);
  auto r2 = fuse_proj ? add_norm(a, Tensor(), b.ln2_w, &b.ln2_b, cfg_.eps, false, 0.f, 0, Tensor(), true)
                      : add_norm(x, a, b.ln2_w, &b.ln2_b, cfg_.eps, false, 0.f, 0);
  x = r2.first;
  // MLP
  Tensor f;
  bool fuse_mlp = false;
  if (active(b.lfc).empty() && active(b.lfcout).empty()) {
    f = mlp_gelu(r2.second, b.fc_w, b.fc_b, b.mproj_w, b.mproj_b, x);
    fuse_mlp = true;
  } else {
    Tensor u = active(b.lfc).empty() ? linear_p(r2.second, b.fc_w, &b.fc_b)
                             : lora_linear(r2.second, b.fc_w, &b.fc_b, active(b.lfc), scale, training, dropout_ctr);
    u = gelu(u, true);
    f = active(b.lfcout).empty() ? linear_p(u, b.mproj_w, &b.mproj_b)
                         : lora_linear(u, b.mproj_w, &b.mproj_b, active(b.lfcout), scale, training, dropout_ctr);
  }
  Param* nw = i + 1 < cfg_.n_layer ? &blocks_[i + 1].ln1_w : &lnf_w_;
  Param* nb = i + 1 < cfg_.n_layer ? &blocks_[i + 1].ln1_b : &lnf_b_;
  const int oc = i + 1 < cfg_.n_layer ? aug(active(blocks_[i + 1].lqkv)) : 0;
  const Tensor la = oc ? lora_fused_a(active(blocks_[i + 1].lqkv), training) : Tensor();
  if (fuse_mlp) return add_norm(f, Tensor(), *nw, nb, cfg_.eps, false, 0.f, oc, la, true);
  return add_norm(x, f, *nw, nb, cfg_.eps, false, 0.f, oc, la);
}

Tensor GPT2::hidden(const Tensor& ids) {
  if (compute_dtype() == DType::F32) return hidden_ref(ids);
  lora_prep_step_begin();  // every LoRA layer's weight prep for this forward, one launch
  const int64_t B = ids.size(0), S = ids.size(1);
  MFT_CHECK(S <= cfg_.n_positions, "sequence ", S, " exceeds n_positions ", cfg_.n_positions);
  const int C = cfg_.n_embd;
  const bool st = streamer_ != nullptr;
  // block weights that are not resident: the host-streaming tier or the ZeRO-3 partitioner
  BlockProvider* bp = st ? streamer_.get() : provider_;
  if (bp) bp->begin_forward();
  Tensor x = embed(ids, wte_, &wpe_, 1.f);
  const int oc0 = (active(blocks_[0].lqkv).empty() || st) ? 0 : lora_aug_cols(C, active(blocks_[0].lqkv));
  // (resid_out: block 0's residual consumers send their gradient through this norm's backward kernel)
  Tensor h;
  std::tie(x, h) = add_norm(x, Tensor(), blocks_[0].ln1_w, &blocks_[0].ln1_b, cfg_.eps, false, 0.f, oc0,
                            oc0 ? lora_fused_a(active(blocks_[0].lqkv), training) : Tensor(), true);
  const bool ckpt = grad_checkpoint && training && grad_enabled();
  for (int i = 0; i < cfg_.n_layer; ++i) {
    if (bp) bp->ensure(i, i + 1);
    if (ckpt) {
      auto o = checkpoint([this, i, B, S](const std::vector<Tensor>& in) {
        auto r = block(i, in[0], in[1], B, S);
        return std::vector<Tensor>{r.first, r.second};
      }, {x, h});
      x = o[0];
      h = o[1];
    } else {
      std::tie(x, h) = block(i, x, h, B, S);
    }
    if (bp) std::tie(x, h) = bp->gate(x, h, i);
  }
  return h;
}

Tensor GPT2::loss(const Tensor& ids, const Tensor& labels, float w_grad_scale) {
  Tensor h = hidden(ids);
  if (compute_dtype() == DType::F32) {  // full logits + the catalog's cross entropy (mean over valid labels)
    Tensor l = cross_entropy(logits_ref(h), labels.reshape({-1}), -100);
    return loss_sum ? mul(l, valid_count(labels)) : l;
  }
  return lm_head_ce(h, wte_, labels, cfg_.vocab_size, ce_chunk, w_grad_scale, loss_sum);
}

std::pair<Tensor, Tensor> GPT2::nll(const Tensor& ids, const Tensor& labels) {
  NoGradGuard ng;
  const bool t = training;
  training = false;
  Tensor h = hidden(ids);
  lora_prep_step_end();  // no backward follows
  training = t;
  if (compute_dtype() == DType::F32) {
    Tensor cnt = valid_count(labels);
    return {mul(cross_entropy(logits_ref(h), labels.reshape({-1}), -100), cnt), cnt};
  }
  return lm_head_nll(h, wte_, labels, cfg_.vocab_size, ce_chunk);
}

// ------------------------------------------------------------------ composite path (--dtype fp32)
// The reference's forward (graph/gpt2_model.cpp:323-442, :530-817) op by op on fp32 tensors: embedding +
// positions, per block LayerNorm -> qkv (+ LoRA) -> masked-softmax attention -> proj (+ LoRA) -> residual
// -> LayerNorm -> fc (+ LoRA) -> GELU-tanh -> proj (+ LoRA) -> residual, final LayerNorm; the tied LM head
// is the full [M, V] logits GEMM.  Unlike the reference, every op has its backward.
Tensor GPT2::hidden_ref(const Tensor& ids) {
  MFT_CHECK(!streamer_ && !provider_, "--dtype fp32: weight streaming / ZeRO-3 run the bf16 kernels only");
  const int64_t B = ids.size(0), S = ids.size(1);
  MFT_CHECK(S <= cfg_.n_positions, "sequence ", S, " exceeds n_positions ", cfg_.n_positions);
  const int C = cfg_.n_embd, H = cfg_.n_head, D = cfg_.head_dim();
  const float s = spec_.scale();
  const uint64_t step = training ? (uint64_t)dropout_ctr.item() : 0;  // (eager: capturable() is false)
  std::vector<int64_t> pos((size_t)S);
  for (int64_t i = 0; i < S; ++i) pos[(size_t)i] = i;
  Tensor x = add(embedding(ids.reshape({-1}), cw(wte_)).view({B, S, C}), embedding(from_vector(pos, {S}, DType::I64), cw(wpe_)));
  x = x.reshape({B * S, C});
  for (int i = 0; i < cfg_.n_layer; ++i) {
    auto& b = blocks_[i];
    Tensor h = layer_norm(x, cw(b.ln1_w), cw(b.ln1_b), cfg_.eps);
    Tensor qkv = lora_linear_ref(h, b.attn_w, &b.attn_b, active(b.lqkv), s, training, step).view({B, S, 3, H, D});
    Tensor o = attention_ref(qkv.select(2, 0), qkv.select(2, 1), qkv.select(2, 2), 1.f / std::sqrt((float)D), true, 0);
    x = add(x, lora_linear_ref(o.reshape({B * S, C}), b.proj_w, &b.proj_b, active(b.lproj), s, training, step));
    h = layer_norm(x, cw(b.ln2_w), cw(b.ln2_b), cfg_.eps);
    Tensor u = gelu(lora_linear_ref(h, b.fc_w, &b.fc_b, active(b.lfc), s, training, step), true);
    x = add(x, lora_linear_ref(u, b.mproj_w, &b.mproj_b, active(b.lfcout), s, training, step));
  }
  return layer_norm(x, cw(lnf_w_), cw(lnf_b_), cfg_.eps);
}

Tensor GPT2::logits_ref(const Tensor& h) { return matmul(h, cw(wte_).slice(0, 0, cfg_.vocab_size).t()); }

}  // namespace eng
}  // namespace mft
