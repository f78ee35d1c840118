// libmft engine: Gemma-3 model (see gemma3.h).
#include "engine/gemma3.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <regex>
#include <set>
#include <sstream>
#include <tuple>

#include "engine/autograd.h"
#include "engine/gemm.h"
#include "engine/ops.h"
#include "kernels.h"
#include "runtime/json.h"
#include "runtime/safetensors.h"

namespace mft {
namespace eng {

// ------------------------------------------------------------------ config
namespace {
std::vector<bool> pattern_sliding(int n, int pattern) {
  std::vector<bool> s(n);
  for (int i = 0; i < n; ++i) s[i] = (i + 1) % pattern != 0;  // every pattern-th layer is global
  return s;
}
}  // namespace

Gemma3Config Gemma3Config::preset(const std::string& n0) {
  std::string n = n0;
  for (auto& c : n) c = (c == '_') ? '-' : (char)std::tolower(c);
  Gemma3Config c;
  if (n == "gemma3-270m" || n == "gemma-3-270m" || n == "gemma3") {
    // defaults
  } else if (n == "gemma3-1b" || n == "gemma-3-1b") {
    c.hidden = 1152, c.intermediate = 6912, c.n_layer = 26;
  } else if (n == "gemma3-tiny") {
    c.vocab_size = 1024, c.hidden = 128, c.intermediate = 256, c.n_layer = 3, c.n_head = 4, c.n_kv = 2;
    c.head_dim = 64, c.sliding_window = 16, c.max_positions = 512, c.query_pre_attn_scalar = 64.f;
    c.sliding = {true, true, false};
  } else {
    MFT_CHECK(false, "unknown Gemma-3 preset '", n0, "' (gemma3-270m, gemma3-1b, gemma3-tiny)");
  }
  if (c.sliding.empty()) c.sliding = pattern_sliding(c.n_layer, 6);
  return c;
}

Gemma3Config Gemma3Config::from_json(const std::string& path) {
  std::ifstream f(path);
  MFT_CHECK(f.good(), "cannot open ", path);
  std::stringstream ss;
  ss << f.rdbuf();
  json::Value root = json::parse(ss.str());
  const json::Value& v = root.get("text_config") ? root["text_config"] : root;
  Gemma3Config c;
  auto gi = [&](const char* k, int d) { return v.get(k) && v[k].is_number() ? (int)v[k].as_int() : d; };
  auto gf = [&](const char* k, float d) { return v.get(k) && v[k].is_number() ? (float)v[k].as_double() : d; };
  c.vocab_size = gi("vocab_size", c.vocab_size);
  c.hidden = gi("hidden_size", c.hidden);
  c.intermediate = gi("intermediate_size", c.intermediate);
  c.n_layer = gi("num_hidden_layers", c.n_layer);
  c.n_head = gi("num_attention_heads", c.n_head);
  c.n_kv = gi("num_key_value_heads", c.n_kv);
  c.head_dim = gi("head_dim", c.head_dim);
  c.eps = gf("rms_norm_eps", c.eps);
  c.sliding_window = gi("sliding_window", c.sliding_window);
  c.query_pre_attn_scalar = gf("query_pre_attn_scalar", c.query_pre_attn_scalar);
  c.max_positions = gi("max_position_embeddings", c.max_positions);
  c.rope_theta = gf("rope_theta", c.rope_theta);
  c.rope_local = gf("rope_local_base_freq", c.rope_local);
  c.init_range = gf("initializer_range", c.init_range);
  c.bos_id = gi("bos_token_id", c.bos_id);
  c.eos_id = gi("eos_token_id", c.eos_id);
  c.pad_id = gi("pad_token_id", c.pad_id);
  if (v.get("hidden_activation") && v["hidden_activation"].is_string()) {
    const std::string a = v["hidden_activation"].as_string();
    c.act = (a == "silu" || a == "swish") ? 1 : 0;
  }
  if (const json::Value* rs = v.get("rope_scaling")) {
    if (rs->is_object()) {
      const json::Value* t = rs->get("rope_type") ? rs->get("rope_type") : rs->get("type");
      if (t && t->is_string() && t->as_string() == "linear" && rs->get("factor"))
        c.rope_scaling = (float)(*rs)["factor"].as_double();
    }
  }
  if (const json::Value* rp = v.get("rope_parameters")) {  // transformers >= 5 layout
    if (const json::Value* full = rp->get("full_attention")) {
      if (full->get("rope_theta")) c.rope_theta = (float)(*full)["rope_theta"].as_double();
      const json::Value* t = full->get("rope_type");
      if (t && t->is_string() && t->as_string() == "linear" && full->get("factor"))
        c.rope_scaling = (float)(*full)["factor"].as_double();
    }
    if (const json::Value* sl = rp->get("sliding_attention"))
      if (sl->get("rope_theta")) c.rope_local = (float)(*sl)["rope_theta"].as_double();
  }
  c.sliding.clear();
  if (const json::Value* lt = v.get("layer_types")) {
    if (lt->is_array())
      for (auto& e : lt->as_array()) c.sliding.push_back(e.is_string() && e.as_string() == "sliding_attention");
  }
  if ((int)c.sliding.size() != c.n_layer) c.sliding = pattern_sliding(c.n_layer, gi("sliding_window_pattern", 6));
  return c;
}

bool GemmaLoraSpec::has(const std::string& t) const {
  return std::find(targets.begin(), targets.end(), t) != targets.end();
}

std::vector<std::string> GemmaLoraSpec::parse_targets(const std::string& s0) {
  static const std::vector<std::string> all{"q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"};
  std::string key = s0;
  for (auto& c : key) c = (char)std::tolower(c);
  key.erase(std::remove_if(key.begin(), key.end(), ::isspace), key.end());
  if (key == "full" || key == "full_attn_mlp") return all;
  if (key == "attn" || key == "attention_only") return {"q_proj", "k_proj", "v_proj", "o_proj"};
  if (key == "light" || key == "attention_light") return {"q_proj", "v_proj"};
  std::vector<std::string> out;
  std::stringstream ss(key);
  std::string item;
  while (std::getline(ss, item, ',')) {
    if (item.empty()) continue;
    if (item.size() < 5 || item.substr(item.size() - 5) != "_proj") item += "_proj";
    MFT_CHECK(std::find(all.begin(), all.end(), item) != all.end(), "unknown Gemma LoRA target '", item, "'");
    if (std::find(out.begin(), out.end(), item) == out.end()) out.push_back(item);
  }
  return out;
}

// ------------------------------------------------------------------ model
namespace {
Param frozen(Tensor t) {
  Param p;
  p.leaf = t;
  p.c = t;
  return p;
}
DType st_dtype(const std::string& d) {
  if (d == "F32") return DType::F32;
  if (d == "BF16") return DType::BF16;
  if (d == "F16") return DType::F16;
  MFT_CHECK(false, "safetensors: unsupported dtype ", d);
  return DType::F32;
}
float bf16_round(float x) {  // round-to-nearest-even to bf16 (the Python model's embed_scale)
  uint32_t u;
  std::memcpy(&u, &x, 4);
  u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
  float r;
  std::memcpy(&r, &u, 4);
  return r;
}
}  // namespace

Gemma3::Gemma3(const Gemma3Config& cfg) : cfg_(cfg) { alloc(); }

void Gemma3::alloc() {
  const int H = cfg_.hidden, D = cfg_.head_dim, I = cfg_.intermediate;
  const int nqkv = (cfg_.n_head + 2 * cfg_.n_kv) * D;
  MFT_CHECK((int)cfg_.sliding.size() == cfg_.n_layer, "gemma3: layer types do not match num_hidden_layers");
  NoGradGuard ng;
  const DType wd = compute_dtype();  // bf16, or fp32 for --dtype fp32 (norm weights are fp32 either way)
  embed_ = frozen(zeros({cfg_.vocab_padded(), H}, wd));
  final_norm_ = frozen(zeros({H}, DType::F32));
  layers_.resize(cfg_.n_layer);
  for (int i = 0; i < cfg_.n_layer; ++i) {
    auto& L = layers_[i];
    L.sliding = cfg_.sliding[i];
    L.in_norm = frozen(zeros({H}, DType::F32));
    L.qkv_w = frozen(zeros({nqkv, H}, wd));
    L.o_w = frozen(zeros({H, cfg_.n_head * D}, wd));
    L.q_norm = frozen(zeros({D}, DType::F32));
    L.k_norm = frozen(zeros({D}, DType::F32));
    L.post_attn_norm = frozen(zeros({H}, DType::F32));
    L.pre_ff_norm = frozen(zeros({H}, DType::F32));
    L.gu_w = frozen(zeros({2 * I, H}, wd));
    L.down_w = frozen(zeros({H, I}, wd));
    L.post_ff_norm = frozen(zeros({H}, DType::F32));
  }
  dropout_ctr = zeros({1}, DType::I64);
  ce_chunk = default_ce_chunk(cfg_.vocab_padded());
  // (the bf16 model rounds sqrt(H) to bf16 like HF does in that dtype; fp32 keeps it exact)
  embed_scale_ = wd == DType::F32 ? std::sqrt((float)H) : bf16_round(std::sqrt((float)H));
  rope_len_ = std::min(cfg_.max_positions, 4096);
}

void Gemma3::init_random(uint64_t seed) {
  NoGradGuard ng;
  uint64_t s = seed * 1000003ull + 29;
  auto nrm = [&](Param& p) { p.c.copy_(randn(p.c.shape(), ++s, cfg_.init_range, DType::F32)); };
  nrm(embed_);
  embed_.c.slice(0, cfg_.vocab_size, cfg_.vocab_padded()).zero_();
  for (auto& L : layers_) {
    nrm(L.qkv_w);
    nrm(L.o_w);
    nrm(L.gu_w);
    nrm(L.down_w);
  }
}

void Gemma3::load_hf(const std::string& dir) {
  NoGradGuard ng;
  // one file, or the shards of model.safetensors.index.json
  std::vector<std::string> files;
  if (dir.size() >= 12 && dir.substr(dir.size() - 12) == ".safetensors") {
    files.push_back(dir);
  } else {
    std::ifstream idx(dir + "/model.safetensors.index.json");
    if (idx.good()) {
      std::stringstream ss;
      ss << idx.rdbuf();
      json::Value v = json::parse(ss.str());
      std::set<std::string> seen;
      for (auto& kv : v["weight_map"].as_object())
        if (seen.insert(kv.second.as_string()).second) files.push_back(dir + "/" + kv.second.as_string());
    } else {
      files.push_back(dir + "/model.safetensors");
    }
  }
  std::vector<std::unique_ptr<SafeTensorsFile>> fs;
  for (auto& p : files) fs.push_back(std::make_unique<SafeTensorsFile>(p));
  auto find = [&](const std::string& k) -> std::pair<SafeTensorsFile*, const TensorInfo*> {
    for (const char* pre : {"", "model.", "model.language_model.", "language_model.model."})
      for (auto& f : fs)
        if (f->has(pre + k)) return {f.get(), &f->info(pre + k)};
    MFT_CHECK(false, "Gemma checkpoint under ", dir, " has no tensor '", k, "'");
    return {nullptr, nullptr};
  };
  // copy tensor `key` into rows [r0, r0 + rows) of dst (host cast to fp32, then device cast)
  auto load_rows = [&](const Tensor& dst, const std::string& key, int64_t r0) {
    auto ft = find(key);
    const TensorInfo* ti = ft.second;
    Tensor host = from_blob(const_cast<void*>(ft.first->data(ti->name)), ti->shape, st_dtype(ti->dtype), Device::cpu());
    const int64_t rows = ti->shape.empty() ? 1 : ti->shape[0];
    Tensor d = dst.slice(0, r0, r0 + rows);
    MFT_CHECK(host.numel() == d.numel(), "Gemma tensor '", key, "' ", shape_str(ti->shape), " does not fit ", d.str());
    Tensor staged = empty(host.shape(), DType::F32, Device::cpu());
    staged.copy_(host);
    d.copy_(staged.view(d.shape()));
  };
  load_rows(embed_.c, "embed_tokens.weight", 0);
  const int qd = cfg_.n_head * cfg_.head_dim, kd = cfg_.n_kv * cfg_.head_dim;
  for (int i = 0; i < cfg_.n_layer; ++i) {
    auto& L = layers_[i];
    const std::string p = "layers." + std::to_string(i) + ".";
    load_rows(L.qkv_w.c, p + "self_attn.q_proj.weight", 0);
    load_rows(L.qkv_w.c, p + "self_attn.k_proj.weight", qd);
    load_rows(L.qkv_w.c, p + "self_attn.v_proj.weight", qd + kd);
    load_rows(L.o_w.c, p + "self_attn.o_proj.weight", 0);
    load_rows(L.q_norm.c, p + "self_attn.q_norm.weight", 0);
    load_rows(L.k_norm.c, p + "self_attn.k_norm.weight", 0);
    load_rows(L.gu_w.c, p + "mlp.gate_proj.weight", 0);
    load_rows(L.gu_w.c, p + "mlp.up_proj.weight", cfg_.intermediate);
    load_rows(L.down_w.c, p + "mlp.down_proj.weight", 0);
    load_rows(L.in_norm.c, p + "input_layernorm.weight", 0);
    load_rows(L.post_attn_norm.c, p + "post_attention_layernorm.weight", 0);
    load_rows(L.pre_ff_norm.c, p + "pre_feedforward_layernorm.weight", 0);
    load_rows(L.post_ff_norm.c, p + "post_feedforward_layernorm.weight", 0);
    L.waug_qkv = L.waug_o = L.waug_gu = L.waug_down = Tensor();
  }
  load_rows(final_norm_.c, "norm.weight", 0);
  synchronize();
}

size_t Gemma3::num_parameters() const {
  const int H = cfg_.hidden, D = cfg_.head_dim, I = cfg_.intermediate;
  const size_t per = (size_t)(cfg_.n_head + 2 * cfg_.n_kv) * D * H + (size_t)cfg_.n_head * D * H + 3ull * I * H +
                     2ull * D + 4ull * H;
  return (size_t)cfg_.vocab_size * H + per * cfg_.n_layer + H;
}

// ------------------------------------------------------------------ LoRA
void Gemma3::inject_lora(const GemmaLoraSpec& spec) {
  spec_ = spec;
  const int H = cfg_.hidden, D = cfg_.head_dim, I = cfg_.intermediate;
  const int qd = cfg_.n_head * D, kd = cfg_.n_kv * D;
  std::vector<int> layers = spec.layers;
  if (layers.empty())
    for (int i = 0; i < cfg_.n_layer; ++i) layers.push_back(i);
  uint64_t s = spec.seed;
  for (int i : layers) {
    auto& L = layers_[i];
    const std::string pre = "layer." + std::to_string(i) + ".";
    auto add = [&](std::vector<LoraAdapter>& ads, std::vector<std::string>& names, int col0, int n, int in,
                   const std::string& nm) {
      // PEFT init (reference gemma_lora_injector.cpp:30-46): A [r, in] ~ U(+-1/sqrt(in)), B = 0
      const float bound = 1.f / std::sqrt((float)in);
      Tensor A = rand_uniform({spec.rank, in}, ++s * 7919ull + (uint64_t)i, -bound, bound, DType::F32);
      ads.push_back(make_adapter(col0, n, spec.rank, A, spec.dropout, pre + nm));
      names.push_back(pre + nm);
    };
    if (spec.has("q_proj")) add(L.lqkv, L.names_qkv, 0, qd, H, "attn.q");
    if (spec.has("k_proj")) add(L.lqkv, L.names_qkv, qd, kd, H, "attn.k");
    if (spec.has("v_proj")) add(L.lqkv, L.names_qkv, qd + kd, kd, H, "attn.v");
    if (spec.has("o_proj")) add(L.lo, L.names_o, 0, H, qd, "attn.proj");
    if (spec.has("gate_proj")) add(L.lgu, L.names_gu, 0, I, H, "mlp.gate");
    if (spec.has("up_proj")) add(L.lgu, L.names_gu, I, I, H, "mlp.up");
    if (spec.has("down_proj")) add(L.ldown, L.names_down, 0, H, I, "mlp.down");
  }
}

std::vector<std::pair<std::string, Param*>> Gemma3::trainable() {
  std::vector<std::pair<std::string, Param*>> v;
  for (auto& L : layers_) {
    auto add = [&](std::vector<LoraAdapter>& ads, std::vector<std::string>& names) {
      for (size_t j = 0; j < ads.size(); ++j) {
        v.push_back({names[j] + ".lora_A", &ads[j].A});
        v.push_back({names[j] + ".lora_B", &ads[j].B});
      }
    };
    add(L.lqkv, L.names_qkv);
    add(L.lo, L.names_o);
    add(L.lgu, L.names_gu);
    add(L.ldown, L.names_down);
  }
  return v;
}

void Gemma3::load_lora(const std::string& path) {
  SafeTensorsFile f(path);
  const auto& meta = f.metadata();
  auto mget = [&](const char* k) -> std::string {
    auto it = meta.find(k);
    return it == meta.end() ? "" : it->second;
  };
  std::map<std::string, const TensorInfo*> A, B;
  std::regex re(R"(layer\.(\d+)\.(attn\.q|attn\.k|attn\.v|attn\.proj|mlp\.gate|mlp\.up|mlp\.down)\.lora_(A|B))");
  std::set<int> layers;
  std::set<std::string> parts;
  for (auto& ti : f.tensors()) {
    std::smatch m;
    if (!std::regex_match(ti.name, m, re)) continue;
    (m[3].str() == "A" ? A : B)["layer." + m[1].str() + "." + m[2].str()] = &ti;
    layers.insert(std::stoi(m[1].str()));
    parts.insert(m[2].str());
  }
  MFT_CHECK(!A.empty(), "no Gemma LoRA tensors in ", path);
  GemmaLoraSpec spec;
  spec.rank = mget("rank").empty() ? (int)A.begin()->second->shape[0] : std::stoi(mget("rank"));
  spec.alpha = mget("alpha").empty() ? 2.f * spec.rank : std::stof(mget("alpha"));
  spec.dropout = mget("dropout").empty() ? 0.f : std::stof(mget("dropout"));
  spec.targets.clear();
  const std::pair<const char*, const char*> names[] = {{"attn.q", "q_proj"},   {"attn.k", "k_proj"},
                                                       {"attn.v", "v_proj"},   {"attn.proj", "o_proj"},
                                                       {"mlp.gate", "gate_proj"}, {"mlp.up", "up_proj"},
                                                       {"mlp.down", "down_proj"}};
  for (auto& nm : names)
    if (parts.count(nm.first)) spec.targets.push_back(nm.second);
  spec.layers.assign(layers.begin(), layers.end());
  for (auto& L : layers_) {
    L.lqkv.clear(), L.lo.clear(), L.lgu.clear(), L.ldown.clear();
    L.names_qkv.clear(), L.names_o.clear(), L.names_gu.clear(), L.names_down.clear();
    L.waug_qkv = L.waug_o = L.waug_gu = L.waug_down = Tensor();
  }
  inject_lora(spec);
  NoGradGuard ng;
  for (auto& kv : trainable()) {
    const std::string& name = kv.first;
    const bool isA = name.substr(name.size() - 7) == ".lora_A";
    const std::string stem = name.substr(0, name.size() - 7);
    auto& mp = isA ? A : B;
    auto it = mp.find(stem);
    MFT_CHECK(it != mp.end(), "Gemma LoRA checkpoint lacks ", name);
    const TensorInfo* ti = it->second;
    Tensor host = from_blob(const_cast<void*>(f.data(ti->name)), ti->shape, st_dtype(ti->dtype), Device::cpu());
    Tensor src = isA ? host : host.t();  // A [r, in] as stored; B [out, r] -> [r, out]
    Tensor staged = empty(src.shape(), DType::F32, Device::cpu());
    staged.copy_(src);
    Param* p = kv.second;
    MFT_CHECK(staged.numel() == p->leaf.numel() && staged.size(0) == p->leaf.size(0), "Gemma LoRA tensor ", name,
              " shape ", shape_str(ti->shape), " does not fit ", p->leaf.str());
    p->leaf.copy_(staged);
    p->c.copy_(p->leaf);
  }
}

void Gemma3::save_lora(const std::string& path) {
  std::vector<Tensor> keep;
  std::vector<TensorBlob> blobs;
  std::set<std::string> present;
  for (auto& kv : trainable()) {
    const std::string& name = kv.first;
    const bool isA = name.substr(name.size() - 7) == ".lora_A";
    Tensor src = kv.second->leaf.detach();
    if (!isA) src = src.t();  // [r, out] -> PEFT [out, r]
    Tensor h = empty(src.shape(), DType::F32, Device::cpu());
    h.copy_(src);
    keep.push_back(h);
    blobs.push_back({name, "F32", h.shape(), h.data_ptr(), h.nbytes()});
    const size_t d1 = name.find('.', 6);
    present.insert(name.substr(d1 + 1, name.size() - 7 - d1 - 1));
  }
  std::string targets;
  for (const char* t : {"attn.q", "attn.k", "attn.v", "attn.proj", "mlp.gate", "mlp.up", "mlp.down"})
    if (present.count(t)) targets += (targets.empty() ? "" : ",") + std::string(t);
  auto fmt = [](double x) {
    std::ostringstream os;
    os << x;
    return os.str();
  };
  safetensors_save(path, blobs,
                   {{"rank", std::to_string(spec_.rank)},
                    {"alpha", fmt(spec_.alpha)},
                    {"dropout", fmt(spec_.dropout)},
                    {"targets", targets}},
                   true, false);
}

void Gemma3::merge_lora(float sign) {
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
  for (auto& L : layers_) {
    merge(L.qkv_w, L.lqkv);
    merge(L.o_w, L.lo);
    merge(L.gu_w, L.lgu);
    merge(L.down_w, L.ldown);
    L.waug_qkv = L.waug_o = L.waug_gu = L.waug_down = Tensor();
  }
}

void Gemma3::enable_weight_streaming(size_t budget_bytes, const DiskTier& disk) {
  std::vector<std::vector<Param*>> groups;
  for (auto& L : layers_) {
    groups.push_back({&L.qkv_w, &L.o_w, &L.gu_w, &L.down_w});
    L.waug_qkv = L.waug_o = L.waug_gu = L.waug_down = Tensor();
  }
  streamer_ = std::make_unique<WeightStreamer>(groups, budget_bytes, disk);
}

// ------------------------------------------------------------------ forward
std::pair<Tensor, Tensor> Gemma3::rope(bool local, int S) {
  const int key = local ? 1 : 0;
  auto it = rope_.find(key);
  if (it != rope_.end() && it->second.first.size(0) >= S) return it->second;
  // HF default rope in fp64 on the host (ops/rope_tables.py): f = (pos / scaling) * theta^(-2j/D)
  const int n = std::max(S, rope_len_), half = cfg_.head_dim / 2;
  const double theta = local ? cfg_.rope_local : cfg_.rope_theta, sc = local ? 1.0 : cfg_.rope_scaling;
  std::vector<float> c((size_t)n * half), s((size_t)n * half);
  for (int p = 0; p < n; ++p)
    for (int j = 0; j < half; ++j) {
      const double inv = 1.0 / std::pow(theta, (2.0 * j) / cfg_.head_dim);
      const double f = ((double)p / sc) * inv;
      c[(size_t)p * half + j] = (float)std::cos(f);
      s[(size_t)p * half + j] = (float)std::sin(f);
    }
  NoGradGuard ng;
  auto t = std::make_pair(from_host(c.data(), {n, half}, DType::F32), from_host(s.data(), {n, half}, DType::F32));
  rope_[key] = t;
  return t;
}

std::pair<Tensor, Tensor> Gemma3::layer(int i, const Tensor& x0, const Tensor& h, int64_t B, int64_t S) {
  const int H = cfg_.hidden, D = cfg_.head_dim, nq = cfg_.n_head, nkv = cfg_.n_kv, I = cfg_.intermediate;
  const float s = spec_.scale(), eps = cfg_.eps;
  const float attn_scale = 1.f / std::sqrt(cfg_.query_pre_attn_scalar);
  // streamed weights: no resident augmented-K copy [W | s B^T], the adapters run beside the GEMM
  const bool st = streamer_ != nullptr;
  auto aug = [&](std::vector<LoraAdapter>& ads, int in) { return (ads.empty() || st) ? 0 : lora_aug_cols(in, ads); };
  // the fused A stack when the producing RMSNorm computes u = y A^T itself (no dropout, sum r <= 32)
  auto fused_a = [&](std::vector<LoraAdapter>& ads) { return (ads.empty() || st) ? Tensor() : lora_fused_a(ads, training); };
  // (geglu_h / geglu_gu: the GeGLU MLP fused into the gate|up and down GEMM epilogues, nn.h linear_p)
  auto proj = [&](const Tensor& x, int K, Param& w, std::vector<LoraAdapter>& ads, Tensor& waug, bool u_ready,
                  Tensor* geglu_h = nullptr, const Tensor& geglu_gu = Tensor()) {
    if (ads.empty()) return linear_p(x, w, nullptr, geglu_h, geglu_gu);
    if (st) return lora_linear(x, w, nullptr, ads, s, training, dropout_ctr);
    return lora_linear_aug(x, K, w, nullptr, ads, s, waug, training, dropout_ctr, u_ready, Tensor(), geglu_h, geglu_gu);
  };
  auto& L = layers_[i];
  const auto cs = rope(L.sliding, (int)S);
  Tensor x = x0;
  // attention
  Tensor qkv = proj(h, H, L.qkv_w, active(L.lqkv), L.waug_qkv, fused_a(active(L.lqkv)).defined()).view({B, S, nq + 2 * nkv, D});
  Tensor o;
  if (attn_naive) {  // --attn_impl naive: per-head RMSNorm + RoPE + materialized GQA masked softmax
    Tensor q = rms_norm(qkv.slice(2, 0, nq), L.q_norm.c.to(qkv.dtype()), eps, 1.f);
    Tensor k = rms_norm(qkv.slice(2, nq, nq + nkv), L.k_norm.c.to(qkv.dtype()), eps, 1.f);
    Tensor c = cs.first.slice(0, 0, S), sn = cs.second.slice(0, 0, S);
    q = apply_rope(q, c, sn, interleaved_rope);
    k = apply_rope(k, c, sn, interleaved_rope);
    o = attention_ref(q, k, qkv.slice(2, nq + nkv, nq + 2 * nkv), attn_scale, true, L.sliding ? cfg_.sliding_window : 0);
    o = pad_cols(o.view({B * S, nq * D}), std::max(nq * D, aug(active(L.lo), nq * D)));
  } else {
    o = qknorm_rope_attention(qkv, nq, nkv, L.q_norm, L.k_norm, cs.first, cs.second, eps, 1.f, interleaved_rope,
                              attn_scale, L.sliding ? cfg_.sliding_window : 0, aug(active(L.lo), nq * D));
  }
  o = o.view({B * S, o.size(-1)});
  Tensor a = proj(o, nq * D, L.o_w, active(L.lo), L.waug_o, false);
  a = add_norm(a, Tensor(), L.post_attn_norm, nullptr, eps, true, 1.f, 0).second;
  const Tensor agu = fused_a(active(L.lgu));
  auto r = add_norm(x, a, L.pre_ff_norm, nullptr, eps, true, 1.f, aug(active(L.lgu), H), agu);
  x = r.first;
  // GeGLU MLP: h = gelu(g) u comes out of the gate|up GEMM's epilogue and d gu out of the down data
  // gradient's (no gated_fwd / gated_bwd pass over [M, 2I]); else the gated_act kernels
  const int64_t M = B * S;
  const int hc = std::max(I, aug(active(L.ldown), I));  // h with the down adapter's augmented columns
  const int64_t Kgu = active(L.lgu).empty() || st ? H : aug(active(L.lgu), H);
  Tensor f;
  if (!st && cfg_.act == 0 && geglu_fusable(M, I, Kgu, H)) {
    Tensor hbuf = empty({M, (int64_t)hc}, DType::BF16, x.device());
    if (hc > I) ::mft::zero_cols((::mft::bf16_t*)hbuf.data_ptr(), hc, M, I, hc - I, current_stream());
    Tensor gu = proj(r.second, H, L.gu_w, active(L.lgu), L.waug_gu, agu.defined(), &hbuf);
    f = proj(hbuf, I, L.down_w, active(L.ldown), L.waug_down, false, nullptr, gu);
  } else {
    Tensor gu = proj(r.second, H, L.gu_w, active(L.lgu), L.waug_gu, agu.defined());
    Tensor g = gated_act(gu, cfg_.act, aug(active(L.ldown), I));
    f = proj(g, I, L.down_w, active(L.ldown), L.waug_down, false);
  }
  f = add_norm(f, Tensor(), L.post_ff_norm, nullptr, eps, true, 1.f, 0).second;
  if (!capture_layers.empty() && std::find(capture_layers.begin(), capture_layers.end(), i) != capture_layers.end()) {
    NoGradGuard ng;
    captured[i] = f.detach().clone();
  }
  Param& nw = i + 1 < cfg_.n_layer ? layers_[i + 1].in_norm : final_norm_;
  const int oc = i + 1 < cfg_.n_layer ? aug(active(layers_[i + 1].lqkv), H) : 0;
  return add_norm(x, f, nw, nullptr, eps, true, 1.f, oc, oc ? fused_a(active(layers_[i + 1].lqkv)) : Tensor());
}

Tensor Gemma3::embed_tokens(const Tensor& ids) {
  NoGradGuard ng;
  return embed(ids, embed_, nullptr, embed_scale_);
}

Tensor Gemma3::hidden(const Tensor& ids) {
  if (compute_dtype() == DType::F32) return hidden_ref(ids);
  lora_prep_step_begin();  // every LoRA layer's weight prep for this forward, one launch
  const int64_t B = ids.size(0), S = ids.size(1);
  const int H = cfg_.hidden;
  const bool st = streamer_ != nullptr;
  rope(false, (int)S), rope(true, (int)S);  // tables before any capture / checkpoint
  Tensor x = embed(ids, embed_, nullptr, embed_scale_);
  const int oc0 = (active(layers_[0].lqkv).empty() || st) ? 0 : lora_aug_cols(H, active(layers_[0].lqkv));
  Tensor h = add_norm(x, Tensor(), layers_[0].in_norm, nullptr, cfg_.eps, true, 1.f, oc0,
                      oc0 ? lora_fused_a(active(layers_[0].lqkv), training) : Tensor())
                 .second;
  const bool ckpt = grad_checkpoint && training && grad_enabled();
  for (int i = 0; i < cfg_.n_layer; ++i) {
    if (st) streamer_->ensure(i, i + 1);
    if (ckpt) {
      auto o = checkpoint([this, i, B, S](const std::vector<Tensor>& in) {
        auto r = layer(i, in[0], in[1], B, S);
        return std::vector<Tensor>{r.first, r.second};
      }, {x, h});
      x = o[0];
      h = o[1];
    } else {
      std::tie(x, h) = layer(i, x, h, B, S);
    }
    if (st) std::tie(x, h) = streamer_->gate(x, h, i);
  }
  return h;
}

Tensor Gemma3::loss(const Tensor& ids, const Tensor& labels, float w_grad_scale) {
  Tensor h = hidden(ids);
  if (compute_dtype() == DType::F32) {
    Tensor l = cross_entropy(logits_ref(h), labels.reshape({-1}), -100);
    return loss_sum ? mul(l, valid_count(labels)) : l;
  }
  return lm_head_ce(h, embed_, labels, cfg_.vocab_size, ce_chunk, w_grad_scale, loss_sum);
}

std::pair<Tensor, Tensor> Gemma3::nll(const Tensor& ids, const Tensor& labels) {
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
  return lm_head_nll(h, embed_, labels, cfg_.vocab_size, ce_chunk);
}

// ------------------------------------------------------------------ composite path (--dtype fp32)
// The reference's Gemma-3 forward (graph/gemma_model.cpp:179-944) op by op on fp32 tensors: scaled
// embedding, per layer RMSNorm(1 + w) -> q|k|v (+ LoRA) -> q / k RMSNorm over head_dim -> RoPE (rotate-half,
// or the reference's interleaved pairs) -> GQA masked softmax (sliding window on local layers) -> o (+ LoRA)
// -> post-attention norm -> residual -> pre-FF norm -> gate|up (+ LoRA) -> GeGLU -> down (+ LoRA) ->
// post-FF norm -> residual; final norm; tied LM head (no transposed copy kept).
Tensor Gemma3::hidden_ref(const Tensor& ids) {
  MFT_CHECK(!streamer_, "--dtype fp32: weight streaming runs the bf16 kernels only");
  const int64_t B = ids.size(0), S = ids.size(1);
  const int H = cfg_.hidden, D = cfg_.head_dim, nq = cfg_.n_head, nkv = cfg_.n_kv, I = cfg_.intermediate;
  const float s = spec_.scale(), eps = cfg_.eps, attn_scale = 1.f / std::sqrt(cfg_.query_pre_attn_scalar);
  const uint64_t step = training ? (uint64_t)dropout_ctr.item() : 0;
  rope(false, (int)S), rope(true, (int)S);
  Tensor x = mul_scalar(embedding(ids.reshape({-1}), cw(embed_)), embed_scale_);
  for (int i = 0; i < cfg_.n_layer; ++i) {
    auto& L = layers_[i];
    const auto cs = rope(L.sliding, (int)S);
    Tensor c = cs.first.slice(0, 0, S), sn = cs.second.slice(0, 0, S);
    Tensor h = rms_norm(x, cw(L.in_norm), eps, 1.f);
    Tensor qkv = lora_linear_ref(h, L.qkv_w, nullptr, active(L.lqkv), s, training, step).view({B, S, nq + 2 * nkv, D});
    Tensor q = apply_rope(rms_norm(qkv.slice(2, 0, nq), cw(L.q_norm), eps, 1.f), c, sn, interleaved_rope);
    Tensor k = apply_rope(rms_norm(qkv.slice(2, nq, nq + nkv), cw(L.k_norm), eps, 1.f), c, sn, interleaved_rope);
    Tensor o = attention_ref(q, k, qkv.slice(2, nq + nkv, nq + 2 * nkv), attn_scale, true,
                             L.sliding ? cfg_.sliding_window : 0);
    Tensor a = lora_linear_ref(o.reshape({B * S, nq * D}), L.o_w, nullptr, active(L.lo), s, training, step);
    x = add(x, rms_norm(a, cw(L.post_attn_norm), eps, 1.f));
    h = rms_norm(x, cw(L.pre_ff_norm), eps, 1.f);
    Tensor gu = lora_linear_ref(h, L.gu_w, nullptr, active(L.lgu), s, training, step);
    Tensor g = cfg_.act == 1 ? swiglu(gu.slice(1, 0, I), gu.slice(1, I, 2 * I)) : geglu(gu.slice(1, 0, I), gu.slice(1, I, 2 * I));
    Tensor f = rms_norm(lora_linear_ref(g, L.down_w, nullptr, active(L.ldown), s, training, step), cw(L.post_ff_norm), eps, 1.f);
    if (!capture_layers.empty() && std::find(capture_layers.begin(), capture_layers.end(), i) != capture_layers.end()) {
      NoGradGuard ng;
      captured[i] = f.detach().clone();
    }
    x = add(x, f);
  }
  return rms_norm(x, cw(final_norm_), eps, 1.f);
}

Tensor Gemma3::logits_ref(const Tensor& h) { return matmul(h, cw(embed_).slice(0, 0, cfg_.vocab_size).t()); }

}  // namespace eng
}  // namespace mft
