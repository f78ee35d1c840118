#include "dataset.h"

#include <algorithm>
#include <cctype>
#include <fstream>
#include <numeric>
#include <sstream>
#include <stdexcept>
#include <thread>

#include "json.h"

namespace mft {

static std::string trim(const std::string& s) {
  size_t l = 0, r = s.size();
  while (l < r && std::isspace((unsigned char)s[l])) ++l;
  while (r > l && std::isspace((unsigned char)s[r - 1])) --r;
  return s.substr(l, r - l);
}

std::vector<std::string> read_lines(const std::string& path, bool keep_blank) {
  std::ifstream in(path);
  if (!in) throw std::runtime_error("dataset: cannot open " + path);
  std::vector<std::string> lines;
  std::string line;
  while (std::getline(in, line)) {
    if (!keep_blank && trim(line).empty()) continue;
    lines.push_back(line);
  }
  return lines;
}

std::vector<int32_t> pack_lines(const std::vector<std::string>& lines,
                                const std::function<std::vector<int>(const std::string&)>& encode, int eos_id,
                                bool insert_eos, float data_fraction, int seq_len, int threads) {
  const size_t n = lines.size();
  threads = std::max(1, std::min<int>(threads, (int)std::max<size_t>(1, n / 256)));
  std::vector<std::vector<int32_t>> parts(threads);
  auto work = [&](int t) {
    const size_t a = n * t / threads, b = n * (t + 1) / threads;
    auto& out = parts[t];
    for (size_t i = a; i < b; ++i) {
      auto enc = encode(lines[i]);
      out.insert(out.end(), enc.begin(), enc.end());
      if (insert_eos) out.push_back(eos_id);
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  std::vector<int32_t> ids;
  size_t total = 0;
  for (auto& p : parts) total += p.size();
  ids.reserve(total + 1);
  for (auto& p : parts) ids.insert(ids.end(), p.begin(), p.end());
  if (ids.empty() || ids.back() != eos_id) ids.push_back(eos_id);
  const float frac = std::clamp(data_fraction, 0.0f, 1.0f);
  if (frac < 1.0f) {
    size_t limit = (size_t)((double)ids.size() * frac);
    limit = std::max(limit, (size_t)(seq_len + 1));
    limit = std::min(limit, ids.size());
    ids.resize(limit);
    if (ids.empty() || ids.back() != eos_id) ids.push_back(eos_id);
  }
  return ids;
}

PretokMeta read_pretok_meta(const std::string& path) {
  std::ifstream in(path);
  if (!in) throw std::runtime_error("dataset: cannot open meta " + path);
  std::stringstream ss;
  ss << in.rdbuf();
  auto j = json::parse(ss.str());
  PretokMeta m;
  m.total_tokens = j["total_tokens"].as_int();
  auto geti = [&](const char* k, int& dst) {
    if (const json::Value* v = j.get(k))
      if (v->is_number()) dst = (int)v->as_int();
  };
  geti("eos_token_id", m.eos_id);
  geti("pad_token_id", m.pad_id);
  geti("bos_token_id", m.bos_id);
  geti("unk_token_id", m.unk_id);
  geti("vocab_size", m.vocab_size);
  if (const json::Value* v = j.get("insert_eos_between_lines"))
    if (v->type == json::Value::Bool) m.insert_eos_between_lines = v->b;
  if (const json::Value* sp = j.get("splits")) {
    const char* names[3][2] = {{"train", "train"}, {"valid", "validation"}, {"test", "test"}};
    for (int s = 0; s < 3; ++s)
      for (int a = 0; a < 2; ++a)
        if (const json::Value* e = sp->get(names[s][a])) {
          m.off[s] = (*e)["offset"].as_int();
          m.len[s] = (*e)["length"].as_int();
          break;
        }
  }
  return m;
}

std::vector<int32_t> read_pretok_split(const std::string& bin_path, const PretokMeta& m, int split, float data_fraction,
                                       int seq_len) {
  if (split < 0 || split > 2 || m.off[split] < 0) throw std::runtime_error("dataset: split not found in meta");
  int64_t use = m.len[split];
  const float frac = std::clamp(data_fraction, 0.0f, 1.0f);
  if (frac < 1.0f) use = std::max<int64_t>(seq_len + 1, std::min<int64_t>(use, (int64_t)((double)use * frac)));
  if (m.off[split] >= m.total_tokens) throw std::runtime_error("dataset: split offset exceeds total tokens");
  use = std::min<int64_t>(use, m.total_tokens - m.off[split]);
  std::vector<int32_t> ids((size_t)use);
  std::ifstream bin(bin_path, std::ios::binary);
  if (!bin) throw std::runtime_error("dataset: cannot open " + bin_path);
  bin.seekg((std::streamoff)(m.off[split] * 4), std::ios::beg);
  bin.read(reinterpret_cast<char*>(ids.data()), (std::streamsize)(use * 4));
  ids.resize((size_t)bin.gcount() / 4);
  if (ids.empty()) throw std::runtime_error("dataset: zero tokens read");
  return ids;
}

TokenDataset::TokenDataset(const DataConfig& cfg) : cfg_(cfg), rng_(cfg.seed) {
  if (cfg_.world < 1) cfg_.world = 1;
}

void TokenDataset::set_tokens(std::vector<int32_t> ids) {
  ids_ = std::move(ids);
  build_chunks();
  order_.resize(starts_.size());
  std::iota(order_.begin(), order_.end(), 0);
  cursor_ = 0;
  epoch_ = 0;
  if (cfg_.shuffle) std::shuffle(order_.begin(), order_.end(), rng_);
  build_local();
}

void TokenDataset::build_chunks() {
  starts_.clear();
  const long long S = cfg_.seq_len, need = S + 1, N = (long long)ids_.size();
  const long long stride = cfg_.stride <= 0 ? S : cfg_.stride;
  for (long long s = 0; s + need <= N; s += stride) starts_.push_back((size_t)s);
  if (!cfg_.drop_last) {
    if (starts_.empty() || (long long)starts_.back() + need < N) {
      const long long s = std::max(0LL, N - need);
      if (starts_.empty() || starts_.back() != (size_t)s) starts_.push_back((size_t)s);
    }
  }
}

void TokenDataset::build_local() {
  local_.clear();
  const size_t W = (size_t)cfg_.world, R = (size_t)cfg_.rank;
  if (W == 1) {
    local_ = order_;
    return;
  }
  const size_t per = order_.size() / W;  // equal share per rank (drop the remainder)
  for (size_t i = 0; i < per; ++i) local_.push_back(order_[i * W + R]);
}

void TokenDataset::shuffle() {
  std::shuffle(order_.begin(), order_.end(), rng_);
  build_local();
  cursor_ = 0;
}

void TokenDataset::get_batch(const size_t* chunk_idx, int B, int64_t* input_ids, int64_t* targets, float* mask,
                             int32_t* lengths) const {
  const int S = cfg_.seq_len;
  for (int b = 0; b < B; ++b) {
    int64_t* in = input_ids + (size_t)b * S;
    int64_t* tg = targets + (size_t)b * S;
    float* mk = mask + (size_t)b * S;
    std::fill(in, in + S, (int64_t)cfg_.pad_id);
    std::fill(tg, tg + S, (int64_t)-100);
    std::fill(mk, mk + S, 0.0f);
    if (chunk_idx[b] == (size_t)-1) {
      if (lengths) lengths[b] = 0;
      continue;
    }
    const size_t st = starts_.at(chunk_idx[b]);
    const size_t avail = std::min((size_t)S + 1, ids_.size() - st);
    const size_t tok_len = avail >= 2 ? avail - 1 : 0;
    for (size_t i = 0; i < tok_len && i < (size_t)S; ++i) {
      in[i] = ids_[st + i];
      mk[i] = 1.0f;
      // labels = inputs, shifted by the loss: target of position i is input i+1
      if (i + 1 < tok_len) tg[i] = ids_[st + i + 1];
    }
    if (lengths) lengths[b] = (int32_t)std::min(tok_len, (size_t)S);
  }
}

int TokenDataset::next_batch(int B, bool need_loop, int64_t* input_ids, int64_t* targets, float* mask,
                             int32_t* lengths) {
  if (local_.empty()) throw std::runtime_error("dataset: not loaded (or fewer chunks than ranks)");
  if (cursor_ >= local_.size()) {
    if (!need_loop) return 0;
    ++epoch_;
    shuffle();
  }
  const size_t start = cursor_;
  cursor_ = std::min(cursor_ + (size_t)B, local_.size());
  const int got = (int)(cursor_ - start);
  std::vector<size_t> idx((size_t)B, (size_t)-1);
  for (int b = 0; b < got; ++b) idx[b] = local_[start + b];
  get_batch(idx.data(), B, input_ids, targets, mask, lengths);
  return got;
}

std::string TokenDataset::rng_state() const {
  std::ostringstream ss;
  ss << rng_;
  return ss.str();
}

void TokenDataset::restore(int64_t epoch, size_t cursor, const std::string& rng_state) {
  // Re-create the order of `epoch`: replay the shuffles from the initial state.
  rng_.seed(cfg_.seed);
  order_.resize(starts_.size());
  std::iota(order_.begin(), order_.end(), 0);
  if (cfg_.shuffle) std::shuffle(order_.begin(), order_.end(), rng_);
  for (int64_t e = 0; e < epoch; ++e) std::shuffle(order_.begin(), order_.end(), rng_);
  build_local();
  epoch_ = epoch;
  cursor_ = cursor;
  if (!rng_state.empty()) {
    std::istringstream ss(rng_state);
    ss >> rng_;
  }
}

}  // namespace mft
