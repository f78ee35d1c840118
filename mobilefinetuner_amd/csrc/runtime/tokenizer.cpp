#include "tokenizer.h"

#include <atomic>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <queue>
#include <sstream>
#include <stdexcept>

#include "json.h"
#include "unicode_tables.h"

namespace mft {

namespace {

std::string read_file(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) throw std::runtime_error("tokenizer: cannot open " + path);
  std::ostringstream ss;
  ss << in.rdbuf();
  return ss.str();
}

struct CP {
  uint32_t cp;
  uint32_t off;
  uint32_t len;
};

std::vector<CP> decode_utf8(const std::string& s) {
  std::vector<CP> out;
  out.reserve(s.size());
  size_t i = 0;
  while (i < s.size()) {
    unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    uint32_t n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6 && i + 1 < s.size()) { cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); n = 2; }
    else if ((c >> 4) == 14 && i + 2 < s.size()) { cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F); n = 3; }
    else if ((c >> 3) == 30 && i + 3 < s.size()) {
      cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F); n = 4;
    } else { cp = c; n = 1; }  // invalid byte: treat as a 1-byte symbol
    out.push_back({cp, (uint32_t)i, n});
    i += n;
  }
  return out;
}

void put_utf8(std::string& s, uint32_t cp) {
  if (cp < 0x80) s += (char)cp;
  else if (cp < 0x800) { s += (char)(0xC0 | (cp >> 6)); s += (char)(0x80 | (cp & 0x3F)); }
  else if (cp < 0x10000) {
    s += (char)(0xE0 | (cp >> 12)); s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
  } else {
    s += (char)(0xF0 | (cp >> 18)); s += (char)(0x80 | ((cp >> 12) & 0x3F));
    s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
  }
}

bool in_ranges(uint32_t cp, const uint32_t (*r)[2], int n) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    int mid = (lo + hi) / 2;
    if (cp < r[mid][0]) hi = mid - 1;
    else if (cp > r[mid][1]) lo = mid + 1;
    else return true;
  }
  return false;
}
inline bool is_L(uint32_t c) {
  if (c < 0x80) return (c | 32) >= 'a' && (c | 32) <= 'z';
  return in_ranges(c, uni::kLetter, uni::kLetterN);
}
inline bool is_N(uint32_t c) {
  if (c < 0x80) return c >= '0' && c <= '9';
  return in_ranges(c, uni::kNumber, uni::kNumberN);
}
inline bool is_S(uint32_t c) {
  for (int i = 0; i < uni::kSpaceN; ++i)
    if (uni::kSpace[i] == c) return true;
  return false;
}

}  // namespace

// ------------------------------------------------------------------------------------ BPECore
void BPECore::add_token(const std::string& s, int id) {
  if (id < 0) return;
  if ((int)id_to_tok_.size() <= id) id_to_tok_.resize(id + 1);
  id_to_tok_[id] = s;
  tok_to_id_[s] = id;
}

int BPECore::token_id(const std::string& s) const {
  auto it = tok_to_id_.find(s);
  return it == tok_to_id_.end() ? -1 : it->second;
}

const std::string& BPECore::token_str(int id) const {
  static const std::string empty;
  if (id < 0 || id >= (int)id_to_tok_.size()) return empty;
  return id_to_tok_[id];
}

void BPECore::add_merge(const std::string& a, const std::string& b, int rank) {
  const int ia = token_id(a), ib = token_id(b), im = token_id(a + b);
  if (ia < 0 || ib < 0 || im < 0) return;  // merge producing an unknown token: never applicable
  const uint64_t key = ((uint64_t)(uint32_t)ia << 32) | (uint32_t)ib;
  if (!merges_.count(key)) merges_[key] = MergeInfo{rank, im};
}

void BPECore::merge(std::vector<int>& syms) const {
  const int n = (int)syms.size();
  if (n < 2 || merges_.empty()) return;
  std::vector<int> prv(n), nxt(n);
  for (int i = 0; i < n; ++i) { prv[i] = i - 1; nxt[i] = i + 1 < n ? i + 1 : -1; }
  struct Cand {
    int rank, pos, left, right;
    bool operator>(const Cand& o) const { return rank != o.rank ? rank > o.rank : pos > o.pos; }
  };
  std::priority_queue<Cand, std::vector<Cand>, std::greater<Cand>> pq;
  auto push = [&](int i) {
    if (i < 0) return;
    const int j = nxt[i];
    if (j < 0) return;
    auto it = merges_.find(((uint64_t)(uint32_t)syms[i] << 32) | (uint32_t)syms[j]);
    if (it != merges_.end()) pq.push(Cand{it->second.rank, i, syms[i], syms[j]});
  };
  for (int i = 0; i + 1 < n; ++i) push(i);
  std::vector<char> dead(n, 0);
  while (!pq.empty()) {
    Cand c = pq.top();
    pq.pop();
    const int i = c.pos;
    if (dead[i] || syms[i] != c.left) continue;
    const int j = nxt[i];
    if (j < 0 || syms[j] != c.right) continue;
    auto it = merges_.find(((uint64_t)(uint32_t)c.left << 32) | (uint32_t)c.right);
    syms[i] = it->second.id;
    dead[j] = 1;
    nxt[i] = nxt[j];
    if (nxt[j] >= 0) prv[nxt[j]] = i;
    push(prv[i]);
    push(i);
  }
  int w = 0;
  for (int i = 0; i >= 0 && i < n; i = nxt[i]) syms[w++] = syms[i];
  syms.resize(w);
}

// ------------------------------------------------------------------------------------ ByteLevelBPE
void ByteLevelBPE::init_byte_map() {
  std::vector<int> bs;
  for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
  for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
  for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
  std::vector<int> cs = bs;
  int n = 0;
  for (int b = 0; b < 256; ++b) {
    if (std::find(bs.begin(), bs.end(), b) == bs.end()) {
      bs.push_back(b);
      cs.push_back(256 + n++);
    }
  }
  for (size_t k = 0; k < bs.size(); ++k) {
    std::string s;
    put_utf8(s, (uint32_t)cs[k]);
    byte_to_uni_[bs[k]] = s;
    uni_to_byte_[(uint32_t)cs[k]] = (uint8_t)bs[k];
  }
}

std::unique_ptr<ByteLevelBPE> ByteLevelBPE::from_files(const std::string& vocab_json, const std::string& merges_txt) {
  auto t = std::make_unique<ByteLevelBPE>();
  t->init_byte_map();
  auto v = json::parse(read_file(vocab_json));
  for (auto& kv : v.as_object()) t->add_token(kv.first, (int)kv.second.as_int());
  std::ifstream in(merges_txt);
  if (!in) throw std::runtime_error("tokenizer: cannot open " + merges_txt);
  std::string line;
  int rank = 0;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty() || line.rfind("#version", 0) == 0) continue;
    const size_t sp = line.find(' ');
    if (sp == std::string::npos) continue;
    t->add_merge(line.substr(0, sp), line.substr(sp + 1), rank++);
  }
  const int eot = t->token_id("<|endoftext|>");
  if (eot >= 0) {
    t->eos_id = t->bos_id = t->pad_id = eot;
    t->special["<|endoftext|>"] = eot;
  }
  return t;
}

std::unique_ptr<ByteLevelBPE> ByteLevelBPE::from_tokenizer_json(const std::string& path) {
  auto t = std::make_unique<ByteLevelBPE>();
  t->init_byte_map();
  auto j = json::parse(read_file(path));
  auto& model = j["model"];
  for (auto& kv : model["vocab"].as_object()) t->add_token(kv.first, (int)kv.second.as_int());
  int rank = 0;
  for (auto& m : model["merges"].as_array()) {
    if (m.is_string()) {
      const std::string& s = m.as_string();
      const size_t sp = s.find(' ');
      if (sp != std::string::npos) t->add_merge(s.substr(0, sp), s.substr(sp + 1), rank);
    } else {
      t->add_merge(m.as_array().at(0).as_string(), m.as_array().at(1).as_string(), rank);
    }
    ++rank;
  }
  if (const json::Value* at = j.get("added_tokens"))
    if (at->is_array())
      for (auto& a : at->as_array()) {
        t->add_token(a["content"].as_string(), (int)a["id"].as_int());
        t->special[a["content"].as_string()] = (int)a["id"].as_int();
      }
  const int eot = t->token_id("<|endoftext|>");
  if (eot >= 0) t->eos_id = t->bos_id = t->pad_id = eot;
  return t;
}

std::vector<std::string> ByteLevelBPE::pretokenize(const std::string& text) const {
  std::vector<std::string> out;
  const auto cps = decode_utf8(text);
  const size_t n = cps.size();
  auto emit = [&](size_t a, size_t b) {
    const uint32_t off = cps[a].off;
    const uint32_t end = b < n ? cps[b].off : (uint32_t)text.size();
    out.emplace_back(text.substr(off, end - off));
  };
  size_t i = 0;
  while (i < n) {
    const uint32_t c = cps[i].cp;
    // 's 't 're 've 'm 'll 'd
    if (c == '\'' && i + 1 < n) {
      const uint32_t c1 = cps[i + 1].cp;
      if (c1 == 's' || c1 == 't' || c1 == 'm' || c1 == 'd') { emit(i, i + 2); i += 2; continue; }
      if (i + 2 < n) {
        const uint32_t c2 = cps[i + 2].cp;
        if ((c1 == 'r' && c2 == 'e') || (c1 == 'v' && c2 == 'e') || (c1 == 'l' && c2 == 'l')) { emit(i, i + 3); i += 3; continue; }
      }
    }
    const size_t j0 = (c == ' ' && i + 1 < n) ? i + 1 : i;  // optional leading space
    const uint32_t d = cps[j0].cp;
    if (is_L(d)) {
      size_t j = j0;
      while (j < n && is_L(cps[j].cp)) ++j;
      emit(i, j); i = j; continue;
    }
    if (is_N(d)) {
      size_t j = j0;
      while (j < n && is_N(cps[j].cp)) ++j;
      emit(i, j); i = j; continue;
    }
    if (!is_S(d) && !is_L(d) && !is_N(d)) {
      size_t j = j0;
      while (j < n && !is_S(cps[j].cp) && !is_L(cps[j].cp) && !is_N(cps[j].cp)) ++j;
      emit(i, j); i = j; continue;
    }
    // whitespace: \s+(?!\S) | \s+
    size_t j = i;
    while (j < n && is_S(cps[j].cp)) ++j;
    if (j == i) { emit(i, i + 1); i += 1; continue; }  // lone ' ' before end-of-text handled above
    if (j < n && j - i >= 2) { emit(i, j - 1); i = j - 1; continue; }
    emit(i, j); i = j;
  }
  return out;
}

uint64_t ByteLevelBPE::next_uid() {
  static std::atomic<uint64_t> n{1};
  return n.fetch_add(1, std::memory_order_relaxed);
}

void ByteLevelBPE::encode_word(const std::string& w, std::vector<int>& out) const {
  // per-thread word cache (the dataset tokenises WikiText lines on several threads), keyed by the
  // tokenizer's serial; caches of tokenizers that no longer exist are dropped wholesale
  static thread_local std::unordered_map<uint64_t, std::unordered_map<std::string, std::vector<int>>> tl;
  if (tl.size() > 8 && !tl.count(uid_)) tl.clear();
  auto& cache_ = tl[uid_];
  auto it = cache_.find(w);
  if (it != cache_.end()) {
    out.insert(out.end(), it->second.begin(), it->second.end());
    return;
  }
  std::vector<int> syms;
  syms.reserve(w.size());
  for (unsigned char b : w) {
    const int id = token_id(byte_to_uni_[b]);
    if (id < 0) throw std::runtime_error("tokenizer: byte symbol missing from vocab");
    syms.push_back(id);
  }
  merge(syms);
  if (cache_.size() < (1u << 20)) cache_.emplace(w, syms);
  out.insert(out.end(), syms.begin(), syms.end());
}

std::vector<int> ByteLevelBPE::encode(const std::string& text) const {
  std::vector<int> out;
  // split on special tokens first (e.g. <|endoftext|>)
  size_t pos = 0;
  while (pos <= text.size()) {
    size_t best = std::string::npos, blen = 0;
    int bid = -1;
    for (auto& kv : special) {
      const size_t f = text.find(kv.first, pos);
      if (f != std::string::npos && (f < best || (f == best && kv.first.size() > blen))) {
        best = f; blen = kv.first.size(); bid = kv.second;
      }
    }
    const size_t stop = best == std::string::npos ? text.size() : best;
    if (stop > pos)
      for (auto& w : pretokenize(text.substr(pos, stop - pos))) encode_word(w, out);
    if (best == std::string::npos) break;
    out.push_back(bid);
    pos = best + blen;
  }
  return out;
}

std::string ByteLevelBPE::decode(const std::vector<int>& ids, bool skip_special) const {
  std::string s;
  for (int id : ids) {
    const std::string& t = token_str(id);
    if (special.count(t)) {
      if (!skip_special) s += t;
      continue;
    }
    for (auto& c : decode_utf8(t)) {
      auto it = uni_to_byte_.find(c.cp);
      if (it != uni_to_byte_.end()) s += (char)it->second;
      else s.append(t, c.off, c.len);
    }
  }
  return s;
}

// ------------------------------------------------------------------------------------ SentencePieceBPE
std::unique_ptr<SentencePieceBPE> SentencePieceBPE::from_tokenizer_json(const std::string& path) {
  auto t = std::make_unique<SentencePieceBPE>();
  auto j = json::parse(read_file(path));
  auto& model = j["model"];
  for (auto& kv : model["vocab"].as_object()) t->add_token(kv.first, (int)kv.second.as_int());
  int rank = 0;
  for (auto& m : model["merges"].as_array()) {
    if (m.is_string()) {
      const std::string& s = m.as_string();
      const size_t sp = s.find(' ');
      if (sp != std::string::npos) t->add_merge(s.substr(0, sp), s.substr(sp + 1), rank);
    } else {
      t->add_merge(m.as_array().at(0).as_string(), m.as_array().at(1).as_string(), rank);
    }
    ++rank;
  }
  if (const json::Value* bf = model.get("byte_fallback")) t->byte_fallback = bf->type == json::Value::Bool && bf->b;
  if (const json::Value* unk = model.get("unk_token"))
    if (unk->is_string()) t->unk_id = t->token_id(unk->as_string());
  // normaliser: Replace(" ", "▁") possibly preceded by Prepend("▁")
  std::vector<const json::Value*> norms;
  if (const json::Value* nz = j.get("normalizer")) {
    if (nz->is_object()) {
      if (nz->get("type") && (*nz)["type"].as_string() == "Sequence") {
        for (auto& x : (*nz)["normalizers"].as_array()) norms.push_back(&x);
      } else {
        norms.push_back(nz);
      }
    }
  }
  for (auto* nz : norms) {
    const std::string ty = (*nz)["type"].as_string();
    if (ty == "Prepend") t->add_prefix_space = true;
    if (ty == "Replace") {
      const json::Value& pat = (*nz)["pattern"];
      if (pat.get("String")) t->replace_from = pat["String"].as_string();
      t->replace_to = (*nz)["content"].as_string();
    }
  }
  t->is_special.assign(t->vocab_size(), false);
  if (const json::Value* at = j.get("added_tokens"))
    if (at->is_array())
      for (auto& a : at->as_array()) {
        const int id = (int)a["id"].as_int();
        t->add_token(a["content"].as_string(), id);
        t->added.emplace_back(a["content"].as_string(), id);
        if ((int)t->is_special.size() <= id) t->is_special.resize(id + 1, false);
        const json::Value* sp = a.get("special");
        t->is_special[id] = sp && sp->type == json::Value::Bool && sp->b;
      }
  std::sort(t->added.begin(), t->added.end(),
            [](const std::pair<std::string, int>& x, const std::pair<std::string, int>& y) { return x.first.size() > y.first.size(); });
  for (int b = 0; b < 256; ++b) {
    char buf[8];
    snprintf(buf, sizeof(buf), "<0x%02X>", b);
    t->byte_tok_[b] = t->token_id(buf);
  }
  auto sid = [&](const char* s, int dflt) { const int v = t->token_id(s); return v >= 0 ? v : dflt; };
  t->bos_id = sid("<bos>", t->bos_id);
  t->eos_id = sid("<eos>", t->eos_id);
  t->pad_id = sid("<pad>", t->pad_id);
  if (t->unk_id < 0) t->unk_id = sid("<unk>", 3);
  return t;
}

void SentencePieceBPE::encode_chunk(const std::string& raw, std::vector<int>& out) const {
  std::string s;
  if (add_prefix_space) s = replace_to;
  // normalise: replace every occurrence of replace_from
  if (!replace_from.empty()) {
    size_t p = 0;
    while (true) {
      const size_t f = raw.find(replace_from, p);
      if (f == std::string::npos) { s.append(raw, p, std::string::npos); break; }
      s.append(raw, p, f - p);
      s += replace_to;
      p = f + replace_from.size();
    }
  } else {
    s += raw;
  }
  // symbols = code points; unknown code points -> byte fallback (break the merge run)
  std::vector<int> run;
  auto flush = [&]() {
    merge(run);
    out.insert(out.end(), run.begin(), run.end());
    run.clear();
  };
  for (auto& c : decode_utf8(s)) {
    const int id = token_id(s.substr(c.off, c.len));
    if (id >= 0) {
      run.push_back(id);
      continue;
    }
    flush();
    if (byte_fallback) {
      for (uint32_t k = 0; k < c.len; ++k) {
        const int bt = byte_tok_[(unsigned char)s[c.off + k]];
        out.push_back(bt >= 0 ? bt : unk_id);
      }
    } else {
      out.push_back(unk_id);
    }
  }
  flush();
}

std::vector<int> SentencePieceBPE::encode(const std::string& text, bool add_bos) const {
  std::vector<int> out;
  if (add_bos) out.push_back(bos_id);
  size_t pos = 0;
  while (pos < text.size()) {
    size_t best = std::string::npos, blen = 0;
    int bid = -1;
    for (auto& a : added) {  // longest first
      const size_t f = text.find(a.first, pos);
      if (f != std::string::npos && f < best) { best = f; blen = a.first.size(); bid = a.second; }
    }
    const size_t stop = best == std::string::npos ? text.size() : best;
    if (stop > pos) encode_chunk(text.substr(pos, stop - pos), out);
    if (best == std::string::npos) break;
    out.push_back(bid);
    pos = best + blen;
  }
  return out;
}

std::string SentencePieceBPE::decode(const std::vector<int>& ids, bool skip_special) const {
  std::string s;
  for (int id : ids) {
    if (skip_special && id >= 0 && id < (int)is_special.size() && is_special[id]) continue;
    const std::string& t = token_str(id);
    if (t.size() == 6 && t[0] == '<' && t[1] == '0' && t[2] == 'x' && t[5] == '>') {
      s += (char)std::stoi(t.substr(3, 2), nullptr, 16);
      continue;
    }
    size_t p = 0;
    while (true) {
      const size_t f = t.find(replace_to, p);
      if (f == std::string::npos) { s.append(t, p, std::string::npos); break; }
      s.append(t, p, f - p);
      s += replace_from;
      p = f + replace_to.size();
    }
  }
  if (add_prefix_space && !s.empty() && s[0] == ' ') s.erase(0, 1);
  return s;
}

}  // namespace mft
