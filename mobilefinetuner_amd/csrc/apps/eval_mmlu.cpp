// Native CLI `eval_mmlu` on the libmft engine: MMLU multiple-choice accuracy of GPT-2 or Gemma-3
// (+ optional LoRA adapter, merged by default).
//
// Reference: gpt2_lora_finetune/eval_mmlu.cpp:60-167 and mmlu/mmlu_runner.cpp (flags --mmlu_root
// --split --fewshot --pretrained_dir --lora_path --lora_merge --out --debug; <root>/<split>/*.csv
// with header subject,question,a,b,c,d,answer or the headerless Hendrycks layout; prompt
// "Question: ...\nA. ...\nB. ...\nC. ...\nD. ...\nAnswer: " after k same-subject examples each
// followed by its letter and a blank line; log-softmax of the last position over the tokens of
// "A".."D", argmax; macro / micro accuracy).  Same evaluation as the Python CLI
// (eval/mmlu.py): prompts in length-sorted right-padded batches (causal attention keeps the last
// real position exact), a few-shot example never the item itself, GPT-2 prompts keep their last
// n_positions tokens.  Extras: --model_type gpt2|gemma --tokenizer_dir D --batch_size N --model P
// --random_init --scores_out F (the [N, 4] letter log-probs, subject-sorted, for parity checks).
#include <dirent.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "apps/app_common.h"
#include "engine/autograd.h"
#include "engine/gemma3.h"
#include "engine/gpt2.h"
#include "engine/ops.h"
#include "runtime/tokenizer.h"

using namespace mft;
using namespace mft::eng;
using mft::apps::Args;

namespace {

const std::set<std::string> kBool = {"debug", "random_init", "help"};
const std::set<std::string> kValued = {"mmlu_root",  "split", "fewshot",    "pretrained_dir", "lora_path", "lora_merge",
                                       "out",        "batch_size", "model_type", "tokenizer_dir",  "model",     "device",
                                       "scores_out", "dtype"};

struct MCQ {
  std::string subject, question, a, b, c, d, answer;
};

// RFC 4180 CSV: quoted fields ("" escapes, embedded separators / newlines), CRLF or LF rows
std::vector<std::vector<std::string>> parse_csv(const std::string& t) {
  std::vector<std::vector<std::string>> rows;
  std::vector<std::string> row;
  std::string f;
  bool q = false, any = false;
  for (size_t i = 0; i < t.size(); ++i) {
    const char c = t[i];
    if (q) {
      if (c == '"') {
        if (i + 1 < t.size() && t[i + 1] == '"') f += '"', ++i;
        else q = false;
      } else {
        f += c;
      }
      continue;
    }
    if (c == '"') {
      q = any = true;
    } else if (c == ',') {
      row.push_back(f), f.clear(), any = true;
    } else if (c == '\n' || c == '\r') {
      if (c == '\r' && i + 1 < t.size() && t[i + 1] == '\n') ++i;
      row.push_back(f), f.clear();
      rows.push_back(row), row.clear();
      any = false;
    } else {
      f += c, any = true;
    }
  }
  if (any || !f.empty() || !row.empty()) {
    row.push_back(f);
    rows.push_back(row);
  }
  return rows;
}

std::string strip(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) ++a;
  while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}

std::map<std::string, std::vector<MCQ>> read_split(const std::string& root, const std::string& split) {
  std::map<std::string, std::vector<MCQ>> by;
  const std::string dir = root + "/" + split;
  std::vector<std::string> files;
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      const std::string n = e->d_name;
      if (n.size() > 4 && n.substr(n.size() - 4) == ".csv") files.push_back(n);
    }
    closedir(d);
  }
  MFT_CHECK(!files.empty(), "no *.csv under ", dir);
  std::sort(files.begin(), files.end());
  for (auto& fn : files) {
    std::ifstream in(dir + "/" + fn, std::ios::binary);
    std::stringstream ss;
    ss << in.rdbuf();
    auto rows = parse_csv(ss.str());
    if (rows.empty()) continue;
    std::map<std::string, int> idx;
    for (const char* k : {"subject", "question", "a", "b", "c", "d", "answer"}) idx[k] = -1;
    for (size_t i = 0; i < rows[0].size(); ++i) {
      std::string h = strip(rows[0][i]);
      for (auto& ch : h) ch = (char)std::tolower((unsigned char)ch);
      if (idx.count(h) && idx[h] < 0) idx[h] = (int)i;
    }
    size_t body = 1;
    int mn = 1 << 30;
    for (const char* k : {"question", "a", "b", "c", "d", "answer"}) mn = std::min(mn, idx[k]);
    if (mn < 0) {  // headerless Hendrycks layout: question,a,b,c,d,answer; subject from the file name
      idx = {{"subject", -1}, {"question", 0}, {"a", 1}, {"b", 2}, {"c", 3}, {"d", 4}, {"answer", 5}};
      body = 0;
    }
    const size_t us = fn.rfind('_');
    const std::string subj_file = us != std::string::npos ? fn.substr(0, us) : fn.substr(0, fn.size() - 4);
    int mx = -1;
    for (auto& kv : idx) mx = std::max(mx, kv.second);
    for (size_t r = body; r < rows.size(); ++r) {
      const auto& row = rows[r];
      bool blank = true;
      for (auto& x : row) blank = blank && strip(x).empty();
      if ((int)row.size() <= mx || blank) continue;
      MCQ m;
      std::string ans = strip(row[idx["answer"]]);
      m.answer = ans.empty() ? "A" : std::string(1, (char)std::toupper((unsigned char)ans[0]));
      m.subject = idx["subject"] >= 0 ? strip(row[idx["subject"]]) : subj_file;
      m.question = strip(row[idx["question"]]);
      m.a = strip(row[idx["a"]]), m.b = strip(row[idx["b"]]), m.c = strip(row[idx["c"]]), m.d = strip(row[idx["d"]]);
      by[m.subject].push_back(m);
    }
  }
  return by;
}

std::string one(const MCQ& q) {
  return "Question: " + q.question + "\nA. " + q.a + "\nB. " + q.b + "\nC. " + q.c + "\nD. " + q.d + "\nAnswer: ";
}

int run(int argc, char** argv) {
  Args a = mft::apps::parse_args(argc, argv, kBool, kValued);
  if (a.b("help") || a.get("mmlu_root").empty()) {
    std::printf(
        "eval_mmlu -- native MI355X engine (libmft)\n"
        "  --mmlu_root D --split dev|val|test --fewshot K --pretrained_dir P [--lora_path F --lora_merge 0|1]\n"
        "  [--out F] [--debug]  extras: --model_type gpt2|gemma --tokenizer_dir D --batch_size N --model P\n"
        "  --random_init --scores_out F\n");
    return a.b("help") ? 0 : 2;
  }
  HIP_OK(hipSetDevice(0));
  hipStream_t stream;
  HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  set_current_stream(stream);
  mft::apps::apply_dtype_flag(a);
  const std::string mtype = a.get("model_type", "gpt2"), pdir = a.get("pretrained_dir");
  const std::string tdir = a.get("tokenizer_dir", pdir);
  const bool random_init = a.b("random_init") || pdir.empty();
  const bool cfg_file = !random_init && mft::apps::file_exists(pdir + "/config.json");
  const std::string lora = a.get("lora_path");
  const bool merge = a.i("lora_merge", 1) != 0;
  std::unique_ptr<LanguageModel> model;
  std::function<std::vector<int>(const std::string&, bool)> enc;
  int max_len = 0;
  if (mtype == "gpt2") {
    GPT2Config cfg = cfg_file ? GPT2Config::from_json(pdir + "/config.json") : GPT2Config::preset(a.get("model", "gpt2"));
    auto m = std::make_unique<GPT2>(cfg);
    if (random_init) m->init_random(1234);
    else m->load_hf(pdir);
    if (!lora.empty()) {
      m->load_lora(lora);
      if (merge) m->merge_lora(1.f);
    }
    max_len = cfg.n_positions;
    std::shared_ptr<ByteLevelBPE> tok = mft::apps::file_exists(tdir + "/vocab.json")
                                            ? std::shared_ptr<ByteLevelBPE>(ByteLevelBPE::from_files(tdir + "/vocab.json", tdir + "/merges.txt"))
                                            : std::shared_ptr<ByteLevelBPE>(ByteLevelBPE::from_tokenizer_json(tdir + "/tokenizer.json"));
    enc = [tok](const std::string& s, bool) { return tok->encode(s); };
    mft::apps::apply_model_flags(a, *m);
    model = std::move(m);
  } else if (mtype == "gemma") {
    Gemma3Config cfg = cfg_file ? Gemma3Config::from_json(pdir + "/config.json")
                                : Gemma3Config::preset(a.get("model", "gemma3-270m"));
    auto m = std::make_unique<Gemma3>(cfg);
    if (random_init) m->init_random(1234);
    else m->load_hf(pdir);
    if (!lora.empty()) {
      m->load_lora(lora);
      if (merge) m->merge_lora(1.f);
    }
    std::shared_ptr<SentencePieceBPE> tok = SentencePieceBPE::from_tokenizer_json(tdir + "/tokenizer.json");
    enc = [tok](const std::string& s, bool bos) { return tok->encode(s, bos); };
    mft::apps::apply_model_flags(a, *m);
    model = std::move(m);
  } else {
    throw std::runtime_error("--model_type must be gpt2 or gemma");
  }
  model->training = false;
  const bool gemma = mtype == "gemma";
  const int fewshot = a.i("fewshot", 0), bs = std::max(1, a.i("batch_size", 16)), V = model->vocab();
  const std::string split = a.get("split", "dev");
  auto data = read_split(a.get("mmlu_root"), split);
  size_t nq = 0;
  for (auto& kv : data) nq += kv.second.size();
  std::printf("[eval_mmlu] %zu questions in %zu subjects (split=%s, fewshot=%d)\n", nq, data.size(), split.c_str(),
              fewshot);
  int letters[4];
  for (int i = 0; i < 4; ++i) {
    auto ids = enc(std::string(1, "ABCD"[i]), false);
    letters[i] = ids.empty() ? 0 : ids[0];
  }
  std::ofstream scores;
  if (!a.get("scores_out").empty()) scores.open(a.get("scores_out"));
  scores.precision(9);
  NoGradGuard ng;
  Param& W = model->output_embedding();
  struct Row {
    std::string subject;
    int correct, total;
  };
  std::vector<Row> per;
  int tc = 0, tn = 0;
  for (auto& kv : data) {
    const auto& items = kv.second;
    std::vector<std::vector<int>> toks(items.size());
    for (size_t i = 0; i < items.size(); ++i) {
      std::string p;
      if (fewshot > 0)
        for (size_t j = 0; j < std::min<size_t>(fewshot, items.size()); ++j)
          if (j != i) p += one(items[j]) + items[j].answer + "\n\n";
      p += one(items[i]);
      toks[i] = enc(p, gemma);
      if (max_len > 0 && (int)toks[i].size() > max_len) toks[i].erase(toks[i].begin(), toks[i].end() - max_len);
    }
    std::vector<size_t> order(items.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return toks[x].size() < toks[y].size(); });
    std::vector<std::array<float, 4>> lp(items.size());
    for (size_t s = 0; s < order.size(); s += bs) {
      const size_t nb = std::min<size_t>(bs, order.size() - s);
      size_t L = 1;
      for (size_t r = 0; r < nb; ++r) L = std::max(L, toks[order[s + r]].size());
      std::vector<int64_t> ids(nb * L, 0), last(nb);
      for (size_t r = 0; r < nb; ++r) {
        const auto& t = toks[order[s + r]];
        for (size_t j = 0; j < t.size(); ++j) ids[r * L + j] = t[j];
        last[r] = (int64_t)(r * L + std::max<size_t>(t.size(), 1) - 1);
      }
      Tensor h = model->hidden(from_host(ids.data(), {(int64_t)nb, (int64_t)L}, DType::I64));
      Tensor hl = embedding(from_host(last.data(), {(int64_t)nb}, DType::I64), h.view({-1, h.size(-1)}));
      Tensor logits = linear(hl, W.c).slice(1, 0, V).to(DType::F32);
      Tensor lsm = log_softmax(logits.contiguous()).to(Device::cpu());
      const float* p = lsm.data<float>();
      for (size_t r = 0; r < nb; ++r)
        for (int c = 0; c < 4; ++c) lp[order[s + r]][c] = p[r * V + letters[c]];
    }
    int correct = 0;
    for (size_t i = 0; i < items.size(); ++i) {
      int best = 0;
      for (int c = 1; c < 4; ++c)
        if (lp[i][c] > lp[i][best]) best = c;
      correct += std::string(1, "ABCD"[best]) == items[i].answer;
      if (scores.is_open()) scores << lp[i][0] << " " << lp[i][1] << " " << lp[i][2] << " " << lp[i][3] << "\n";
    }
    per.push_back({kv.first, correct, (int)items.size()});
    tc += correct;
    tn += (int)items.size();
    std::printf("  %-40s %5d/%-5d acc=%.4f\n", kv.first.c_str(), correct, (int)items.size(),
                correct / (double)std::max<size_t>(1, items.size()));
  }
  double macro = 0.0;
  for (auto& r : per) macro += r.correct / (double)std::max(1, r.total);
  macro /= std::max<size_t>(1, per.size());
  const double micro = tc / (double)std::max(1, tn);
  std::printf("[eval_mmlu] macro=%.4f micro=%.4f total=%d\n", macro, micro, tn);
  if (!a.get("out").empty()) {
    std::ofstream o(a.get("out"), std::ios::app);
    o.precision(9);
    for (auto& r : per)
      o << "{\"task\": \"mmlu\", \"split\": \"" << split << "\", \"subject\": \"" << r.subject << "\", \"correct\": " << r.correct
        << ", \"total\": " << r.total << ", \"acc\": " << r.correct / (double)std::max(1, r.total) << "}\n";
    o << "{\"task\": \"mmlu\", \"split\": \"" << split << "\", \"macro\": " << macro << ", \"micro\": " << micro
      << ", \"total\": " << tn << ", \"fewshot\": " << fewshot << ", \"lora\": \"" << lora << "\"}\n";
  }
  std::printf("{\"macro\": %.9g, \"micro\": %.9g, \"total\": %d}\n", macro, micro, tn);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  mft::apps::install_crash_report();
  try {
    return run(argc, argv);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "eval_mmlu: error: %s\n", e.what());
    return 1;
  }
}
