// Shared plumbing of the native CLIs (csrc/apps): reference-style "--flag value" / "--flag=value"
// parsing against per-program flag sets, file helpers, the token-data sources every training /
// eval CLI accepts (pretokenized stream, synthetic stream, raw WikiText-2 text) and the
// power-monitor flags.
#pragma once
#include <sys/stat.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "runtime/dataset.h"
#include "runtime/power_monitor.h"

namespace mft {
namespace apps {

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

// kBool flags may appear bare; kValued flags take a value; anything else is an error (lenient: it
// is recorded in Args::unknown and skipped with its value, like the reference Gemma CLI parser)
inline Args parse_args(int argc, char** argv, const std::set<std::string>& kBool, const std::set<std::string>& kValued,
                       bool lenient = false) {
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

// --pm_* flags (reference energy options) -> PowerMonitor, or null when off
inline std::unique_ptr<PowerMonitor> power_monitor_from(const Args& a) {
  if (a.i("pm_interval", 0) <= 0 && a.get("pm_schedule").empty()) return nullptr;
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
  pc.use_gpu_telemetry = a.b("pm_gpu_telemetry");
  auto pm = std::make_unique<PowerMonitor>(pc);
  pm->set_manual_readings(a.f("pm_manual_batt", 100.f), a.f("pm_manual_temp", 30.f));
  if (!a.get("pm_schedule").empty()) pm->set_step_schedule(PowerMonitor::parse_schedule(a.get("pm_schedule")));
  return pm;
}

}  // namespace apps
}  // namespace mft
