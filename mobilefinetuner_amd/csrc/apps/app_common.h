// Shared plumbing of the native CLIs (csrc/apps): reference-style "--flag value" / "--flag=value"
// parsing against per-program flag sets, file helpers.
#pragma once
#include <sys/stat.h>

#include <cstdint>
#include <map>
#include <set>
#include <stdexcept>
#include <string>

namespace mft {
namespace apps {

struct Args {
  std::map<std::string, std::string> kv;
  std::set<std::string> flags;
  std::string get(const std::string& k, const std::string& d = "") const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
  int i(const std::string& k, int d) const { return kv.count(k) ? std::stoi(kv.at(k)) : d; }
  int64_t l(const std::string& k, int64_t d) const { return kv.count(k) ? std::stoll(kv.at(k)) : d; }
  float f(const std::string& k, float d) const { return kv.count(k) ? std::stof(kv.at(k)) : d; }
  bool b(const std::string& k) const { return flags.count(k) || (kv.count(k) && kv.at(k) != "0" && kv.at(k) != "false"); }
};

// kBool flags may appear bare; kValued flags take a value; anything else is an error
inline Args parse_args(int argc, char** argv, const std::set<std::string>& kBool, const std::set<std::string>& kValued) {
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
    if (!kValued.count(key)) throw std::runtime_error("unknown flag --" + key + " (see --help)");
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

}  // namespace apps
}  // namespace mft
