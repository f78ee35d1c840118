#include "power_monitor.h"

#include <dirent.h>

#include <algorithm>
#include <cmath>
#include <fstream>
#include <sstream>

namespace mft {

static bool read_num(const std::string& path, double& v) {
  std::ifstream in(path);
  if (!in) return false;
  in >> v;
  return (bool)in;
}

GpuTelemetry read_gpu_telemetry(int gpu_index) {
  // amdgpu exposes hwmon under /sys/class/drm/cardN/device/hwmon/hwmonM/{temp*_input, power1_average,
  // power1_cap}.  Card numbering follows the DRM minor order; we take the gpu_index-th amdgpu card.
  GpuTelemetry t;
  std::vector<std::string> cards;
  if (DIR* d = opendir("/sys/class/drm")) {
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n.rfind("card", 0) == 0 && n.find('-') == std::string::npos) cards.push_back(n);
    }
    closedir(d);
  }
  std::sort(cards.begin(), cards.end(), [](const std::string& a, const std::string& b) {
    return std::atoi(a.c_str() + 4) < std::atoi(b.c_str() + 4);
  });
  int seen = 0;
  for (auto& c : cards) {
    const std::string base = "/sys/class/drm/" + c + "/device/hwmon";
    DIR* d = opendir(base.c_str());
    if (!d) continue;
    std::string hw;
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n.rfind("hwmon", 0) == 0) hw = base + "/" + n;
    }
    closedir(d);
    if (hw.empty()) continue;
    std::ifstream nm(hw + "/name");
    std::string name;
    nm >> name;
    if (name != "amdgpu") continue;
    if (seen++ != gpu_index) continue;
    double v;
    // prefer junction (temp2) then edge (temp1); values in millidegrees C
    if (read_num(hw + "/temp2_input", v) || read_num(hw + "/temp1_input", v)) t.temp_c = (float)(v / 1000.0);
    if (read_num(hw + "/power1_average", v) || read_num(hw + "/power1_input", v)) t.power_w = (float)(v / 1e6);
    if (read_num(hw + "/power1_cap", v)) t.power_cap_w = (float)(v / 1e6);
    t.ok = true;
    break;
  }
  return t;
}

std::vector<StepSleep> PowerMonitor::parse_schedule(const std::string& spec) {
  std::vector<StepSleep> out;
  size_t pos = 0;
  while (pos < spec.size()) {
    size_t comma = spec.find(',', pos);
    std::string tok = spec.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
    pos = comma == std::string::npos ? spec.size() : comma + 1;
    if (tok.empty()) continue;
    const size_t colon = tok.find(':');
    if (colon == std::string::npos) continue;
    StepSleep ss;
    try {
      ss.sleep_ms = std::max(0, std::stoi(tok.substr(colon + 1)));
    } catch (...) {
      continue;
    }
    const std::string range = tok.substr(0, colon);
    const size_t dash = range.find('-');
    if (dash == std::string::npos) continue;
    try {
      ss.start_step = std::stoll(range.substr(0, dash));
    } catch (...) {
      continue;
    }
    const std::string e = range.substr(dash + 1);
    if (e.empty()) ss.end_step = -1;
    else {
      try {
        ss.end_step = std::stoll(e);
      } catch (...) {
        ss.end_step = -1;
      }
    }
    out.push_back(ss);
  }
  std::sort(out.begin(), out.end(), [](const StepSleep& a, const StepSleep& b) { return a.start_step < b.start_step; });
  return out;
}

int PowerMonitor::freq_to_sleep_ms(float f) {
  if (f <= 0.f) return 0;
  return (int)std::lround(std::min(1000.f / f, 5000.f));
}

void PowerMonitor::refresh_telemetry() {
  if (!cfg_.use_gpu_telemetry) return;
  GpuTelemetry t = read_gpu_telemetry(cfg_.gpu_index);
  if (!t.ok) return;
  temp_ = t.temp_c;
  if (t.power_cap_w > 0.f) battery_ = std::clamp(100.f * (1.f - t.power_w / t.power_cap_w), 0.f, 100.f);
}

int PowerMonitor::recompute() {
  refresh_telemetry();
  float fb = cfg_.freq_b_high;
  if (cfg_.enable_battery && battery_ < cfg_.battery_threshold) fb = cfg_.freq_b_low;
  float ft = cfg_.freq_t_high;
  if (cfg_.enable_temp && temp_ > cfg_.temp_threshold) ft = cfg_.freq_t_low;
  last_ = freq_to_sleep_ms(std::min(fb, ft));
  return last_;
}

int PowerMonitor::suggest_sleep_ms(int64_t step) {
  for (const auto& ss : schedule_) {
    if (step < ss.start_step) break;
    if (ss.end_step < 0 || step <= ss.end_step) return ss.sleep_ms;
  }
  if (cfg_.check_interval_steps <= 0) return last_;
  if (step % cfg_.check_interval_steps == 0) return recompute();
  return last_;
}

std::string PowerMonitor::debug_state() const {
  std::ostringstream o;
  o << "PowerMonitor{battery=" << battery_ << "%, temp=" << temp_ << "C, last_sleep_ms=" << last_
    << ", interval=" << cfg_.check_interval_steps << ", schedule_items=" << schedule_.size()
    << ", gpu_telemetry=" << (cfg_.use_gpu_telemetry ? "on" : "off") << "}";
  return o.str();
}

}  // namespace mft
