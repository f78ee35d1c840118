#include "power_monitor.h"

#include <dirent.h>

#include <stdlib.h>

#include <algorithm>
#include <cctype>
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

namespace {
// hwmon directory of an amdgpu card ("" if none), its PCI address (basename of the device link)
std::string amdgpu_hwmon(const std::string& card, std::string* bus) {
  const std::string dev = "/sys/class/drm/" + card + "/device";
  if (bus) {
    char buf[4096];
    if (char* rp = realpath(dev.c_str(), buf)) {
      std::string r(rp);
      const size_t sl = r.rfind('/');
      *bus = sl == std::string::npos ? r : r.substr(sl + 1);
    } else {
      bus->clear();
    }
  }
  const std::string base = dev + "/hwmon";
  DIR* d = opendir(base.c_str());
  if (!d) return "";
  std::string hw;
  while (dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n.rfind("hwmon", 0) == 0) hw = base + "/" + n;
  }
  closedir(d);
  if (hw.empty()) return "";
  std::ifstream nm(hw + "/name");
  std::string name;
  nm >> name;
  return name == "amdgpu" ? hw : "";
}

std::vector<std::string> drm_cards() {
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
  return cards;
}

GpuTelemetry read_hwmon(const std::string& hw) {
  GpuTelemetry t;
  double v;
  // prefer junction (temp2) then edge (temp1); values in millidegrees C
  if (read_num(hw + "/temp2_input", v) || read_num(hw + "/temp1_input", v)) t.temp_c = (float)(v / 1000.0);
  if (read_num(hw + "/power1_average", v) || read_num(hw + "/power1_input", v)) t.power_w = (float)(v / 1e6);
  if (read_num(hw + "/power1_cap", v)) t.power_cap_w = (float)(v / 1e6);
  t.ok = true;
  return t;
}

std::string lower(std::string s) {
  for (char& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}
}  // namespace

GpuTelemetry read_gpu_telemetry_bus(const std::string& pci_bus) {
  const std::string want = lower(pci_bus);
  for (auto& c : drm_cards()) {
    std::string bus;
    const std::string hw = amdgpu_hwmon(c, &bus);
    if (!hw.empty() && lower(bus) == want) return read_hwmon(hw);
  }
  return GpuTelemetry{};
}

int power_cap_sleep_ms(float power_w, float cap_w, float step_ms, int prev) {
  if (cap_w <= 0.f || power_w <= 0.f || step_ms <= 0.f) return prev;
  // P was measured with the previous sleep in place: the busy power is P (t + s) / t
  const float busy_w = power_w * (step_ms + (float)prev) / step_ms;
  const float target = busy_w > cap_w ? step_ms * (busy_w / cap_w - 1.f) : 0.f;
  // move halfway toward the target (the sensor averages over ~1 s), at least 1 ms when above cap
  float s = 0.5f * ((float)prev + target);
  if (power_w > cap_w) s = std::max(s, (float)prev + 1.f);
  return (int)std::lround(std::min(std::max(s, 0.f), 5000.f));
}

GpuTelemetry read_gpu_telemetry(int gpu_index) {
  // amdgpu exposes hwmon under /sys/class/drm/cardN/device/hwmon/hwmonM/{temp*_input, power1_average,
  // power1_cap}.  Card numbering follows the DRM minor order; we take the gpu_index-th amdgpu card
  // (a multi-GPU job should name its card by PCI address instead: read_gpu_telemetry_bus).
  int seen = 0;
  for (auto& c : drm_cards()) {
    const std::string hw = amdgpu_hwmon(c, nullptr);
    if (hw.empty()) continue;
    if (seen++ == gpu_index) return read_hwmon(hw);
  }
  return GpuTelemetry{};
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
  GpuTelemetry t = cfg_.pci_bus.empty() ? read_gpu_telemetry(cfg_.gpu_index) : read_gpu_telemetry_bus(cfg_.pci_bus);
  if (!t.ok) return;
  temp_ = t.temp_c;
  power_w_ = t.power_w;
  have_power_ = true;
  if (t.power_cap_w > 0.f) battery_ = std::clamp(100.f * (1.f - t.power_w / t.power_cap_w), 0.f, 100.f);
}

int PowerMonitor::recompute() {
  refresh_telemetry();
  float fb = cfg_.freq_b_high;
  if (cfg_.enable_battery && battery_ < cfg_.battery_threshold) fb = cfg_.freq_b_low;
  float ft = cfg_.freq_t_high;
  if (cfg_.enable_temp && temp_ > cfg_.temp_threshold) ft = cfg_.freq_t_low;
  last_ = freq_to_sleep_ms(std::min(fb, ft));
  if (cfg_.power_cap_w > 0.f && have_power_) {
    cap_sleep_ = power_cap_sleep_ms(power_w_, cfg_.power_cap_w, step_ms_, cap_sleep_);
    // the battery / temperature policy applies on top only when enabled by its flags
    const int pol = (cfg_.enable_battery || cfg_.enable_temp) ? last_ : 0;
    last_ = std::max(pol, cap_sleep_);
  }
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
    << ", gpu_telemetry=" << (cfg_.use_gpu_telemetry ? "on" : "off") << (cfg_.pci_bus.empty() ? "" : " @")
    << cfg_.pci_bus << ", power_cap_w=" << cfg_.power_cap_w << ", cap_sleep_ms=" << cap_sleep_ << "}";
  return o.str();
}

}  // namespace mft
