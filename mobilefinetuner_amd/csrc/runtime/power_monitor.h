// Energy-aware step throttling.
// Policy identical to the reference PowerMonitor (opt_ops/energy/power_monitor.h:20-72,
// .cpp:19-112): battery / temperature thresholds select high or low target step frequencies,
// sleep = round(1000 / min(f_b, f_t)) ms capped at 5000, recomputed every check_interval_steps;
// a deterministic "a-b:ms,c-:ms" schedule overrides.  The reference only had manual (mock)
// readings; here readings can also come from the MI355X itself: GPU junction temperature and
// socket power from the amdgpu hwmon sysfs nodes, with "battery" mapped to the remaining power
// headroom under the board power cap (100% = idle, 0% = at cap).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mft {

struct PowerConfig {
  int check_interval_steps = 0;
  float battery_threshold = 20.0f;
  float freq_b_high = 2.0f, freq_b_low = 0.5f;
  bool enable_battery = true;
  float temp_threshold = 42.0f;
  float freq_t_high = 2.0f, freq_t_low = 0.5f;
  bool enable_temp = true;
  bool use_gpu_telemetry = false;
  int gpu_index = 0;       // n-th amdgpu card in DRM minor order (when pci_bus is empty)
  std::string pci_bus;     // this rank's GPU ("0000:05:00.0", hipDeviceGetPCIBusId): its own sensors
  float power_cap_w = 0.f;  // > 0: software power cap -- sleep so the average socket power stays <= cap
};

struct StepSleep {
  int64_t start_step = 0, end_step = -1;
  int sleep_ms = 0;
};

struct GpuTelemetry {
  bool ok = false;
  float temp_c = 0.f;       // junction / edge temperature
  float power_w = 0.f;      // average socket power
  float power_cap_w = 0.f;  // board power cap
};

GpuTelemetry read_gpu_telemetry(int gpu_index);
// the amdgpu card whose PCI device is `pci_bus` (case-insensitive, e.g. "0000:05:00.0")
GpuTelemetry read_gpu_telemetry_bus(const std::string& pci_bus);

// Software power cap (no root needed, the board cap is untouched): with the step's busy time t and
// the measured average power P, a sleep s per step keeps P * t / (t + s) <= cap, i.e.
// s >= t (P / cap - 1).  P is a running average (hwmon power1_average), so the sleep is adjusted
// multiplicatively toward that target each check instead of jumping to it.
int power_cap_sleep_ms(float power_w, float cap_w, float step_ms, int prev_sleep_ms);

class PowerMonitor {
 public:
  explicit PowerMonitor(const PowerConfig& cfg = PowerConfig()) : cfg_(cfg) {}
  void set_manual_readings(float battery_percent, float temp_c) {
    battery_ = battery_percent;
    temp_ = temp_c;
  }
  void set_step_schedule(const std::vector<StepSleep>& s) { schedule_ = s; }
  static std::vector<StepSleep> parse_schedule(const std::string& spec);
  int suggest_sleep_ms(int64_t global_step);
  // the last step's busy time (the trainer's host-side step period minus the previous sleep); the
  // power-cap mode sizes its sleep from it
  void note_step_ms(float ms) { step_ms_ = ms; }
  std::string debug_state() const;
  float battery() const { return battery_; }
  float temperature() const { return temp_; }

 private:
  int recompute();
  float step_ms_ = 0.f, power_w_ = 0.f;
  bool have_power_ = false;
  int cap_sleep_ = 0;
  void refresh_telemetry();
  static int freq_to_sleep_ms(float f);
  PowerConfig cfg_;
  float battery_ = 100.f, temp_ = 30.f;
  std::vector<StepSleep> schedule_;
  int last_ = 0;
};

}  // namespace mft
