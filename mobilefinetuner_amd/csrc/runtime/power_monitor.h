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
  int gpu_index = 0;
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
  std::string debug_state() const;
  float battery() const { return battery_; }
  float temperature() const { return temp_; }

 private:
  int recompute();
  void refresh_telemetry();
  static int freq_to_sleep_ms(float f);
  PowerConfig cfg_;
  float battery_ = 100.f, temp_ = 30.f;
  std::vector<StepSleep> schedule_;
  int last_ = 0;
};

}  // namespace mft
