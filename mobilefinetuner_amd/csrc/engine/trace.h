// libmft engine: roctx ranges around the native trainer's phases -- step, graph
// capture, evaluation, checkpoint -- so `rocprofv3 --marker-trace` shows them next to the kernel
// trace of a native CLI run.  Without a profiler tool attached the calls are no-ops.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace mft {
namespace eng {

class TraceRange {
 public:
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

// --profile_steps a:b: collection paused outside the window (rocprofv3 --selected-regions honours
// roctxProfilerPause / Resume; without a tool attached both are no-ops)
inline void profiler_pause() { roctxProfilerPause(0); }
inline void profiler_resume() { roctxProfilerResume(0); }

}  // namespace eng
}  // namespace mft
