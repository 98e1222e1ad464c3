// roctx ranges around the engine's host-side phases (SURVEY §5 "Tracing /
// profiling").  `rocprofv3 --marker-trace` (or any rocprofiler-sdk tool)
// records them next to the kernel / copy traces; with no tool attached a
// push/pop is a few ns.  Names: twtml.<engine>.<phase>.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace twtml {

class TraceRange {
 public:
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace twtml
