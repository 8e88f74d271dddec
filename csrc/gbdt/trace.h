// Scoped roctx ranges (host side): each range names one engine phase on the rocprofv3 timeline
// (`rocprofv3 --marker-trace`), so a trace shows where a fit's wall clock goes - dataset encode, row upload,
// tree growth, score update, validation, prediction, collectives - next to the kernels each phase enqueued.
// The ranges mark host-side spans: for asynchronous phases they cover the enqueue, and the kernels carry
// the device time.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace sml {

class TraceRange {
 public:
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace sml
