// roctx ranges (SURVEY §5 tracing) around the engine's host-side phases:
// encode calls, E-step accumulate chunks, seed-mining stages, the trainer's
// RCCL reductions.  Visible with `rocprofv3 --marker-trace --kernel-trace`;
// without a tool attached a range is two cheap calls into librocprofiler-
// sdk-roctx.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

namespace spm_amd {

class TraceRange {
 public:
  explicit TraceRange(const char *name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange &) = delete;
  TraceRange &operator=(const TraceRange &) = delete;
};

}  // namespace spm_amd
