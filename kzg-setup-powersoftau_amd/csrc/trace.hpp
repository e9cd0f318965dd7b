// roctx ranges around the host-side stages of the library (SURVEY §5 tracing): H2D staging, the
// wait for a chunk's output (kernel + D2H), each preprocess section per shard thread, the two
// BLAKE2b digests, pread / pwrite, the multi-GPU enqueue. rocprofv3 --marker-trace records them
// beside the kernel and memory-copy traces (tools/stage_summary.py turns the three into a
// per-stage breakdown); without a profiler attached a range is two cheap library calls.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace kzgpot {

struct TraceRange {
  explicit TraceRange(const char* what) { roctxRangePushA(what); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

inline void trace_thread(const char* name) { roctxNameOsThread(name); }

}  // namespace kzgpot
