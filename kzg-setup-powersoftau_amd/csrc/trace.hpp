// roctx ranges around the host-side stages of the library (SURVEY §5 tracing): H2D staging, the
// wait for a chunk's output (kernel + D2H), each preprocess section per shard thread, the two
// BLAKE2b digests, pread / pwrite, the multi-GPU enqueue. rocprofv3 --marker-trace records them
// beside the kernel and memory-copy traces (tools/stage_summary.py turns the three into a
// per-stage breakdown).
//
// roctx is optional at run time: librocprofiler-sdk-roctx.so.1 is bound with dlopen on first use
// (as comm.hip binds RCCL), so the library loads on a host without rocprofiler-sdk and every range
// is then a no-op. Under rocprofv3 the tool has already loaded the same library, and dlopen
// returns that copy, so the ranges reach the tracer as before.
#pragma once
#include <dlfcn.h>

namespace kzgpot {

struct RoctxApi {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  int (*name_thread)(const char*) = nullptr;
};

inline const RoctxApi& roctx() {
  static const RoctxApi api = [] {
    RoctxApi a;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return a;
    a.push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
    a.pop = (int (*)())dlsym(h, "roctxRangePop");
    a.name_thread = (int (*)(const char*))dlsym(h, "roctxNameOsThread");
    if (!a.push || !a.pop) a.push = nullptr, a.pop = nullptr;  // ranges need both ends
    return a;
  }();
  return api;
}

struct TraceRange {
  explicit TraceRange(const char* what) : on_(roctx().push != nullptr) {
    if (on_) roctx().push(what);
  }
  ~TraceRange() {
    if (on_) roctx().pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

inline void trace_thread(const char* name) {
  if (roctx().name_thread) roctx().name_thread(name);
}

}  // namespace kzgpot
