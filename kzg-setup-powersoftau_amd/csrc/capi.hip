// C ABI (include/kzgpot.h): host-buffer and device-buffer entry points for the point codec, and
// the kgz / fastkzg file pipeline. No CPU fallback exists: without a GPU every entry point
// returns KZGPOT_E_DEVICE.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <strings.h>

#include <ctype.h>
#include <errno.h>
#include <fcntl.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "blake2b.hpp"
#include "codec.hpp"
#include "trace.hpp"

using namespace kzgpot;

namespace {

constexpr uint64_t kNoBad = ~0ull;

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "kzgpot: %s failed: %s (%s:%d)\n", #expr, hipGetErrorString(e_), \
              __FILE__, __LINE__);                                                       \
      return KZGPOT_E_DEVICE;                                                            \
    }                                                                                    \
  } while (0)

// ---------------------------------------------------------------- host resources at the C ABI
// No exception may cross an extern "C" entry (it would std::terminate the caller's process, where
// the reference returns a Result, preprocess-kgz.rs:105-110). Host threads are started through
// start_thread, which reports a failed start (std::system_error EAGAIN under a process or thread
// limit, std::bad_alloc) as false; every thread body catches its own exceptions; every entry that
// allocates runs under api_guard; and the threads a call started are joined on every exit path
// (JoinOnExit, ThreadGroup) before it returns.

#ifdef KZGPOT_TEST_HOOKS
// Fault injection, test build only (tests/kzgpot_test_hooks.h, kzgpot_test_inject_host_fault):
// from the (skip + 1)-th event of `site` on, every such event fails until the site is cleared.
std::atomic<int> g_fault_site{0};
std::atomic<long> g_fault_skip{0};
bool injected(int site) {
  if (g_fault_site.load() != site) return false;
  return g_fault_skip.fetch_sub(1) <= 0;
}
#endif
enum { kFaultThread = 1, kFaultHostBuf = 2 };

template <class F>
bool start_thread(std::thread& t, F&& f) noexcept {
  try {
#ifdef KZGPOT_TEST_HOOKS
    if (injected(kFaultThread)) throw std::system_error(EAGAIN, std::generic_category(), "injected thread fault");
#endif
    t = std::thread(std::forward<F>(f));
    return true;
  } catch (...) {
    return false;
  }
}

template <class F>
int api_guard(F&& f) noexcept {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return KZGPOT_E_OUT_OF_MEMORY;
  } catch (const std::system_error&) {  // a host thread or lock could not be obtained
    return KZGPOT_E_OUT_OF_MEMORY;
  } catch (...) {
    return KZGPOT_E_DEVICE;
  }
}

// Joins a thread on scope exit (after running `before`, e.g. telling it to stop), so that an
// early return or an exception never destroys a joinable std::thread.
struct JoinOnExit {
  std::thread& t;
  std::function<void()> before;
  ~JoinOnExit() {
    if (!t.joinable()) return;
    if (before) before();
    t.join();
  }
};

// The shard threads of one section: joined on destruction whatever path leaves the scope.
class ThreadGroup {
 public:
  explicit ThreadGroup(size_t n) { th_.reserve(n); }
  ~ThreadGroup() { join(); }
  template <class F>
  bool start(F&& f) noexcept {
    std::thread t;
    if (!start_thread(t, std::forward<F>(f))) return false;
    th_.push_back(std::move(t));  // no reallocation: reserved
    return true;
  }
  void join() {
    for (auto& t : th_)
      if (t.joinable()) t.join();
  }

 private:
  std::vector<std::thread> th_;
};

// Per-device staging for the host-buffer API (grown on demand, reused across calls): two slots,
// each with its own stream, so chunk k's kernel runs while the host thread moves chunk k-1's
// output back and chunk k+1's input in (run_host).
struct Slot {
  hipStream_t stream = nullptr;
  void* d_in = nullptr;
  void* d_out = nullptr;
  uint8_t* d_status = nullptr;
  unsigned long long* d_key = nullptr;
  size_t cap_in = 0, cap_out = 0, cap_status = 0;
};
struct DevCtx {
  std::mutex mu;
  Slot slot[2];
};
DevCtx g_ctx[64];

int ensure(void** p, size_t* cap, size_t need) {
  if (*cap >= need) return 0;
  if (*p) HIP_TRY(hipFree(*p));
  *p = nullptr;
  *cap = 0;
  HIP_TRY(hipMalloc(p, need));
  *cap = need;
  return 0;
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Restores the caller's current HIP device on scope exit: the library switches devices per
// shard, and a torch rank on cuda:3 must still be on cuda:3 after any call.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Bytes [0, ready) of a transcript that is still being read from disk are valid; consumers (the
// GPU chunk loop, the transcript hasher) wait for the range they need.
class Watermark {
 public:
  void advance(size_t to) {
    std::lock_guard<std::mutex> l(mu_);
    ready_ = to;
    cv_.notify_all();
  }
  void fail() {
    std::lock_guard<std::mutex> l(mu_);
    failed_ = true;
    cv_.notify_all();
  }
  bool failed() {
    std::lock_guard<std::mutex> l(mu_);
    return failed_;
  }
  // false if the reader failed before `upto` bytes arrived
  bool wait(size_t upto) {
    std::unique_lock<std::mutex> l(mu_);
    cv_.wait(l, [&] { return failed_ || ready_ >= upto; });
    return ready_ >= upto;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  size_t ready_ = 0;
  bool failed_ = false;
};

// Where a run_host input lives while the file is still being read: wait until `end` is readable.
struct InputWait {
  Watermark* wm;
  const uint8_t* base;
  bool operator()(const uint8_t* end) const { return !wm || wm->wait((size_t)(end - base)); }
};

int decode_key(uint64_t key, int64_t* first_bad) {
  // no kernel writes key 0 (every rejection has status >= 1): it is the multi-rank "a rank failed"
  // word (KZGPOT_KEY_RANK_FAILED), never "point 0 accepted"
  if (key == kNoBad || key == KZGPOT_KEY_RANK_FAILED) {
    if (first_bad) *first_bad = -1;
    return key == kNoBad ? 0 : KZGPOT_E_RANK_FAILED;
  }
  if (first_bad) *first_bad = (int64_t)(key >> 8);
  return -(int)(key & 0xff);
}

// The chunks of a host-buffer call (run_host). Only the first chunk's input copy and the last
// chunk's output copy are exposed (every other copy runs while a kernel does), so a long call
// starts with a 2^17-point chunk (one wave of blocks on 256 CUs) growing x4 per chunk below cmax,
// and ends with chunks halving from <= cmax / 2 down to 2^17: chunk k's output copy then hides
// behind chunk k + 1's kernel, which is at least half as long, and the exposed copies are of
// 2^17-point chunks instead of cmax-point ones (2^25 G1 points: 100 + 201 MB at cmax = 2^21). A
// call too short for both ramps keeps equal chunks. Chunks are multiples of 256 points but one.
struct ChunkPlan {
  size_t n = 0, cmax = 0, first = 0, last = 0;  // equal-chunk plan: [first, cmax, ..., ragged, last]
  bool ramp = false;
  size_t up = 0, mid = 0, down = 0, sum_up = 0, rest = 0;  // ramp plan: up x4, mid x cmax, down /2
#ifndef KZGPOT_CHUNK_END_LOG2  // build knobs for chunk-plan experiments (tools/ab_host_plans.sh)
#define KZGPOT_CHUNK_END_LOG2 17
#endif
#ifndef KZGPOT_CHUNK_FLOOR_LOG2
#define KZGPOT_CHUNK_FLOOR_LOG2 17
#endif
  static constexpr size_t kMin = (size_t)1 << KZGPOT_CHUNK_END_LOG2;      // the ramps' end chunks
  static constexpr size_t kFloor = (size_t)1 << KZGPOT_CHUNK_FLOOR_LOG2;  // the smallest cmax
  ChunkPlan(size_t n_, bool small_first) : n(n_) {
    cmax = std::min<size_t>(n, (size_t)1 << 21);
    // up to 2^24 points: at least 8 chunks, so that copies overlap kernels at all
    if (n > 2 * kFloor) cmax = std::min(cmax, std::max(kFloor, ((n + 7) / 8 + 255) & ~(size_t)255));
    // a streaming consumer (the output digest) starts on the first chunk's records: 2^16 points
    first = (small_first && n > cmax) ? std::min<size_t>(cmax, (size_t)1 << 16) : cmax;
    if (cmax < 2 * kMin) {  // no room for a ramp (calls below ~2^21 points)
      // half-size end chunks shorten the exposed first input and last output copies there: 2^20
      // G2 / G1 points 12.7-13.9 / 14.4-16.4 % over device-resident against 16.0-16.3 / 18.1-18.6 %
      // with equal chunks, same box (profiles/r06za_ab_plans, variants A and old)
      if (n > 2 * kMin && cmax == kMin) first = last = kMin / 2;
      return;
    }
    for (size_t x = kMin; x < cmax; x *= 4) up++, sum_up += x;
    for (size_t x = kMin; 2 * x <= cmax; x *= 2) down++;  // down: kMin 2^(down-1), ..., 2 kMin, kMin
    const size_t sum_down = kMin * (((size_t)1 << down) - 1);
    if (n <= sum_up + sum_down + cmax) return;  // too short: equal chunks
    ramp = true;
    rest = n - sum_up - sum_down;
    mid = (rest + cmax - 1) / cmax;
  }
  size_t count() const {
    if (ramp) return up + mid + down;
    return first >= n ? 1 : 1 + (n - first - last + cmax - 1) / cmax + (last ? 1 : 0);
  }
  void span(size_t j, size_t& off, size_t& m) const {  // chunk j = points [off, off + m)
    if (!ramp) {
      if (last && j + 1 == count()) {
        off = n - last, m = last;
        return;
      }
      off = j == 0 ? 0 : first + (j - 1) * cmax;
      m = std::min(j == 0 ? first : cmax, n - last - off);
    } else if (j < up) {
      off = kMin * ((((size_t)1 << (2 * j)) - 1) / 3);
      m = kMin << (2 * j);
    } else if (j < up + mid) {
      off = sum_up + (j - up) * cmax;
      m = std::min(cmax, sum_up + rest - off);
    } else {
      const size_t k = j - up - mid;
      off = sum_up + rest + kMin * (((size_t)1 << down) - ((size_t)1 << (down - k)));
      m = kMin << (down - 1 - k);
    }
  }
  size_t max_chunk() const { return cmax; }
};

// Run one op over host buffers on device `dev`, in chunks that bound the staging memory. Chunks
// alternate between two slots/streams: while the GPU decodes chunk k, this thread copies chunk
// k-1's output out and chunk k+1's input in (pageable copies block the host, not the other
// stream), so PCIe time hides behind the kernels except for the first input and last output.
// on_chunk (may be null) is called with (first point, count) of each chunk once its output is
// in `out`, in order — the end-to-end preprocess streams the output digest from it.
// keep_out = false: the records are validated but not copied back (out may be null).
// in_wait (may be null): called before each chunk's input is copied, for inputs still streaming
// in from disk.
int run_host(int dev, CodecOp op, const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad,
             uint8_t* status, const std::function<void(size_t, size_t)>* on_chunk = nullptr, bool keep_out = true,
             const InputWait* in_wait = nullptr) {
  if (first_bad) *first_bad = -1;
  if (n == 0) return 0;
  if (!in || (keep_out && !out)) return KZGPOT_E_INVALID_ARG;
  if (dev < 0 || dev >= device_count() || dev >= 64) return KZGPOT_E_DEVICE;
  DevCtx& c = g_ctx[dev];
  std::lock_guard<std::mutex> lock(c.mu);
  DeviceGuard guard;
  HIP_TRY(hipSetDevice(dev));
  const uint64_t rin = in_record(op), rout = out_record(op);
  // 2 x 2^21 x 288 B of staging at most. A call of up to 2^24 points is cut into at least 8 chunks
  // so that its PCIe copies overlap its kernels (2^20 G2 points in one chunk: 31 % over the
  // device-resident time, profiles/r04a_bench_n1.json); longer calls ramp their chunk sizes up and
  // down (ChunkPlan). A streaming consumer (on_chunk: the output digest of the e2e pipeline) can
  // only start on the first chunk's records, so an equal-chunk call gives it a 2^16-point first chunk.
  const ChunkPlan plan(n, on_chunk != nullptr);
  const size_t chunk = plan.max_chunk(), nchunks = plan.count();
  auto span = [&](size_t j, size_t& off, size_t& m) { plan.span(j, off, m); };
  for (int k = 0; k < (nchunks > 1 ? 2 : 1); k++) {
    Slot& sl = c.slot[k];
    if (!sl.stream) HIP_TRY(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
    if (ensure(&sl.d_in, &sl.cap_in, chunk * rin)) return KZGPOT_E_DEVICE;
    if (ensure(&sl.d_out, &sl.cap_out, chunk * rout)) return KZGPOT_E_DEVICE;
    if (status && ensure((void**)&sl.d_status, &sl.cap_status, chunk)) return KZGPOT_E_DEVICE;
    if (!sl.d_key) HIP_TRY(hipMalloc(&sl.d_key, sizeof(unsigned long long)));
  }
  uint64_t best = kNoBad;
  // an error exit leaves no copy or kernel of this call in flight (the slots are reused)
  auto quiesce = [&](int code) {
    for (int k = 0; k < 2; k++)
      if (c.slot[k].stream) (void)hipStreamSynchronize(c.slot[k].stream);
    return code;
  };
  // drain chunk j: its output (and status, key) back to the host
  auto drain = [&](size_t j) -> int {
    TraceRange tr_("kzgpot.d2h");  // waits for chunk j's kernel, then its output copy
    Slot& sl = c.slot[j & 1];
    size_t off, m;
    span(j, off, m);
    if (keep_out) HIP_TRY(hipMemcpyAsync(out + off * rout, sl.d_out, m * rout, hipMemcpyDeviceToHost, sl.stream));
    if (status) HIP_TRY(hipMemcpyAsync(status + off, sl.d_status, m, hipMemcpyDeviceToHost, sl.stream));
    unsigned long long key = kNoBad;
    HIP_TRY(hipMemcpyAsync(&key, sl.d_key, sizeof key, hipMemcpyDeviceToHost, sl.stream));
    HIP_TRY(hipStreamSynchronize(sl.stream));
    if (key != kNoBad && best == kNoBad) best = ((uint64_t)(key >> 8) + off) << 8 | (key & 0xff);
    if (on_chunk && best == kNoBad) {
      TraceRange tc_("kzgpot.handoff");
      try {
        (*on_chunk)(off, m);
      } catch (...) {  // the consumer could not queue the range (std::bad_alloc)
        return quiesce(KZGPOT_E_OUT_OF_MEMORY);
      }
    }
    return 0;
  };
  for (size_t j = 0; j < nchunks; j++) {
    Slot& sl = c.slot[j & 1];
    size_t off, m;
    span(j, off, m);
    if (in_wait) {
      TraceRange tw_("kzgpot.wait_input");  // the transcript still streaming in from disk
      if (!(*in_wait)(in + (off + m) * rin)) return quiesce(KZGPOT_E_IO);  // the transcript read failed
    }
    {
      TraceRange th_("kzgpot.h2d");  // a pageable copy: the host thread stages it
      HIP_TRY(hipMemcpyAsync(sl.d_in, in + off * rin, m * rin, hipMemcpyHostToDevice, sl.stream));
    }
    HIP_TRY(hipMemsetAsync(sl.d_key, 0xff, sizeof(unsigned long long), sl.stream));
    HIP_TRY(launch_codec(op, sl.d_in, sl.d_out, m, flags, sl.d_key, status ? sl.d_status : nullptr, sl.stream));
    if (j > 0)
      if (const int r = drain(j - 1)) return quiesce(r);  // chunks finish in order: best stays the first
  }
  if (const int r = drain(nchunks - 1)) return quiesce(r);
  return decode_key(best, first_bad);
}

int current_device() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return -1;
  return d;
}

int run_dev(CodecOp op, const void* d_in, size_t n, void* d_out, uint32_t flags, uint64_t* d_bad_key,
            uint8_t* d_status, void* stream) {
  if (!d_bad_key) return KZGPOT_E_INVALID_ARG;
  if (n && (!d_in || !d_out)) return KZGPOT_E_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemsetAsync(d_bad_key, 0xff, sizeof(uint64_t), s));
  HIP_TRY(launch_codec(op, d_in, d_out, n, flags, (unsigned long long*)d_bad_key, d_status, s));
  return 0;
}

}  // namespace

extern "C" {

int kzgpot_g1_decompress_ex(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad,
                            uint8_t* status) {
  return api_guard(
      [&] { return run_host(current_device(), CodecOp::G1Decompress, in, n, out, flags, first_bad, status); });
}
int kzgpot_g2_decompress_ex(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad,
                            uint8_t* status) {
  return api_guard(
      [&] { return run_host(current_device(), CodecOp::G2Decompress, in, n, out, flags, first_bad, status); });
}
int kzgpot_g1_transcode_uncompressed_ex(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags,
                                        int64_t* first_bad, uint8_t* status) {
  return api_guard([&] {
    return run_host(current_device(), CodecOp::G1Transcode, in, n, out, flags & KZGPOT_SUBGROUP_REF, first_bad,
                    status);
  });
}
int kzgpot_g2_transcode_uncompressed_ex(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags,
                                        int64_t* first_bad, uint8_t* status) {
  return api_guard([&] {
    return run_host(current_device(), CodecOp::G2Transcode, in, n, out, flags & KZGPOT_SUBGROUP_REF, first_bad,
                    status);
  });
}
int kzgpot_g1_decompress(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad) {
  return kzgpot_g1_decompress_ex(in, n, out, flags, first_bad, nullptr);
}
int kzgpot_g2_decompress(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad) {
  return kzgpot_g2_decompress_ex(in, n, out, flags, first_bad, nullptr);
}
int kzgpot_g1_transcode_uncompressed(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags,
                                     int64_t* first_bad) {
  return kzgpot_g1_transcode_uncompressed_ex(in, n, out, flags, first_bad, nullptr);
}
int kzgpot_g2_transcode_uncompressed(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags,
                                     int64_t* first_bad) {
  return kzgpot_g2_transcode_uncompressed_ex(in, n, out, flags, first_bad, nullptr);
}

int kzgpot_g1_decompress_dev(const void* d_in, size_t n, void* d_out, uint32_t flags, uint64_t* d_bad_key,
                             uint8_t* d_status, void* stream) {
  return run_dev(CodecOp::G1Decompress, d_in, n, d_out, flags, d_bad_key, d_status, stream);
}
int kzgpot_g2_decompress_dev(const void* d_in, size_t n, void* d_out, uint32_t flags, uint64_t* d_bad_key,
                             uint8_t* d_status, void* stream) {
  return run_dev(CodecOp::G2Decompress, d_in, n, d_out, flags, d_bad_key, d_status, stream);
}
int kzgpot_g1_transcode_uncompressed_dev(const void* d_in, size_t n, void* d_out, uint32_t flags,
                                         uint64_t* d_bad_key, uint8_t* d_status, void* stream) {
  return run_dev(CodecOp::G1Transcode, d_in, n, d_out, flags & KZGPOT_SUBGROUP_REF, d_bad_key, d_status, stream);
}
int kzgpot_g2_transcode_uncompressed_dev(const void* d_in, size_t n, void* d_out, uint32_t flags,
                                         uint64_t* d_bad_key, uint8_t* d_status, void* stream) {
  return run_dev(CodecOp::G2Transcode, d_in, n, d_out, flags & KZGPOT_SUBGROUP_REF, d_bad_key, d_status, stream);
}
int kzgpot_decode_bad_key(uint64_t key, int64_t* first_bad) { return decode_key(key, first_bad); }

// ------------------------------------------------------------------------------- file pipeline
uint64_t kzgpot_contribution_size(uint32_t n_log2) {
  const uint64_t n = 1ull << n_log2;
  return (2 * n - 1) * 48 + n * 96 + 2 * n * 48 + 96 + (3 * 192 + 6 * 96) + 64;
}
uint64_t kzgpot_output_size(uint32_t n_log2, int mode) {
  const uint64_t n = 1ull << n_log2;
  return mode == KZGPOT_MODE_FASTKZG ? (2 * n - 1) * 96 + n * 96 + 2 * 192 + n * 192
                                     : (2 * n - 1) * 96 + n * 96 + 576;
}

}  // extern "C"

namespace {

// Consumes byte ranges in submission order on its own thread: the output digest (BLAKE2b is one
// sequential stream) and the output file writer, so both run while the GPU is still decoding
// later sections.
class OrderedWorker {
 public:
  OrderedWorker(const char* name, std::function<bool(const uint8_t*, size_t)> fn)
      : name_(name), fn_(std::move(fn)) {}
  ~OrderedWorker() { finish(); }
  // false if the thread could not be started (the worker is then unusable)
  bool start() { return start_thread(th_, [this] { run(); }); }
  // may throw std::bad_alloc (the queue)
  void push(const uint8_t* p, size_t n) {
    std::lock_guard<std::mutex> l(mu_);
    q_.emplace_back(p, n);
    cv_.notify_one();
  }
  // waits for every pushed range; false if any range failed
  bool finish() {
    {
      std::lock_guard<std::mutex> l(mu_);
      if (done_) return ok_;
      done_ = true;
      cv_.notify_one();
    }
    if (!th_.joinable()) return ok_ = false;
    th_.join();
    return ok_;
  }

 private:
  void run() {
    try {
      trace_thread(name_);
    } catch (...) {
    }
    for (;;) {
      std::pair<const uint8_t*, size_t> item;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [this] { return done_ || !q_.empty(); });
        if (q_.empty()) return;
        item = q_.front();
        q_.pop_front();
      }
      try {
        TraceRange tr_(name_);
        if (ok_ && !fn_(item.first, item.second)) ok_ = false;
      } catch (...) {
        ok_ = false;
      }
    }
  }
  const char* name_;
  std::function<bool(const uint8_t*, size_t)> fn_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<const uint8_t*, size_t>> q_;
  bool done_ = false;
  bool ok_ = true;
  std::thread th_;
};

bool pwrite_all(int fd, const uint8_t* p, size_t n, uint64_t off) {
  while (n) {
    const ssize_t w = pwrite(fd, p, std::min<size_t>(n, (size_t)1 << 30), (off_t)off);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    p += w, n -= (size_t)w, off += (uint64_t)w;
  }
  return true;
}

// Where the transcript comes from and where the output goes, besides the two buffers.
struct PipelineIo {
  Watermark* in_wm = nullptr;  // non-null: the transcript is still being read from disk
  int out_fd = -1;             // >= 0: output ranges are written here (file order offsets) as they land
};

// 128 hex digits (either case): the form of expect_transcript_digest
bool is_hex128(const char* s) {
  for (int i = 0; i < 128; i++)
    if (!isxdigit((unsigned char)s[i])) return false;
  return s[128] == '\0';
}

int preprocess_run(const uint8_t* tr, size_t len, uint8_t* out, int mode, uint32_t n_log2, int n_shards,
                   const char* expect_in_hex, char* in_hex, char* out_hex, int* bad_section, int64_t* bad_index,
                   const PipelineIo& io) {
  // transcript digest (download_parameters' check, preprocess-kgz.rs:51-61) beside the GPU pass;
  // a transcript still streaming from disk is hashed as it arrives. It is the call's critical path
  // (one sequential BLAKE2b stream), so it starts before anything touches HIP: in a fresh process
  // (the CLI drop-ins) the runtime's initialisation then overlaps it instead of preceding it.
  uint8_t in_digest[64];
  bool in_ok = true;
  std::atomic<bool> abandon{false};  // set when the call fails: the hasher stops at its next piece
  std::thread in_hash;
  JoinOnExit in_hash_join{in_hash, [&abandon] { abandon = true; }};  // any early exit
  const bool want_in = expect_in_hex || in_hex;
  TraceRange call_("kzgpot.preprocess");
  if (want_in && !start_thread(in_hash, [&] {
        try {
          trace_thread("kzgpot.blake2b.transcript");
          TraceRange tr_("kzgpot.blake2b.transcript");
          Blake2b h;
          for (size_t off = 0; off < len;) {
            const size_t m = std::min<size_t>(len - off, (size_t)32 << 20);
            if (abandon.load(std::memory_order_relaxed) || (io.in_wm && !io.in_wm->wait(off + m))) {
              in_ok = false;
              return;
            }
            h.update(tr + off, m);
            off += m;
          }
          h.finalize(in_digest);
        } catch (...) {
          in_ok = false;
        }
      }))
    return KZGPOT_E_OUT_OF_MEMORY;
  const int ndev = device_count();
  if (ndev <= 0) return KZGPOT_E_DEVICE;
  if (n_shards <= 0) n_shards = ndev;
  n_shards = std::min(n_shards, 64);
  int dev0 = current_device();
  if (dev0 < 0 || dev0 >= ndev) dev0 = 0;
  const uint64_t n = 1ull << n_log2;
  const InputWait in_wait{io.in_wm, tr};
  // output consumers, fed the file's byte ranges in file order
  Blake2b out_h;
  std::unique_ptr<OrderedWorker> out_hash, out_write;
  if (out_hex) {
    out_hash.reset(new OrderedWorker("kzgpot.blake2b.output", [&](const uint8_t* p, size_t m) {
      out_h.update(p, m);
      return true;
    }));
    if (!out_hash->start()) return KZGPOT_E_OUT_OF_MEMORY;
  }
  if (io.out_fd >= 0) {
    out_write.reset(new OrderedWorker(
        "kzgpot.pwrite", [&](const uint8_t* p, size_t m) { return pwrite_all(io.out_fd, p, m, (uint64_t)(p - out)); }));
    if (!out_write->start()) return KZGPOT_E_OUT_OF_MEMORY;
  }
  const bool sink = out_hash || out_write;
  auto push = [&](const uint8_t* p, size_t m) {
    if (out_hash) out_hash->push(p, m);
    if (out_write) out_write->push(p, m);
  };

  // powersoftau Accumulator section order (after the 64-B hash)
  const uint64_t cnt[5] = {2 * n - 1, n, n, n, 1};
  static const char* const kSectionRange[5] = {"kzgpot.section.tau_g1", "kzgpot.section.tau_g2",
                                               "kzgpot.section.alpha_tau_g1", "kzgpot.section.beta_tau_g1",
                                               "kzgpot.section.beta_g2"};
  const bool g2[5] = {false, true, false, false, true};
  // read back by read_g1/read_g2 (checked) in each binary: kgz τG1, τG2, ατG1; fastkgz + βτG1
  const bool checked[5] = {true, true, true, mode == KZGPOT_MODE_FASTKZG, false};
  // output layout (A7): τG1 and ατG1 are decoded straight into their place in `out`; fastkzg's
  // powers_of_h (= τG2) too; sections the file does not hold (kgz τG2 beyond h, beta_h; βτG1;
  // βG2) are decoded and checked on the GPU but never copied back (dst = null)
  const uint64_t off_gamma = (2 * n - 1) * 96, off_tail = off_gamma + n * 96;
  uint8_t* dst[5] = {out, nullptr, out + off_gamma, nullptr, nullptr};
  if (mode == KZGPOT_MODE_FASTKZG) dst[1] = out + off_tail + 2 * 192;
  int ret = 0;
  const uint8_t* p = tr + 64;
  for (int s = 0; s < 5 && !ret; s++) {
    const CodecOp op = g2[s] ? CodecOp::G2Decompress : CodecOp::G1Decompress;
    const uint64_t rin = in_record(op), rout = out_record(op);
    const uint32_t fl = checked[s] ? 0u : KZGPOT_NO_SUBGROUP_CHECK;
    // contiguous shards, one host thread each
    std::vector<int> rc(n_shards, 0);
    std::vector<int64_t> fb(n_shards, -1);
    const uint64_t per = (cnt[s] + n_shards - 1) / n_shards;
    // The τG1 / ατG1 output (file order) is handed to the digest and writer threads chunk by chunk
    // as it lands, so hashing and writing overlap the GPU pass instead of following it. Each shard
    // reports its chunks in order; a record goes out once every shard before it has landed up to
    // it (cursor), so the consumers see the file in order at any shard count.
    const bool stream = sink && (s == 0 || s == 2);
    std::mutex land_mu;
    std::vector<uint64_t> landed(n_shards, 0);  // shard g: points [g per, g per + landed[g]) are in `out`
    uint64_t cursor = 0;                         // section points [0, cursor) have been pushed
    auto land = [&, s, rout](int g, size_t off, size_t m) {
      std::lock_guard<std::mutex> l(land_mu);
      landed[g] = off + m;
      while (cursor < cnt[s]) {
        const uint64_t h = cursor / per, avail = h * per + landed[h];
        if (avail <= cursor) break;
        push(dst[s] + cursor * rout, (avail - cursor) * rout);
        cursor = avail;
      }
    };
    {
      // declared after everything the shards use, so it joins them first on any exit
      ThreadGroup th(n_shards);
      for (int g = 0; g < n_shards; g++) {
        const uint64_t lo = std::min(cnt[s], g * per), hi = std::min(cnt[s], lo + per);
        const bool started = th.start([&, g, lo, hi] {
          try {
            trace_thread("kzgpot.shard");
            TraceRange tr_(kSectionRange[s]);
            const std::function<void(size_t, size_t)> on_chunk = [&, g](size_t off, size_t m) { land(g, off, m); };
            rc[g] = run_host((dev0 + g) % ndev, op, p + lo * rin, hi - lo, dst[s] ? dst[s] + lo * rout : nullptr,
                             fl, &fb[g], nullptr, stream ? &on_chunk : nullptr, dst[s] != nullptr, &in_wait);
          } catch (...) {
            rc[g] = KZGPOT_E_OUT_OF_MEMORY;
          }
          if (fb[g] >= 0) fb[g] += (int64_t)lo;
        });
        if (!started) {  // the shards already running finish their ranges; this one and the rest never run
          for (int k = g; k < n_shards; k++) rc[k] = KZGPOT_E_OUT_OF_MEMORY;
          break;
        }
      }
    }  // joined
    // shards are contiguous and in index order: the first failing shard holds the smallest index
    for (int g = 0; g < n_shards && !ret; g++)
      if (rc[g]) {
        ret = rc[g];
        if (bad_section) *bad_section = s;
        if (bad_index) *bad_index = fb[g];
      }
    p += cnt[s] * rin;
    if (!ret && stream && cursor != cnt[s]) ret = KZGPOT_E_IO;  // cannot happen: every shard succeeded, so every chunk landed
  }
  uint8_t h_beta_h[2 * 192];  // kgz: τG2[0..1] for the VerifierKey (the section itself was checked)
  if (!ret && mode == KZGPOT_MODE_KZG) {
    int64_t fb2 = -1;
    ret = run_host(dev0, CodecOp::G2Decompress, tr + 64 + cnt[0] * 48, 2, h_beta_h, 0, &fb2, nullptr, nullptr, true,
                   &in_wait);
  }
  if (!ret) {
    uint8_t* o = out + off_tail;
    const uint8_t* tau_g2 = mode == KZGPOT_MODE_FASTKZG ? dst[1] : h_beta_h;
    if (mode == KZGPOT_MODE_KZG) {  // VerifierKey{g, gamma_g, h, beta_h} (preprocess-kgz.rs:177-194)
      memcpy(o, out, 96);
      memcpy(o + 96, out + off_gamma, 96);
      memcpy(o + 192, tau_g2, 384);
      if (sink) push(o, 576);
    } else {  // h, beta_h, neg_powers_of_h (empty), powers_of_h (preprocess-fastkgz.rs:200-208)
      memcpy(o, tau_g2, 384);
      if (sink) push(o, 384 + n * 192);
    }
  }
  if (out_write && !out_write->finish() && !ret) ret = KZGPOT_E_IO;
  if (out_hash) {
    out_hash->finish();
    if (!ret) {
      uint8_t d[64];
      out_h.finalize(d);
      to_hex(d, out_hex);
    }
  }
  if (want_in) {
    in_hash.join();
    if (!in_ok) {
      if (!ret) ret = KZGPOT_E_IO;
    } else {
      char hex[129];
      to_hex(in_digest, hex);
      if (in_hex) memcpy(in_hex, hex, 129);
      // The reference checks the digest before it decodes anything (download_parameters runs
      // first), so a wrong transcript is reported as such even if it also holds a bad point.
      if (expect_in_hex && strncasecmp(hex, expect_in_hex, 128) != 0) {
        ret = KZGPOT_E_DIGEST;
        if (bad_section) *bad_section = -1;
        if (bad_index) *bad_index = -1;
      }
    }
  }
  return ret;
}

// The two `main`s (preprocess-kgz.rs:162-199, preprocess-fastkgz.rs:180-213) minus the download.
// n_shards host threads each decode a contiguous shard of every section; shard g runs on device
// (current + g) % device_count, so n_shards above the device count oversubscribes (the shards of
// one device then run one after another) — which is how the multi-shard path is tested on one GPU.
// Host resources that run out (memory, a thread) end the call with KZGPOT_E_OUT_OF_MEMORY after
// every thread it started has been joined.
int preprocess_impl(const uint8_t* tr, size_t len, uint8_t* out, int mode, uint32_t n_log2, int n_shards,
                    const char* expect_in_hex, char* in_hex, char* out_hex, int* bad_section, int64_t* bad_index,
                    const PipelineIo& io = PipelineIo()) noexcept {
  if (bad_section) *bad_section = -1;
  if (bad_index) *bad_index = -1;
  if (!tr || !out || n_log2 < 1 || n_log2 > 30 || (mode != KZGPOT_MODE_KZG && mode != KZGPOT_MODE_FASTKZG))
    return KZGPOT_E_INVALID_ARG;
  if (expect_in_hex && !is_hex128(expect_in_hex)) return KZGPOT_E_INVALID_ARG;
  if (len != kzgpot_contribution_size(n_log2)) return KZGPOT_E_SIZE;
  const int r = api_guard([&] {
    return preprocess_run(tr, len, out, mode, n_log2, n_shards, expect_in_hex, in_hex, out_hex, bad_section,
                          bad_index, io);
  });
  if (r == KZGPOT_E_OUT_OF_MEMORY) {
    if (bad_section) *bad_section = -1;
    if (bad_index) *bad_index = -1;
  }
  return r;
}

}  // namespace

extern "C" {

int kzgpot_blake2b(const uint8_t* data, size_t len, uint8_t* digest64) {
  if ((!data && len) || !digest64) return KZGPOT_E_INVALID_ARG;
  blake2b_512(data, len, digest64);
  return 0;
}

int kzgpot_preprocess_buffer_ex(const uint8_t* tr, size_t len, uint8_t* out, int mode, uint32_t n_log2,
                                int n_gpus, const char* expect_transcript_digest, char* transcript_digest,
                                char* output_digest, int* bad_section, int64_t* bad_index) {
  return preprocess_impl(tr, len, out, mode, n_log2, n_gpus, expect_transcript_digest, transcript_digest,
                         output_digest, bad_section, bad_index);
}
int kzgpot_preprocess_buffer(const uint8_t* tr, size_t len, uint8_t* out, int mode, uint32_t n_log2, int n_gpus,
                             int* bad_section, int64_t* bad_index) {
  return preprocess_impl(tr, len, out, mode, n_log2, n_gpus, nullptr, nullptr, nullptr, bad_section, bad_index);
}

}  // extern "C"

namespace {
// A large host buffer of the file path (the 604 MB transcript, the 0.6-1.0 GB output): a 2 MiB
// aligned anonymous mapping with MADV_HUGEPAGE, so faulting it in (pread, the D2H copies) and
// unmapping it at the end costs one fault / one free per 2 MiB instead of per 4 KiB page (with
// transparent huge pages in "madvise" mode; elsewhere it is an ordinary mapping).
class HostBuf {
 public:
  explicit HostBuf(size_t n) {
    constexpr size_t kHuge = (size_t)2 << 20;
    map_ = n + kHuge;
#ifdef KZGPOT_TEST_HOOKS
    void* m = injected(kFaultHostBuf) ? MAP_FAILED
                                      : mmap(nullptr, map_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
#else
    void* m = mmap(nullptr, map_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
#endif
    if (m == MAP_FAILED) {
      map_ = 0;
      return;
    }
    base_ = (uint8_t*)m;
    p_ = (uint8_t*)(((uintptr_t)m + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
    (void)madvise(p_, n, MADV_HUGEPAGE);
  }
  ~HostBuf() {
    if (map_) munmap(base_, map_);
  }
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  uint8_t* get() const { return p_; }

 private:
  size_t map_ = 0;
  uint8_t* base_ = nullptr;
  uint8_t* p_ = nullptr;
};

// Unmapping a file call's 1.2-1.6 GB of faulted-in pages takes ~77 ms of kernel time
// (profiles/r04e_e2e_stages.json, after_pipeline_ms) that the caller need not wait for, so it
// runs on a helper thread. At most one release is outstanding when a call returns: the next file
// call joins the previous helper when it hands over its own buffers (by then, ~300 ms into its
// pipeline, the helper has long finished — joining at entry instead cost back-to-back calls up to
// 67 ms, profiles/r05b_e2e_stages.json), so at most two calls' buffers ever coexist, and the
// library's unload joins the last one (this object's destructor runs at exit / dlclose), so no
// helper outlives the library's code. The helper calls nothing but munmap (no roctx, no HIP). If
// no thread can be started the buffers are released on the calling thread.
class Releaser {
 public:
  ~Releaser() { join(); }
  void join() {
    std::lock_guard<std::mutex> l(mu_);
    if (th_.joinable()) th_.join();
  }
  void release(std::unique_ptr<HostBuf> a, std::unique_ptr<HostBuf> b) {
    std::lock_guard<std::mutex> l(mu_);
    if (th_.joinable()) th_.join();
    // if no thread starts, the callable (and the buffers it owns) is destroyed with the failed
    // start: released here, on the calling thread
    (void)start_thread(th_, [a = std::move(a), b = std::move(b)]() mutable noexcept {
      a.reset();
      b.reset();
    });
  }

 private:
  std::mutex mu_;
  std::thread th_;
};
Releaser g_release;
}  // namespace

extern "C" {

// File to file, as the reference runs (preprocess-kgz.rs:69-126,187-194): a reader thread streams
// the transcript in 32 MiB pread()s while the GPU decodes what has arrived; a writer thread
// pwrite()s each output range as it lands. The output goes to a temporary file in the same
// directory, renamed over `out_path` only on success (the reference's File::create leaves a
// truncated file behind on a panic).
int kzgpot_preprocess_ex(const char* transcript_path, const char* out_path, int mode, uint32_t n_log2, int n_gpus,
                         const char* expect_transcript_digest, char* transcript_digest, char* output_digest,
                         int* bad_section, int64_t* bad_index) {
  if (bad_section) *bad_section = -1;
  if (bad_index) *bad_index = -1;
  if (!transcript_path || !out_path || n_log2 < 1 || n_log2 > 30) return KZGPOT_E_INVALID_ARG;
  TraceRange call_("kzgpot.preprocess_file");
  // Everything the call opens, creates or starts is undone on every exit path, including an
  // exception (std::bad_alloc) caught by api_guard below: the reader is joined, both descriptors
  // closed, and the temporary output removed unless it was renamed over out_path.
  struct Files {
    int fd = -1, ofd = -1;
    std::string tmp;
    bool committed = false;
    ~Files() {
      if (fd >= 0) close(fd);
      if (ofd >= 0) close(ofd);
      if (!tmp.empty() && !committed) unlink(tmp.c_str());
    }
  };
  std::unique_ptr<HostBuf> tr, out;
  const int ret = api_guard([&]() -> int {
    Files f;
    f.fd = open(transcript_path, O_RDONLY | O_CLOEXEC);
    if (f.fd < 0) return KZGPOT_E_IO;
    const off_t flen = lseek(f.fd, 0, SEEK_END);
    if (flen < 0) return KZGPOT_E_IO;
    if ((uint64_t)flen != kzgpot_contribution_size(n_log2)) return KZGPOT_E_SIZE;
    const size_t len = (size_t)flen;
    (void)posix_fadvise(f.fd, 0, flen, POSIX_FADV_SEQUENTIAL);
    tr.reset(new HostBuf(len));
    out.reset(new HostBuf(kzgpot_output_size(n_log2, mode)));
    if (!tr->get() || !out->get()) return KZGPOT_E_OUT_OF_MEMORY;  // the 0.6-1.6 GB mappings
    // unique per call (mkstemp), so concurrent calls for one out_path never share a temporary
    std::string tmp = std::string(out_path) + ".kzgpot-tmp-XXXXXX";
    f.ofd = mkostemp(&tmp[0], O_CLOEXEC);
    if (f.ofd < 0) return KZGPOT_E_IO;
    f.tmp.swap(tmp);
    (void)fchmod(f.ofd, 0644);  // mkstemp creates 0600: a setup file is meant to be read by others
    Watermark wm;
    std::thread reader;
    JoinOnExit reader_join{reader, [&wm] { wm.fail(); }};  // stops at its next piece, then joined
    uint8_t* const trp = tr->get();
    const int fd = f.fd;
    if (!start_thread(reader, [&wm, trp, fd, len]() noexcept {
          try {
            trace_thread("kzgpot.pread");
          } catch (...) {
          }
          // stops at the next piece once the pipeline failed
          for (size_t off = 0; off < len && !wm.failed();) {
            const ssize_t k = pread(fd, trp + off, std::min<size_t>(len - off, (size_t)32 << 20), (off_t)off);
            if (k < 0 && errno == EINTR) continue;
            if (k <= 0) return wm.fail();
            off += (size_t)k;
            wm.advance(off);
          }
        }))
      return KZGPOT_E_OUT_OF_MEMORY;
    PipelineIo io;
    io.in_wm = &wm;
    io.out_fd = f.ofd;
    int r = preprocess_impl(trp, len, out->get(), mode, n_log2, n_gpus, expect_transcript_digest, transcript_digest,
                            output_digest, bad_section, bad_index, io);
    if (r) wm.fail();  // the reader finishes its current pread and stops; nothing waits on it
    reader.join();
    TraceRange fin_("kzgpot.file_finish");  // closes and rename
    const int ofd = f.ofd;
    f.ofd = -1;
    if (close(ofd) != 0 && !r) r = KZGPOT_E_IO;
    if (!r && rename(f.tmp.c_str(), out_path) != 0) r = KZGPOT_E_IO;
    f.committed = r == 0;
    return r;
  });
  if (tr || out) g_release.release(std::move(tr), std::move(out));  // unmapped behind the return (Releaser)
  if (ret == KZGPOT_E_OUT_OF_MEMORY) {
    if (bad_section) *bad_section = -1;
    if (bad_index) *bad_index = -1;
  }
  return ret;
}
int kzgpot_preprocess(const char* transcript_path, const char* out_path, int mode, uint32_t n_log2, int n_gpus,
                      int* bad_section, int64_t* bad_index) {
  return kzgpot_preprocess_ex(transcript_path, out_path, mode, n_log2, n_gpus, nullptr, nullptr, nullptr,
                              bad_section, bad_index);
}
// ------------------------------------------------------------------------------- loader mirror
int kzgpot_g1_deserialize_unchecked_ex(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad,
                                       uint8_t* status) {
  return api_guard([&] { return run_host(current_device(), CodecOp::G1Load, in, n, out, 0, first_bad, status); });
}
int kzgpot_g2_deserialize_unchecked_ex(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad,
                                       uint8_t* status) {
  return api_guard([&] { return run_host(current_device(), CodecOp::G2Load, in, n, out, 0, first_bad, status); });
}
int kzgpot_g1_deserialize_unchecked(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad) {
  return kzgpot_g1_deserialize_unchecked_ex(in, n, out, first_bad, nullptr);
}
int kzgpot_g2_deserialize_unchecked(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad) {
  return kzgpot_g2_deserialize_unchecked_ex(in, n, out, first_bad, nullptr);
}
int kzgpot_g1_deserialize_unchecked_dev(const void* d_in, size_t n, void* d_out, uint64_t* d_bad_key,
                                        uint8_t* d_status, void* stream) {
  return run_dev(CodecOp::G1Load, d_in, n, d_out, 0, d_bad_key, d_status, stream);
}
int kzgpot_bn254_g1_decompress_ex(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad, uint8_t* status) {
  return api_guard([&] { return run_host(current_device(), CodecOp::Bn254G1Decompress, in, n, out, 0, first_bad, status); });
}
int kzgpot_bn254_g1_decompress(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad) {
  return kzgpot_bn254_g1_decompress_ex(in, n, out, first_bad, nullptr);
}
int kzgpot_bn254_g1_decompress_dev(const void* d_in, size_t n, void* d_out, uint64_t* d_bad_key, uint8_t* d_status,
                                   void* stream) {
  return run_dev(CodecOp::Bn254G1Decompress, d_in, n, d_out, 0, d_bad_key, d_status, stream);
}
int kzgpot_g2_deserialize_unchecked_dev(const void* d_in, size_t n, void* d_out, uint64_t* d_bad_key,
                                        uint8_t* d_status, void* stream) {
  return run_dev(CodecOp::G2Load, d_in, n, d_out, 0, d_bad_key, d_status, stream);
}

}  // extern "C"

namespace {
// One sequential pass over a setup file: each section is `count` ark-uncompressed points read
// with deserialize_unchecked into `dst`. Mirrors the reference's BufReader loop (no size check
// beyond "enough bytes").
struct LoadSection {
  CodecOp op;
  uint64_t count;
  uint8_t* dst;
  int section;  // reported in *bad_section
};
int load_sections(const uint8_t* file, size_t len, const LoadSection* secs, int nsec, int* bad_section,
                  int64_t* bad_index) {
  if (bad_section) *bad_section = -1;
  if (bad_index) *bad_index = -1;
  if (!file) return KZGPOT_E_INVALID_ARG;
  uint64_t need = 0;
  for (int k = 0; k < nsec; k++) {
    if (!secs[k].dst) return KZGPOT_E_INVALID_ARG;
    need += secs[k].count * in_record(secs[k].op);
  }
  if (len < need) return KZGPOT_E_SIZE;
  if (device_count() <= 0) return KZGPOT_E_DEVICE;
  const uint8_t* p = file;
  for (int k = 0; k < nsec; k++) {
    int64_t fb = -1;
    const int r = run_host(current_device(), secs[k].op, p, secs[k].count, secs[k].dst, 0, &fb, nullptr);
    if (r) {
      if (bad_section) *bad_section = secs[k].section;
      if (bad_index) *bad_index = fb;
      return r;
    }
    p += secs[k].count * in_record(secs[k].op);
  }
  return 0;
}
int read_file(const char* path, std::vector<uint8_t>& buf) {
  if (!path) return KZGPOT_E_INVALID_ARG;
  FILE* f = fopen(path, "rb");
  if (!f) return KZGPOT_E_IO;
  fseek(f, 0, SEEK_END);
  const long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (len < 0) {
    fclose(f);
    return KZGPOT_E_IO;
  }
  try {
    buf.resize((size_t)len);
  } catch (const std::bad_alloc&) {
    fclose(f);
    return KZGPOT_E_OUT_OF_MEMORY;
  }
  const size_t got = fread(buf.data(), 1, buf.size(), f);
  fclose(f);
  return got == buf.size() ? 0 : KZGPOT_E_IO;
}
}  // namespace

extern "C" {

int kzgpot_load_kzg_setup_buffer(const uint8_t* file, size_t len, uint32_t n_log2, uint8_t* powers_of_g,
                                 uint8_t* powers_of_gamma_g, uint8_t* vk, int* bad_section, int64_t* bad_index) {
  if (n_log2 > 30 || !vk) return KZGPOT_E_INVALID_ARG;
  const uint64_t n = 1ull << n_log2;
  const uint64_t g1 = KZGPOT_G1_ARK_MONT_BYTES;
  const LoadSection secs[] = {
      {CodecOp::G1Load, 2 * n - 1, powers_of_g, 0},      // TAU_POWERS_G1_LENGTH (src/lib.rs:179-181)
      {CodecOp::G1Load, n, powers_of_gamma_g, 1},        // TAU_POWERS_LENGTH (src/lib.rs:182-184)
      {CodecOp::G1Load, 2, vk, 2},                       // VerifierKey g, gamma_g
      {CodecOp::G2Load, 2, vk + 2 * g1, 2},              // VerifierKey h, beta_h
  };
  return api_guard([&] { return load_sections(file, len, secs, 4, bad_section, bad_index); });
}
int kzgpot_load_kzg_setup(const char* path, uint32_t n_log2, uint8_t* powers_of_g, uint8_t* powers_of_gamma_g,
                          uint8_t* vk, int* bad_section, int64_t* bad_index) {
  return api_guard([&] {
    std::vector<uint8_t> buf;
    const int r = read_file(path, buf);
    if (r) return r;
    return kzgpot_load_kzg_setup_buffer(buf.data(), buf.size(), n_log2, powers_of_g, powers_of_gamma_g, vk,
                                        bad_section, bad_index);
  });
}
uint64_t kzgpot_phase1_size(uint32_t exp) {
  if (exp > 30) return 0;
  const uint64_t m = 1ull << exp;
  return 2 * 96 + 192 + m * (3 * 96 + 192);
}
int kzgpot_load_phase1_buffer(const uint8_t* file, size_t len, uint32_t exp, uint8_t* alpha, uint8_t* beta_g1,
                              uint8_t* beta_g2, uint8_t* coeffs_g1, uint8_t* coeffs_g2, uint8_t* alpha_coeffs_g1,
                              uint8_t* beta_coeffs_g1, int* bad_section, int64_t* bad_index) {
  if (exp > 30) return KZGPOT_E_INVALID_ARG;
  const uint64_t m = 1ull << exp;
  const LoadSection secs[] = {
      {CodecOp::G1Phase1, 1, alpha, 0},            // src/lib.rs:92
      {CodecOp::G1Phase1, 1, beta_g1, 1},          // src/lib.rs:93
      {CodecOp::G2Phase1, 1, beta_g2, 2},          // src/lib.rs:94
      {CodecOp::G1Phase1, m, coeffs_g1, 3},        // src/lib.rs:95-98
      {CodecOp::G2Phase1, m, coeffs_g2, 4},        // src/lib.rs:99-102
      {CodecOp::G1Phase1, m, alpha_coeffs_g1, 5},  // src/lib.rs:103-106
      {CodecOp::G1Phase1, m, beta_coeffs_g1, 6},   // src/lib.rs:107-110
  };
  return api_guard([&] { return load_sections(file, len, secs, 7, bad_section, bad_index); });
}
int kzgpot_load_phase1(const char* path, uint32_t exp, uint8_t* alpha, uint8_t* beta_g1, uint8_t* beta_g2,
                       uint8_t* coeffs_g1, uint8_t* coeffs_g2, uint8_t* alpha_coeffs_g1, uint8_t* beta_coeffs_g1,
                       int* bad_section, int64_t* bad_index) {
  return api_guard([&] {
    std::vector<uint8_t> buf;
    const int r = read_file(path, buf);
    if (r) return r;
    return kzgpot_load_phase1_buffer(buf.data(), buf.size(), exp, alpha, beta_g1, beta_g2, coeffs_g1, coeffs_g2,
                                     alpha_coeffs_g1, beta_coeffs_g1, bad_section, bad_index);
  });
}
int kzgpot_load_fastkzg_setup_buffer(const uint8_t* file, size_t len, uint32_t n_log2, uint8_t* powers_of_g,
                                     uint8_t* powers_of_gamma_g, uint8_t* h_beta_h, uint8_t* powers_of_h,
                                     int* bad_section, int64_t* bad_index) {
  if (n_log2 > 30) return KZGPOT_E_INVALID_ARG;
  const uint64_t n = 1ull << n_log2;
  const LoadSection secs[] = {
      {CodecOp::G1Load, 2 * n - 1, powers_of_g, 0},  // src/lib.rs:204-206
      {CodecOp::G1Load, n, powers_of_gamma_g, 1},    // src/lib.rs:207-209 (BTreeMap keys 0..N-1)
      {CodecOp::G2Load, 2, h_beta_h, 2},             // h, beta_h (src/lib.rs:211-212)
      {CodecOp::G2Load, n, powers_of_h, 3},          // src/lib.rs:214-217
  };
  return api_guard([&] { return load_sections(file, len, secs, 4, bad_section, bad_index); });
}
int kzgpot_load_fastkzg_setup(const char* path, uint32_t n_log2, uint8_t* powers_of_g, uint8_t* powers_of_gamma_g,
                              uint8_t* h_beta_h, uint8_t* powers_of_h, int* bad_section, int64_t* bad_index) {
  return api_guard([&] {
    std::vector<uint8_t> buf;
    const int r = read_file(path, buf);
    if (r) return r;
    return kzgpot_load_fastkzg_setup_buffer(buf.data(), buf.size(), n_log2, powers_of_g, powers_of_gamma_g,
                                            h_beta_h, powers_of_h, bad_section, bad_index);
  });
}

const char* kzgpot_status_name(int s) {
  switch (s < 0 && s > -100 ? -s : s) {
    case KZGPOT_OK: return "ok";
    case KZGPOT_ST_COMPRESSION_MODE: return "UnexpectedCompressionMode";
    case KZGPOT_ST_UNEXPECTED_INFO: return "UnexpectedInformation";
    case KZGPOT_ST_NOT_IN_FIELD: return "NotInField";
    case KZGPOT_ST_NOT_ON_CURVE: return "NotOnCurve";
    case KZGPOT_ST_NOT_IN_SUBGROUP: return "NotInSubgroup";
    case KZGPOT_ST_UNEXPECTED_FLAGS: return "UnexpectedFlags";
    case KZGPOT_ST_INFINITY: return "Infinity";
    case KZGPOT_E_INVALID_ARG: return "InvalidArgument";
    case KZGPOT_E_DEVICE: return "DeviceError";
    case KZGPOT_E_IO: return "IoError";
    case KZGPOT_E_SIZE: return "SizeMismatch";
    case KZGPOT_E_DIGEST: return "DigestMismatch";
    case KZGPOT_E_NETWORK: return "NetworkUnavailable";
    case KZGPOT_E_RANK_FAILED: return "RankFailed";
    case KZGPOT_E_TIMEOUT: return "Timeout";
    case KZGPOT_E_OUT_OF_MEMORY: return "OutOfMemory";
    default: return "unknown";
  }
}
int kzgpot_device_count(void) { return device_count(); }
const char* kzgpot_version(void) { return "kzgpot 0.1.0 (gfx950)"; }

#ifdef KZGPOT_TEST_HOOKS
// test build only (tests/kzgpot_test_hooks.h)
// The chunk plan of a host-buffer call of n points (run_host): writes up to cap (offset, count)
// pairs and returns the number of chunks (tests/test_host.py checks the tiling on the CPU).
long kzgpot_test_chunk_plan(uint64_t n, int streaming_consumer, uint64_t* spans, long cap) {
  if (n == 0) return 0;
  const ChunkPlan plan((size_t)n, streaming_consumer != 0);
  const long k = (long)plan.count();
  for (long j = 0; j < k && j < cap; j++) {
    size_t off, m;
    plan.span((size_t)j, off, m);
    spans[2 * j] = off;
    spans[2 * j + 1] = m;
  }
  return k;
}
int kzgpot_test_inject_host_fault(int site, long skip) {
  if (site < 0 || site > kFaultHostBuf || skip < 0) return KZGPOT_E_INVALID_ARG;
  g_fault_site = 0;
  g_fault_skip = skip;
  g_fault_site = site;
  return 0;
}
#endif

}  // extern "C"
