// Multi-GPU path inside the library (north_star "the τ^i array shards trivially across
// the 8 GPUs of one node with a final RCCL all-gather over xGMI to produce one contiguous arkworks
// buffer"): one process (or thread) per GPU, each holding a kzgpot communicator (an RCCL comm plus
// a private comm stream), and one call that decodes the rank's share of a point stream and
// assembles the whole arkworks buffer in HBM on every rank.
//
// The reference has no parallel exchange at all: its only parallel stage is the chunked
// decompression inside powersoftau's Accumulator::deserialize (src/bin/preprocess-kgz.rs:105-110),
// whose workers write disjoint slices of one Vec. Here the slices are block-cyclic over the ranks
// so that the exchange can be pipelined behind the decoding:
//
//   n points = nranks x chunks blocks of B = floor(n / (nranks chunks)) points + a tail of
//   r = n - nranks chunks B points (r < nranks chunks, e.g. τG1's 2^22 - 1 points);
//   rank k owns blocks c nranks + k (c < chunks); chunk c's nranks blocks are adjacent in the
//   output, so after the rank's chunk-c decode ONE in-place ncclAllGather fills that contiguous
//   region, on the comm stream, while the caller's stream decodes chunk c + 1. Only the last
//   chunk's gather is exposed. The tail is decoded by every rank (no exchange; it is < 64 points
//   in any layout a caller would pick).
//
// The first rejected point over all ranks is one 8-byte ncclAllReduce(min) of the per-launch keys
// shifted to global indices (k_merge_keys), so every rank returns the same deterministic answer.
//
// Failures never desynchronise the ranks (the reference's workers share one process, so it has
// no such problem; ranks on different GPUs do). A rank whose local HIP work fails keeps issuing
// every collective of the call — its peers receive garbage for its blocks — and all-reduces the
// key 0 (KZGPOT_KEY_RANK_FAILED, below every real key), so every rank learns of the failure from
// the same key. Only a failing RCCL call aborts the communicator. kzgpot_comm_wait bounds the
// host's wait and aborts on timeout, which is what makes a peer's lost collective recoverable.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "codec.hpp"
#include "trace.hpp"

using namespace kzgpot;

namespace {

// RCCL is bound at first use, not at link time: a process that already holds an RCCL (torch does:
// its own librccl.so with the same SONAME) must keep using that one — a second copy loaded ahead
// of torch corrupts the heap at exit — and single-GPU users never load it at all.
// Test builds only (libkzgpot_test.so, -DKZGPOT_TEST_HOOKS): KZGPOT_RCCL_LIB names another library
// with the same symbols (tests/fake_rccl: N ranks as threads on one GPU), opened RTLD_LOCAL so that
// it never interposes on torch's RCCL. The product library binds librccl.so.1 and nothing else.
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;  // optional
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommCount) comm_count = nullptr;
  decltype(&ncclCommCuDevice) comm_device = nullptr;
  decltype(&ncclCommUserRank) comm_user_rank = nullptr;
  bool ok = false;
};
const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
#ifdef KZGPOT_TEST_HOOKS
    const char* over = getenv("KZGPOT_RCCL_LIB");
#else
    const char* over = nullptr;
#endif
    void* h = nullptr;
    if (over && *over) {
      h = dlopen(over, RTLD_NOW | RTLD_LOCAL);
    } else {
      h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);  // the process's own RCCL
      if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    }
    if (!h) {
      fprintf(stderr, "kzgpot: cannot load %s: %s\n", over && *over ? over : "librccl.so.1", dlerror());
      return;
    }
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.comm_abort = (decltype(r.comm_abort))dlsym(h, "ncclCommAbort");
    r.async_error = (decltype(r.async_error))dlsym(h, "ncclCommGetAsyncError");
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.comm_count = (decltype(r.comm_count))dlsym(h, "ncclCommCount");
    r.comm_device = (decltype(r.comm_device))dlsym(h, "ncclCommCuDevice");
    r.comm_user_rank = (decltype(r.comm_user_rank))dlsym(h, "ncclCommUserRank");
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.comm_abort && r.all_gather && r.all_reduce &&
           r.error_string && r.comm_count && r.comm_device && r.comm_user_rank;
    if (!r.ok) fprintf(stderr, "kzgpot: %s lacks an RCCL entry point\n", over && *over ? over : "librccl.so.1");
  });
  return r;
}

#define HIP_OK(expr)                                                                                        \
  do {                                                                                                      \
    hipError_t e_ = (expr);                                                                                 \
    if (e_ != hipSuccess) {                                                                                 \
      fprintf(stderr, "kzgpot: %s failed: %s (%s:%d)\n", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return KZGPOT_E_DEVICE;                                                                               \
    }                                                                                                       \
  } while (0)
#define NCCL_OK(expr)                                                                                          \
  do {                                                                                                         \
    ncclResult_t e_ = (expr);                                                                                  \
    if (e_ != ncclSuccess) {                                                                                   \
      fprintf(stderr, "kzgpot: %s failed: %s (%s:%d)\n", #expr, rccl().error_string(e_), __FILE__, __LINE__); \
      return KZGPOT_E_DEVICE;                                                                                  \
    }                                                                                                          \
  } while (0)

struct Comm {
  ncclComm_t nccl = nullptr;
  int rank = 0, nranks = 1, device = -1;
  bool aborted = false;
  hipStream_t cs = nullptr;               // the comm stream: gathers + the key all-reduce
  std::vector<hipEvent_t> ev;             // one per chunk (decode done) + 1 (keys merged)
  hipEvent_t done = nullptr;              // recorded on cs after the last collective of a call
  bool done_recorded = false;
  unsigned long long* d_keys = nullptr;   // per-launch keys (chunks + tail)
  uint64_t* d_local = nullptr;            // [0] this rank's global-index min key, [1] = 0 (a failed rank's key)
  size_t cap_keys = 0;
  int fault_site = 0;                     // kzgpot_comm_inject_fault (test builds), one shot
  uint32_t fault_at = 0;
  hipEvent_t entry = nullptr;             // recorded on the caller's stream at each call's entry
  std::mutex mu;                          // one call at a time per communicator
};

// fault sites of the test-only kzgpot_comm_inject_fault (tests/kzgpot_test_hooks.h: KZGPOT_FAULT_*);
// a product build never sets one
enum { kFaultLaunch = 1, kFaultCollective = 2 };

bool op_from_code(int code, CodecOp* op) {
  switch (code) {
    case KZGPOT_OP_G1_DECOMPRESS: *op = CodecOp::G1Decompress; return true;
    case KZGPOT_OP_G2_DECOMPRESS: *op = CodecOp::G2Decompress; return true;
    case KZGPOT_OP_G1_TRANSCODE: *op = CodecOp::G1Transcode; return true;
    case KZGPOT_OP_G2_TRANSCODE: *op = CodecOp::G2Transcode; return true;
    case KZGPOT_OP_BN254_G1_DECOMPRESS: *op = CodecOp::Bn254G1Decompress; return true;
    default: return false;
  }
}

// keys[j] (j < chunks: block j nranks + rank, j == chunks: the tail) hold (local index << 8) |
// status or all ones; out = min over j of the key shifted to the global index.
__global__ void k_merge_keys(const unsigned long long* __restrict__ keys, uint32_t chunks, uint64_t block,
                             uint32_t nranks, uint32_t rank, uint64_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t best = ~0ull;
  for (uint32_t j = 0; j <= chunks; j++) {
    const uint64_t k = keys[j];
    if (k == ~0ull) continue;
    const uint64_t base = j < chunks ? ((uint64_t)j * nranks + rank) * block : (uint64_t)chunks * nranks * block;
    const uint64_t g = (((k >> 8) + base) << 8) | (k & 0xff);
    best = g < best ? g : best;
  }
  out[0] = best;
}

int ensure_events(Comm& c, size_t need) {
  try {
    c.ev.reserve(need);  // push_back below cannot throw then
  } catch (const std::bad_alloc&) {  // never across the C ABI: the caller still issues its collectives
    return KZGPOT_E_OUT_OF_MEMORY;
  }
  while (c.ev.size() < need) {
    hipEvent_t e;
    HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c.ev.push_back(e);
  }
  return 0;
}

// A failing RCCL call: the communicator cannot be trusted to line up with its peers any more.
int abort_comm(Comm& c, ncclResult_t r, const char* what) {
  fprintf(stderr, "kzgpot: %s failed on rank %d of %d: %s; aborting the communicator\n", what, c.rank, c.nranks,
          r == ncclSuccess ? "timeout" : rccl().error_string(r));
  if (c.nccl) rccl().comm_abort(c.nccl);
  c.nccl = nullptr;
  c.aborted = true;
  return KZGPOT_E_DEVICE;
}

}  // namespace

extern "C" {

int kzgpot_comm_unique_id(uint8_t* id) {
  if (!id) return KZGPOT_E_INVALID_ARG;
  static_assert(sizeof(ncclUniqueId) == KZGPOT_COMM_ID_BYTES, "RCCL unique id size");
  if (!rccl().ok) return KZGPOT_E_DEVICE;
  ncclUniqueId u;
  NCCL_OK(rccl().get_unique_id(&u));
  memcpy(id, &u, sizeof u);
  return 0;
}

int kzgpot_comm_init(void** comm, const uint8_t* id, int nranks, int rank) {
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) return KZGPOT_E_INVALID_ARG;
  *comm = nullptr;
  if (!rccl().ok) return KZGPOT_E_DEVICE;
  int dev = -1;
  HIP_OK(hipGetDevice(&dev));
  Comm* c = new (std::nothrow) Comm;
  if (!c) return KZGPOT_E_OUT_OF_MEMORY;
  c->rank = rank;
  c->nranks = nranks;
  c->device = dev;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  const ncclResult_t r = rccl().comm_init_rank(&c->nccl, nranks, u, rank);
  if (r != ncclSuccess) {
    fprintf(stderr, "kzgpot: ncclCommInitRank(%d of %d) failed: %s\n", rank, nranks, rccl().error_string(r));
    delete c;
    return KZGPOT_E_DEVICE;
  }
  if (hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->entry, hipEventDisableTiming) != hipSuccess ||
      hipMalloc(&c->d_local, 2 * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(c->d_local, 0, 2 * sizeof(uint64_t)) != hipSuccess) {
    if (c->d_local) (void)hipFree(c->d_local);
    if (c->entry) (void)hipEventDestroy(c->entry);
    if (c->done) (void)hipEventDestroy(c->done);
    if (c->cs) (void)hipStreamDestroy(c->cs);
    rccl().comm_destroy(c->nccl);
    delete c;
    return KZGPOT_E_DEVICE;
  }
  *comm = c;
  return 0;
}

int kzgpot_comm_destroy(void* comm) {
  if (!comm) return KZGPOT_E_INVALID_ARG;
  Comm* c = (Comm*)comm;
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(c->device);
  if (!c->aborted) (void)hipStreamSynchronize(c->cs);  // an aborted comm's kernels have exited or never will
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  (void)hipEventDestroy(c->done);
  (void)hipEventDestroy(c->entry);
  if (!c->aborted) {
    if (c->d_keys) (void)hipFree(c->d_keys);
    if (c->d_local) (void)hipFree(c->d_local);
    (void)hipStreamDestroy(c->cs);
  }  // else: leaked on purpose — a stuck stream may still reference them
  const ncclResult_t r = c->nccl ? rccl().comm_destroy(c->nccl) : ncclSuccess;
  if (prev >= 0) (void)hipSetDevice(prev);
  delete c;
  return r == ncclSuccess ? 0 : KZGPOT_E_DEVICE;
}

int kzgpot_shard_layout(uint64_t n, int nranks, uint32_t chunks, uint64_t* block, uint64_t* tail) {
  if (nranks < 1 || chunks < 1 || !block || !tail) return KZGPOT_E_INVALID_ARG;
  *block = n / ((uint64_t)nranks * chunks);
  *tail = n - *block * (uint64_t)nranks * chunks;
  return 0;
}

int kzgpot_comm_size(void* comm, int* nranks, int* rank, int* device) {
  if (!comm) return KZGPOT_E_INVALID_ARG;
  Comm& c = *(Comm*)comm;
  std::lock_guard<std::mutex> lock(c.mu);
  if (c.aborted || !c.nccl) return KZGPOT_E_DEVICE;
  int n = -1, r = -1, d = -1;  // what RCCL itself reports for the communicator, not our copies
  NCCL_OK(rccl().comm_count(c.nccl, &n));
  NCCL_OK(rccl().comm_user_rank(c.nccl, &r));
  NCCL_OK(rccl().comm_device(c.nccl, &d));
  if (nranks) *nranks = n;
  if (rank) *rank = r;
  if (device) *device = d;
  return 0;
}

#ifdef KZGPOT_TEST_HOOKS
// Failure injection, test builds only (declared in tests/kzgpot_test_hooks.h): the NEXT
// kzgpot_decode_allgather_dev on this communicator fails at `site`, step `at`, once.
int kzgpot_comm_inject_fault(void* comm, int site, uint32_t at) {
  if (!comm || site < 0 || site > kFaultCollective) return KZGPOT_E_INVALID_ARG;
  Comm& c = *(Comm*)comm;
  std::lock_guard<std::mutex> lock(c.mu);
  c.fault_site = site;
  c.fault_at = at;
  return 0;
}
#endif

int kzgpot_decode_allgather_dev(void* comm, int op_code, const void* d_in_local, uint64_t n, uint32_t chunks,
                                void* d_out, uint32_t flags, uint64_t* d_bad_key, void* stream) {
  CodecOp op;
  if (!comm || !op_from_code(op_code, &op) || chunks < 1 || !d_bad_key || (n && (!d_in_local || !d_out)))
    return KZGPOT_E_INVALID_ARG;
  Comm& c = *(Comm*)comm;
  std::lock_guard<std::mutex> lock(c.mu);
  TraceRange tr_("kzgpot.decode_allgather.enqueue");
  if (c.aborted) return KZGPOT_E_DEVICE;
  int dev = -1;
  HIP_OK(hipGetDevice(&dev));
  if (dev != c.device) return KZGPOT_E_INVALID_ARG;  // the communicator's GPU must be current
  if (op == CodecOp::Bn254G1Decompress || op == CodecOp::G1Transcode || op == CodecOp::G2Transcode)
    flags &= KZGPOT_SUBGROUP_REF;
  const int fault = c.fault_site;
  const uint32_t fault_at = c.fault_at;
  c.fault_site = 0;

  // From here on every collective of the call is issued whatever happens locally (file comment).
  hipStream_t s = (hipStream_t)stream;
  bool failed = false;
  auto local = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && !failed) {
      fprintf(stderr, "kzgpot: rank %d of %d: %s failed: %s; the gathered buffer will be incomplete\n", c.rank,
              c.nranks, what, hipGetErrorString(e));
      failed = true;
    }
    return !failed;
  };
  // The comm stream runs behind everything the caller queued on `stream` before this call (a
  // memset of d_bad_key, a reader of the previous d_out), whatever fails later: the collectives
  // below write d_out and d_bad_key on cs even when no chunk event ever links the two streams.
  if (hipEventRecord(c.entry, s) != hipSuccess || hipStreamWaitEvent(c.cs, c.entry, 0) != hipSuccess) {
    fprintf(stderr, "kzgpot: rank %d of %d: cannot order the comm stream after the caller's stream\n", c.rank,
            c.nranks);
    failed = true;
    (void)hipStreamSynchronize(s);  // the same order, the slow way
  }
  // the previous call's collectives read d_keys / d_local and used the events: wait for them
  if (c.done_recorded) local(hipStreamWaitEvent(s, c.done, 0), "hipStreamWaitEvent(previous call)");
  if (!failed && c.cap_keys < chunks + 1) {
    if (c.d_keys && local(hipEventSynchronize(c.done), "hipEventSynchronize(previous call)"))
      local(hipFree(c.d_keys), "hipFree(keys)");
    c.d_keys = nullptr;
    c.cap_keys = 0;
    if (local(hipMalloc(&c.d_keys, (chunks + 1) * sizeof(unsigned long long)), "hipMalloc(keys)"))
      c.cap_keys = chunks + 1;
  }
  if (!failed && ensure_events(c, chunks + 1)) local(hipErrorOutOfMemory, "hipEventCreate");
  if (!failed) local(hipMemsetAsync(c.d_keys, 0xff, (chunks + 1) * sizeof(unsigned long long), s), "hipMemsetAsync(keys)");

  const uint64_t rin = in_record(op), rout = out_record(op);
  uint64_t B = 0, tail = 0;
  kzgpot_shard_layout(n, c.nranks, chunks, &B, &tail);
  const uint8_t* in = (const uint8_t*)d_in_local;
  uint8_t* out = (uint8_t*)d_out;
  const size_t bytes = (size_t)(B * rout);
  for (uint32_t ch = 0; B && ch < chunks; ch++) {
    if (!failed) {
      const uint64_t g0 = ((uint64_t)ch * c.nranks + c.rank) * B;
      const hipError_t e = fault == kFaultLaunch && fault_at == ch
                               ? hipErrorLaunchFailure
                               : launch_codec(op, in + ch * B * rin, out + g0 * rout, B, flags, c.d_keys + ch, nullptr, s);
      if (local(e, "decode launch") && local(hipEventRecord(c.ev[ch], s), "hipEventRecord"))
        local(hipStreamWaitEvent(c.cs, c.ev[ch], 0), "hipStreamWaitEvent");
    }
    uint8_t* region = out + (uint64_t)ch * c.nranks * B * rout;
    const ncclResult_t r = fault == kFaultCollective && fault_at == ch
                               ? ncclSystemError
                               : rccl().all_gather(region + (size_t)c.rank * bytes, region, bytes, ncclUint8, c.nccl, c.cs);
    if (r != ncclSuccess) return abort_comm(c, r, "ncclAllGather");
  }
  if (!failed && tail) {
    const hipError_t e = fault == kFaultLaunch && fault_at == chunks
                             ? hipErrorLaunchFailure
                             : launch_codec(op, in + (uint64_t)chunks * B * rin,
                                            out + (uint64_t)chunks * c.nranks * B * rout, tail, flags,
                                            c.d_keys + chunks, nullptr, s);
    local(e, "tail decode launch");
  }
  if (!failed) {
    hipLaunchKernelGGL(k_merge_keys, dim3(1), dim3(64), 0, s, c.d_keys, chunks, B, (uint32_t)c.nranks,
                       (uint32_t)c.rank, c.d_local);
    if (local(hipGetLastError(), "key merge launch") && local(hipEventRecord(c.ev[chunks], s), "hipEventRecord"))
      local(hipStreamWaitEvent(c.cs, c.ev[chunks], 0), "hipStreamWaitEvent");
  }
  // a failed rank contributes the constant 0 word (d_local[1], never written after init): the
  // min over ranks is then KZGPOT_KEY_RANK_FAILED on every rank
  const ncclResult_t r = fault == kFaultCollective && fault_at == chunks
                             ? ncclSystemError
                             : rccl().all_reduce(failed ? c.d_local + 1 : c.d_local, d_bad_key, 1, ncclUint64,
                                                 ncclMin, c.nccl, c.cs);
  if (r != ncclSuccess) return abort_comm(c, r, "ncclAllReduce");
  HIP_OK(hipEventRecord(c.done, c.cs));
  c.done_recorded = true;
  HIP_OK(hipStreamWaitEvent(s, c.done, 0));  // the caller's stream sees the whole buffer
  return failed ? KZGPOT_E_DEVICE : 0;
}

int kzgpot_comm_wait(void* comm, const uint64_t* d_bad_key, int64_t* first_bad, uint32_t timeout_ms, void* stream) {
  if (first_bad) *first_bad = -1;
  if (!comm || !d_bad_key) return KZGPOT_E_INVALID_ARG;
  Comm& c = *(Comm*)comm;
  hipStream_t s = (hipStream_t)stream;
  {
    std::lock_guard<std::mutex> lock(c.mu);
    if (c.aborted) return KZGPOT_E_DEVICE;
  }
  TraceRange tr_("kzgpot.comm_wait");
  const auto t0 = std::chrono::steady_clock::now();
  for (int spin = 0;; spin++) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) {
      fprintf(stderr, "kzgpot: rank %d: stream error while waiting: %s\n", c.rank, hipGetErrorString(q));
      return KZGPOT_E_DEVICE;
    }
    std::lock_guard<std::mutex> lock(c.mu);
    if (c.aborted) return KZGPOT_E_DEVICE;
    ncclResult_t ae = ncclSuccess;
    if (rccl().async_error && c.nccl && rccl().async_error(c.nccl, &ae) == ncclSuccess && ae != ncclSuccess &&
        ae != ncclInProgress)
      return abort_comm(c, ae, "asynchronous RCCL operation");
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_ms && ms > timeout_ms) {
      abort_comm(c, ncclSuccess, "kzgpot_comm_wait");
      return KZGPOT_E_TIMEOUT;
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  {
    // a stream that drained is not proof that the collectives moved the data: an RCCL error
    // reported asynchronously (a peer aborted) voids the buffer and the key
    std::lock_guard<std::mutex> lock(c.mu);
    if (c.aborted) return KZGPOT_E_DEVICE;
    ncclResult_t ae = ncclSuccess;
    if (rccl().async_error && c.nccl && rccl().async_error(c.nccl, &ae) == ncclSuccess && ae != ncclSuccess &&
        ae != ncclInProgress)
      return abort_comm(c, ae, "asynchronous RCCL operation");
  }
  uint64_t key = ~0ull;
  HIP_OK(hipMemcpy(&key, d_bad_key, sizeof key, hipMemcpyDeviceToHost));
  if (key == KZGPOT_KEY_RANK_FAILED) return KZGPOT_E_RANK_FAILED;
  return kzgpot_decode_bad_key(key, first_bad);
}

}  // extern "C"
