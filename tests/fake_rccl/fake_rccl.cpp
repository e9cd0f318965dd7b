// TEST-ONLY stand-in for librccl.so.1: N ranks running as threads of ONE process on ONE GPU.
//
// Why: the pool's GPU boxes have one MI355X, and RCCL refuses two ranks on one device, so the
// library's multi-rank path (kzgpot_decode_allgather_dev, csrc/comm.hip) could otherwise only run
// at nranks = 1, where an in-place all-gather moves nothing. Bound through KZGPOT_RCCL_LIB, this
// library implements the RCCL entry points the product binds, with RCCL's semantics for them:
//   ncclGetUniqueId / ncclCommInitRank (collective: blocks until all ranks joined) /
//   ncclCommDestroy / ncclCommAbort (wakes every peer blocked in a collective: they return
//   ncclRemoteError) / ncclCommGetAsyncError / ncclAllGather / ncclAllReduce (u64/i64 min, max,
//   sum) / ncclGetErrorString.
// A collective is host-synchronous here: the calling thread waits for its stream (so the data it
// sends is final), meets its peers at a barrier, copies every peer's contribution device to
// device on its own stream, and meets them again (so no peer reuses a buffer being read). RCCL
// proper returns at once and moves data in kernels; the bytes that land are the same.
// Every collective also checks that all ranks issued the same operation with the same size —
// the mismatch that would hang real RCCL is reported as ncclInvalidUsage instead.
// A barrier that waits longer than FAKE_RCCL_TIMEOUT_S (default 60) returns ncclSystemError.
//
// Async-error mode (fake_rccl_set_async_errors(1), per process): once a peer aborted, a collective
// returns ncclSuccess at once without moving anything, as real RCCL's enqueue does, and the
// failure is visible only through ncclCommGetAsyncError — so the peers learn of it where real
// peers do, in kzgpot_comm_wait, instead of from the enqueue's return code.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

enum Kind { kNone, kAllGather, kAllReduce };

struct Slot {
  Kind kind = kNone;
  const void* send = nullptr;
  size_t bytes = 0;
  int dtype = 0, redop = 0;
  std::vector<uint64_t> host;  // all-reduce contributions
};

struct Group {
  int nranks = 0;
  std::mutex mu;
  std::condition_variable cv;
  int joined = 0;
  int live = 0;
  bool aborted = false;
  uint64_t gen = 0;
  int arrived = 0;
  std::vector<Slot> slots;
};

struct FakeComm {
  Group* g;
  int rank;
  int device;  // the HIP device current at ncclCommInitRank, as RCCL records it
};

std::mutex g_reg_mu;
std::map<std::string, Group*> g_reg;
std::atomic<uint64_t> g_counter{0};
std::atomic<int> g_async_errors{0};

double timeout_s() {
  const char* e = getenv("FAKE_RCCL_TIMEOUT_S");
  return e && *e ? atof(e) : 60.0;
}

// generation barrier; lk holds g->mu
ncclResult_t barrier(Group* g, std::unique_lock<std::mutex>& lk, int rank, const char* what) {
  if (g->aborted) return g_async_errors ? ncclInProgress : ncclRemoteError;
  const uint64_t my = g->gen;
  if (++g->arrived == g->nranks) {
    g->arrived = 0;
    g->gen++;
    g->cv.notify_all();
    return ncclSuccess;
  }
  const bool woke = g->cv.wait_for(lk, std::chrono::duration<double>(timeout_s()),
                                   [&] { return g->gen != my || g->aborted; });
  if (g->gen != my) return ncclSuccess;
  if (g->aborted) return g_async_errors ? ncclInProgress : ncclRemoteError;
  if (!woke) fprintf(stderr, "fake_rccl: rank %d timed out in %s (%d of %d arrived)\n", rank, what, g->arrived, g->nranks);
  return ncclSystemError;
}

size_t dtype_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

// a collective's result as its caller sees it: in async-error mode an aborted group's collective
// "was enqueued" (ncclSuccess); the error is reported by ncclCommGetAsyncError
ncclResult_t enqueue_result(ncclResult_t r) { return r == ncclInProgress ? ncclSuccess : r; }

}  // namespace

extern "C" {

void fake_rccl_set_async_errors(int on) { g_async_errors = on; }

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (fake_rccl)";
    case ncclUnhandledCudaError: return "unhandled HIP error (fake_rccl)";
    case ncclSystemError: return "system error / timeout (fake_rccl)";
    case ncclInternalError: return "internal error (fake_rccl)";
    case ncclInvalidArgument: return "invalid argument (fake_rccl)";
    case ncclInvalidUsage: return "invalid usage: ranks issued different collectives (fake_rccl)";
    case ncclRemoteError: return "remote error: a peer aborted (fake_rccl)";
    default: return "unknown (fake_rccl)";
  }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  memset(id, 0, sizeof *id);
  snprintf(id->internal, sizeof id->internal, "fake_rccl:%d:%llu", (int)getpid(),
           (unsigned long long)g_counter.fetch_add(1));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  Group* g;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    const std::string key(id.internal, strnlen(id.internal, sizeof id.internal));
    auto it = g_reg.find(key);
    if (it == g_reg.end()) {
      g = new Group;
      g->nranks = nranks;
      g->slots.resize(nranks);
      g_reg[key] = g;
    } else {
      g = it->second;
    }
  }
  std::unique_lock<std::mutex> lk(g->mu);
  if (g->nranks != nranks) return ncclInvalidUsage;
  g->joined++;
  g->live++;
  const ncclResult_t r = barrier(g, lk, rank, "ncclCommInitRank");
  if (r != ncclSuccess) return r;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return ncclUnhandledCudaError;
  *comm = (ncclComm_t) new FakeComm{g, rank, dev};
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  delete (FakeComm*)comm;  // the group stays registered (tests create few)
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  FakeComm* c = (FakeComm*)comm;
  {
    std::lock_guard<std::mutex> lk(c->g->mu);
    c->g->aborted = true;
    c->g->cv.notify_all();
  }
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* err) {
  if (!comm || !err) return ncclInvalidArgument;
  FakeComm* c = (FakeComm*)comm;
  std::lock_guard<std::mutex> lk(c->g->mu);
  *err = c->g->aborted ? ncclRemoteError : ncclSuccess;
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  if (!comm || !count) return ncclInvalidArgument;
  *count = ((FakeComm*)comm)->g->nranks;
  return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  if (!comm || !rank) return ncclInvalidArgument;
  *rank = ((FakeComm*)comm)->rank;
  return ncclSuccess;
}

ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device) {
  if (!comm || !device) return ncclInvalidArgument;
  *device = ((FakeComm*)comm)->device;
  return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclComm_t comm,
                           hipStream_t stream) {
  if (!comm || !dtype_size(dt)) return ncclInvalidArgument;
  FakeComm* c = (FakeComm*)comm;
  Group* g = c->g;
  const size_t bytes = count * dtype_size(dt);
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  std::unique_lock<std::mutex> lk(g->mu);
  Slot& mine = g->slots[c->rank];
  mine.kind = kAllGather;
  mine.send = send;
  mine.bytes = bytes;
  ncclResult_t r = barrier(g, lk, c->rank, "ncclAllGather");
  if (r != ncclSuccess) return enqueue_result(r);
  std::vector<const void*> src(g->nranks);
  for (int i = 0; i < g->nranks; i++) {
    if (g->slots[i].kind != kAllGather || g->slots[i].bytes != bytes) {
      fprintf(stderr, "fake_rccl: rank %d: ncclAllGather(%zu B) met rank %d's op %d (%zu B)\n", c->rank, bytes, i,
              (int)g->slots[i].kind, g->slots[i].bytes);
      return ncclInvalidUsage;
    }
    src[i] = g->slots[i].send;
  }
  lk.unlock();
  for (int i = 0; i < (int)src.size(); i++) {
    uint8_t* dst = (uint8_t*)recv + (size_t)i * bytes;
    if (bytes && dst != src[i] && hipMemcpyAsync(dst, src[i], bytes, hipMemcpyDeviceToDevice, stream) != hipSuccess)
      return ncclUnhandledCudaError;
  }
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  lk.lock();  // slots stay as they are: a slower peer may still be reading them until this barrier
  return enqueue_result(barrier(g, lk, c->rank, "ncclAllGather (release)"));
}

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
  if (!comm || (dt != ncclUint64 && dt != ncclInt64) || (op != ncclMin && op != ncclMax && op != ncclSum))
    return ncclInvalidArgument;
  FakeComm* c = (FakeComm*)comm;
  Group* g = c->g;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  std::vector<uint64_t> v(count);
  if (count && hipMemcpy(v.data(), send, count * 8, hipMemcpyDeviceToHost) != hipSuccess) return ncclUnhandledCudaError;
  std::unique_lock<std::mutex> lk(g->mu);
  Slot& mine = g->slots[c->rank];
  mine.kind = kAllReduce;
  mine.bytes = count * 8;
  mine.dtype = (int)dt;
  mine.redop = (int)op;
  mine.host = v;
  ncclResult_t r = barrier(g, lk, c->rank, "ncclAllReduce");
  if (r != ncclSuccess) return enqueue_result(r);
  std::vector<uint64_t> acc = g->slots[0].host;
  for (int i = 0; i < g->nranks; i++) {
    const Slot& s = g->slots[i];
    if (s.kind != kAllReduce || s.bytes != count * 8 || s.dtype != (int)dt || s.redop != (int)op) {
      fprintf(stderr, "fake_rccl: rank %d: ncclAllReduce met rank %d's op %d\n", c->rank, i, (int)s.kind);
      return ncclInvalidUsage;
    }
    for (size_t k = 0; i && k < count; k++) {
      const uint64_t a = acc[k], b = s.host[k];
      if (op == ncclSum) acc[k] = a + b;
      else if (dt == ncclUint64) acc[k] = op == ncclMin ? (a < b ? a : b) : (a > b ? a : b);
      else acc[k] = op == ncclMin ? ((int64_t)a < (int64_t)b ? a : b) : ((int64_t)a > (int64_t)b ? a : b);
    }
  }
  lk.unlock();
  if (count && (hipMemcpyAsync(recv, acc.data(), count * 8, hipMemcpyHostToDevice, stream) != hipSuccess ||
                hipStreamSynchronize(stream) != hipSuccess))
    return ncclUnhandledCudaError;
  lk.lock();  // slots stay as they are: a slower peer may still be reading them until this barrier
  return enqueue_result(barrier(g, lk, c->rank, "ncclAllReduce (release)"));
}

}  // extern "C"
