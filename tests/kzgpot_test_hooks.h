/*
 * Test-only entry points of libkzgpot_test.so (kzg-setup-powersoftau_amd/Makefile, built with
 * -DKZGPOT_TEST_HOOKS). The product library (libkzgpot.so) exports none of this and binds only
 * librccl.so.1.
 *
 * In the test build, KZGPOT_RCCL_LIB=<path> binds another library exporting RCCL's entry points
 * instead of librccl.so.1, read once per process: tests/fake_rccl runs N ranks as threads of one
 * process on one GPU (tests/test_gpu_multirank.py).
 */
#ifndef KZGPOT_TEST_HOOKS_H
#define KZGPOT_TEST_HOOKS_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* Failure injection (SURVEY §5 "failure detection"): the NEXT kzgpot_decode_allgather_dev on this
 * communicator fails at site `site`, step `at`, once:
 *   KZGPOT_FAULT_LAUNCH: the decode launch of chunk `at` (at == chunks: the tail) reports a HIP
 *   launch failure; KZGPOT_FAULT_COLLECTIVE: the `at`-th all-gather (0-based; at == chunks: the
 *   key all-reduce) reports an RCCL error. site 0 clears. */
#define KZGPOT_FAULT_LAUNCH 1
#define KZGPOT_FAULT_COLLECTIVE 2
int kzgpot_comm_inject_fault(void* comm, int site, uint32_t at);
/* Host-resource failure injection (csrc/capi.hip): from the (skip + 1)-th event of `site` on, every
 * such event in the process fails, until site 0 clears it:
 *   KZGPOT_HOST_FAULT_THREAD: a library host thread fails to start, as std::thread does with
 *   std::system_error(EAGAIN) under RLIMIT_NPROC; KZGPOT_HOST_FAULT_HOSTBUF: the file path's
 *   large anonymous mapping fails (mmap MAP_FAILED). The entry points must return
 *   KZGPOT_E_OUT_OF_MEMORY with every started thread joined and no temporary file left. */
#define KZGPOT_HOST_FAULT_THREAD 1
#define KZGPOT_HOST_FAULT_HOSTBUF 2
int kzgpot_test_inject_host_fault(int site, long skip);
/* The chunk plan of a host-buffer call of n points (csrc/capi.hip ChunkPlan): up to cap (offset,
 * count) pairs into spans; returns the number of chunks. streaming_consumer: the e2e output digest
 * reads the chunks as they land (its first chunk is small). */
long kzgpot_test_chunk_plan(uint64_t n, int streaming_consumer, uint64_t* spans, long cap);
#ifdef __cplusplus
}
#endif
#endif
