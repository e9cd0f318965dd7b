// Field-operation census (measurement build, not the product): the codec kernels compiled with
// fp381.hpp's KZG_FPOP hook counting every Montgomery reduction by kind, so that the per-point
// reduction counts the DESIGN states (doublings x reductions, square-root chain) are measured
// rather than derived, and the codec's field-op rate can be set against the microbenchmarked
// peak of each primitive (tools/microbench/fpops_peak.hip; tools/fpops/census.py combines them).
//
// One translation unit: the kernel sources are included here with the hook defined, so the
// counters are this module's own device globals. Counting costs an atomic per reduction per
// lane, so this build is run on a few thousand points only.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ unsigned long long g_fpops[8];
#define KZG_FPOP(kind) atomicAdd(&g_fpops[(int)(kind)], 1ull)

#include "../../kzg-setup-powersoftau_amd/csrc/bn254_kernels.hip"
#include "../../kzg-setup-powersoftau_amd/csrc/codec_kernels.hip"
#include "../../kzg-setup-powersoftau_amd/csrc/g1_kernels.hip"
#include "../../kzg-setup-powersoftau_amd/csrc/load_kernels.hip"

// op: kzgpot::CodecOp as an int (0 G1Decompress, 1 G2Decompress, 2 G1Transcode, 3 G2Transcode,
// 4 G1Load, 5 G2Load, 6 Bn254G1Decompress). d_in / d_out / d_status: device buffers sized for n
// records. counts: host array of kzgpot::FpOp::Count totals over the launch. *first_bad: the
// launch's rejection key (all ones when every point was accepted). Returns a hipError_t.
extern "C" int fp_census_run(int op, const void* d_in, uint64_t n, void* d_out, uint32_t flags, uint8_t* d_status,
                             unsigned long long* counts, unsigned long long* first_bad) {
  constexpr int K = (int)kzgpot::FpOp::Count;
  static_assert(K <= 8, "census slots");
  if (op < 0 || op > (int)kzgpot::CodecOp::Bn254G1Decompress) return (int)hipErrorInvalidValue;
  unsigned long long zero[8] = {0}, *d_key = nullptr;
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_fpops), zero, sizeof zero);
  if (e == hipSuccess) e = hipMalloc(&d_key, sizeof *d_key);
  if (e == hipSuccess) e = hipMemset(d_key, 0xff, sizeof *d_key);
  if (e == hipSuccess)
    e = kzgpot::launch_codec((kzgpot::CodecOp)op, d_in, d_out, n, flags, d_key, d_status, nullptr);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  unsigned long long got[8];
  if (e == hipSuccess) e = hipMemcpyFromSymbol(got, HIP_SYMBOL(g_fpops), sizeof got);
  if (e == hipSuccess) e = hipMemcpy(first_bad, d_key, sizeof *d_key, hipMemcpyDeviceToHost);
  if (e == hipSuccess)
    for (int k = 0; k < K; k++) counts[k] = got[k];
  if (d_key) (void)hipFree(d_key);
  return (int)e;
}
