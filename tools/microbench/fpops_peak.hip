// Chip-wide throughput peak of each Montgomery primitive the codecs use (csrc/fp381.hpp, the
// product's own functions): fp_mul, fp_sqr, fp_mul_sum2, fp_mul_sum3, fp_mul_addsqr<1> on
// 14 x 28-bit limbs and f30_mul / f30_sqr on the square root's 13 x 30-bit balanced limbs. Each
// lane runs CH independent chains of the op on register operands; the launch holds 256 blocks per
// CU's worth of waves, with LDS padding capping the waves per SIMD (2 = the codecs' occupancy, 4).
// tools/fpops/census.py sets the codec's per-point reduction census against these peaks.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-use-divergent-register-indexing=1
//        -o bin/fpops_peak fpops_peak.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../kzg-setup-powersoftau_amd/csrc/fp381.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using kzgpot::fp;
using kzgpot::f30;
constexpr int N28 = kzgpot::NL;
constexpr int NOPS = 7;
const char* kName[NOPS] = {"fp_mul", "fp_sqr", "fp_mul_sum2", "fp_mul_sum3", "fp_mul_addsqr", "f30_mul", "f30_sqr"};

__device__ void load_fp(fp& x, const uint32_t* in, int base) {
#pragma unroll
  for (int j = 0; j < N28; j++) x.v[j] = in[(base + j) & 1023] & (j == N28 - 1 ? 0xffffu : kzgpot::LMASK);
}

// V: index into kName. CH independent chains per lane.
template <int V, int CH>
__global__ void __launch_bounds__(256) kpeak(uint32_t* out, const uint32_t* in, int iters, int lds_pad) {
  extern __shared__ uint32_t pad[];
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  // Every product of an op has an operand from the chain (x the newest value, x1 / x2 the two
  // before it), and no two products share one: with a loop-invariant product (z w) or a common
  // factor (x y + x z) the compiler hoists or factors work the kernels cannot.
  fp x[CH], x1[CH], x2[CH], y, z, w;
  load_fp(y, in, tid * 7);
  load_fp(z, in, tid * 5 + 300);
  load_fp(w, in, tid * 3 + 600);
#pragma unroll
  for (int c = 0; c < CH; c++) {
    load_fp(x[c], in, tid * 13 + 14 * c + 100);
    load_fp(x1[c], in, tid * 11 + 14 * c + 400);
    load_fp(x2[c], in, tid * 17 + 14 * c + 800);
  }
  uint32_t s = 0;
  if constexpr (V < 5) {
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int c = 0; c < CH; c++) {
        fp r;
        if (V == 0) kzgpot::fp_mul(r, x[c], y);
        if (V == 1) kzgpot::fp_sqr(r, x[c]);
        if (V == 2) kzgpot::fp_mul_sum2(r, x[c], y, x1[c], z);
        if (V == 3) kzgpot::fp_mul_sum3(r, x[c], y, x1[c], z, x2[c], w);
        if (V == 4) kzgpot::fp_mul_addsqr<1>(r, x[c], y, x1[c]);
        if (V >= 3) x2[c] = x1[c];
        if (V >= 2) x1[c] = x[c];
        x[c] = r;
      }
    }
#pragma unroll
    for (int c = 0; c < CH; c++)
#pragma unroll
      for (int j = 0; j < N28; j++) s += x[c].v[j] * (j + 1);
  } else {
    f30 a[CH], b;
    kzgpot::f30_from_fp(b, y);
#pragma unroll
    for (int c = 0; c < CH; c++) kzgpot::f30_from_fp(a[c], x[c]);
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int c = 0; c < CH; c++) {
        if (V == 5) kzgpot::f30_mul(a[c], a[c], b);
        if (V == 6) kzgpot::f30_sqr(a[c], a[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < CH; c++)
#pragma unroll
      for (int j = 0; j < kzgpot::N30; j++) s += (uint32_t)a[c].v[j] * (j + 1);
  }
  if (lds_pad < 0) pad[threadIdx.x] = s;
  out[tid] = s;
}

template <int V, int CH>
void launch(int blocks, size_t lds, uint32_t* out, const uint32_t* in, int iters) {
  hipLaunchKernelGGL((kpeak<V, CH>), blocks, 256, lds, 0, out, in, iters / CH, 0);
}
template <int CH>
void launch_op(int v, int blocks, size_t lds, uint32_t* out, const uint32_t* in, int iters) {
  switch (v) {
    case 0: launch<0, CH>(blocks, lds, out, in, iters); break;
    case 1: launch<1, CH>(blocks, lds, out, in, iters); break;
    case 2: launch<2, CH>(blocks, lds, out, in, iters); break;
    case 3: launch<3, CH>(blocks, lds, out, in, iters); break;
    case 4: launch<4, CH>(blocks, lds, out, in, iters); break;
    case 5: launch<5, CH>(blocks, lds, out, in, iters); break;
    case 6: launch<6, CH>(blocks, lds, out, in, iters); break;
  }
}

int main() {
  uint32_t *out, *in;
  const int blocks = 256 * 16, threads = 256, iters = 64;
  CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
  CHECK(hipMalloc(&in, 1024 * 4));
  static uint32_t hin[1024];
  uint64_t s = 0x9e3779b97f4a7c15ULL;
  for (int i = 0; i < 1024; i++) { s = s * 6364136223846793005ULL + 1; hin[i] = (uint32_t)(s >> 32); }
  CHECK(hipMemcpy(in, hin, sizeof hin, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int pass = 0; pass < 3; pass++)  // two passes through the clock ramp, the third printed
    for (int v = 0; v < NOPS; v++)
      for (int ch = 1; ch <= 2; ch++)
        for (int occ = 2; occ <= 4; occ += 2) {
          const size_t lds = (160 * 1024) / occ - 1024;
          float ms = 0;
          CHECK(hipEventRecord(e0));
          if (ch == 1) launch_op<1>(v, blocks, lds, out, in, iters);
          else launch_op<2>(v, blocks, lds, out, in, iters);
          CHECK(hipEventRecord(e1));
          CHECK(hipEventSynchronize(e1));
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          if (pass == 2)
            printf("%-14s chains %d waves/SIMD<=%d: %8.3f ms  %7.2f G ops/s\n", kName[v], ch, occ, ms,
                   (double)blocks * threads * iters / ms / 1e6);
        }
  CHECK(hipGetLastError());
  return 0;
}
