// Radix-2^28 Montgomery multiply (14 limbs, R = 2^392) vs the radix-2^32 FIPS (B6 grouping).
// With 28-bit limbs every column sum (<= 28 products of < 2^60 each when both operands have
// limbs < 2^30, plus a < 2^36 carry) fits one 64-bit accumulator, so each product is ONE
// v_mad_u64_u32 and no carry ever goes through an SGPR: plain C++, compiler-scheduled.
// Build: hipcc --offload-arch=gfx950 -O3 -o mont28 mont28.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

static constexpr uint32_t P28[14] = {0xfffaaab, 0xfefffff, 0x3ffffb9, 0xfffeb15, 0x6241eab, 0xa0f6b0f, 0xf6730d2,
                                     0xf38512b, 0x4774b84, 0x4bacd76, 0xba7b643, 0xe69a4b1, 0x1ea397f, 0x1a011};
#define PINV28 0xffcfffdu
#define M28 0xfffffffu

// variant 0: single accumulator, straight FIPS
template <int V>
__device__ __forceinline__ void mont28(uint32_t r[14], const uint32_t a[14], const uint32_t b[14]) {
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 28; i++) {
    const int j0 = i < 14 ? 0 : i - 13, j1 = i < 14 ? i : 13;
    if (V == 0) {
#pragma unroll
      for (int j = j0; j <= j1; j++) {
        if (i < 14 && j == i) continue;
        acc += (uint64_t)a[j] * b[i - j];
        acc += (uint64_t)m[j] * P28[i - j];
      }
    } else {  // two accumulators (a*b and m*p) to shorten the dependency chain
      uint64_t acc2 = 0;
#pragma unroll
      for (int j = j0; j <= j1; j++) {
        if (i < 14 && j == i) continue;
        acc += (uint64_t)a[j] * b[i - j];
        acc2 += (uint64_t)m[j] * P28[i - j];
      }
      acc += acc2;
    }
    if (i < 14) {
      acc += (uint64_t)a[i] * b[0];
      m[i] = ((uint32_t)acc * PINV28) & M28;
      acc += (uint64_t)m[i] * P28[0];
    } else {
      r[i - 14] = (uint32_t)acc & M28;
    }
    acc >>= 28;
  }
}

// dedicated squaring: cross products once (a_j * 2 a_k), then the same interleaved REDC
__device__ __forceinline__ void sqr28(uint32_t r[14], const uint32_t a[14]) {
  uint32_t d[14], m[14];
#pragma unroll
  for (int j = 0; j < 14; j++) d[j] = a[j] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 27; i++) {
    const int j0 = i < 14 ? 0 : i - 13;
    uint64_t accp = 0;
#pragma unroll
    for (int j = j0; 2 * j < i; j++) acc += (uint64_t)a[j] * d[i - j];
    if ((i & 1) == 0) acc += (uint64_t)a[i / 2] * a[i / 2];
    const int k1 = i < 14 ? i - 1 : 13;
#pragma unroll
    for (int k = j0; k <= k1; k++) accp += (uint64_t)m[k] * P28[i - k];
    acc += accp;
    if (i < 14) {
      m[i] = ((uint32_t)acc * PINV28) & M28;
      acc += (uint64_t)m[i] * P28[0];
    } else {
      r[i - 14] = (uint32_t)acc & M28;
    }
    acc >>= 28;
  }
  r[13] = (uint32_t)acc & M28;
}

template <int V, int CH>
__global__ void __launch_bounds__(256) kmont(uint32_t* out, const uint32_t* in, int iters, int lds_pad) {
  extern __shared__ uint32_t pad[];
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[CH][14], y[14];
#pragma unroll
  for (int j = 0; j < 14; j++) {
    y[j] = in[(tid * 7 + j) & 1023] & (j == 13 ? 0xffffu : M28);
#pragma unroll
    for (int c = 0; c < CH; c++) x[c][j] = in[(tid * 13 + j + 14 * c + 100) & 1023] & (j == 13 ? 0xffffu : M28);
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      if (V == 2) sqr28(x[c], x[c]);
      else mont28<V>(x[c], x[c], y);
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int j = 0; j < 14; j++) s += x[c][j] * (j + 1);
  if (lds_pad < 0) pad[threadIdx.x] = s;
  out[tid] = s;
}

template <int V>
__global__ void kcheck(uint32_t* out, const uint32_t* in) {
  int t = threadIdx.x;
  uint32_t a[14], b[14], r[14];
  for (int j = 0; j < 14; j++) a[j] = in[t * 28 + j], b[j] = in[t * 28 + 14 + j];
  if (V == 2) sqr28(r, a);
  else mont28<V>(r, a, b);
  for (int j = 0; j < 14; j++) out[t * 14 + j] = r[j];
}

// CPU model: big-integer Montgomery with R = 2^392 using __int128 limbs of 28 bits
static void mont_ref(uint32_t r[14], const uint32_t a[14], const uint32_t b[14]) {
  // schoolbook product into 28 limbs of 64 bits, then REDC word by word
  unsigned __int128 t[30] = {0};
  for (int i = 0; i < 14; i++)
    for (int j = 0; j < 14; j++) t[i + j] += (unsigned __int128)a[i] * b[j];
  for (int i = 0; i < 14; i++) {
    uint32_t m = ((uint32_t)(uint64_t)t[i] * PINV28) & M28;
    for (int j = 0; j < 14; j++) t[i + j] += (unsigned __int128)m * P28[j];
    t[i + 1] += t[i] >> 28;
    t[i] = 0;
  }
  for (int i = 14; i < 28; i++) {
    t[i + 1] += t[i] >> 28;
    r[i - 14] = (uint32_t)(t[i] & M28);
  }
}

int main() {
  uint32_t *out, *in;
  const int blocks = 256 * 16, threads = 256;
  CHECK(hipMalloc(&out, (size_t)blocks * threads * 4 * 16));
  CHECK(hipMalloc(&in, 1024 * 4 * 4));
  static uint32_t hin[4096];
  uint64_t s = 0x9e3779b97f4a7c15ULL;
  for (int i = 0; i < 4096; i++) { s = s * 6364136223846793005ULL + 1; hin[i] = (uint32_t)(s >> 32); }
  // check inputs: limbs up to 30 bits (the widest the design feeds in), top limb small
  static uint32_t cin[64 * 28];
  for (int t = 0; t < 64; t++)
    for (int j = 0; j < 28; j++) cin[t * 28 + j] = hin[t * 28 + j] & ((j % 14) == 13 ? 0x3ffffu : 0x3fffffffu);
  CHECK(hipMemcpy(in, cin, sizeof cin, hipMemcpyHostToDevice));
  for (int v = 0; v < 2; v++) {
    uint32_t hout[64 * 14], ref[14];
    if (v == 0) hipLaunchKernelGGL(kcheck<0>, 1, 64, 0, 0, out, in);
    else hipLaunchKernelGGL(kcheck<1>, 1, 64, 0, 0, out, in);
    CHECK(hipMemcpy(hout, out, sizeof hout, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int t = 0; t < 64; t++) {
      mont_ref(ref, cin + t * 28, cin + t * 28 + 14);
      for (int j = 0; j < 14; j++) if (ref[j] != hout[t * 14 + j]) { bad++; break; }
    }
    printf("check V=%d: %d/64 mismatches\n", v, bad);
  }
  {
    uint32_t hout[64 * 14], ref[14];
    hipLaunchKernelGGL(kcheck<2>, 1, 64, 0, 0, out, in);
    CHECK(hipMemcpy(hout, out, sizeof hout, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int t = 0; t < 64; t++) {
      mont_ref(ref, cin + t * 28, cin + t * 28);
      for (int j = 0; j < 14; j++) if (ref[j] != hout[t * 14 + j]) { bad++; break; }
    }
    printf("check sqr: %d/64 mismatches\n", bad);
  }
  CHECK(hipMemcpy(in, hin, 4096 * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int occ[4] = {1, 2, 4, 8};
  for (int v = 0; v < 5; v++)
    for (int oi = 0; oi < 4; oi++) {
      size_t lds = (160 * 1024) / occ[oi] - 1024;
      int iters = 100;
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        CHECK(hipEventRecord(e0));
        if (v == 0) hipLaunchKernelGGL((kmont<0, 1>), blocks, threads, lds, 0, out, in, iters, 0);
        if (v == 1) hipLaunchKernelGGL((kmont<1, 1>), blocks, threads, lds, 0, out, in, iters, 0);
        if (v == 2) hipLaunchKernelGGL((kmont<0, 2>), blocks, threads, lds, 0, out, in, iters / 2, 0);
        if (v == 3) hipLaunchKernelGGL((kmont<2, 1>), blocks, threads, lds, 0, out, in, iters, 0);
        if (v == 4) hipLaunchKernelGGL((kmont<2, 2>), blocks, threads, lds, 0, out, in, iters / 2, 0);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
      }
      const char* nm[5] = {"R28 single acc", "R28 two acc", "R28 2 chains", "R28 sqr", "R28 sqr 2 chains"};
      printf("%-16s waves/SIMD<=%d: %8.3f ms  %7.2f G fp-mul/s\n", nm[v], occ[oi], ms,
             (double)blocks * threads * iters / ms / 1e6);
    }
  CHECK(hipGetLastError());
  return 0;
}
