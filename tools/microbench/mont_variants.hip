// Montgomery-multiply variants on gfx950: how much do hazard wait states around the carry chain
// cost, and does grouping the hand-issued MACs into larger asm statements help?
//   B1 : one asm statement per product (mad + addc)  — hipcc inserts s_nop 0 between statements
//   B6 : the same products, six per asm statement     — 6x fewer inserted nops
//   BI : B1 with two independent multiplies interleaved (ILP across chains)
// Each variant is checked against a CPU model before timing.
// Build: hipcc --offload-arch=gfx950 -O3 -o mont_variants mont_variants.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

static constexpr uint32_t P[12] = {0xffffaaab,0xb9feffff,0xb153ffff,0x1eabfffe,0xf6b0f624,0x6730d2a0,
                                   0xf38512bf,0x64774b84,0x434bacd7,0x4b1ba7b6,0x397fe69a,0x1a0111ea};
#define PINV 0xfffcfffdu

__device__ __forceinline__ void mac1(uint64_t& lo, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(lo), "=&s"(cc), "+v"(hi) : "v"(x), "v"(y));
}
#define MAC_STR(x, y) "v_mad_u64_u32 %0, %1, %" #x ", %" #y ", %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1\n\t"

// up to 6 products in one statement; unused slots get x = y = 0 (harmless)
__device__ __forceinline__ void mac6(uint64_t& lo, uint32_t& hi, const uint32_t* x, const uint32_t* y, int n) {
  uint64_t cc;
  if (n == 6)
    asm(MAC_STR(3, 4) MAC_STR(5, 6) MAC_STR(7, 8) MAC_STR(9, 10) MAC_STR(11, 12) MAC_STR(13, 14)
        : "+v"(lo), "=&s"(cc), "+v"(hi)
        : "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]), "v"(x[4]),
          "v"(y[4]), "v"(x[5]), "v"(y[5]));
  else
    for (int k = 0; k < n; k++) mac1(lo, hi, x[k], y[k]);
}

template <int G>
__device__ __forceinline__ void mont(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  uint32_t m[12];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 24; i++) {
    // gather this column's operand pairs
    uint32_t xs[24], ys[24];
    int n = 0;
    const int j0 = i < 12 ? 0 : i - 11, j1 = i < 12 ? i : 11;
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      if (i < 12 && j == i) continue;  // a_i b_0 and m_i p_0 handled below for low columns
      xs[n] = a[j], ys[n] = b[i - j], n++;
      xs[n] = m[j], ys[n] = P[i - j], n++;
    }
    if (G == 6) {
#pragma unroll
      for (int k = 0; k < 24; k += 6)
        if (k < n) mac6(lo, hi, xs + k, ys + k, (n - k) >= 6 ? 6 : n - k);
    } else {
#pragma unroll
      for (int k = 0; k < 24; k++)
        if (k < n) mac1(lo, hi, xs[k], ys[k]);
    }
    if (i < 12) {
      mac1(lo, hi, a[i], b[0]);
      m[i] = (uint32_t)lo * PINV;
      mac1(lo, hi, m[i], P[0]);
    } else {
      r[i - 12] = (uint32_t)lo;
    }
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
}

template <int G, int CH>
__global__ void __launch_bounds__(256) kmont(uint32_t* out, const uint32_t* in, int iters, int lds_pad) {
  extern __shared__ uint32_t pad[];
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[CH][12], y[12];
#pragma unroll
  for (int j = 0; j < 12; j++) {
    y[j] = in[(tid * 7 + j) & 1023] & (j == 11 ? 0x0fffffffu : 0xffffffffu);
#pragma unroll
    for (int c = 0; c < CH; c++) x[c][j] = in[(tid * 13 + j + 12 * c + 100) & 1023] & (j == 11 ? 0x0fffffffu : 0xffffffffu);
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) mont<G>(x[c], x[c], y);
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int j = 0; j < 12; j++) s += x[c][j] * (j + 1);
  if (lds_pad < 0) pad[threadIdx.x] = s;  // never true; keeps the LDS allocation
  out[tid] = s;
}

template <int G>
__global__ void kcheck(uint32_t* out, const uint32_t* in) {
  int t = threadIdx.x;
  uint32_t a[12], b[12], r[12];
  for (int j = 0; j < 12; j++) a[j] = in[t * 24 + j], b[j] = in[t * 24 + 12 + j];
  mont<G>(r, a, b);
  for (int j = 0; j < 12; j++) out[t * 12 + j] = r[j];
}

static void mont_ref(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  uint32_t t[14] = {0};
  for (int i = 0; i < 12; i++) {
    uint64_t C = 0;
    for (int j = 0; j < 12; j++) { C = (uint64_t)a[j] * b[i] + t[j] + (C >> 32); t[j] = (uint32_t)C; }
    C = (uint64_t)t[12] + (C >> 32); t[12] = (uint32_t)C; t[13] = (uint32_t)(C >> 32);
    uint32_t m = t[0] * PINV;
    C = (uint64_t)m * P[0] + t[0];
    for (int j = 1; j < 12; j++) { C = (uint64_t)m * P[j] + t[j] + (C >> 32); t[j - 1] = (uint32_t)C; }
    C = (uint64_t)t[12] + (C >> 32); t[11] = (uint32_t)C;
    t[12] = t[13] + (uint32_t)(C >> 32);
  }
  for (int j = 0; j < 12; j++) r[j] = t[j];
}

int main() {
  uint32_t *out, *in;
  const int blocks = 256 * 16, threads = 256;
  CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
  CHECK(hipMalloc(&in, 64 * 24 * 4));
  uint32_t hin[64 * 24];
  uint64_t s = 0x9e3779b97f4a7c15ULL;
  for (int i = 0; i < 64 * 24; i++) { s = s * 6364136223846793005ULL + 1; hin[i] = (uint32_t)(s >> 32); }
  for (int t = 0; t < 64; t++) { hin[t * 24 + 11] &= 0x1fffffff; hin[t * 24 + 23] &= 0x1fffffff; }
  CHECK(hipMemcpy(in, hin, sizeof hin, hipMemcpyHostToDevice));
  // correctness: one wave alone (back-to-back issue, the worst case for any hazard)
  for (int g = 0; g < 2; g++) {
    uint32_t hout[64 * 12], ref[12];
    if (g == 0) hipLaunchKernelGGL(kcheck<1>, 1, 64, 0, 0, out, in);
    else hipLaunchKernelGGL(kcheck<6>, 1, 64, 0, 0, out, in);
    CHECK(hipMemcpy(hout, out, sizeof hout, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int t = 0; t < 64; t++) {
      mont_ref(ref, hin + t * 24, hin + t * 24 + 12);
      for (int j = 0; j < 12; j++) if (ref[j] != hout[t * 12 + j]) { bad++; break; }
    }
    printf("check G=%d: %d/64 mismatches\n", g ? 6 : 1, bad);
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // occupancy control: LDS per block = 160 KiB / (blocks per CU); 256 threads = 4 waves per block
  const int occ_blocks[4] = {1, 2, 4, 8};  // blocks/CU -> waves/SIMD = blocks/CU
  for (int v = 0; v < 3; v++) {
    for (int oi = 0; oi < 4; oi++) {
      int bpc = occ_blocks[oi];
      size_t lds = (160 * 1024) / bpc - 1024;
      int iters = 100;
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        CHECK(hipEventRecord(e0));
        if (v == 0) hipLaunchKernelGGL((kmont<1, 1>), blocks, threads, lds, 0, out, in, iters, 0);
        if (v == 1) hipLaunchKernelGGL((kmont<6, 1>), blocks, threads, lds, 0, out, in, iters, 0);
        if (v == 2) hipLaunchKernelGGL((kmont<1, 2>), blocks, threads, lds, 0, out, in, iters / 2, 0);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
      }
      double nm = (double)blocks * threads * iters;
      const char* nm_[3] = {"B1 (asm/product)", "B6 (asm/6 products)", "BI (2 chains interleaved)"};
      printf("%-26s waves/SIMD<=%d: %8.3f ms  %7.2f G fp-mul/s\n", nm_[v], bpc, ms, nm / ms / 1e6);
    }
  }
  CHECK(hipGetLastError());
  return 0;
}
