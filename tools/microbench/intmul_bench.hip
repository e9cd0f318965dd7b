// Integer-VALU microbenchmark for gfx950: the roof of the BLS12-381 point codec.
//
// The hot path is bound by 381-bit Montgomery multiplies, not by HBM.
// This measures (1) raw issue rates of the 32-bit multiply primitives CDNA4 offers and
// (2) full 12x32-bit-limb Montgomery multiplies in three formulations, chip-wide, so the
// kernel design and the reported "Fp-mul peak" rest on measurements.
//
// Build:  hipcc --offload-arch=gfx950 -O3 -o intmul_bench intmul_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__constant__ uint32_t P[12] = {0xffffaaab,0xb9feffff,0xb153ffff,0x1eabfffe,0xf6b0f624,0x6730d2a0,
                               0xf38512bf,0x64774b84,0x434bacd7,0x4b1ba7b6,0x397fe69a,0x1a0111ea};
#define PINV 0xfffcfffdu

// ---------------- primitives ----------------
template <int OP>
__global__ void prim(uint32_t* out, int iters, uint32_t seed) {
  uint32_t x[16];
#pragma unroll
  for (int k = 0; k < 16; k++) x[k] = seed * (threadIdx.x + 17 * k + 1);
  uint32_t y = seed ^ blockIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if constexpr (OP == 0) {  // v_mad_u64_u32 (64-bit accumulate)
        uint64_t acc = ((uint64_t)x[k] << 32) | x[(k + 1) & 15];
        uint64_t cc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(x[k]), "v"(y));
        x[k] = (uint32_t)acc ^ (uint32_t)(acc >> 32);
      } else if constexpr (OP == 1) {  // v_mul_lo_u32
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "v"(y));
      } else if constexpr (OP == 2) {  // v_mul_hi_u32
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[k]) : "v"(y));
      } else if constexpr (OP == 3) {  // v_add_co_u32 (carry to sgpr pair)
        asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x[k]) : "v"(y) : "vcc");
      } else if constexpr (OP == 4) {  // v_mul_u32_u24
        asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[k]) : "v"(y));
      } else if constexpr (OP == 5) {  // v_mad_u64_u32 only (no xor), pure
        uint64_t acc = ((uint64_t)x[k] << 32) | x[(k + 3) & 15];
        uint64_t cc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
                     "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
                     "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
                     "v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(x[k]), "v"(y));
        x[k] = (uint32_t)acc;
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) s ^= x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---------------- Montgomery multiply variants (inputs < 2p, output < 2p) ----------------
// A: plain C++ CIOS, 64-bit intermediates (compiler picks the instructions).
__device__ __forceinline__ void mont_A(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  uint32_t t[13];
#pragma unroll
  for (int j = 0; j < 13; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t C = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
      C = (uint64_t)a[j] * b[i] + t[j] + (C >> 32);
      t[j] = (uint32_t)C;
    }
    t[12] += (uint32_t)(C >> 32);
    uint32_t m = t[0] * PINV;
    C = (uint64_t)m * P[0] + t[0];
#pragma unroll
    for (int j = 1; j < 12; j++) {
      C = (uint64_t)m * P[j] + t[j] + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    C = (uint64_t)t[12] + (C >> 32);
    t[11] = (uint32_t)C;
    t[12] = (uint32_t)(C >> 32);
  }
#pragma unroll
  for (int j = 0; j < 12; j++) r[j] = t[j];
}

// B: finely-integrated product scanning (FIPS), 3-word column accumulator, hand-issued
// v_mad_u64_u32 with its carry-out folded into the third word by v_addc_co_u32.
__device__ __forceinline__ void mac3(uint64_t& lo, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(lo), "=&s"(cc), "+v"(hi) : "v"(x), "v"(y));
}
__device__ __forceinline__ void mont_B(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  uint32_t m[12];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      mac3(lo, hi, a[j], b[i - j]);
      mac3(lo, hi, m[j], P[i - j]);
    }
    mac3(lo, hi, a[i], b[0]);
    m[i] = (uint32_t)lo * PINV;
    mac3(lo, hi, m[i], P[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int i = 12; i < 24; i++) {
#pragma unroll
    for (int j = i - 11; j < 12; j++) {
      mac3(lo, hi, a[j], b[i - j]);
      mac3(lo, hi, m[j], P[i - j]);
    }
    r[i - 12] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
}

// C: FIPS in plain C++ (carry detected by compare), to see what the compiler makes of it.
__device__ __forceinline__ void mac3c(uint64_t& lo, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t p = (uint64_t)x * y;
  lo += p;
  hi += (lo < p);
}
__device__ __forceinline__ void mont_C(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  uint32_t m[12];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      mac3c(lo, hi, a[j], b[i - j]);
      mac3c(lo, hi, m[j], P[i - j]);
    }
    mac3c(lo, hi, a[i], b[0]);
    m[i] = (uint32_t)lo * PINV;
    mac3c(lo, hi, m[i], P[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int i = 12; i < 24; i++) {
#pragma unroll
    for (int j = i - 11; j < 12; j++) {
      mac3c(lo, hi, a[j], b[i - j]);
      mac3c(lo, hi, m[j], P[i - j]);
    }
    r[i - 12] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
}

template <int V, int CHAINS>
__global__ void montk(uint32_t* out, const uint32_t* in, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[CHAINS][12], y[12];
#pragma unroll
  for (int j = 0; j < 12; j++) {
    y[j] = in[(tid * 7 + j) & 1023] & (j == 11 ? 0x0fffffffu : 0xffffffffu);
#pragma unroll
    for (int c = 0; c < CHAINS; c++)
      x[c][j] = in[(tid * 13 + j + 12 * c + 100) & 1023] & (j == 11 ? 0x0fffffffu : 0xffffffffu);
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) {
      if constexpr (V == 0) mont_A(x[c], x[c], y);
      if constexpr (V == 1) mont_B(x[c], x[c], y);
      if constexpr (V == 2) mont_C(x[c], x[c], y);
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++)
#pragma unroll
    for (int j = 0; j < 12; j++) s += x[c][j] * (j + 1);
  out[tid] = s;
}

// Host-side check: all variants compute the same Montgomery product (vs a 64-bit CPU model).
static void mont_ref(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  static const uint32_t Ph[12] = {0xffffaaab,0xb9feffff,0xb153ffff,0x1eabfffe,0xf6b0f624,0x6730d2a0,
                                  0xf38512bf,0x64774b84,0x434bacd7,0x4b1ba7b6,0x397fe69a,0x1a0111ea};
  uint32_t t[14] = {0};
  for (int i = 0; i < 12; i++) {
    uint64_t C = 0;
    for (int j = 0; j < 12; j++) { C = (uint64_t)a[j] * b[i] + t[j] + (C >> 32); t[j] = (uint32_t)C; }
    C = (uint64_t)t[12] + (C >> 32); t[12] = (uint32_t)C; t[13] = (uint32_t)(C >> 32);
    uint32_t m = t[0] * PINV;
    C = (uint64_t)m * Ph[0] + t[0];
    for (int j = 1; j < 12; j++) { C = (uint64_t)m * Ph[j] + t[j] + (C >> 32); t[j - 1] = (uint32_t)C; }
    C = (uint64_t)t[12] + (C >> 32); t[11] = (uint32_t)C;
    t[12] = t[13] + (uint32_t)(C >> 32);
  }
  for (int j = 0; j < 12; j++) r[j] = t[j];
}

template <int V>
__global__ void montcheck(uint32_t* out, const uint32_t* in) {
  int tid = threadIdx.x;
  uint32_t a[12], b[12], r[12];
  for (int j = 0; j < 12; j++) { a[j] = in[tid * 24 + j]; b[j] = in[tid * 24 + 12 + j]; }
  if constexpr (V == 0) mont_A(r, a, b);
  if constexpr (V == 1) mont_B(r, a, b);
  if constexpr (V == 2) mont_C(r, a, b);
  for (int j = 0; j < 12; j++) out[tid * 12 + j] = r[j];
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  const int blocks = 256 * 16, threads = 256;
  uint32_t *out, *in;
  CHECK(hipMalloc(&out, (size_t)blocks * threads * 4 * 16));
  CHECK(hipMalloc(&in, 1024 * 4 * 8));
  uint32_t hin[8192];
  uint64_t s = 0x12345678abcdefULL;
  for (int i = 0; i < 8192; i++) { s = s * 6364136223846793005ULL + 1442695040888963407ULL; hin[i] = (uint32_t)(s >> 33) ^ (uint32_t)s; }
  // keep check operands < 2p: top limb masked
  for (int t = 0; t < 64; t++) { hin[t * 24 + 11] &= 0x1fffffff; hin[t * 24 + 23] &= 0x1fffffff; }
  CHECK(hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float ms;

  // correctness of the variants
  {
    uint32_t hout[64 * 12], ref[12];
    int bad[3] = {0, 0, 0};
    for (int v = 0; v < 3; v++) {
      if (v == 0) hipLaunchKernelGGL(montcheck<0>, 1, 64, 0, 0, out, in);
      if (v == 1) hipLaunchKernelGGL(montcheck<1>, 1, 64, 0, 0, out, in);
      if (v == 2) hipLaunchKernelGGL(montcheck<2>, 1, 64, 0, 0, out, in);
      CHECK(hipMemcpy(hout, out, sizeof(hout), hipMemcpyDeviceToHost));
      for (int t = 0; t < 64; t++) {
        mont_ref(ref, hin + t * 24, hin + t * 24 + 12);
        for (int j = 0; j < 12; j++) if (ref[j] != hout[t * 12 + j]) { bad[v]++; break; }
      }
    }
    printf("montcheck mismatches: A=%d B=%d C=%d (of 64)\n", bad[0], bad[1], bad[2]);
  }

  const char* pname[6] = {"v_mad_u64_u32(+xor)", "v_mul_lo_u32", "v_mul_hi_u32", "v_add_co_u32", "v_mul_u32_u24", "v_mad_u64_u32 x4"};
  for (int op = 0; op < 6; op++) {
    int iters = 2000;
    for (int rep = 0; rep < 2; rep++) {
      CHECK(hipEventRecord(e0));
      switch (op) {
        case 0: hipLaunchKernelGGL(prim<0>, blocks, threads, 0, 0, out, iters, 3u); break;
        case 1: hipLaunchKernelGGL(prim<1>, blocks, threads, 0, 0, out, iters, 3u); break;
        case 2: hipLaunchKernelGGL(prim<2>, blocks, threads, 0, 0, out, iters, 3u); break;
        case 3: hipLaunchKernelGGL(prim<3>, blocks, threads, 0, 0, out, iters, 3u); break;
        case 4: hipLaunchKernelGGL(prim<4>, blocks, threads, 0, 0, out, iters, 3u); break;
        case 5: hipLaunchKernelGGL(prim<5>, blocks, threads, 0, 0, out, iters, 3u); break;
      }
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    }
    double nops = (double)blocks * threads * iters * 16 * (op == 5 ? 4 : 1);
    printf("%-22s %8.3f ms  %8.2f Tlane-op/s  (%.1f lane-op/clk/CU @2.4GHz)\n", pname[op], ms, nops / ms / 1e9,
           nops / (ms * 1e-3) / 256 / 2.4e9);
  }

  const char* vname[3] = {"A: C++ CIOS", "B: asm FIPS", "C: C++ FIPS"};
  for (int v = 0; v < 3; v++) {
    for (int chains = 1; chains <= 2; chains++) {
      int iters = 200;
      for (int rep = 0; rep < 2; rep++) {
        CHECK(hipEventRecord(e0));
        if (v == 0 && chains == 1) hipLaunchKernelGGL((montk<0, 1>), blocks, threads, 0, 0, out, in, iters);
        if (v == 0 && chains == 2) hipLaunchKernelGGL((montk<0, 2>), blocks, threads, 0, 0, out, in, iters);
        if (v == 1 && chains == 1) hipLaunchKernelGGL((montk<1, 1>), blocks, threads, 0, 0, out, in, iters);
        if (v == 1 && chains == 2) hipLaunchKernelGGL((montk<1, 2>), blocks, threads, 0, 0, out, in, iters);
        if (v == 2 && chains == 1) hipLaunchKernelGGL((montk<2, 1>), blocks, threads, 0, 0, out, in, iters);
        if (v == 2 && chains == 2) hipLaunchKernelGGL((montk<2, 2>), blocks, threads, 0, 0, out, in, iters);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
      }
      double nm = (double)blocks * threads * iters * chains;
      printf("mont %-12s chains=%d %8.3f ms  %8.2f G fp-mul/s\n", vname[v], chains, ms, nm / ms / 1e6);
    }
  }
  CHECK(hipGetLastError());
  return 0;
}
