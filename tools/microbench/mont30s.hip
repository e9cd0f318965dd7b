// Montgomery multiply per-instruction floor: the product's 14 x 28-bit unsigned limbs
// (csrc/fp381.hpp, R = 2^392) against 13 x 30-bit BALANCED signed limbs (R = 2^390, limbs in
// [-2^29, 2^29), v_mad_i64_i32). With signed limbs every product is < 2^58 in magnitude, so the
// a*b and m*p column chains (13 products each) still fit one 64-bit accumulator, and a multiply
// costs 169 + 169 mads instead of 196 + 196. The price is headroom: an operand may not exceed
// ~1.46 x 2^29 per limb, so lazy (un-normalized) sums must be normalized before they are
// multiplied.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mont30s mont30s.hip
// Run:   ./mont30s dump.bin && python3 mont30s_check.py dump.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../kzg-setup-powersoftau_amd/csrc/fp381.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int N30 = 13;
__device__ constexpr int32_t P30[N30] = {-21845,     -402915328, 356515836,  -352321620, -252304353,
                                         55215067,   288093811,  316751073,  -321428361, 517541167,
                                         -375082566, -91332614,  1704210};
constexpr uint32_t PINV30 = 0x3ffcfffdu;  // -p^-1 mod 2^30
constexpr uint32_t M30 = (1u << 30) - 1;

__device__ __forceinline__ int32_t sext30(uint32_t x) { return __builtin_amdgcn_sbfe((int32_t)x, 0, 30); }
// r = a b 2^-390 mod p (|value| < p/2 + |a||b|/R), balanced limbs in and out. The upper
// columns start their a*b partial sum at +2^29, so that limb = (acc & M30) - 2^29 and
// carry = acc >> 30 give the balanced digit and its exact quotient.
__device__ __forceinline__ void mul30(int32_t (&r)[N30], const int32_t (&a)[N30], const int32_t (&b)[N30]) {
  constexpr int N = N30;
  int32_t m[N];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N - 1; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int j1 = i < N ? i - 1 : N - 1;
    int64_t accab = i < N ? 0 : (int64_t)1 << 29, accp = 0;
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      accab += (int64_t)a[j] * b[i - j];
      accp += (int64_t)m[j] * P30[i - j];
    }
    acc += accab;
    if (i < N) {
      acc += (int64_t)a[i] * b[0];
      acc += accp;
      m[i] = sext30((uint32_t)acc * PINV30);
      acc += (int64_t)m[i] * P30[0];
    } else {
      acc += accp;
      r[i - N] = (int32_t)((uint32_t)acc & M30) - (1 << 29);
    }
    acc >>= 30;
  }
  r[N - 1] = (int32_t)acc;
}

__device__ __forceinline__ void sqr30(int32_t (&r)[N30], const int32_t (&a)[N30]) {
  constexpr int N = N30;
  int32_t d[N], m[N];
#pragma unroll
  for (int j = 0; j < N; j++) d[j] = a[j] + a[j];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N - 1; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int k1 = i < N ? i - 1 : N - 1;
    int64_t accab = i < N ? 0 : (int64_t)1 << 29, accp = 0;
#pragma unroll
    for (int j = j0; 2 * j < i; j++) accab += (int64_t)a[j] * d[i - j];
    if ((i & 1) == 0) accab += (int64_t)a[i / 2] * a[i / 2];
    acc += accab;
#pragma unroll
    for (int k = j0; k <= k1; k++) accp += (int64_t)m[k] * P30[i - k];
    acc += accp;
    if (i < N) {
      m[i] = sext30((uint32_t)acc * PINV30);
      acc += (int64_t)m[i] * P30[0];
    } else {
      r[i - N] = (int32_t)((uint32_t)acc & M30) - (1 << 29);
    }
    acc >>= 30;
  }
  r[N - 1] = (int32_t)acc;
}

// a b + c as an opaque v_mad_i64_i32 (carry-out to a scratch SGPR pair): a chain of these is not
// re-associated, so each upper column merges its a*b products onto the carry with one add fewer
__device__ __forceinline__ int64_t mad_v(int32_t a, int32_t b, int64_t c) {
  int64_t r;
  uint64_t dummy;
  asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(dummy) : "v"(a), "v"(b), "v"(c));
  return r;
}
// variants with the upper columns chained on the carry (V = 4: mul30c, 5: sqr30c)
__device__ __forceinline__ void mul30c(int32_t (&r)[N30], const int32_t (&a)[N30], const int32_t (&b)[N30]) {
  constexpr int N = N30;
  int32_t m[N];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N - 1; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int j1 = i < N ? i - 1 : N - 1;
    int64_t accp = 0;
    if (i >= N) acc += (int64_t)1 << 29;
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      acc = i >= N ? mad_v(a[j], b[i - j], acc) : acc + (int64_t)a[j] * b[i - j];
      accp += (int64_t)m[j] * P30[i - j];
    }
    if (i < N) {
      acc += (int64_t)a[i] * b[0];
      acc += accp;
      m[i] = sext30((uint32_t)acc * PINV30);
      acc += (int64_t)m[i] * P30[0];
    } else {
      acc += accp;
      r[i - N] = (int32_t)((uint32_t)acc & M30) - (1 << 29);
    }
    acc >>= 30;
  }
  r[N - 1] = (int32_t)acc;
}
__device__ __forceinline__ void sqr30c(int32_t (&r)[N30], const int32_t (&a)[N30]) {
  constexpr int N = N30;
  int32_t d[N], m[N];
#pragma unroll
  for (int j = 0; j < N; j++) d[j] = a[j] + a[j];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N - 1; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int k1 = i < N ? i - 1 : N - 1;
    int64_t accp = 0;
    if (i >= N) acc += (int64_t)1 << 29;
#pragma unroll
    for (int j = j0; 2 * j < i; j++) acc = i >= N ? mad_v(a[j], d[i - j], acc) : acc + (int64_t)a[j] * d[i - j];
    if ((i & 1) == 0) acc = i >= N ? mad_v(a[i / 2], a[i / 2], acc) : acc + (int64_t)a[i / 2] * a[i / 2];
#pragma unroll
    for (int k = j0; k <= k1; k++) accp += (int64_t)m[k] * P30[i - k];
    acc += accp;
    if (i < N) {
      m[i] = sext30((uint32_t)acc * PINV30);
      acc += (int64_t)m[i] * P30[0];
    } else {
      r[i - N] = (int32_t)((uint32_t)acc & M30) - (1 << 29);
    }
    acc >>= 30;
  }
  r[N - 1] = (int32_t)acc;
}

using kzgpot::fp;
constexpr int N28 = kzgpot::NL;

// V: 0 fp_mul (14 x 28), 1 fp_sqr (14 x 28), 2 mul30, 3 sqr30. CH independent chains per lane.
template <int V, int CH>
__global__ void __launch_bounds__(256) kbench(uint32_t* out, const uint32_t* in, int iters, int lds_pad) {
  extern __shared__ uint32_t pad[];
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t s = 0;
  if constexpr (V < 2) {
    fp x[CH], y;
#pragma unroll
    for (int j = 0; j < N28; j++) {
      y.v[j] = in[(tid * 7 + j) & 1023] & (j == 13 ? 0xffffu : kzgpot::LMASK);
#pragma unroll
      for (int c = 0; c < CH; c++)
        x[c].v[j] = in[(tid * 13 + j + 14 * c + 100) & 1023] & (j == 13 ? 0xffffu : kzgpot::LMASK);
    }
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int c = 0; c < CH; c++) {
        if (V == 1) kzgpot::fp_sqr(x[c], x[c]);
        else kzgpot::fp_mul(x[c], x[c], y);
      }
    }
#pragma unroll
    for (int c = 0; c < CH; c++)
#pragma unroll
      for (int j = 0; j < N28; j++) s += x[c].v[j] * (j + 1);
  } else {
    int32_t x[CH][N30], y[N30];
#pragma unroll
    for (int j = 0; j < N30; j++) {
      y[j] = j == 12 ? (int32_t)(in[(tid * 7 + j) & 1023] & 0xfffffu) : sext30(in[(tid * 7 + j) & 1023]);
#pragma unroll
      for (int c = 0; c < CH; c++) {
        const uint32_t w = in[(tid * 13 + j + 13 * c + 100) & 1023];
        x[c][j] = j == 12 ? (int32_t)(w & 0xfffffu) : sext30(w);
      }
    }
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int c = 0; c < CH; c++) {
        if (V == 3) sqr30(x[c], x[c]);
        else if (V == 5) sqr30c(x[c], x[c]);
        else if (V == 4) mul30c(x[c], x[c], y);
        else mul30(x[c], x[c], y);
      }
    }
#pragma unroll
    for (int c = 0; c < CH; c++)
#pragma unroll
      for (int j = 0; j < N30; j++) s += (uint32_t)x[c][j] * (j + 1);
  }
  if (lds_pad < 0) pad[threadIdx.x] = s;
  out[tid] = s;
}

// correctness dump: 256 lanes, a (13 limbs), b, a*b, a^2
__global__ void kcheck30(int32_t* out, const int32_t* in) {
  const int t = threadIdx.x;
  int32_t a[N30], b[N30], r[N30];
  for (int j = 0; j < N30; j++) a[j] = in[t * 26 + j], b[j] = in[t * 26 + 13 + j];
  mul30(r, a, b);
  for (int j = 0; j < N30; j++) out[t * 52 + j] = a[j], out[t * 52 + 13 + j] = b[j], out[t * 52 + 26 + j] = r[j];
  sqr30(r, a);
  for (int j = 0; j < N30; j++) out[t * 52 + 39 + j] = r[j];
  int32_t r2[N30];
  mul30c(r2, a, b);
  sqr30c(r, a);
  for (int j = 0; j < N30; j++) out[256 * 52 + t * 26 + j] = r2[j], out[256 * 52 + t * 26 + 13 + j] = r[j];
}

int main(int argc, char** argv) {
  uint32_t *out, *in;
  const int blocks = 256 * 16, threads = 256;
  CHECK(hipMalloc(&out, (size_t)blocks * threads * 4 * 16));
  CHECK(hipMalloc(&in, 1024 * 4 * 8));
  static uint32_t hin[4096];
  uint64_t s = 0x9e3779b97f4a7c15ULL;
  for (int i = 0; i < 4096; i++) { s = s * 6364136223846793005ULL + 1; hin[i] = (uint32_t)(s >> 32); }
  {  // check inputs: random balanced limbs, plus extreme lanes (every limb at -2^29 or 2^29 - 1)
    static int32_t cin[256 * 26], cout[256 * 52 + 256 * 26];
    for (int t = 0; t < 256; t++)
      for (int j = 0; j < 26; j++) {
        const int k = j % 13;
        int32_t v = (int32_t)(hin[(t * 26 + j) & 4095] << 2) >> 2;
        if (k == 12) v = (int32_t)(hin[(t * 26 + j) & 4095] & 0x1fffff) - (1 << 20);
        if (t < 4) v = k == 12 ? ((t & 1) ? (1 << 20) : -(1 << 20)) : ((t & 1) ? (1 << 29) - 1 : -(1 << 29));
        if (t >= 4 && t < 8) v = k == 12 ? 0 : (((t + j) & 1) ? (1 << 29) - 1 : -(1 << 29));
        cin[t * 26 + j] = v;
      }
    int32_t* dev;
    CHECK(hipMalloc(&dev, sizeof cin));
    CHECK(hipMemcpy(dev, cin, sizeof cin, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(kcheck30, 1, 256, 0, 0, (int32_t*)out, dev);
    CHECK(hipMemcpy(cout, out, sizeof cout, hipMemcpyDeviceToHost));
    if (argc > 1) {
      FILE* f = fopen(argv[1], "wb");
      fwrite(cout, sizeof cout, 1, f);
      fclose(f);
      printf("check dump: %s\n", argv[1]);
    }
  }
  CHECK(hipMemcpy(in, hin, 4096 * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* nm[6] = {"fp_mul 14x28", "fp_sqr 14x28", "mul30 13x30s", "sqr30 13x30s", "mul30 chained", "sqr30 chained"};
  for (int pass = 0; pass < 2; pass++)
    for (int v = 0; v < 6; v++)
      for (int ch = 1; ch <= 2; ch++)
        for (int occ = 2; occ <= 4; occ += 2) {
          const size_t lds = (160 * 1024) / occ - 1024;
          const int iters = 64;
          float ms = 0;
          CHECK(hipEventRecord(e0));
#define L(VV, CC) hipLaunchKernelGGL((kbench<VV, CC>), blocks, threads, lds, 0, out, in, iters / CC, 0)
          if (ch == 1) {
            if (v == 0) L(0, 1);
            if (v == 1) L(1, 1);
            if (v == 2) L(2, 1);
            if (v == 3) L(3, 1);
            if (v == 4) L(4, 1);
            if (v == 5) L(5, 1);
          } else {
            if (v == 0) L(0, 2);
            if (v == 1) L(1, 2);
            if (v == 2) L(2, 2);
            if (v == 3) L(3, 2);
            if (v == 4) L(4, 2);
            if (v == 5) L(5, 2);
          }
#undef L
          CHECK(hipEventRecord(e1));
          CHECK(hipEventSynchronize(e1));
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          if (pass == 1)
            printf("%-14s chains %d waves/SIMD<=%d: %8.3f ms  %7.2f G ops/s\n", nm[v], ch, occ, ms,
                   (double)blocks * threads * iters / ms / 1e6);
        }
  CHECK(hipGetLastError());
  return 0;
}
