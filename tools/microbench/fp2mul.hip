// Fp2 multiply on 14 x 28-bit limbs: the schoolbook-with-shared-reduction form of the G2 ladders
// (curve.hpp f2_mul_lz: 4 products, 2 reductions) against Karatsuba (3 products, 2 reductions):
//   P00 = a0 b0, P11 = a1 b1, S = (a0 + a1)(b0 + b1) column by column,
//   c0 = P00 - P11 + K2, c1 = S - P00 - P11,
// where K2 is a multiple of p written in COLUMN form (28 uint64 column values) that dominates every
// possible P11 column, so the c0 column stays non-negative; S may wrap 2^64, c1 is exact mod 2^64.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/fp2mul fp2mul.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../kzg-setup-powersoftau_amd/csrc/curve.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using namespace kzgpot;
__device__ constexpr uint64_t K2[28] = {0x04984461b1e2a14cull, 0x093088c36699db31ull, 0x0dc8cd25178d5ffcull, 0x12611186c2320badull, 0x16f955e86c6796c3ull, 0x1b919a4a233f5dbeull, 0x2029deabd3f26fcbull, 0x24c2230d79a78be7ull, 0x295a676f2b73f300ull, 0x2df2abd0d8fa468dull, 0x328af0328c88977cull, 0x3723349434aabc08ull, 0x3bbb78f5e14bd6abull, 0x37b63d2064b4b6a8ull, 0x331df8beb5f9dd40ull, 0x2e85b45d07403d80ull, 0x29ed6ffb58869dc0ull, 0x25552b99a9ccfe00ull, 0x20bce737fb135e40ull, 0x1c24a2d64c59be80ull, 0x178c5e749da01ec0ull, 0x12f41a12eee67f00ull, 0x0e5bd5b1402cdf40ull, 0x09c3914f91733f80ull, 0x052b4cede2b99fc0ull, 0x0093088c34000000ull, 0x0001000000000000ull, 0x0000000000000000ull};

KZG_DEV void f2_mul_ks(fp2& r, const fp2& a, const fp2& b) {
  constexpr int N = NL;
  uint32_t sa[N], sb[N], m0[N], m1[N];
#pragma unroll
  for (int j = 0; j < N; j++) sa[j] = a.c0.v[j] + a.c1.v[j], sb[j] = b.c0.v[j] + b.c1.v[j];
  uint64_t acc0 = 0, acc1 = 0;
#pragma unroll
  for (int i = 0; i < 2 * N; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int j1 = i < N ? i : N - 1;
    uint64_t p00 = K2[i], p11 = 0, s = K2[i], ap0 = 0, ap1 = 0;
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      p00 += (uint64_t)a.c0.v[j] * b.c0.v[i - j];
      p11 += (uint64_t)a.c1.v[j] * b.c1.v[i - j];
      s += (uint64_t)sa[j] * sb[i - j];
      if (j < i || i >= N) {
        ap0 += (uint64_t)m0[j] * BlsFp::P[i - j];
        ap1 += (uint64_t)m1[j] * BlsFp::P[i - j];
      }
    }
    acc0 += p00 - p11 + ap0;
    acc1 += s - p00 - p11 + ap1;
    if (i < N) {
      m0[i] = ((uint32_t)acc0 * BlsFp::PINV) & BlsFp::MASK;
      acc0 += (uint64_t)m0[i] * BlsFp::P[0];
      m1[i] = ((uint32_t)acc1 * BlsFp::PINV) & BlsFp::MASK;
      acc1 += (uint64_t)m1[i] * BlsFp::P[0];
    } else {
      r.c0.v[i - N] = (uint32_t)acc0 & BlsFp::MASK;
      r.c1.v[i - N] = (uint32_t)acc1 & BlsFp::MASK;
    }
    acc0 >>= 28;
    acc1 >>= 28;
  }
}

template <int V>
__global__ void __launch_bounds__(256) kbench(uint32_t* out, const uint32_t* in, int iters, int lds_pad) {
  extern __shared__ uint32_t pad[];
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fp2 x, y;
#pragma unroll
  for (int j = 0; j < NL; j++) {
    const uint32_t m = j == 13 ? 0xffffu : LMASK;
    y.c0.v[j] = in[(tid * 7 + j) & 1023] & m;
    y.c1.v[j] = in[(tid * 5 + j + 300) & 1023] & m;
    x.c0.v[j] = in[(tid * 13 + j + 100) & 1023] & m;
    x.c1.v[j] = in[(tid * 11 + j + 600) & 1023] & m;
  }
  for (int it = 0; it < iters; it++) {
    if (V == 0) f2_mul_lz(x, x, y, BlsFp::KB_2_28);
    else f2_mul_ks(x, x, y);
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < NL; j++) s += (x.c0.v[j] ^ x.c1.v[j]) * (j + 1);
  if (lds_pad < 0) pad[threadIdx.x] = s;
  out[tid] = s;
}

// correctness dump: a, b (28 words each: c0 limbs, c1 limbs), then f2_mul_lz and f2_mul_ks results
__global__ void kcheck(uint32_t* out, const uint32_t* in) {
  const int t = threadIdx.x;
  fp2 a, b, r;
  for (int j = 0; j < NL; j++) {
    a.c0.v[j] = in[t * 56 + j], a.c1.v[j] = in[t * 56 + 14 + j];
    b.c0.v[j] = in[t * 56 + 28 + j], b.c1.v[j] = in[t * 56 + 42 + j];
  }
  uint32_t* o = out + t * 112;
  for (int j = 0; j < 56; j++) o[j] = in[t * 56 + j];
  f2_mul_lz(r, a, b, BlsFp::KB_2_28);
  for (int j = 0; j < NL; j++) o[56 + j] = r.c0.v[j], o[70 + j] = r.c1.v[j];
  f2_mul_ks(r, a, b);
  for (int j = 0; j < NL; j++) o[84 + j] = r.c0.v[j], o[98 + j] = r.c1.v[j];
}

int main(int argc, char** argv) {
  uint32_t *out, *in;
  const int blocks = 256 * 16, threads = 256;
  CHECK(hipMalloc(&out, (size_t)blocks * threads * 4 * 16));
  CHECK(hipMalloc(&in, 256 * 56 * 4));
  static uint32_t hin[256 * 56];
  uint64_t s = 0x9e3779b97f4a7c15ULL;
  for (int i = 0; i < 256 * 56; i++) {
    s = s * 6364136223846793005ULL + 1;
    uint32_t v = (uint32_t)(s >> 32);
    const int k = (i % 56) % 14, op = (i % 56) / 14;  // a0 a1 b0 b1
    // a: lazy (limbs up to 2^30, top up to 2^24: values up to ~84 p); b: normalized (top 2^17)
    v = op < 2 ? (k == 13 ? v & 0xffffffu : v & 0x3fffffffu) : (k == 13 ? v & 0x1ffffu : v & LMASK);
    if (i / 56 < 4) v = op < 2 ? (k == 13 ? 0xffffffu : 0x3fffffffu) : (k == 13 ? 0x1ffffu : LMASK);
    hin[i] = v;
  }
  CHECK(hipMemcpy(in, hin, sizeof hin, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(kcheck, 1, 256, 0, 0, out, in);
  static uint32_t hout[256 * 112];
  CHECK(hipMemcpy(hout, out, sizeof hout, hipMemcpyDeviceToHost));
  if (argc > 1) {
    FILE* f = fopen(argv[1], "wb");
    fwrite(hout, sizeof hout, 1, f);
    fclose(f);
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* nm[2] = {"f2_mul_lz (4 products)", "f2_mul_ks (Karatsuba)"};
  for (int pass = 0; pass < 2; pass++)
    for (int v = 0; v < 2; v++)
      for (int occ = 2; occ <= 4; occ += 2) {
        const size_t lds = (160 * 1024) / occ - 1024;
        const int iters = 32;
        float ms = 0;
        CHECK(hipEventRecord(e0));
        if (v == 0) hipLaunchKernelGGL(kbench<0>, blocks, threads, lds, 0, out, in, iters, 0);
        else hipLaunchKernelGGL(kbench<1>, blocks, threads, lds, 0, out, in, iters, 0);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (pass == 1)
          printf("%-24s waves/SIMD<=%d: %8.3f ms  %7.2f G Fp2-mul/s\n", nm[v], occ, ms,
                 (double)blocks * threads * iters / ms / 1e6);
      }
  CHECK(hipGetLastError());
  return 0;
}
