// Synthetic transcript generator (bench / test utility, NOT the product path; built into its own
// libkzgpot_synth.so). Produces valid, distinct, subgroup G1/G2 points directly in HBM so the
// 2^27-point bench workload never crosses PCIe, plus the ark bytes each point must decode to —
// a full-size round-trip parity check that needs no CPU oracle.
//
// Point i = [k_i] G with k_i a 128-bit scalar from SplitMix64(seed, i) (bit 0 and bit 127 set),
// by a fixed-base comb: table T[w][j] = [j 2^(4w)] G (w < 32, j < 16, built on the GPU), so each
// point costs 31 mixed additions + one inversion (~800 Fp multiplies) instead of a full ladder.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "curve.hpp"

namespace kzgpot {
namespace {

constexpr int kSynthBlock = 256;
constexpr int kWindows = 32;  // 128-bit scalars, 4-bit windows

KZG_DEV uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

KZG_DEV void gen_point(fp& x, fp& y) {
  fp_set(x, G1_GEN_X);
  fp_set(y, G1_GEN_Y);
}
KZG_DEV void gen_point(fp2& x, fp2& y) {
  fp_set(x.c0, G2_GEN_X0);
  fp_set(x.c1, G2_GEN_X1);
  fp_set(y.c0, G2_GEN_Y0);
  fp_set(y.c1, G2_GEN_Y1);
}

// a^(p-2) = (a^((p-3)/4))^4 a
KZG_DEV void f_inv(fp& r, const fp& a) {
  fp t;
  fp_pow_pm3d4(t, a);
  fp_sqr(t, t);
  fp_sqr(t, t);
  fp_mul(r, t, a);
}
KZG_DEV void f_inv(fp2& r, const fp2& a) {  // (a0 - a1 u) / (a0^2 + a1^2); reduced in and out
  fp n, t;
  fp_sqr(n, a.c0);
  fp_sqr(t, a.c1);
  fp_add(n, n, t);
  f_inv(n, n);
  fp_mul(r.c0, a.c0, n);
  fp_mul(t, a.c1, n);
  fp_zero(n);
  fp_sub_red(r.c1, n, t);
}

template <typename F>
KZG_DEV void to_affine(F& x, F& y, const jac<F>& p) {
  F zi, z2;
  f_inv(zi, p.z);
  f_sqr(z2, zi);
  f_mul(x, p.x, z2);
  f_mul(z2, z2, zi);
  f_mul(y, p.y, z2);
}

template <typename F>
KZG_DEV void store_f(uint32_t* dst, const F& a) {
  const uint32_t* s = (const uint32_t*)&a;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(F) / 4); k++) dst[k] = s[k];
}
template <typename F>
KZG_DEV void load_f(F& a, const uint32_t* src) {
  uint32_t* d = (uint32_t*)&a;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(F) / 4); k++) d[k] = src[k];
}

// T[w][j] = [j 2^(4w)] G, affine Montgomery (x ‖ y); j = 0 slots unused
template <typename F>
__global__ void k_synth_table(uint32_t* __restrict__ table) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kWindows * 16) return;
  const int w = t >> 4, j = t & 15;
  if (j == 0) return;
  F gx, gy;
  gen_point(gx, gy);
  jac<F> acc;  // [j] G by double-and-add over j's 4 bits, then 4w doublings
  acc.x = gx;
  acc.y = gy;
  f_one(acc.z);
  const int top = 31 - __builtin_clz(j);
  for (int b = top - 1; b >= 0; b--) {
    jac_dbl(acc);
    if ((j >> b) & 1) jac_madd(acc, [&](F& x, F& y) { x = gx, y = gy; });
  }
  for (int k = 0; k < 4 * w; k++) jac_dbl(acc);
  F x, y;
  to_affine(x, y, acc);
  const int words = sizeof(F) / 4;
  store_f(table + (size_t)t * 2 * words, x);
  store_f(table + (size_t)t * 2 * words + words, y);
}

KZG_DEV void canon_pair(fp& xc, fp& yc, bool& greatest, const fp& x, const fp& y) {
  fp_from_mont(xc, x);
  fp_from_mont(yc, y);
  // greatest: y > p - y (pairing G1Compressed::from_affine)
  fp ny;
  fp_neg_canon(ny, yc);
  greatest = fp_lt_canon(ny, yc);
}

KZG_DEV void store_be(uint32_t* dst, const fp& c) {  // canonical -> 48 big-endian bytes
  uint32_t w[12];
  fp_to_words(w, c);
#pragma unroll
  for (int k = 0; k < 12; k++) dst[k] = __builtin_bswap32(w[11 - k]);
}
KZG_DEV void store_le(uint32_t* dst, const fp& c) {  // canonical -> 48 little-endian bytes
  uint32_t w[12];
  fp_to_words(w, c);
#pragma unroll
  for (int k = 0; k < 12; k++) dst[k] = w[k];
}

template <typename F>
__global__ void __launch_bounds__(kSynthBlock) k_synth(const uint32_t* __restrict__ table, uint64_t seed,
                                                       uint64_t start, uint64_t n, uint32_t* __restrict__ comp,
                                                       uint32_t* __restrict__ ark) {
  const uint64_t i = (uint64_t)blockIdx.x * kSynthBlock + threadIdx.x;
  if (i >= n) return;
  const uint64_t gi = start + i;
  const uint64_t klo = splitmix64(seed ^ (2 * gi)) | 1ull;
  const uint64_t khi = splitmix64(seed ^ (2 * gi + 1)) | (1ull << 63);
  const int words = sizeof(F) / 4;
  jac<F> acc;
  {
    const int d = (int)(klo & 15);
    load_f(acc.x, table + (size_t)d * 2 * words);
    load_f(acc.y, table + (size_t)d * 2 * words + words);
    f_one(acc.z);
  }
#pragma unroll 1
  for (int w = 1; w < kWindows; w++) {
    const int d = (int)(((w < 16 ? klo >> (4 * w) : khi >> (4 * (w - 16)))) & 15);
    if (d) {
      const uint32_t* e = table + (size_t)(w * 16 + d) * 2 * words;
      jac_madd(acc, [&](F& x, F& y) {
        load_f(x, e);
        load_f(y, e + words);
      });
    }
  }
  F x, y;
  to_affine(x, y, acc);
  if constexpr (sizeof(F) == sizeof(fp)) {
    fp xc, yc;
    bool greatest;
    canon_pair(xc, yc, greatest, x, y);
    uint32_t* c = comp + i * 12;
    store_be(c, xc);
    c[0] |= 0x80u | (greatest ? 0x20u : 0u);
    if (ark) {
      uint32_t* a = ark + i * 24;
      store_le(a, xc);
      store_le(a + 12, yc);
    }
  } else {
    const fp2& x2 = *(const fp2*)&x;
    const fp2& y2 = *(const fp2*)&y;
    fp2 xc, yc;
    fp_from_mont(xc.c0, x2.c0);
    fp_from_mont(xc.c1, x2.c1);
    fp_from_mont(yc.c0, y2.c0);
    fp_from_mont(yc.c1, y2.c1);
    // greatest: y > -y lexicographically (c1 first)
    fp n0, n1;
    fp_neg_canon(n0, yc.c0);
    fp_neg_canon(n1, yc.c1);
    bool c1eq = true;
#pragma unroll
    for (int k = 0; k < NL; k++) c1eq = c1eq && (yc.c1.v[k] == n1.v[k]);
    const bool greatest = c1eq ? fp_lt_canon(n0, yc.c0) : fp_lt_canon(n1, yc.c1);
    uint32_t* c = comp + i * 24;
    store_be(c, xc.c1);
    store_be(c + 12, xc.c0);
    c[0] |= 0x80u | (greatest ? 0x20u : 0u);
    if (ark) {
      uint32_t* a = ark + i * 48;
      store_le(a, xc.c0);
      store_le(a + 12, xc.c1);
      store_le(a + 24, yc.c0);
      store_le(a + 36, yc.c1);
    }
  }
}

template <typename F>
int synth(uint64_t seed, uint64_t start, size_t n, void* d_comp, void* d_ark, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const size_t tbytes = (size_t)kWindows * 16 * 2 * sizeof(F);
  uint32_t* table = nullptr;
  if (hipMallocAsync((void**)&table, tbytes, s) != hipSuccess) return -101;
  hipLaunchKernelGGL(k_synth_table<F>, dim3((kWindows * 16 + 63) / 64), dim3(64), 0, s, table);
  if (n)
    hipLaunchKernelGGL(k_synth<F>, dim3((unsigned)((n + kSynthBlock - 1) / kSynthBlock)), dim3(kSynthBlock), 0, s,
                       table, seed, start, (uint64_t)n, (uint32_t*)d_comp, (uint32_t*)d_ark);
  if (hipFreeAsync(table, s) != hipSuccess) return -101;
  return hipGetLastError() == hipSuccess ? 0 : -101;
}

// BN254 G1 (cofactor 1: every curve point is in the group): x_i = 252 random bits, then the
// first x_i + j with x^3 + 3 a square; y or -y by a random bit; the compressed encoding sets
// PositiveY when the chosen y > -y.
__global__ void __launch_bounds__(kSynthBlock) k_synth_bn254(uint64_t seed, uint64_t start, uint64_t n,
                                                             uint32_t* __restrict__ comp, uint32_t* __restrict__ ark) {
  const uint64_t i = (uint64_t)blockIdx.x * kSynthBlock + threadIdx.x;
  if (i >= n) return;
  const uint64_t gi = start + i;
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t r = splitmix64(seed ^ (0x6a09e667f3bcc909ull * (4 * gi + k + 1)));
    w[2 * k] = (uint32_t)r;
    w[2 * k + 1] = (uint32_t)(r >> 32);
  }
  w[7] &= 0x0fffffffu;  // < 2^252 < p
  const bool flip = splitmix64(seed ^ ~gi) & 1;
  fpbn x, y;
  fp_from_words(x, w);
#pragma unroll 1
  for (int attempt = 0; attempt < 64; attempt++) {
    fpbn xm, a, t, three;
    fp_to_mont(xm, x);
    fp_sqr(a, xm);
    fp_mul(a, a, xm);
    fp_set(three, BN_THREE);
    fp_add(a, a, three);
    fp_pow_pm3d4(t, a);
    fp_mul(y, t, a);
    fp_sqr(t, y);
    if (fp_eq(t, a)) break;
    x.v[0] += 1;  // x + 1 (normalize: the carry may run up the limbs)
    fp_norm(x, x);
  }
  fpbn yc, nyc, ncho;
  fp_from_mont(yc, y);
  fp_neg_canon(nyc, yc);
  fp_select(yc, flip, nyc, yc);  // the chosen root
  fp_neg_canon(ncho, yc);
  const bool positive = fp_lt_canon(ncho, yc);
  uint32_t xw[8], yw[8];
  fp_to_words(xw, x);
  fp_to_words(yw, yc);
  uint32_t* c = comp + i * 8;
#pragma unroll
  for (int k = 0; k < 8; k++) c[k] = xw[k];
  if (positive) c[7] |= 0x80000000u;
  if (ark) {
    uint32_t* a = ark + i * 16;
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = xw[k], a[8 + k] = yw[k];
  }
}

// Clock probe for bench.py (measurement only, not the product): each of the launch's blocks records
// its XCD (HW_REG_XCC_ID), the shader-clock counter (s_memtime) and the 100 MHz real-time counter
// (s_memrealtime). Two probes around a timed region give each XCD's average shader clock over it.
__global__ void k_clock_probe(unsigned long long* out) {
  if (threadIdx.x) return;
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const uint64_t t = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 3 + 0] = xcc;
  out[blockIdx.x * 3 + 1] = t;
  out[blockIdx.x * 3 + 2] = r;
}

}  // namespace
}  // namespace kzgpot

extern "C" {
// 64 one-wave blocks (every XCD several times): d_out receives 64 x (xcc id, s_memtime, s_memrealtime).
int kzgpot_synth_clock_probe(void* d_out, void* stream) {
  hipLaunchKernelGGL(kzgpot::k_clock_probe, dim3(64), dim3(64), 0, (hipStream_t)stream, (unsigned long long*)d_out);
  return hipGetLastError() == hipSuccess ? 0 : -101;
}
// Points start .. start+n-1 of stream `seed`: compressed pairing encodings into d_comp (48 / 96 B
// each) and, if d_ark != NULL, the expected ark uncompressed bytes (96 / 192 B each). Async.
int kzgpot_synth_g1_dev(uint64_t seed, uint64_t start, size_t n, void* d_comp, void* d_ark, void* stream) {
  return kzgpot::synth<kzgpot::fp>(seed, start, n, d_comp, d_ark, stream);
}
int kzgpot_synth_g2_dev(uint64_t seed, uint64_t start, size_t n, void* d_comp, void* d_ark, void* stream) {
  return kzgpot::synth<kzgpot::fp2>(seed, start, n, d_comp, d_ark, stream);
}
// BN254 G1: ark compressed (32 B) into d_comp, expected ark uncompressed (64 B) into d_ark.
int kzgpot_synth_bn254_dev(uint64_t seed, uint64_t start, size_t n, void* d_comp, void* d_ark, void* stream) {
  if (n)
    hipLaunchKernelGGL(kzgpot::k_synth_bn254, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       seed, start, (uint64_t)n, (uint32_t*)d_comp, (uint32_t*)d_ark);
  return hipGetLastError() == hipSuccess ? 0 : -101;
}
}
