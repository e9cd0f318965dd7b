// BLS12-381 base-field arithmetic for gfx950 (CDNA4), one field element per lane.
//
// Representation: 12 x 32-bit limbs, Montgomery form with R = 2^384, LAZILY reduced: every value
// lives in [0, 2p] (p < 2^381, so 4p < R and the Montgomery product of two such values stays
// < 1.5p without a final subtraction). Canonical [0, p) form is produced only where bytes leave
// the kernel or an order/equality test needs it (fp_canon).
//
// The multiply is finely-integrated product scanning (FIPS): each 32x32 product is one
// v_mad_u64_u32 into a 64-bit column accumulator whose carry-out is folded into a third word by
// v_addc_co_u32 — two VALU instructions per product, no separate carry chain. gfx950 has no
// 64x64 multiply, so this is the widest MAC the ISA offers; measured 63.7 G Fp-mul/s chip-wide
// vs 45.3 for a compiler-scheduled CIOS (profiles/r01_intmul_microbench.txt).
//
// The reference does the same arithmetic on the CPU in ark-ff 0.2 (6 x u64 limbs, CIOS over u128)
// and pairing 0.14.2; only the boolean / canonical outputs are observable, and they are identical.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls12_381_consts.hpp"

#define KZG_DEV __device__ __forceinline__

namespace kzgpot {

struct fp {
  uint32_t v[12];
};

KZG_DEV void fp_set(fp& r, const uint32_t (&c)[12]) {
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = c[i];
}
KZG_DEV void fp_zero(fp& r) {
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = 0;
}

// (hi:lo) += x * y with the 64-bit carry-out of the accumulate folded into hi.
KZG_DEV void mac3(uint64_t& lo, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(lo), "=&s"(cc), "+v"(hi)
      : "v"(x), "v"(y));
}
// same, with y a wave-uniform constant kept in an SGPR (modulus limbs)
KZG_DEV void mac3s(uint64_t& lo, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(lo), "=&s"(cc), "+v"(hi)
      : "v"(x), "s"(y));
}

// Three products (a_j b_k pairs interleaved with m_j p_k pairs) in ONE asm statement. hipcc
// cannot see inside inline asm, so it separates consecutive SGPR-writing asm statements by an
// s_nop; packing products cuts those nops 3-6x (+9 % Fp-mul/s at 2 waves/SIMD,
// tools/microbench/mont_variants.hip). The mad -> addc carry hand-off inside one statement needs
// no wait state (verified with a single wave issuing back to back).
#define KZG_MAC_STR(x, y) "v_mad_u64_u32 %0, %1, %" #x ", %" #y ", %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1\n\t"
KZG_DEV void mac3x3(uint64_t& lo, uint32_t& hi, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t x2,
                    uint32_t y2) {
  uint64_t cc;
  asm(KZG_MAC_STR(3, 4) KZG_MAC_STR(5, 6) KZG_MAC_STR(7, 8)
      : "+v"(lo), "=&s"(cc), "+v"(hi)
      : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2));
}
KZG_DEV void mac3x2(uint64_t& lo, uint32_t& hi, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
  uint64_t cc;
  asm(KZG_MAC_STR(3, 4) KZG_MAC_STR(5, 6) : "+v"(lo), "=&s"(cc), "+v"(hi) : "v"(x0), "v"(y0), "v"(x1), "v"(y1));
}

// Accumulate the products x[k] * y[k], k < N, into (hi:lo), N known at compile time.
template <int N>
KZG_DEV void mac_run(uint64_t& lo, uint32_t& hi, const uint32_t (&x)[N], const uint32_t (&y)[N]) {
  int k = 0;
#pragma unroll
  for (; k + 3 <= N; k += 3) mac3x3(lo, hi, x[k], y[k], x[k + 1], y[k + 1], x[k + 2], y[k + 2]);
  if constexpr (N % 3 == 2) mac3x2(lo, hi, x[N - 2], y[N - 2], x[N - 1], y[N - 1]);
  if constexpr (N % 3 == 1) mac3(lo, hi, x[N - 1], y[N - 1]);
}

// Column i of the finely-integrated product scan: all a_j b_{i-j} and m_j p_{i-j} terms except the
// (a_i b_0, m_i p_0) pair of a low column, which the caller handles (m_i is born there).
template <int I>
KZG_DEV void fips_column(uint64_t& lo, uint32_t& hi, const fp& a, const fp& b, const uint32_t (&m)[12]) {
  constexpr int J0 = I < 12 ? 0 : I - 11;
  constexpr int J1 = I < 12 ? I - 1 : 11;
  constexpr int N = 2 * (J1 - J0 + 1);
  if constexpr (N > 0) {
    uint32_t x[N], y[N];
#pragma unroll
    for (int j = J0; j <= J1; j++) {
      x[2 * (j - J0)] = a.v[j];
      y[2 * (j - J0)] = b.v[I - j];
      x[2 * (j - J0) + 1] = m[j];
      y[2 * (j - J0) + 1] = FP_P[I - j];
    }
    mac_run<N>(lo, hi, x, y);
  }
}

template <int I>
KZG_DEV void fips_step(uint64_t& lo, uint32_t& hi, const fp& a, const fp& b, uint32_t (&m)[12], uint32_t (&out)[12]) {
  fips_column<I>(lo, hi, a, b, m);
  if constexpr (I < 12) {
    mac3(lo, hi, a.v[I], b.v[0]);
    m[I] = (uint32_t)lo * FP_PINV;
    mac3s(lo, hi, m[I], FP_P[0]);
  } else {
    out[I - 12] = (uint32_t)lo;
  }
  lo = (lo >> 32) | ((uint64_t)hi << 32);
  hi = 0;
  if constexpr (I < 23) fips_step<I + 1>(lo, hi, a, b, m, out);
}

// r = a * b * R^-1 mod p  (inputs in [0, 2p], output in [0, 1.5p))
KZG_DEV void fp_mul(fp& r, const fp& a, const fp& b) {
  uint32_t m[12];
  uint32_t out[12];
  uint64_t lo = 0;
  uint32_t hi = 0;
  fips_step<0>(lo, hi, a, b, m, out);
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = out[i];
}
KZG_DEV void fp_sqr(fp& r, const fp& a) { fp_mul(r, a, a); }

// r = a + b, reduced into [0, 2p]
KZG_DEV void fp_add(fp& r, const fp& a, const fp& b) {
  uint32_t s[12], t[12];
  uint32_t c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
#pragma unroll
  for (int i = 0; i < 12; i++) t[i] = __builtin_subc(s[i], FP_2P[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = br ? s[i] : t[i];
}
// r = a - b, lifted into [0, 2p] by adding 2p on borrow
KZG_DEV void fp_sub(fp& r, const fp& a, const fp& b) {
  uint32_t d[12];
  uint32_t br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  const uint32_t mask = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = __builtin_addc(d[i], FP_2P[i] & mask, c, &c);
}
KZG_DEV void fp_dbl(fp& r, const fp& a) { fp_add(r, a, a); }
KZG_DEV void fp_neg(fp& r, const fp& a) {
  fp z;
  fp_zero(z);
  fp_sub(r, z, a);
}

// [0, 2p] -> [0, p)
KZG_DEV void fp_canon(fp& r, const fp& a) {
  uint32_t x[12], t[12];
#pragma unroll
  for (int i = 0; i < 12; i++) x[i] = a.v[i];
#pragma unroll
  for (int round = 0; round < 2; round++) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) t[i] = __builtin_subc(x[i], FP_P[i], br, &br);
#pragma unroll
    for (int i = 0; i < 12; i++) x[i] = br ? x[i] : t[i];
  }
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = x[i];
}
KZG_DEV bool fp_is_zero_canon(const fp& c) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) o |= c.v[i];
  return o == 0;
}
KZG_DEV bool fp_is_zero(const fp& a) {
  fp c;
  fp_canon(c, a);
  return fp_is_zero_canon(c);
}
KZG_DEV bool fp_eq(const fp& a, const fp& b) {
  fp d;
  fp_sub(d, a, b);
  return fp_is_zero(d);
}
// canonical a < canonical b (both already canonical)
KZG_DEV bool fp_lt_canon(const fp& a, const fp& b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)__builtin_subc(a.v[i], b.v[i], br, &br);
  return br != 0;
}
// canonical value (< 2^384) compared with p: true if v >= p
KZG_DEV bool limbs_geq_p(const uint32_t (&v)[12]) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)__builtin_subc(v[i], FP_P[i], br, &br);
  return br == 0;
}
KZG_DEV void fp_select(fp& r, bool c, const fp& a, const fp& b) {  // r = c ? a : b
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = c ? a.v[i] : b.v[i];
}
KZG_DEV void fp_to_mont(fp& r, const fp& canon) {
  fp r2;
  fp_set(r2, FP_R2);
  fp_mul(r, canon, r2);
}
KZG_DEV void fp_from_mont(fp& canon, const fp& a) {
  fp one;
  fp_zero(one);
  one.v[0] = 1;
  fp_mul(canon, a, one);
  fp_canon(canon, canon);
}

// r = a^((p-3)/4): fixed sliding-window schedule (tools/gen_constants.py), identical for every
// lane, so the whole wave follows one instruction stream. Loops stay rolled so one square and
// one multiply body serve all 453 operations (I-cache).
KZG_DEV void fp_pow_pm3d4(fp& r, const fp& a) {
  fp tab[SQRT_TABLE];
  fp a2;
  tab[0] = a;
  fp_sqr(a2, a);
#pragma unroll
  for (int k = 1; k < SQRT_TABLE; k++) fp_mul(tab[k], tab[k - 1], a2);
  fp acc = tab[SQRT_STEP_IDX[0]];
#pragma unroll 1
  for (int s = 1; s < SQRT_STEPS; s++) {
    const int nsq = __builtin_amdgcn_readfirstlane(SQRT_STEP_SQ[s]);
    const int idx = __builtin_amdgcn_readfirstlane(SQRT_STEP_IDX[s]);
#pragma unroll 1
    for (int k = 0; k < nsq; k++) fp_sqr(acc, acc);
    if (idx >= 0) {
      fp t = tab[0];
#pragma unroll
      for (int k = 1; k < SQRT_TABLE; k++)
        if (idx == k) t = tab[k];
      fp_mul(acc, acc, t);
    }
  }
  r = acc;
}

// ------------------------------------------------------------------------------- Fp2 = Fp[u]/(u^2+1)
struct fp2 {
  fp c0, c1;
};
KZG_DEV void f_add(fp& r, const fp& a, const fp& b) { fp_add(r, a, b); }
KZG_DEV void f_sub(fp& r, const fp& a, const fp& b) { fp_sub(r, a, b); }
KZG_DEV void f_dbl(fp& r, const fp& a) { fp_add(r, a, a); }
KZG_DEV void f_mul(fp& r, const fp& a, const fp& b) { fp_mul(r, a, b); }
KZG_DEV void f_sqr(fp& r, const fp& a) { fp_mul(r, a, a); }
KZG_DEV bool f_is_zero(const fp& a) { return fp_is_zero(a); }
KZG_DEV void f_one(fp& r) { fp_set(r, FP_ONE); }

KZG_DEV void f_add(fp2& r, const fp2& a, const fp2& b) {
  fp_add(r.c0, a.c0, b.c0);
  fp_add(r.c1, a.c1, b.c1);
}
KZG_DEV void f_sub(fp2& r, const fp2& a, const fp2& b) {
  fp_sub(r.c0, a.c0, b.c0);
  fp_sub(r.c1, a.c1, b.c1);
}
KZG_DEV void f_dbl(fp2& r, const fp2& a) { f_add(r, a, a); }
// Karatsuba: 3 Fp multiplies
KZG_DEV void f_mul(fp2& r, const fp2& a, const fp2& b) {
  fp t0, t1, s0, s1;
  fp_mul(t0, a.c0, b.c0);
  fp_mul(t1, a.c1, b.c1);
  fp_add(s0, a.c0, a.c1);
  fp_add(s1, b.c0, b.c1);
  fp_mul(s0, s0, s1);
  fp_sub(r.c0, t0, t1);
  fp_sub(s0, s0, t0);
  fp_sub(r.c1, s0, t1);
}
// (a0 + a1 u)^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u : 2 Fp multiplies
KZG_DEV void f_sqr(fp2& r, const fp2& a) {
  fp s, d, m;
  fp_add(s, a.c0, a.c1);
  fp_sub(d, a.c0, a.c1);
  fp_mul(m, a.c0, a.c1);
  fp_mul(r.c0, s, d);
  fp_add(r.c1, m, m);
}
KZG_DEV bool f_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
KZG_DEV void f_one(fp2& r) {
  fp_set(r.c0, FP_ONE);
  fp_zero(r.c1);
}

}  // namespace kzgpot
