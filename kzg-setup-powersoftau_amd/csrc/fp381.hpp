// Prime-field arithmetic for gfx950 (CDNA4), one field element per lane — generic over the field
// (traits struct: BlsFp = BLS12-381 Fq, Bn254Fp = BN254 Fq; tools/gen_constants.py).
//
// Representation: NL limbs of LB bits, each held in a 32-bit VGPR, Montgomery form with
// R = 2^(LB NL) (BLS12-381: 14 x 28 bits, R = 2^392; BN254: 9 x 29 bits, R = 2^261). The spare
// bits per limb are the point of the design (numbers below for BLS12-381's 4):
//
//  * Multiply (fp_mul): finely-integrated product scanning where every column sum fits ONE
//    64-bit accumulator — up to 14 products a_j b_k < 2^60 (operand limbs < 2^30 / 2^32 x 2^28)
//    plus 14 products m_j p_k < 2^56 plus a < 2^36 carry stays below 2^63.9 — so each 32x32
//    product is a single v_mad_u64_u32 and no carry ever passes through an SGPR. The radix-2^32
//    alternative needs mad + addc per product and gfx950 requires wait states around SGPR carry
//    hand-offs; measured 75.5 vs 63.7 G Fp-mul/s (tools/microbench/mont28.hip, mont_variants.hip).
//  * Add / subtract are limb-wise and carry-free: a + b, and a - b as a + KB - b where KB is a
//    multiple of p in a "borrowed" limb form whose every limb dominates b's (bls12_381_consts.hpp).
//    NL VALU instructions, no carry chain, no wait states.
//
// Bounds discipline (checked for every formula by tests/test_field_bounds.py): a value is
// "normalized" (N) when all limbs < 2^28; fp_mul needs limb-bit(a) + limb-bit(b) <= 60 and returns
// N with value < p (1 + v(a) v(b) p / R); loose values (limbs up to 2^30-2^32 after a few
// limb-wise adds) only ever feed fp_mul or a further limb-wise op, never storage-to-bytes or a
// comparison, which go through fp_norm / fp_canon.
//
// The reference does this arithmetic on the CPU with ark-ff 0.2 (6 x u64 limbs, CIOS over u128)
// and pairing 0.14.2; only canonical outputs and booleans are observable, and those are identical.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "bls12_381_consts.hpp"
#include "bn254_consts.hpp"

#define KZG_DEV __device__ __forceinline__

// Field-operation census hook: every Montgomery reduction below names its kind. The product build
// compiles it away; tools/fpops/fp_census.hip defines it to count the reductions per point.
#ifndef KZG_FPOP
#define KZG_FPOP(kind) ((void)0)
#endif

namespace kzgpot {

enum class FpOp { Mul, Sqr, MulSum2, MulSum3, MulAddSqr, Mul30, Sqr30, Count };

constexpr uint32_t LMASK = (1u << 28) - 1;  // BLS12-381 limbs (BlsFp::MASK)

template <class Tr>
struct Fe {
  uint32_t v[Tr::NL];
};
using fp = Fe<BlsFp>;        // BLS12-381 Fq
using fpbn = Fe<Bn254Fp>;    // BN254 Fq
constexpr int NL = BlsFp::NL;

template <class Tr>
KZG_DEV void fp_set(Fe<Tr>& r, const uint32_t (&c)[Tr::NL]) {
#pragma unroll
  for (int i = 0; i < Tr::NL; i++) r.v[i] = c[i];
}
template <class Tr>
KZG_DEV void fp_zero(Fe<Tr>& r) {
#pragma unroll
  for (int i = 0; i < Tr::NL; i++) r.v[i] = 0;
}

// 2x as a VOP2 add: a wave64 v_add_u32 issues in ~2 SIMD cycles, the v_lshlrev_b32 the compiler
// emits for x << 1 in ~4 (profiles/r02_valu_issue_microbench.txt). asm, or the compiler folds it back.
KZG_DEV uint32_t dbl_u32(uint32_t x) {
  uint32_t r;
  asm("v_add_u32_e32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
}

// ------------------------------------------------------------------------------- multiply
// r = a b R^-1 mod p. Requires limb-bit(a) + limb-bit(b) <= 60 (see header). Output normalized.
template <class Tr>
KZG_DEV void fp_mul(Fe<Tr>& r, const Fe<Tr>& a, const Fe<Tr>& b) {
  KZG_FPOP(FpOp::Mul);
  constexpr int N = Tr::NL;
  uint32_t m[N];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int j1 = i < N ? i - 1 : N - 1;
    uint64_t accp = 0;  // m*p terms in their own chain: two independent mad chains per column
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      acc += (uint64_t)a.v[j] * b.v[i - j];
      accp += (uint64_t)m[j] * Tr::P[i - j];
    }
    if (i < N) {
      acc += (uint64_t)a.v[i] * b.v[0];
      acc += accp;
      m[i] = ((uint32_t)acc * Tr::PINV) & Tr::MASK;
      acc += (uint64_t)m[i] * Tr::P[0];
    } else {
      acc += accp;
      r.v[i - N] = (uint32_t)acc & Tr::MASK;
    }
    acc >>= Tr::LB;
  }
}
// r = (a b + c d) R^-1 mod p: both products and the m*p terms share one column scan and one
// reduction (three independent mad chains per column) — the Fp2 multiply's building block.
// Column sums are checked by tests/field_bounds_model.py mul_sum2 for the operand bounds used.
template <class Tr>
KZG_DEV void fp_mul_sum2(Fe<Tr>& r, const Fe<Tr>& a, const Fe<Tr>& b, const Fe<Tr>& c,
                         const Fe<Tr>& d) {
  KZG_FPOP(FpOp::MulSum2);
  constexpr int N = Tr::NL;
  uint32_t m[N];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int j1 = i < N ? i - 1 : N - 1;
    uint64_t acc2 = 0, accp = 0;
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      acc += (uint64_t)a.v[j] * b.v[i - j];
      acc2 += (uint64_t)c.v[j] * d.v[i - j];
      accp += (uint64_t)m[j] * Tr::P[i - j];
    }
    if (i < N) {
      acc += (uint64_t)a.v[i] * b.v[0];
      acc2 += (uint64_t)c.v[i] * d.v[0];
      acc += acc2 + accp;
      m[i] = ((uint32_t)acc * Tr::PINV) & Tr::MASK;
      acc += (uint64_t)m[i] * Tr::P[0];
    } else {
      acc += acc2 + accp;
      r.v[i - N] = (uint32_t)acc & Tr::MASK;
    }
    acc >>= Tr::LB;
  }
}
// r = (a b + c d + e f) R^-1 mod p: three products and the m*p terms in one column scan, one
// reduction — the folded G2 doubling's Y3 components (curve.hpp). Bounds: field_bounds_model mul_sum3.
template <class Tr>
KZG_DEV void fp_mul_sum3(Fe<Tr>& r, const Fe<Tr>& a, const Fe<Tr>& b, const Fe<Tr>& c, const Fe<Tr>& d,
                         const Fe<Tr>& e, const Fe<Tr>& f) {
  KZG_FPOP(FpOp::MulSum3);
  constexpr int N = Tr::NL;
  uint32_t m[N];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int j1 = i < N ? i - 1 : N - 1;
    uint64_t acc2 = 0, acc3 = 0, accp = 0;
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      acc += (uint64_t)a.v[j] * b.v[i - j];
      acc2 += (uint64_t)c.v[j] * d.v[i - j];
      acc3 += (uint64_t)e.v[j] * f.v[i - j];
      accp += (uint64_t)m[j] * Tr::P[i - j];
    }
    if (i < N) {
      acc += (uint64_t)a.v[i] * b.v[0];
      acc2 += (uint64_t)c.v[i] * d.v[0];
      acc3 += (uint64_t)e.v[i] * f.v[0];
      acc += acc2 + acc3 + accp;
      m[i] = ((uint32_t)acc * Tr::PINV) & Tr::MASK;
      acc += (uint64_t)m[i] * Tr::P[0];
    } else {
      acc += acc2 + acc3 + accp;
      r.v[i - N] = (uint32_t)acc & Tr::MASK;
    }
    acc >>= Tr::LB;
  }
}
// r = (a b + 8 c^2) R^-1 mod p in one column scan and one reduction, the c^2 half as a squaring:
// cross products c_j (16 c_k) once, squares c_j (8 c_j) — the G1 doubling's -Y3 = E (X3 - D) + 8 B^2
// (curve.hpp), 105 instead of 196 mads for the 8 B^2 term. c must be normalized (16 c_k < 2^32);
// column sums: tests/field_bounds_model.py mul_add8sqr.
// fp_mul_addsqr<S>: (a b + S c^2) R^-1 for S = 8 (the Y-form doubling) or S = 1 (the W = 2Y form,
// whose B'^2 = 16 B^2 needs no scale: curve.hpp jac_dbl_w; bounds field_bounds_model.mul_addsqr).
template <int S, class Tr>
KZG_DEV void fp_mul_addsqr(Fe<Tr>& r, const Fe<Tr>& a, const Fe<Tr>& b, const Fe<Tr>& c) {
  KZG_FPOP(FpOp::MulAddSqr);
  static_assert(S == 1 || S == 8, "scale");
  constexpr int N = Tr::NL;
  uint32_t c8[N], c16[N], m[N];  // S c and 2 S c
#pragma unroll
  for (int j = 0; j < N; j++) {
    c8[j] = S == 1 ? c.v[j] : c.v[j] << 3;
    c16[j] = dbl_u32(c8[j]);
  }
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int j1 = i < N ? i - 1 : N - 1;
    uint64_t acc2 = 0, accp = 0;
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      acc += (uint64_t)a.v[j] * b.v[i - j];
      accp += (uint64_t)m[j] * Tr::P[i - j];
    }
#pragma unroll
    for (int j = j0; 2 * j < i; j++) acc2 += (uint64_t)c.v[j] * c16[i - j];
    if ((i & 1) == 0 && i / 2 < N) acc2 += (uint64_t)c.v[i / 2] * c8[i / 2];
    if (i < N) {
      acc += (uint64_t)a.v[i] * b.v[0];
      acc += acc2 + accp;
      m[i] = ((uint32_t)acc * Tr::PINV) & Tr::MASK;
      acc += (uint64_t)m[i] * Tr::P[0];
    } else {
      acc += acc2 + accp;
      r.v[i - N] = (uint32_t)acc & Tr::MASK;
    }
    acc >>= Tr::LB;
  }
}
template <class Tr>
KZG_DEV void fp_mul_add8sqr(Fe<Tr>& r, const Fe<Tr>& a, const Fe<Tr>& b, const Fe<Tr>& c) {
  fp_mul_addsqr<8>(r, a, b, c);
}
// r = a^2 R^-1 mod p: each cross product a_j a_k (j < k) once, as a_j (2 a_k), plus the squares —
// NL(NL+1)/2 instead of NL^2 products for the a*a half (the NL^2 m*p products of the reduction
// stay). Every column partial sum is at most fp_mul(a, a)'s, so the same bounds hold; in addition
// a's limbs must be < 2^31 so that 2 a_k fits 32 bits.
template <class Tr>
KZG_DEV void fp_sqr(Fe<Tr>& r, const Fe<Tr>& a) {
  KZG_FPOP(FpOp::Sqr);
  constexpr int N = Tr::NL;
  uint32_t d[N], m[N];
#pragma unroll
  for (int j = 0; j < N; j++) d[j] = dbl_u32(a.v[j]);
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N - 1; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    uint64_t accp = 0;
#pragma unroll
    for (int j = j0; 2 * j < i; j++) acc += (uint64_t)a.v[j] * d[i - j];
    if ((i & 1) == 0) acc += (uint64_t)a.v[i / 2] * a.v[i / 2];
    const int k1 = i < N ? i - 1 : N - 1;
#pragma unroll
    for (int k = j0; k <= k1; k++) accp += (uint64_t)m[k] * Tr::P[i - k];
    acc += accp;
    if (i < N) {
      m[i] = ((uint32_t)acc * Tr::PINV) & Tr::MASK;
      acc += (uint64_t)m[i] * Tr::P[0];
    } else {
      r.v[i - N] = (uint32_t)acc & Tr::MASK;
    }
    acc >>= Tr::LB;
  }
  r.v[N - 1] = (uint32_t)acc & Tr::MASK;  // column 2 NL - 1 holds only the carry
}

// ------------------------------------------------------------------------------- limb-wise ops
template <class Tr>
KZG_DEV void fp_add_nr(Fe<Tr>& r, const Fe<Tr>& a, const Fe<Tr>& b) {
#pragma unroll
  for (int i = 0; i < Tr::NL; i++) r.v[i] = a.v[i] + b.v[i];
}
template <int S, class Tr>
KZG_DEV void fp_shl_nr(Fe<Tr>& r, const Fe<Tr>& a) {  // 2^S a, limb-wise
#pragma unroll
  for (int i = 0; i < Tr::NL; i++) r.v[i] = S == 1 ? dbl_u32(a.v[i]) : a.v[i] << S;
}
template <class Tr>
KZG_DEV void fp_mul3_nr(Fe<Tr>& r, const Fe<Tr>& a) {
#pragma unroll
  for (int i = 0; i < Tr::NL; i++) r.v[i] = (a.v[i] << 1) + a.v[i];
}
// K - b with the constant K in the instruction: a VOP2 v_sub_u32 with a literal. Written so because
// the compiler otherwise hoists the borrowed constants into SGPRs, and the codecs' SGPR budget is
// spent: every use then reloads a spilled SGPR with a v_readlane (a VALU instruction plus hazard
// wait states) inside the ladders.
template <uint32_t C>
KZG_DEV uint32_t lit_sub(uint32_t b) {
  uint32_t r;
  asm("v_sub_u32_e32 %0, %1, %2" : "=v"(r) : "n"(C), "v"(b));
  return r;
}
// a + C, the same way. a + K - b is formed as (a + K) - b rather than a + (K - b): K - b would
// depend on b alone, and the scheduler then hoists it (for the G2 mixed addition's H = U2 - X1 and
// r' = S2 - Y1: to the end of the preceding doubling), where the 2 x 14 results occupied VGPRs
// across the whole multiply chain and were spilled to scratch at every ladder step.
template <uint32_t C>
KZG_DEV uint32_t lit_add(uint32_t a) {
  uint32_t r;
  asm("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "n"(C), "v"(a));
  return r;
}
template <const auto& K, class Tr, size_t... I>
KZG_DEV void subk_lit(Fe<Tr>& r, const Fe<Tr>& a, const Fe<Tr>& b, std::index_sequence<I...>) {
  ((r.v[I] = lit_add<K[I]>(a.v[I]) - b.v[I]), ...);
}
template <const auto& K, class Tr, size_t... I>
KZG_DEV void negk_lit(Fe<Tr>& r, const Fe<Tr>& b, std::index_sequence<I...>) {
  ((r.v[I] = lit_sub<K[I]>(b.v[I])), ...);
}
// r = a + K - b with K a borrowed multiple of p dominating b limb by limb
template <const auto& K, class Tr>
KZG_DEV void fp_subk_nr(Fe<Tr>& r, const Fe<Tr>& a, const Fe<Tr>& b) {
  subk_lit<K>(r, a, b, std::make_index_sequence<Tr::NL>{});
}
// r = K - b (the additive inverse of b, as a borrowed multiple K of p minus b, limb by limb)
template <const auto& K, class Tr>
KZG_DEV void fp_negk_nr(Fe<Tr>& r, const Fe<Tr>& b) {
  negk_lit<K>(r, b, std::make_index_sequence<Tr::NL>{});
}
// carry-propagate to 28-bit limbs (value unchanged; top limb keeps the excess)
template <class Tr>
KZG_DEV void fp_norm(Fe<Tr>& r, const Fe<Tr>& a) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < Tr::NL - 1; i++) {
    const uint32_t t = a.v[i] + c;
    r.v[i] = t & Tr::MASK;
    c = t >> Tr::LB;
  }
  r.v[Tr::NL - 1] = a.v[Tr::NL - 1] + c;
}
template <class Tr>
KZG_DEV void fp_select(Fe<Tr>& r, bool c, const Fe<Tr>& a, const Fe<Tr>& b) {  // r = c ? a : b
#pragma unroll
  for (int i = 0; i < Tr::NL; i++) r.v[i] = c ? a.v[i] : b.v[i];
}

// r = a / 2 (mod p) for a normalized a (limbs < 2^LB but the top one, top + p's top + 1 < 2^32):
// a + p if a is odd, then one right shift across the limbs. Normalized out, value (v(a) + 1) / 2.
// Halving the Montgomery representative halves the element, so this replaces a multiply by
// Montgomery 1/2 (~490 VALU instructions) with ~4 NL. Bounds: field_bounds_model.half.
template <class Tr>
KZG_DEV void fp_half(Fe<Tr>& r, const Fe<Tr>& a) {
  const uint32_t odd = 0u - (a.v[0] & 1u);
  Fe<Tr> t;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < Tr::NL - 1; i++) {
    const uint32_t s = a.v[i] + (Tr::P[i] & odd) + c;
    t.v[i] = s & Tr::MASK;
    c = s >> Tr::LB;
  }
  t.v[Tr::NL - 1] = a.v[Tr::NL - 1] + (Tr::P[Tr::NL - 1] & odd) + c;
#pragma unroll
  for (int i = 0; i < Tr::NL - 1; i++) r.v[i] = (t.v[i] >> 1) | ((t.v[i + 1] & 1u) << (Tr::LB - 1));
  r.v[Tr::NL - 1] = t.v[Tr::NL - 1] >> 1;
}

// normalized a - k (k normalized constant): returns borrow (true if a < k); d = a - k if not
template <class Tr>
KZG_DEV bool fp_sub_const_borrow(Fe<Tr>& d, const Fe<Tr>& a, const uint32_t (&k)[Tr::NL]) {
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < Tr::NL; i++) {
    const int32_t t = (int32_t)a.v[i] - (int32_t)k[i] + br;
    d.v[i] = (uint32_t)t & Tr::MASK;
    br = t >> Tr::LB;  // arithmetic: 0 or -1
  }
  return br != 0;
}
// normalized, value < 2 p -> canonical (one conditional subtraction)
template <class Tr>
KZG_DEV void fp_reduce_once(Fe<Tr>& r, const Fe<Tr>& a) {
  Fe<Tr> d;
  const bool b = fp_sub_const_borrow(d, a, Tr::P);
  fp_select(r, b, a, d);
}
// normalized, value < 256 p  ->  canonical (normalized, value in [0, p))
template <class Tr>
KZG_DEV void fp_reduce_canon(Fe<Tr>& r, const Fe<Tr>& a) {
  Fe<Tr> x = a, d;
#define KZG_RED_STEP(K)                          \
  {                                              \
    const bool b = fp_sub_const_borrow(d, x, K); \
    fp_select(x, b, x, d);                       \
  }
  KZG_RED_STEP(Tr::P_X128)
  KZG_RED_STEP(Tr::P_X64)
  KZG_RED_STEP(Tr::P_X32)
  KZG_RED_STEP(Tr::P_X16)
  KZG_RED_STEP(Tr::P_X8)
  KZG_RED_STEP(Tr::P_X4)
  KZG_RED_STEP(Tr::P_X2)
  KZG_RED_STEP(Tr::P_X1)
#undef KZG_RED_STEP
  r = x;
}
// any value with limbs < 2^32 - 16 and value < 256 p -> canonical
template <class Tr>
KZG_DEV void fp_canon(Fe<Tr>& r, const Fe<Tr>& a) {
  Fe<Tr> n;
  fp_norm(n, a);
  fp_reduce_canon(r, n);
}
template <class Tr>
KZG_DEV bool fp_is_zero_canon(const Fe<Tr>& c) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < Tr::NL; i++) o |= c.v[i];
  return o == 0;
}
// a == 0 (mod p) for any a with limbs < 2^32 - 16 and value < 256 p (fp_canon's precondition),
// without reducing: after normalization a is a multiple k p (k < 256) iff it equals k p for
// k = floor((top + 1) 2^(28 (NL-1)) / p) — the only candidate, computed in double precision
// (exact to ~1e-14 against a >= 4.6e-8 margin for every k; tests/test_fast_paths_math.py) — so
// the test is one normalization, NL small MACs and a compare (~130 instructions) instead of the
// 8-step conditional-subtraction chain (~600).
// A filter runs first: a = k p forces a = k p (mod 2^LB), and limb 0 of a's normalization is
// a.v[0] mod 2^LB (no carry comes in), so k can only be (a.v[0] mod 2^LB) p^-1 mod 2^LB — one
// v_mul_lo. A lane whose candidate is >= 256 holds a nonzero value. A nonzero value passes with
// probability 2^-20 (BLS) / 2^-21 (BN254), so the wave almost always skips the full test through
// one wave-uniform branch (the ladders' exceptional-case tests: 24 calls per G1 point).
template <class Tr>
KZG_DEV bool fp_is_zero(const Fe<Tr>& a) {
  constexpr int N = Tr::NL;
  const uint32_t kc = ((a.v[0] & Tr::MASK) * (0u - Tr::PINV)) & Tr::MASK;  // PINV = -p^-1
  const bool maybe = kc < 256u;
  if (__builtin_amdgcn_ballot_w64(maybe) == 0) return false;
  if (!maybe) return false;
  Fe<Tr> n;
  fp_norm(n, a);
  const uint32_t k = (uint32_t)((double)(n.v[N - 1] + 1u) * Tr::INV_RHO);
  uint64_t c = 0;
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < N - 1; i++) {
    c += (uint64_t)k * Tr::P[i];
    diff |= ((uint32_t)c & Tr::MASK) ^ n.v[i];
    c >>= Tr::LB;
  }
  c += (uint64_t)k * Tr::P[N - 1];
  diff |= (uint32_t)c ^ n.v[N - 1];
  return diff == 0;
}
// a == b (mod p) for b dominated by Tr::KB_EQ (BLS: limbs < 2^31 - 8, value < 63 p;
// BN254: normalized, value < 4 p)
template <class Tr>
KZG_DEV bool fp_eq(const Fe<Tr>& a, const Fe<Tr>& b) {
  Fe<Tr> d;
  fp_subk_nr<Tr::KB_EQ>(d, a, b);
  return fp_is_zero(d);
}
// canonical a < canonical b
template <class Tr>
KZG_DEV bool fp_lt_canon(const Fe<Tr>& a, const Fe<Tr>& b) {
  Fe<Tr> d;
  return fp_sub_const_borrow(d, a, b.v);
}
// canonical p - c, with p - 0 mapped to 0
template <class Tr>
KZG_DEV void fp_neg_canon(Fe<Tr>& r, const Fe<Tr>& c) {
  int32_t br = 0;
  const bool z = fp_is_zero_canon(c);
#pragma unroll
  for (int i = 0; i < Tr::NL; i++) {
    const int32_t t = (int32_t)Tr::P[i] - (int32_t)c.v[i] + br;
    r.v[i] = z ? 0u : ((uint32_t)t & Tr::MASK);
    br = t >> Tr::LB;
  }
}

// "safe" ops for the cold paths: results normalized
template <class Tr>
KZG_DEV void fp_add(Fe<Tr>& r, const Fe<Tr>& a, const Fe<Tr>& b) {
  Fe<Tr> t;
  fp_add_nr(t, a, b);
  fp_norm(r, t);
}
// a - b for b with limbs < 2^31 - 8 and value < 63 p (BLS12-381)
KZG_DEV void fp_sub(fp& r, const fp& a, const fp& b) {
  fp t;
  fp_subk_nr<BlsFp::KB_64_31>(t, a, b);
  fp_norm(r, t);
}
KZG_DEV void fp_neg(fp& r, const fp& a) {
  fp z;
  fp_zero(z);
  fp_sub(r, z, a);
}

// ------------------------------------------------------------------------------- bytes <-> limbs
// NW little-endian 32-bit words (the serialized integer) <-> NL x 28-bit limbs
template <class Tr>
KZG_DEV void fp_from_words(Fe<Tr>& r, const uint32_t (&w)[Tr::NW]) {
#pragma unroll
  for (int k = 0; k < Tr::NL; k++) {
    const int bit = Tr::LB * k, i = bit >> 5, off = bit & 31;
    const uint32_t lo = i < Tr::NW ? w[i] >> off : 0u;
    const uint32_t hi = (off > 32 - Tr::LB && i + 1 < Tr::NW) ? (w[i + 1] << (32 - off)) : 0u;
    r.v[k] = (lo | hi) & Tr::MASK;
  }
}
template <class Tr>
KZG_DEV void fp_to_words(uint32_t (&w)[Tr::NW], const Fe<Tr>& c) {  // c normalized, value < 2^(32 NW)
#pragma unroll
  for (int j = 0; j < Tr::NW; j++) {
    const int bit = 32 * j, k = bit / Tr::LB, off = bit % Tr::LB;
    uint32_t v = c.v[k] >> off;
    if (k + 1 < Tr::NL) v |= c.v[k + 1] << (Tr::LB - off);
    if (2 * Tr::LB - off < 32 && k + 2 < Tr::NL) v |= c.v[k + 2] << (2 * Tr::LB - off);
    w[j] = v;
  }
}
// canonical word vector compared with p: true if v >= p
template <class Tr>
KZG_DEV bool words_geq_p_t(const uint32_t (&v)[Tr::NW]) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < Tr::NW; i++) (void)__builtin_subc(v[i], Tr::P_WORDS[i], br, &br);
  return br == 0;
}
KZG_DEV bool words_geq_p(const uint32_t (&v)[BlsFp::NW]) { return words_geq_p_t<BlsFp>(v); }

template <class Tr>
KZG_DEV void fp_to_mont(Fe<Tr>& r, const Fe<Tr>& canon) {
  Fe<Tr> r2;
  fp_set(r2, Tr::R2);
  fp_mul(r, canon, r2);
}
// Montgomery -> canonical (normalized, [0, p)). For normalized a (< R) the Montgomery product
// a * 1 is (a + m p) / R < 1 + p, so one conditional subtraction finishes it.
template <class Tr>
KZG_DEV void fp_from_mont(Fe<Tr>& canon, const Fe<Tr>& a) {
  Fe<Tr> one;
  fp_zero(one);
  one.v[0] = 1;
  fp_mul(canon, a, one);
  fp_reduce_once(canon, canon);
}

// ------------------------------------------------------------------------------- radix-2^30 core
// BLS12-381's square-root exponentiation (382 squarings + 75 multiplies per call: a third of the
// G1 codec's instruction stream, 40 % of the G2 codec's) runs on 13 x 30-bit BALANCED limbs:
// int32 digits in [-2^29, 2^29), R30 = 2^390, each product one v_mad_i64_i32. Signed digits keep
// every product below 2^58 in magnitude, so the a*b and m*p column chains (13 products each) still
// fit one 64-bit accumulator, and a multiply is 169 + 169 mads instead of 196 + 196: 75.8 against
// 67.9 G multiplies/s, 91 against 83.6 G squarings/s (tools/microbench/mont30s.hip,
// profiles/r03_mont30_microbench.txt). The price is headroom — an operand digit may not exceed
// ~2^29.5 — which the ladders' lazy sums need and a pure square-and-multiply chain does not, so only
// the exponentiation uses it. Bounds: tests/test_fp30.py (worst-case columns for the actual digits
// of p, and an exact model of every function below against Python integers).
constexpr int N30 = 13;
struct f30 {
  int32_t v[N30];
};
KZG_DEV int32_t sext30(uint32_t x) { return __builtin_amdgcn_sbfe((int32_t)x, 0, 30); }

// r = a b 2^-390 mod p for balanced a, b (|digit| <= 2^29, |top digit| <= 2^23: the bound
// tests/test_fp30.py proves, TOP_IN = 2^23 + 1, and the exponentiation's callers use); r balanced with
// |value| < p/2 + |a| |b| / R30. The lower columns are made divisible by 2^30 by m_i = balanced
// (col * PINV30); the upper columns start their a*b partial sum at +2^29, so that the digit
// (acc & M30) - 2^29 and the carry acc >> 30 are the balanced remainder and its exact quotient.
KZG_DEV void f30_mul(f30& r, const f30& a, const f30& b) {
  KZG_FPOP(FpOp::Mul30);
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
      accab += (int64_t)a.v[j] * b.v[i - j];
      accp += (int64_t)m[j] * P30[i - j];
    }
    acc += accab;
    if (i < N) {
      acc += (int64_t)a.v[i] * b.v[0];
      acc += accp;
      m[i] = sext30((uint32_t)acc * PINV30);
      acc += (int64_t)m[i] * P30[0];
    } else {
      acc += accp;
      r.v[i - N] = (int32_t)((uint32_t)acc & ((1u << 30) - 1)) - (1 << 29);
    }
    acc >>= 30;
  }
  r.v[N - 1] = (int32_t)acc;
}
// a b + c as one opaque v_mad_i64_i32 (its carry-out goes to a scratch SGPR pair): a chain of these
// cannot be re-associated by the compiler
KZG_DEV int64_t mad_i64_chain(int32_t a, int32_t b, int64_t c) {
  int64_t r;
  uint64_t carry_out;
  asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry_out) : "v"(a), "v"(b), "v"(c));
  return r;
}
// r = a^2 2^-390: cross products once as a_j (2 a_k), the same reduction. The upper columns chain
// their a*d products onto the incoming carry (mad_i64_chain), one 64-bit merge fewer per column than
// the compiler's re-associated sums: 94.5 against 92.6 G squarings/s (profiles/r03o_mont30_chained.txt;
// the same chaining made the multiply 1.3 % slower, so f30_mul keeps the compiler's form).
KZG_DEV void f30_sqr(f30& r, const f30& a) {
  KZG_FPOP(FpOp::Sqr30);
  constexpr int N = N30;
  int32_t d[N], m[N];
#pragma unroll
  for (int j = 0; j < N; j++) d[j] = a.v[j] + a.v[j];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 2 * N - 1; i++) {
    const int j0 = i < N ? 0 : i - (N - 1);
    const int k1 = i < N ? i - 1 : N - 1;
    int64_t accp = 0;
    if (i >= N) acc += (int64_t)1 << 29;
#pragma unroll
    for (int j = j0; 2 * j < i; j++)
      acc = i >= N ? mad_i64_chain(a.v[j], d[i - j], acc) : acc + (int64_t)a.v[j] * d[i - j];
    if ((i & 1) == 0)
      acc = i >= N ? mad_i64_chain(a.v[i / 2], a.v[i / 2], acc) : acc + (int64_t)a.v[i / 2] * a.v[i / 2];
#pragma unroll
    for (int k = j0; k <= k1; k++) accp += (int64_t)m[k] * P30[i - k];
    acc += accp;
    if (i < N) {
      m[i] = sext30((uint32_t)acc * PINV30);
      acc += (int64_t)m[i] * P30[0];
    } else {
      r.v[i - N] = (int32_t)((uint32_t)acc & ((1u << 30) - 1)) - (1 << 29);
    }
    acc >>= 30;
  }
  r.v[N - 1] = (int32_t)acc;
}
// the same integer in balanced 30-bit digits; a: limbs < 2^32 - 16, value < 2^383 (proven in
// tests/test_fp30.py and test_field_bounds._pow_pm3d4: fp2_sqrt's norm input reaches ~2.02 p)
KZG_DEV void f30_from_fp(f30& r, const fp& a) {
  fp n;
  fp_norm(n, a);
  int32_t c = 0;
#pragma unroll
  for (int k = 0; k < N30; k++) {
    const int bit = 30 * k, i = bit / 28, off = bit % 28;  // off is even and <= 24: two limbs suffice
    uint32_t u = (n.v[i] >> off) | (i + 1 < NL ? n.v[i + 1] << (28 - off) : 0u);
    if (k < N30 - 1) {
      const int32_t t = (int32_t)(u & ((1u << 30) - 1)) + c;  // [0, 2^30]
      c = (t + (1 << 29)) >> 30;
      r.v[k] = sext30((uint32_t)t);
    } else {
      r.v[k] = (int32_t)u + c;
    }
  }
}
// canonical 14 x 28 limbs of a balanced value with |value| < p: + p, unsigned 30-bit digits,
// 28-bit limbs, one conditional subtraction
KZG_DEV void fp_from_f30(fp& r, const f30& z) {
  uint32_t u[N30];
  int32_t c = 0;
#pragma unroll
  for (int k = 0; k < N30; k++) {
    const int32_t t = z.v[k] + P30[k] + c;
    if (k < N30 - 1) {
      u[k] = (uint32_t)t & ((1u << 30) - 1);
      c = t >> 30;
    } else {
      u[k] = (uint32_t)t;
    }
  }
#pragma unroll
  for (int j = 0; j < NL; j++) {
    const int bit = 28 * j, i = bit / 30, off = bit % 30;
    uint32_t v = u[i] >> off;
    if (off > 2 && i + 1 < N30) v |= u[i + 1] << (30 - off);
    r.v[j] = j < NL - 1 ? v & LMASK : v;
  }
  fp_reduce_once(r, r);
}

// The exponentiation schedule as one int32 per step, squarings | table index << 8 (index -1: no
// multiply), plus one padding step. The step loop reads it with a scalar load (s_load_dword) one
// step ahead: the int8 arrays it replaces can only be read by per-lane global_load_sbyte (SMEM has
// no byte loads), and each step then waited on a vector-memory round trip (s_waitcnt vmcnt(0))
// before it could start — 67 waits per exponentiation per wave.
template <class Tr>
struct SqrtSchedule {
  int32_t step[Tr::SQRT_STEPS + 1];
  constexpr SqrtSchedule() : step{} {
    for (int s = 0; s < Tr::SQRT_STEPS; s++) step[s] = (Tr::SQRT_STEP_SQ[s] & 0xff) | (Tr::SQRT_STEP_IDX[s] * 256);
    step[Tr::SQRT_STEPS] = 0;
  }
};
template <class Tr>
__constant__ constexpr SqrtSchedule<Tr> kSqrtSchedule{};
KZG_DEV int sched_nsq(int32_t packed) { return __builtin_amdgcn_readfirstlane(packed & 0xff); }
KZG_DEV int sched_idx(int32_t packed) { return __builtin_amdgcn_readfirstlane(packed >> 8); }

// BLS12-381 r = a^((p-3)/4) on the radix-2^30 core: a (R = 2^392 Montgomery) read as an R30
// Montgomery integer is the element 4a, so the chain computes (4a)^e and one multiply by
// POW30_OUT = 2^392 4^-e turns it into a^e in R = 2^392 Montgomery form. Output canonical.
// The register table holds the 8 odd powers BlsFp::SQRT_TABLE_EXP = a, a^3, a^7, a^9, a^11, a^13,
// a^21, a^255, chosen for this exponent (tools/gen_constants.py, tools/sqrt_chain_search.py): the
// windows over them take 66 multiplies where the w = 4 sliding window's a, a^3, .., a^15 took 78,
// and building them takes 9 multiplies + 7 squarings instead of 7 + 1.
constexpr bool bls_sqrt_table_is(const int16_t (&e)[8]) {
  constexpr int16_t want[8] = {1, 3, 7, 9, 11, 13, 21, 255};
  for (int k = 0; k < 8; k++)
    if (e[k] != want[k]) return false;
  return true;
}
KZG_DEV void fp_pow_pm3d4_30(fp& r, const fp& a_in) {
  typedef uint32_t v8u __attribute__((ext_vector_type(8)));
  static_assert(BlsFp::SQRT_TABLE == 8, "table held as one 8-wide register vector per limb");
  static_assert(bls_sqrt_table_is(BlsFp::SQRT_TABLE_EXP), "the chain below builds exactly this table");
  v8u tab[N30];
  auto put = [&](int e, const f30& x) {
#pragma unroll
    for (int k = 0; k < N30; k++) tab[k][e] = (uint32_t)x.v[k];
  };
  f30 a, a2, a4, t, u;
  f30_from_fp(a, a_in);
  put(0, a);              // a
  f30_sqr(a2, a);         // a^2
  f30_mul(t, a, a2);      // a^3
  put(1, t);
  f30_sqr(a4, a2);        // a^4
  f30_mul(t, t, a4);      // a^7
  put(2, t);
  f30_mul(t, t, a2);      // a^9
  put(3, t);
  f30_mul(t, t, a2);      // a^11
  put(4, t);
  f30_mul(t, t, a2);      // a^13
  put(5, t);
  f30_sqr(a4, a4);        // a^8
  f30_mul(u, t, a4);      // a^21
  put(6, u);
  f30_mul(t, t, a2);      // a^15
  u = t;
#pragma unroll 1
  for (int k = 0; k < 4; k++) f30_sqr(u, u);  // a^240
  f30_mul(u, u, t);       // a^255
  put(7, u);
  f30 acc;
#pragma unroll
  for (int k = 0; k < N30; k++) acc.v[k] = (int32_t)tab[k][BlsFp::SQRT_STEP_IDX[0]];
  int32_t step = kSqrtSchedule<BlsFp>.step[1];
#pragma unroll 1
  for (int s = 1; s < BlsFp::SQRT_STEPS; s++) {
    const int nsq = sched_nsq(step), idx = sched_idx(step);
    step = kSqrtSchedule<BlsFp>.step[s + 1];  // in flight during this step's squarings
#pragma unroll 1
    for (int k = 0; k < nsq; k++) f30_sqr(acc, acc);
    if (idx >= 0) {
#pragma unroll
      for (int k = 0; k < N30; k++) t.v[k] = (int32_t)tab[k][idx];
      f30_mul(acc, acc, t);
    }
  }
#pragma unroll
  for (int k = 0; k < N30; k++) t.v[k] = POW30_OUT[k];
  f30_mul(acc, acc, t);
  fp_from_f30(r, acc);
}

// r = a^((p-3)/4): fixed sliding-window schedule (tools/gen_constants.py), identical for every
// lane, so the whole wave follows one instruction stream. Loops stay rolled so one square and
// one multiply body serve all operations (I-cache). Input limbs <= 2^30, output normalized.
// The 8-entry table lives in registers, one 8-wide vector per limb read with a wave-uniform
// index (below). An earlier scratch-memory table (per-lane private memory) was cheaper in
// instructions but its per-CU working set overflowed L2 at full occupancy: 1,479 B/point of HBM
// re-reads, against 71 B/point with the register table (PMC FETCH_SIZE, k_g1_decompress), and
// 2,370 -> 2,343 ms per 2^27-point G1 codec pass.
template <class Tr>
KZG_DEV void fp_pow_pm3d4_window(Fe<Tr>& r, const Fe<Tr>& a) {
  static_assert(Tr::SQRT_TABLE == 8, "table held as one 8-wide register vector per limb");
  static_assert(Tr::SQRT_TABLE_EXP[0] == 1 && Tr::SQRT_TABLE_EXP[7] == 15, "sliding-window table a, a^3, .., a^15");
  typedef uint32_t v8u __attribute__((ext_vector_type(8)));
  // tab[k][e] = limb k of a^(2e+1): a wave-uniform (SGPR) index into a register vector becomes
  // one m0-indexed v_movrels_b32 per limb — 14 moves per lookup, no memory traffic (a scratch
  // table costs ~1.4 KB of HBM re-reads per point once the per-CU working set exceeds L2).
  v8u tab[Tr::NL];
  Fe<Tr> a2, t = a;
  fp_sqr(a2, a);
#pragma unroll
  for (int k = 0; k < Tr::NL; k++) tab[k][0] = a.v[k];
#pragma clang loop unroll(full)
  for (int e = 1; e < Tr::SQRT_TABLE; e++) {
    fp_mul(t, t, a2);
#pragma unroll
    for (int k = 0; k < Tr::NL; k++) tab[k][e] = t.v[k];
  }
  Fe<Tr> acc;
#pragma unroll
  for (int k = 0; k < Tr::NL; k++) acc.v[k] = tab[k][Tr::SQRT_STEP_IDX[0]];
  int32_t step = kSqrtSchedule<Tr>.step[1];
#pragma unroll 1
  for (int s = 1; s < Tr::SQRT_STEPS; s++) {
    const int nsq = sched_nsq(step), idx = sched_idx(step);
    step = kSqrtSchedule<Tr>.step[s + 1];  // in flight during this step's squarings
#pragma unroll 1
    for (int k = 0; k < nsq; k++) fp_sqr(acc, acc);
    if (idx >= 0) {
#pragma unroll
      for (int k = 0; k < Tr::NL; k++) t.v[k] = tab[k][idx];
      fp_mul(acc, acc, t);
    }
  }
  r = acc;
}
// a^((p-3)/4) for either field: BLS12-381 on the radix-2^30 core with its own table, BN254 by
// the sliding window above
template <class Tr>
KZG_DEV void fp_pow_pm3d4(Fe<Tr>& r, const Fe<Tr>& a) {
  if constexpr (__is_same(Tr, BlsFp)) fp_pow_pm3d4_30(r, a);
  else fp_pow_pm3d4_window(r, a);
}

// ------------------------------------------------------------------------------- reduced ops
// For the cold Fp2 (G2) formulas every value is kept "reduced": normalized with value < 2p.
// Inputs of these ops must be reduced; outputs are reduced. a + b is < 4p, one conditional
// subtraction of 2p brings it back. (fp_mul of reduced inputs is < 1.002 p: reduced.)
KZG_DEV void fp_cond_sub_2p(fp& r, const fp& a) {
  fp d;
  const bool b = fp_sub_const_borrow(d, a, BlsFp::P_X2);
  fp_select(r, b, a, d);
}
KZG_DEV void fp_add_red(fp& r, const fp& a, const fp& b) {
  fp t;
  fp_add_nr(t, a, b);
  fp_norm(t, t);
  fp_cond_sub_2p(r, t);
}
// a - b for reduced a, b: signed borrow chain, then + 2p if negative (no borrowed constant: a
// reduced b may sit just below 2p, where no borrowed form of 2p dominates its top limb)
KZG_DEV void fp_sub_red(fp& r, const fp& a, const fp& b) {
  fp d, e;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int32_t t = (int32_t)a.v[i] - (int32_t)b.v[i] + br;
    d.v[i] = (uint32_t)t & LMASK;
    br = t >> 28;
  }
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint32_t t = d.v[i] + BlsFp::P_X2[i] + c;
    e.v[i] = t & LMASK;
    c = t >> 28;
  }
  fp_select(r, br != 0, e, d);
}

// ------------------------------------------------------------------------------- Fp2 = Fp[u]/(u^2+1)
struct fp2 {
  fp c0, c1;
};
// Fp versions of the generic field interface used by curve.hpp
KZG_DEV void f_mul(fp& r, const fp& a, const fp& b) { fp_mul(r, a, b); }
KZG_DEV void f_sqr(fp& r, const fp& a) { fp_sqr(r, a); }
KZG_DEV bool f_is_zero(const fp& a) { return fp_is_zero(a); }
KZG_DEV void f_one(fp& r) { fp_set(r, BlsFp::ONE); }
KZG_DEV void f_norm(fp& r, const fp& a) { fp_norm(r, a); }

// Schoolbook with one reduction per component: c0 = REDC(a0 b0 + a1 (4p - b1)),
// c1 = REDC(a0 b1 + a1 b0). Same 4 x 196 product mads + 2 x 196 reduction mads as Karatsuba's
// 3 full multiplies, but none of Karatsuba's serial borrow / carry / conditional-2p chains
// (two fp_sub_red, one fp_add_red). Reduced in, reduced out (value < 1.01 p).
KZG_DEV void f_mul(fp2& r, const fp2& a, const fp2& b) {
  fp nb1, c0;
  fp_negk_nr<BlsFp::KB_4_28>(nb1, b.c1);  // 4p - b1, limbs < 2^29
  fp_mul_sum2(c0, a.c0, b.c0, a.c1, nb1);
  fp_mul_sum2(r.c1, a.c0, b.c1, a.c1, b.c0);
  r.c0 = c0;
}
// (a0 + a1 u)^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u : 2 Fp multiplies; reduced in, reduced out
KZG_DEV void f_sqr(fp2& r, const fp2& a) {
  fp s, d, t;
  fp_add_nr(s, a.c0, a.c1);
  fp_subk_nr<BlsFp::KB_4_28>(d, a.c0, a.c1);
  fp_shl_nr<1>(t, a.c0);
  fp_mul(r.c1, t, a.c1);
  fp_mul(r.c0, s, d);
}
KZG_DEV bool f_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
KZG_DEV void f_one(fp2& r) {
  fp_set(r.c0, BlsFp::ONE);
  fp_zero(r.c1);
}
KZG_DEV void fp2_neg_red(fp2& r, const fp2& a) {
  fp z;
  fp_zero(z);
  fp_sub_red(r.c0, z, a.c0);
  fp_sub_red(r.c1, z, a.c1);
}

}  // namespace kzgpot
