// Short-Weierstrass (a = 0) Jacobian arithmetic over Fp / Fp2 and the two subgroup tests.
//
//  * jac_dbl / jac_madd compute ark-ec 0.2.0 `GroupProjective::double_in_place` (dbl-2009-l,
//    COEFF_A = 0) and `add_assign_mixed` (madd-2007-bl incl. its `self.is_zero()` and equal-point
//    branches). The formulas are re-associated for this machine — a squaring costs the same as a
//    multiply here, so 2((X+B)^2 - A - C) becomes 4XB, (Z+H)^2 - Z^2 - H^2 becomes 2ZH, etc. — which
//    changes no field value: every output is the same element of Fp, so `in_subgroup_ref`
//    (= `mul_bits(r).is_zero()`, the reference's `is_in_correct_subgroup_assuming_on_curve`)
//    returns the reference's boolean for ANY input, on the curve or not.
//  * in_subgroup_fast_g1 / _g2 are endomorphism tests, equal to the reference's boolean for every
//    point ON the curve (tests/test_fast_paths_math.py):
//      G1: phi(P) == [-u^2] P,  phi(x, y) = (BETA x, y)       (126 doublings instead of 254)
//      G2: psi(P) == [u] P,     psi = untwist-Frobenius-twist (63 doublings instead of 254)
//
// Limb / value bounds of every step are annotated (bits = limb bound, v = value bound in units of
// p) and machine-checked by tests/test_field_bounds.py, which mirrors these formulas.
#pragma once
#include "fp381.hpp"

namespace kzgpot {

template <typename F>
struct jac {
  F x, y, z;
};

// ---------------------------------------------------------------- generic helpers
// Fp: carry-free limb-wise forms (bounds proven by tests/test_field_bounds.py).
// Fp2 (cold G2 path): every component stays reduced (< 2p); the borrowed constant is not needed
// and each op reduces its result, so the same formulas hold with no value drift.
KZG_DEV void f_subk(fp& r, const fp& a, const fp& b, const uint32_t (&k)[NL]) { fp_subk_nr(r, a, b, k); }
KZG_DEV void f_subk(fp2& r, const fp2& a, const fp2& b, const uint32_t (&)[NL]) {
  fp_sub_red(r.c0, a.c0, b.c0);
  fp_sub_red(r.c1, a.c1, b.c1);
}
template <int S>
KZG_DEV void f_shl(fp& r, const fp& a) { fp_shl_nr<S>(r, a); }
template <int S>
KZG_DEV void f_shl(fp2& r, const fp2& a) {
  r = a;
#pragma unroll
  for (int k = 0; k < S; k++) {
    fp_add_red(r.c0, r.c0, r.c0);
    fp_add_red(r.c1, r.c1, r.c1);
  }
}
KZG_DEV void f_mul3(fp& r, const fp& a) { fp_mul3_nr(r, a); }
KZG_DEV void f_mul3(fp2& r, const fp2& a) {
  fp2 t;
  fp_add_red(t.c0, a.c0, a.c0);
  fp_add_red(t.c1, a.c1, a.c1);
  fp_add_red(r.c0, t.c0, a.c0);
  fp_add_red(r.c1, t.c1, a.c1);
}
KZG_DEV void f_norm(fp2& r, const fp2& a) { r = a; }
// r = a b - c d. Fp: one reduction for both products (d negated as a borrowed multiple of p);
// Fp2: two multiplies and a reduced subtraction.
KZG_DEV void f_mul_sub(fp& r, const fp& a, const fp& b, const fp& c, const fp& d) {
  fp nd;
  fp_negk_nr(nd, d, BlsFp::KB_4_28);
  fp_mul_sum2(r, a, b, c, nd);
}
KZG_DEV void f_mul_sub(fp2& r, const fp2& a, const fp2& b, const fp2& c, const fp2& d) {
  fp2 t, u;
  f_mul(t, a, b);
  f_mul(u, c, d);
  f_subk(r, t, u, BlsFp::KB_32_28);
}

// ---------------------------------------------------------------- doubling
// Hot path (G1, 126 doublings per point). In: X, Y limbs < 2^30, Z normalized, values <= 110.
// Out: X3 limbs < 2^30 (v <= 4.1), Y3, Z3 normalized. 3S + 2M + one two-product multiply: the
// 8C = 8B^2 term of Y3 = E (D - X3) - 8C is folded into E's product as B (-8B), so both share one
// Montgomery reduction — 105 fewer MACs and one reduction's bookkeeping less than squaring 2B
// separately (3S + 3M + 1S). No carry propagation except -8B's normalization.
KZG_DEV void jac_dbl(jac<fp>& p) {
  fp a, b, d, e, t, n;
  fp_sqr(a, p.x);              // A = X^2                    N
  fp_sqr(b, p.y);              // B = Y^2                    N
  fp_shl_nr<2>(t, p.x);        // 4X                        < 2^32
  fp_mul(d, t, b);             // D = 4 X B                  N
  fp_mul3_nr(e, a);            // E = 3A                    < 3 * 2^28
  fp_shl_nr<1>(t, p.y);        // 2Y                        < 2^31
  fp_mul(p.z, t, p.z);         // Z3 = 2 Y Z                 N
  fp_sqr(a, e);                // F = E^2                    N
  fp_shl_nr<1>(t, d);          // 2D                        < 2^29
  fp_subk_nr(p.x, a, t, BlsFp::KB_8_29);  // X3 = F - 2D           < 2^30 + 2^28
  fp_mul3_nr(t, d);            // 3D
  fp_subk_nr(t, t, a, BlsFp::KB_8_28);    // D - X3 = 3D - F       < 5 * 2^28
  fp_shl_nr<3>(n, b);          // 8B                        < 2^31
  fp_negk_nr(n, n, BlsFp::KB_64_31);      // -8B                   < 2^32
  fp_norm(n, n);               //                            N (v <= 64)
  fp_mul_sum2(p.y, e, t, b, n);  // Y3 = E (D - X3) + B (-8B)  N
}

// Generic (Fp2, cold): all values reduced (< 2p) through the Fp2 helpers above. Ordered so
// that each input dies as early as possible (Y after B and Z3, X after A and D): at most five
// Fp2 temporaries live beside the Karatsuba scratch, which keeps the G2 kernels off AGPR spills.
template <typename F>
KZG_DEV void jac_dbl(jac<F>& p) {
  F b, t, a, d, c8;
  f_sqr(b, p.y);               // B = Y^2
  f_shl<1>(t, p.y);
  f_norm(t, t);
  f_mul(p.z, t, p.z);          // Z3 = 2YZ           (Y dead)
  f_sqr(a, p.x);               // A = X^2
  f_shl<2>(t, p.x);
  f_norm(t, t);
  f_mul(d, t, b);              // D = 4XB            (X dead)
  f_shl<3>(t, b);
  f_norm(t, t);
  f_mul(c8, t, b);             // 8C = 8B^2          (B dead)
  f_mul3(a, a);
  f_norm(a, a);                // E = 3A             (A dead)
  f_sqr(t, a);                 // F = E^2
  f_shl<1>(p.y, d);
  f_subk(p.x, t, p.y, BlsFp::KB_64_29);
  f_norm(p.x, p.x);            // X3 = F - 2D        (F dead)
  f_subk(t, d, p.x, BlsFp::KB_128_28);
  f_norm(t, t);                // D - X3            (D dead)
  f_mul(t, a, t);
  f_subk(p.y, t, c8, BlsFp::KB_32_28);
  f_norm(p.y, p.y);            // Y3 = E (D - X3) - 8C
}

// ---------------------------------------------------------------- mixed addition (cold)
// ark add_assign_mixed: p += (x2, y2) for a finite affine (x2, y2) that `load(x2, y2)` delivers
// (normalized, v <= 2 — or, for the G1 test's second ladder, a ladder state: limbs < 2^30). The
// base point is fetched inside and dies after U2 / S2 (the rare `self.is_zero()` branch fetches it
// again), so it never occupies registers across the formula.
// In: X, Y limbs < 2^30, values <= 40; Z normalized. Out: normalized, values <= 64.
template <typename F, typename Load>
KZG_DEV void jac_madd(jac<F>& p, Load&& load) {
  F z1z1, h, r, t;
  {
    F x2, y2;
    load(x2, y2);
    f_sqr(z1z1, p.z);
    f_mul(h, x2, z1z1);        // U2
    f_subk(h, h, p.x, BlsFp::KB_128_31);
    f_norm(h, h);              // H = U2 - X1
    f_mul(t, y2, p.z);
    f_mul(t, t, z1z1);         // S2
    f_subk(r, t, p.y, BlsFp::KB_64_31);
    f_norm(r, r);              // r' = S2 - Y1   (ark's r = 2 r')
  }
  const bool z1zero = f_is_zero(p.z);
  const bool same = !z1zero && f_is_zero(h) && f_is_zero(r);
  if (__builtin_expect(z1zero || same, 0)) {
    if (same) {
      jac_dbl(p);
    } else {
      load(p.x, p.y);
      f_one(p.z);
    }
    return;
  }
  F hh, j;
  f_sqr(hh, h);                // HH
  f_shl<1>(t, p.z);
  f_norm(t, t);
  f_mul(p.z, t, h);            // Z3 = 2 Z1 H  (= (Z1 + H)^2 - Z1Z1 - HH)
  f_shl<2>(hh, hh);
  f_norm(hh, hh);              // I = 4 HH
  f_mul(j, h, hh);             // J = H I
  f_mul(hh, p.x, hh);          // V = X1 I
  f_sqr(t, r);                 // r'^2
  f_shl<2>(t, t);              // r^2 = 4 r'^2
  f_subk(t, t, j, BlsFp::KB_32_28);
  f_shl<1>(h, hh);             // 2V
  f_subk(t, t, h, BlsFp::KB_64_29);
  f_norm(t, t);                // X3 = r^2 - J - 2V
  f_subk(hh, hh, t, BlsFp::KB_128_28);
  f_norm(hh, hh);              // V - X3
  f_shl<1>(r, r);
  f_norm(r, r);                // r = 2 r'
  f_shl<1>(h, p.y);
  f_norm(h, h);                // 2 Y1
  f_mul_sub(p.y, r, hh, h, j); // Y3 = r (V - X3) - 2 Y1 J
  p.x = t;
}

// [|u|] B for the affine finite base B delivered by load(x, y): 63 doublings, 5 mixed additions.
template <typename F, typename Load>
KZG_DEV void mul_abs_u_affine(jac<F>& acc, Load&& load) {
  load(acc.x, acc.y);
  f_one(acc.z);
#pragma unroll 1
  for (int b = BLS_ABS_U_BITS - 2; b >= 0; b--) {
    jac_dbl(acc);
    if ((BLS_ABS_U >> b) & 1) jac_madd(acc, load);
  }
}
// Jacobian (X, Y, Z) == affine (x, y)?  (X == x Z^2, Y == y Z^3, Z != 0). X, Y limbs < 2^30.
template <typename F>
KZG_DEV bool jac_eq_affine(const jac<F>& p, const F& x, const F& y) {
  F z2, t;
  f_sqr(z2, p.z);
  f_mul(t, x, z2);
  f_subk(t, t, p.x, BlsFp::KB_128_31);
  bool ok = f_is_zero(t);
  f_mul(z2, z2, p.z);
  f_mul(t, y, z2);
  f_subk(t, t, p.y, BlsFp::KB_128_31);
  ok = ok && f_is_zero(t);
  return ok && !f_is_zero(p.z);
}

// ark GroupAffine::mul_bits(BitIteratorBE(r)).is_zero() for a finite affine point.
template <typename F, typename Load>
KZG_DEV bool in_subgroup_ref(Load&& load) {
  jac<F> acc;
  load(acc.x, acc.y);  // the leading 1 bit: zero.double() + P = (x, y, 1)
  f_one(acc.z);
#pragma unroll 1
  for (int b = FR_R_BITS - 2; b >= 0; b--) {
    jac_dbl(acc);
    const uint32_t word = FR_R[b >> 5];
    if ((word >> (b & 31)) & 1) jac_madd(acc, load);
  }
  return f_is_zero(acc.z);
}

// G1: P in G1  <=>  [u^2] P == -phi(P) = (BETA x, -y)   (u^2 = |u|^2)
// The second [|u|] runs on the isomorphic curve E': y^2 = x^3 + Z^6 b, iota(x, y) = (Z^2 x, Z^3 y),
// on which Q1 = [|u|] P = (X : Y : Z) is the AFFINE point (X, Y): a = 0 and neither formula reads
// b, so its 5 additions are mixed additions (8M + 3S) instead of Jacobian ones (12M + 4S), and
// [|u|] iota(Q1) = (X' : Y' : Z') is (X' : Y' : Z' Z) on E. Q1 = O (Z = 0) still ends in O.
// park(q1) stores Q1; load_q(x, y) / load_qz(z) fetch it back (the kernel parks it in LDS).
template <typename Load, typename Park, typename LoadQ, typename LoadQZ>
KZG_DEV bool in_subgroup_fast_g1(Load&& load, Park&& park, LoadQ&& load_q, LoadQZ&& load_qz) {
  jac<fp> q2;
  {
    jac<fp> q1;
    mul_abs_u_affine(q1, load);
    park(q1);
  }
  mul_abs_u_affine(q2, load_q);
  {
    fp z;
    load_qz(z);
    fp_mul(q2.z, q2.z, z);
  }
  fp x, y, beta;
  load(x, y);
  fp_set(beta, FP_BETA);
  fp_mul(x, x, beta);
  fp_neg(y, y);
  return jac_eq_affine(q2, x, y);
}

// psi(x, y) = (conj(x) * (0 + CX1 u), conj(y) * (CY0 + CY1 u))
KZG_DEV void g2_psi(fp2& x, fp2& y) {
  fp cx1, t;
  fp_set(cx1, FP_PSI_CX1);
  // conj(x) = (x0, -x1);  (x0 - x1 u)(c u) = x1 c + x0 c u
  fp_mul(t, x.c1, cx1);
  fp_mul(x.c1, x.c0, cx1);
  x.c0 = t;
  fp2 cy;
  fp_set(cy.c0, FP_PSI_CY0);
  fp_set(cy.c1, FP_PSI_CY1);
  fp zero;
  fp_zero(zero);
  fp_sub_red(y.c1, zero, y.c1);
  f_mul(y, y, cy);
}

// G2: P in G2  <=>  [u] P == psi(P)  <=>  [|u|] P == -psi(P)
template <typename Load>
KZG_DEV bool in_subgroup_fast_g2(Load&& load) {
  jac<fp2> q;
  mul_abs_u_affine(q, load);
  fp2 x, y;
  load(x, y);
  g2_psi(x, y);
  fp2_neg_red(y, y);
  return jac_eq_affine(q, x, y);
}

}  // namespace kzgpot
