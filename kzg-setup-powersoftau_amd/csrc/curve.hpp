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
// Fp forms used by the generic jac_madd / jac_eq_affine (instantiated for Fp; the G2 ladders
// have their own carry-free Fp2 overloads below): carry-free limb-wise forms, bounds proven by
// tests/test_field_bounds.py.
template <const auto& K>
KZG_DEV void f_subk(fp& r, const fp& a, const fp& b) { fp_subk_nr<K>(r, a, b); }
template <int S>
KZG_DEV void f_shl(fp& r, const fp& a) { fp_shl_nr<S>(r, a); }
// r = a b - c d in one reduction (d negated as a borrowed multiple of p)
KZG_DEV void f_mul_sub(fp& r, const fp& a, const fp& b, const fp& c, const fp& d) {
  fp nd;
  fp_negk_nr<BlsFp::KB_4_28>(nd, d);
  fp_mul_sum2(r, a, b, c, nd);
}

// ---------------------------------------------------------------- doubling
// Hot path (G1, 126 doublings per point). In: X, Y limbs < 2^30, Z normalized, values <= 110.
// Out: X3 limbs < 2^30 (v <= 4.1), Y3 limbs < 2^29 (v <= 2), Z3 normalized. 3S + 2M + one
// multiply-plus-square: -Y3 = E (X3 - D) + 8 B^2 is ONE Montgomery reduction whose 8 B^2 half is
// computed as a squaring (fp_mul_add8sqr: 105 mads for it where Y3 = E (D - X3) + B (-8B) took a
// full 196-mad product and a normalized -8B), and Y3 = K - (-Y3) is a limb-wise borrowed
// subtraction. The same field element as ark's Y3 (the reference ladder's boolean is unchanged).
KZG_DEV void jac_dbl(jac<fp>& p) {
  fp a, b, d, e, t;
  fp_sqr(a, p.x);              // A = X^2                    N
  fp_sqr(b, p.y);              // B = Y^2                    N
  fp_shl_nr<2>(t, p.x);        // 4X                        < 2^32
  fp_mul(d, t, b);             // D = 4 X B                  N
  fp_mul3_nr(e, a);
  fp_norm(e, e);               // E = 3A                     N (v <= 3.01)
  fp_shl_nr<1>(t, p.y);        // 2Y                        < 2^31
  fp_mul(p.z, t, p.z);         // Z3 = 2 Y Z                 N
  fp_sqr(a, e);                // F = E^2                    N
  fp_shl_nr<1>(t, d);          // 2D                        < 2^29
  fp_subk_nr<BlsFp::KB_8_29>(p.x, a, t);  // X3 = F - 2D           < 2^30 + 2^28
  fp_mul3_nr(t, d);            // 3D                        < 3 * 2^28
  fp_subk_nr<BlsFp::KB_8_30>(t, a, t);    // X3 - D = F - 3D       < 2^30 + 2^28
  fp_mul_add8sqr(d, e, t, b);  // -Y3 = E (X3 - D) + 8 B^2   N
  fp_negk_nr<BlsFp::KB_2_28>(p.y, d);     // Y3                    < 2^29
}

// ---------------------------------------------------------------- G1 fast ladders, W = 2Y
// The endomorphism test's ladders (in_subgroup_fast_g1) carry W = 2Y instead of Y: then
// B' = W^2 = 4B, D = X B' and Z3 = W Z need no 4X / 2Y, and -W3 = 2E (X3 - D) + B'^2 needs no
// 8 B^2 scaling (fp_mul_addsqr<1>) — per doubling 14 v_lshlrev (4X) and 14 v_lshlrev + 14 adds
// (8B, 16B) fewer, 14 adds (2 (X3 - D)) more. Every formula is ark's scaled by the exact factor 2
// on Y, so equal-point and zero tests decide as before; the reference-algorithm ladder
// (in_subgroup_ref) and the generator keep the Y form. Bounds: tests/field_bounds_model.py
// jac_dbl_w / jac_madd_w / jac_tpl_affine_w / ladder_invariant_w.
KZG_DEV void jac_dbl_w(jac<fp>& p) {
  fp a, b, d, e, t;
  fp_sqr(a, p.x);              // A = X^2                    N
  fp_sqr(b, p.y);              // B' = W^2 = 4 Y^2           N
  fp_mul(d, p.x, b);           // D = X B' = 4 X Y^2         N
  fp_mul3_nr(e, a);
  fp_norm(e, e);               // E = 3A                     N
  fp_mul(p.z, p.y, p.z);       // Z3 = W Z = 2 Y Z           N
  fp_sqr(a, e);                // F = E^2                    N
  fp_shl_nr<1>(t, d);          // 2D                        < 2^29
  fp_subk_nr<BlsFp::KB_8_29>(p.x, a, t);  // X3 = F - 2D           < 2^30 + 2^28
  fp_mul3_nr(t, d);            // 3D                        < 3 * 2^28
  fp_subk_nr<BlsFp::KB_8_30>(t, a, t);    // X3 - D = F - 3D       < 2^30 + 2^28
  fp_shl_nr<1>(t, t);          // 2 (X3 - D)
  fp_mul_addsqr<1>(d, e, t, b);  // -W3 = E 2 (X3 - D) + B'^2   N
  fp_negk_nr<BlsFp::KB_2_28>(p.y, d);     // W3                    < 2^29
}

// 3P from the affine base (x, w = 2y), tpl-2007-bl with Z1 = 1 in W form: YYw = w^2 = 4 YY,
// T = YYw^2 = 16 YYYY, E = 3 x YYw - MM (= 12 x YY - MM), U = (M + E)^2 - MM - EE - T,
// X3 = 4 (x EE - YYw U), W3 = 2 Y3 = 8 w (U (T - U) - E EE), Z3 = 2E.
KZG_DEV void jac_tpl_affine_w(jac<fp>& p) {
  fp x, xx, yy, m, mm, s, e, ee, t, u, n;
  fp_norm(x, p.x);                              // x (the second ladder's base Q1.X is lazy)
  fp_sqr(xx, x);                                // XX                     N
  fp_sqr(yy, p.y);                              // YYw = w^2              N
  fp_sqr(t, yy);                                // T = YYw^2 = 16 YYYY    N
  fp_mul3_nr(m, xx);
  fp_norm(m, m);                                // M = 3 XX               N
  fp_sqr(mm, m);                                // MM                     N
  fp_mul(s, x, yy);                             // x YYw                  N
  fp_mul3_nr(s, s);
  fp_subk_nr<BlsFp::KB_8_28>(s, s, mm);
  fp_norm(e, s);                                // E = 3 x YYw - MM       N
  fp_sqr(ee, e);                                // EE                     N
  fp_add_nr(s, m, e);
  fp_sqr(s, s);                                 // S2 = (M + E)^2         N
  fp_subk_nr<BlsFp::KB_8_28>(s, s, mm);
  fp_subk_nr<BlsFp::KB_16_28>(s, s, ee);
  fp_subk_nr<BlsFp::KB_8_28>(s, s, t);
  fp_norm(u, s);                                // U = S2 - MM - EE - T   N
  fp_negk_nr<BlsFp::KB_128_28>(n, u);           // -U                    < 2^29
  fp_mul_sum2(s, x, ee, yy, n);                 // x EE - YYw U           N
  fp_shl_nr<2>(p.x, s);                         // X3                    < 2^30
  fp_subk_nr<BlsFp::KB_128_28>(t, t, u);        // T - U                 < 2^30
  fp_negk_nr<BlsFp::KB_16_28>(n, ee);           // -EE                   < 2^29
  fp_mul_sum2(s, u, t, e, n);                   // U (T - U) - E EE       N
  fp_mul(s, p.y, s);
  fp_shl_nr<3>(s, s);
  fp_norm(p.y, s);                              // W3 = 8 w (...)         N
  fp_shl_nr<1>(s, e);
  fp_norm(p.z, s);                              // Z3 = 2E                N
}

// jac_madd in W form: load(x2, w2) delivers the base with w2 = 2 y2. r = 2 S2 - W1 is ark's
// r = 2 (S2 - Y1), so X3 = r^2 - J - 2V needs no 4 r'^2, and W3 = 2 Y3 = 2r (V - X3) - 2 W1 J.
template <typename Load>
KZG_DEV void jac_madd_w(jac<fp>& p, Load&& load) {
  fp z1z1, h, r, t;
  {
    fp x2, w2;
    load(x2, w2);
    fp_sqr(z1z1, p.z);
    fp_mul(h, x2, z1z1);       // U2
    f_subk<BlsFp::KB_128_31>(h, h, p.x);
    fp_norm(h, h);             // H = U2 - X1
    fp_mul(t, w2, p.z);
    fp_mul(t, t, z1z1);        // 2 S2
    f_subk<BlsFp::KB_64_31>(r, t, p.y);
    fp_norm(r, r);             // r = 2 S2 - W1 = 2 (S2 - Y1)
  }
  const bool z1zero = fp_is_zero(p.z);
  const bool same = !z1zero && fp_is_zero(h) && fp_is_zero(r);
  if (__builtin_expect(z1zero || same, 0)) {
    if (same) {
      jac_dbl_w(p);
    } else {
      load(p.x, p.y);
      f_one(p.z);
    }
    return;
  }
  fp hh, j;
  fp_sqr(hh, h);               // HH
  fp_shl_nr<1>(t, p.z);
  fp_mul(p.z, t, h);           // Z3 = 2 Z1 H
  fp_shl_nr<2>(hh, hh);
  fp_norm(hh, hh);             // I = 4 HH
  fp_mul(j, h, hh);            // J = H I
  fp_mul(hh, p.x, hh);         // V = X1 I
  fp_sqr(t, r);                // r^2
  f_subk<BlsFp::KB_32_28>(t, t, j);
  fp_shl_nr<1>(h, hh);         // 2V
  f_subk<BlsFp::KB_64_29>(t, t, h);
  fp_norm(t, t);               // X3 = r^2 - J - 2V
  f_subk<BlsFp::KB_128_28>(hh, hh, t);
  fp_norm(hh, hh);             // V - X3
  fp_shl_nr<1>(r, r);          // 2r           < 2^29
  fp_shl_nr<1>(h, p.y);        // 2 W1         < 2^30
  f_mul_sub(p.y, r, hh, h, j); // W3 = 2r (V - X3) - 2 W1 J
  p.x = t;
}

// ---------------------------------------------------------------- Fp2, carry-free (G2 ladders)
// The G1 discipline on both components: limb-wise adds and borrowed-constant subtractions, an
// fp_norm only where the next multiply needs normalized limbs — instead of the reduced (< 2p)
// helpers' serial borrow / carry / conditional-2p chains (~125 instructions each, 24 per
// doubling). Every constant is the one tests/field_bounds_model.py (jac_dbl_fp2_lz,
// jac_madd_fp2_lz, jac_eq_affine_fp2_lz) proves for all inputs; ladder states stay normalized
// with values below ~21 p.
// r = a b with b.c1 negated against k (k must dominate b.c1): two Montgomery reductions
template <const auto& K>
KZG_DEV void f2_mul_lz(fp2& r, const fp2& a, const fp2& b) {
  fp nb1, c0;
  fp_negk_nr<K>(nb1, b.c1);
  fp_mul_sum2(c0, a.c0, b.c0, a.c1, nb1);
  fp_mul_sum2(r.c1, a.c0, b.c1, a.c1, b.c0);
  r.c0 = c0;
}
// r = a^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u, the difference against k (dominating a.c1)
template <const auto& K>
KZG_DEV void f2_sqr_lz(fp2& r, const fp2& a) {
  fp s, d, t;
  fp_add_nr(s, a.c0, a.c1);
  fp_subk_nr<K>(d, a.c0, a.c1);
  fp_shl_nr<1>(t, a.c0);
  fp_mul(r.c1, t, a.c1);
  fp_mul(r.c0, s, d);
}
template <const auto& K>
KZG_DEV void f2_subk(fp2& r, const fp2& a, const fp2& b) {
  fp_subk_nr<K>(r.c0, a.c0, b.c0);
  fp_subk_nr<K>(r.c1, a.c1, b.c1);
}
template <int S>
KZG_DEV void f2_shl(fp2& r, const fp2& a) {
  fp_shl_nr<S>(r.c0, a.c0);
  fp_shl_nr<S>(r.c1, a.c1);
}
KZG_DEV void f2_add_nr(fp2& r, const fp2& a, const fp2& b) {
  fp_add_nr(r.c0, a.c0, b.c0);
  fp_add_nr(r.c1, a.c1, b.c1);
}
KZG_DEV void f2_norm(fp2& r, const fp2& a) {
  fp_norm(r.c0, a.c0);
  fp_norm(r.c1, a.c1);
}

// G2 doubling (63 per point): X, Y, Z normalized in and out. 3 squarings + 2 multiplies in Fp2,
// and Y3 = E (D - X3) - 8 B^2 with C = B^2 folded into E's product as in the G1 doubling: per
// component one three-product reduction,
//   Y3.c0 = e0 t0 + e1 (-t1) + (b0 + b1) (-8 (b0 - b1)),   Y3.c1 = e0 t1 + e1 t0 + (2 b0) (-8 b1)
// (t = D - X3; the negated factors normalized so every product stays below 2^58) — 1,568 product
// MACs and 2 reductions where C's squaring plus E (D - X3) took 1,960 and 4.
KZG_DEV void jac_dbl(jac<fp2>& p) {
  fp2 b, a, d, t;
  f2_sqr_lz<BlsFp::KB_32_28>(b, p.y);        // B = Y^2
  f2_shl<1>(t, p.y);
  f2_mul_lz<BlsFp::KB_16_28>(p.z, t, p.z);   // Z3 = 2 Y Z          (Y dead)
  f2_sqr_lz<BlsFp::KB_16_28>(a, p.x);        // A = X^2
  f2_shl<2>(t, p.x);
  f2_mul_lz<BlsFp::KB_2_28>(d, t, b);        // D = 4 X B           (X dead)
  fp_mul3_nr(a.c0, a.c0);
  fp_mul3_nr(a.c1, a.c1);
  f2_norm(a, a);                             // E = 3 A             (A dead)
  f2_sqr_lz<BlsFp::KB_4_28>(t, a);           // F = E^2
  f2_shl<1>(p.x, d);
  f2_subk<BlsFp::KB_4_29>(p.x, t, p.x);
  f2_norm(p.x, p.x);                         // X3 = F - 2D         (F dead)
  f2_subk<BlsFp::KB_8_28>(d, d, p.x);        // t = D - X3
  fp u, s, n, c0;
  fp_negk_nr<BlsFp::KB_16_30>(u, d.c1);      // -t1
  fp_add_nr(s, b.c0, b.c1);                  // b0 + b1             < 2^29
  fp_subk_nr<BlsFp::KB_2_28>(n, b.c0, b.c1);
  fp_norm(n, n);                             // b0 - b1             N
  fp_shl_nr<3>(n, n);
  fp_negk_nr<BlsFp::KB_64_31>(n, n);
  fp_norm(n, n);                             // -8 (b0 - b1)        N
  fp_mul_sum3(c0, a.c0, d.c0, a.c1, u, s, n);
  fp_shl_nr<3>(n, b.c1);
  fp_negk_nr<BlsFp::KB_16_31>(n, n);
  fp_norm(n, n);                             // -8 b1               N
  fp_shl_nr<1>(s, b.c0);                     // 2 b0                < 2^29
  fp_mul_sum3(p.y.c1, a.c0, d.c1, a.c1, d.c0, s, n);
  p.y.c0 = c0;                               // Y3 = E (D - X3) - 8 B^2
}

// G2 mixed addition (ark add_assign_mixed incl. its zero / equal-point branches, as jac_madd):
// X, Y, Z normalized in and out; the base point (x2, y2) normalized, values < 1.01 p.
template <typename Load>
KZG_DEV void jac_madd(jac<fp2>& p, Load&& load) {
  fp2 z1z1, h, r, t;
  {
    fp2 x2, y2;
    load(x2, y2);
    f2_sqr_lz<BlsFp::KB_16_28>(z1z1, p.z);   // (Z values reach ~14 p: the tripling's Z3 = E)
    f2_mul_lz<BlsFp::KB_2_28>(h, x2, z1z1);  // U2
    f2_subk<BlsFp::KB_32_28>(h, h, p.x);
    f2_norm(h, h);                           // H = U2 - X1
    f2_mul_lz<BlsFp::KB_16_28>(t, y2, p.z);
    f2_mul_lz<BlsFp::KB_2_28>(t, t, z1z1);   // S2
    f2_subk<BlsFp::KB_32_28>(r, t, p.y);
    f2_norm(r, r);                           // r' = S2 - Y1   (ark's r = 2 r')
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
  fp2 hh, j;
  f2_sqr_lz<BlsFp::KB_64_28>(hh, h);         // HH
  f2_shl<1>(t, p.z);
  f2_mul_lz<BlsFp::KB_64_28>(p.z, t, h);     // Z3 = 2 Z1 H
  f2_shl<2>(hh, hh);                         // I = 4 HH
  f2_mul_lz<BlsFp::KB_8_30>(j, h, hh);       // J = H I
  f2_mul_lz<BlsFp::KB_8_30>(hh, p.x, hh);    // V = X1 I
  f2_sqr_lz<BlsFp::KB_64_28>(t, r);          // r'^2
  f2_shl<2>(t, t);                           // r^2 = 4 r'^2
  f2_subk<BlsFp::KB_2_28>(t, t, j);
  f2_shl<1>(h, hh);                          // 2V
  f2_subk<BlsFp::KB_4_29>(t, t, h);
  f2_norm(t, t);                             // X3 = r^2 - J - 2V
  f2_subk<BlsFp::KB_32_28>(hh, hh, t);       // V - X3
  f2_shl<1>(r, r);                           // r = 2 r'
  f2_mul_lz<BlsFp::KB_64_30>(hh, r, hh);     // r (V - X3)
  f2_shl<1>(h, p.y);                         // 2 Y1
  f2_mul_lz<BlsFp::KB_2_28>(j, h, j);        // 2 Y1 J
  f2_subk<BlsFp::KB_4_28>(p.y, hh, j);
  f2_norm(p.y, p.y);                         // Y3 = r (V - X3) - 2 Y1 J
  p.x = t;
}

// ---------------------------------------------------------------- G2 fast ladder, W = 2Y
// As the G1 W form (jac_dbl_w above): B' = W^2, D = X B' and Z3 = W Z need no 4X / 2Y, and
// W3 = (2E)(D - X3) - B'^2 needs no -8 scaling of B^2's factors; the mixed addition's
// r = 2 S2 - W1 is ark's r. W limbs reach 2^29 (the base's w = 2y), so the constants borrowed
// against W are KB_*_29. Bounds: tests/field_bounds_model.py jac_dbl_fp2_w / jac_madd_fp2_w /
// jac_tpl_affine_fp2_w / ladder_invariant_fp2_w.
KZG_DEV void jac_dbl_w(jac<fp2>& p) {
  fp2 b, a, d, t;
  f2_sqr_lz<BlsFp::KB_32_29>(b, p.y);        // B' = W^2
  f2_mul_lz<BlsFp::KB_16_28>(p.z, p.y, p.z); // Z3 = W Z           (W dead)
  f2_sqr_lz<BlsFp::KB_16_28>(a, p.x);        // A = X^2
  f2_mul_lz<BlsFp::KB_2_28>(d, p.x, b);      // D = X B'           (X dead)
  fp_mul3_nr(a.c0, a.c0);
  fp_mul3_nr(a.c1, a.c1);
  f2_norm(a, a);                             // E = 3 A            (A dead)
  f2_sqr_lz<BlsFp::KB_4_28>(t, a);           // F = E^2
  f2_shl<1>(p.x, d);
  f2_subk<BlsFp::KB_4_29>(p.x, t, p.x);
  f2_norm(p.x, p.x);                         // X3 = F - 2D        (F dead)
  f2_subk<BlsFp::KB_8_28>(d, d, p.x);        // t = D - X3
  f2_shl<1>(a, a);                           // 2E
  fp u, s, n, c0;
  fp_negk_nr<BlsFp::KB_16_30>(u, d.c1);      // -t1
  fp_add_nr(s, b.c0, b.c1);                  // b0 + b1             < 2^29
  fp_subk_nr<BlsFp::KB_2_28>(n, b.c1, b.c0);
  fp_norm(n, n);                             // b1 - b0             N
  fp_mul_sum3(c0, a.c0, d.c0, a.c1, u, s, n);
  fp_negk_nr<BlsFp::KB_2_28>(n, b.c1);       // -b1                 < 2^29
  fp_shl_nr<1>(s, b.c0);                     // 2 b0                < 2^29
  fp_mul_sum3(p.y.c1, a.c0, d.c1, a.c1, d.c0, s, n);
  p.y.c0 = c0;                               // W3 = 2E (D - X3) - B'^2
}

// The scaled triple (X3/4, W3/8, E) of 3P from (x, w = 2y): YYw = w^2, T = YYw^2, E = 3 x YYw - MM,
// X3/4 = x EE - YYw U, W3/8 = w (U (T - U) - E EE). load delivers (x, w); fetched twice.
template <typename Load>
KZG_DEV void jac_tpl_affine_w(jac<fp2>& p, Load&& load) {
  fp2 yy, m, s, ee, t;
  load(p.x, p.y);
  f2_sqr_lz<BlsFp::KB_2_28>(m, p.x);         // XX
  f2_sqr_lz<BlsFp::KB_4_29>(yy, p.y);        // YYw = w^2
  f2_mul_lz<BlsFp::KB_2_28>(p.z, p.x, yy);   // x YYw               (x, w dead)
  fp_mul3_nr(m.c0, m.c0);
  fp_mul3_nr(m.c1, m.c1);
  f2_norm(m, m);                             // M = 3 XX
  f2_sqr_lz<BlsFp::KB_4_28>(t, m);           // MM
  fp_mul3_nr(p.z.c0, p.z.c0);
  fp_mul3_nr(p.z.c1, p.z.c1);
  f2_subk<BlsFp::KB_2_28>(p.z, p.z, t);
  f2_norm(p.z, p.z);                         // E = 3 x YYw - MM = Z3
  f2_add_nr(s, m, p.z);
  f2_norm(s, s);
  f2_sqr_lz<BlsFp::KB_32_28>(s, s);          // S2 = (M + E)^2
  f2_subk<BlsFp::KB_2_28>(s, s, t);          // - MM
  f2_sqr_lz<BlsFp::KB_16_28>(ee, p.z);       // EE
  f2_subk<BlsFp::KB_4_28>(s, s, ee);         // - EE
  f2_sqr_lz<BlsFp::KB_2_28>(t, yy);          // T = YYw^2 = 16 YYYY
  f2_subk<BlsFp::KB_2_28>(s, s, t);
  f2_norm(s, s);                             // U = S2 - MM - EE - T
  f2_subk<BlsFp::KB_64_28>(t, t, s);
  f2_norm(t, t);                             // T - U
  f2_mul_lz<BlsFp::KB_128_28>(t, s, t);      // U (T - U)
  f2_mul_lz<BlsFp::KB_64_28>(yy, yy, s);     // YYw U
  f2_mul_lz<BlsFp::KB_2_28>(m, p.z, ee);     // E EE
  f2_subk<BlsFp::KB_2_28>(t, t, m);
  f2_norm(t, t);                             // U (T - U) - E EE
  load(p.x, p.y);
  f2_mul_lz<BlsFp::KB_2_28>(p.x, p.x, ee);   // x EE
  f2_subk<BlsFp::KB_2_28>(p.x, p.x, yy);
  f2_norm(p.x, p.x);                         // X3 / 4 = x EE - YYw U
  f2_mul_lz<BlsFp::KB_8_28>(p.y, p.y, t);    // W3 / 8 = w (U (T - U) - E EE)
}

template <typename Load>
KZG_DEV void jac_madd_w(jac<fp2>& p, Load&& load) {
  fp2 z1z1, h, r, t;
  {
    fp2 x2, w2;
    load(x2, w2);
    f2_sqr_lz<BlsFp::KB_16_28>(z1z1, p.z);
    f2_mul_lz<BlsFp::KB_2_28>(h, x2, z1z1);  // U2
    f2_subk<BlsFp::KB_32_28>(h, h, p.x);
    f2_norm(h, h);                           // H = U2 - X1
    f2_mul_lz<BlsFp::KB_16_28>(t, w2, p.z);
    f2_mul_lz<BlsFp::KB_2_28>(t, t, z1z1);   // 2 S2
    f2_subk<BlsFp::KB_32_29>(r, t, p.y);
    f2_norm(r, r);                           // r = 2 S2 - W1 = 2 (S2 - Y1)
  }
  const bool z1zero = f_is_zero(p.z);
  const bool same = !z1zero && f_is_zero(h) && f_is_zero(r);
  if (__builtin_expect(z1zero || same, 0)) {
    if (same) {
      jac_dbl_w(p);
    } else {
      load(p.x, p.y);
      f_one(p.z);
    }
    return;
  }
  fp2 hh, j;
  f2_sqr_lz<BlsFp::KB_64_28>(hh, h);         // HH
  f2_shl<1>(t, p.z);
  f2_mul_lz<BlsFp::KB_64_28>(p.z, t, h);     // Z3 = 2 Z1 H
  f2_shl<2>(hh, hh);                         // I = 4 HH
  f2_mul_lz<BlsFp::KB_8_30>(j, h, hh);       // J = H I
  f2_mul_lz<BlsFp::KB_8_30>(hh, p.x, hh);    // V = X1 I
  f2_sqr_lz<BlsFp::KB_64_28>(t, r);          // r^2
  f2_subk<BlsFp::KB_2_28>(t, t, j);
  f2_shl<1>(h, hh);                          // 2V
  f2_subk<BlsFp::KB_4_29>(t, t, h);
  f2_norm(t, t);                             // X3 = r^2 - J - 2V
  f2_subk<BlsFp::KB_32_28>(hh, hh, t);       // V - X3
  f2_shl<1>(r, r);                           // 2r
  f2_mul_lz<BlsFp::KB_64_30>(hh, r, hh);     // 2r (V - X3)
  f2_shl<1>(h, p.y);                         // 2 W1
  f2_mul_lz<BlsFp::KB_2_28>(j, h, j);        // 2 W1 J
  f2_subk<BlsFp::KB_4_28>(p.y, hh, j);
  f2_norm(p.y, p.y);                         // W3 = 2r (V - X3) - 2 W1 J
  p.x = t;
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
    f_subk<BlsFp::KB_128_31>(h, h, p.x);
    f_norm(h, h);              // H = U2 - X1
    f_mul(t, y2, p.z);
    f_mul(t, t, z1z1);         // S2
    f_subk<BlsFp::KB_64_31>(r, t, p.y);
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
  f_shl<1>(t, p.z);            // 2 Z1 (Z is a product: normalized, so 2 Z1 < 2^29 needs no carry)
  f_mul(p.z, t, h);            // Z3 = 2 Z1 H  (= (Z1 + H)^2 - Z1Z1 - HH)
  f_shl<2>(hh, hh);
  f_norm(hh, hh);              // I = 4 HH
  f_mul(j, h, hh);             // J = H I
  f_mul(hh, p.x, hh);          // V = X1 I
  f_sqr(t, r);                 // r'^2
  f_shl<2>(t, t);              // r^2 = 4 r'^2
  f_subk<BlsFp::KB_32_28>(t, t, j);
  f_shl<1>(h, hh);             // 2V
  f_subk<BlsFp::KB_64_29>(t, t, h);
  f_norm(t, t);                // X3 = r^2 - J - 2V
  f_subk<BlsFp::KB_128_28>(hh, hh, t);
  f_norm(hh, hh);              // V - X3
  f_shl<1>(r, r);              // r = 2 r'     < 2^29
  f_shl<1>(h, p.y);            // 2 Y1         < 2^30
  f_mul_sub(p.y, r, hh, h, j); // Y3 = r (V - X3) - 2 Y1 J
  p.x = t;
}

// [|u|] B for the affine finite base B delivered by load(x, y): |u| starts with the bits 11, so
// the first doubling and mixed addition are one tripling from the affine base (jac_tpl_affine_w);
// then 62 doublings (bits 61..0), 4 mixed additions.
template <typename F, typename Load>
KZG_DEV void mul_abs_u_affine(jac<F>& acc, Load&& load) {
  static_assert(((BLS_ABS_U >> (BLS_ABS_U_BITS - 2)) & 3) == 3, "|u| starts with the bits 11");
  if constexpr (__is_same(F, fp)) {  // W = 2Y form: load delivers (x, 2y)
    load(acc.x, acc.y);
    jac_tpl_affine_w(acc);  // [3] B
#pragma unroll 1
    for (int b = BLS_ABS_U_BITS - 3; b >= 0; b--) {
      jac_dbl_w(acc);
      if ((BLS_ABS_U >> b) & 1) jac_madd_w(acc, load);
    }
  } else {  // W = 2Y form as well: load delivers (x, y), doubled here
    auto loadw = [&](fp2& x, fp2& w) {
      load(x, w);
      f2_shl<1>(w, w);
    };
    jac_tpl_affine_w(acc, loadw);
#pragma unroll 1
    for (int b = BLS_ABS_U_BITS - 3; b >= 0; b--) {
      jac_dbl_w(acc);
      if ((BLS_ABS_U >> b) & 1) jac_madd_w(acc, loadw);
    }
  }
}
// Jacobian (X, Y, Z) == affine (x, y)?  (X == x Z^2, Y == y Z^3, Z != 0). X, Y limbs < 2^30.
template <typename F>
KZG_DEV bool jac_eq_affine(const jac<F>& p, const F& x, const F& y) {
  F z2, t;
  f_sqr(z2, p.z);
  f_mul(t, x, z2);
  f_subk<BlsFp::KB_128_31>(t, t, p.x);
  bool ok = f_is_zero(t);
  f_mul(z2, z2, p.z);
  f_mul(t, y, z2);
  f_subk<BlsFp::KB_128_31>(t, t, p.y);
  ok = ok && f_is_zero(t);
  return ok && !f_is_zero(p.z);
}

// The same test on a carry-free G2 ladder state; x, y reduced or normalized with value < 1.01 p.
KZG_DEV bool jac_eq_affine(const jac<fp2>& p, const fp2& x, const fp2& y) {
  fp2 z2, t;
  f2_sqr_lz<BlsFp::KB_16_28>(z2, p.z);
  f2_mul_lz<BlsFp::KB_2_28>(t, x, z2);
  f2_subk<BlsFp::KB_32_28>(t, t, p.x);
  bool ok = f_is_zero(t);
  f2_mul_lz<BlsFp::KB_16_28>(z2, z2, p.z);
  f2_mul_lz<BlsFp::KB_2_28>(t, y, z2);
  f2_subk<BlsFp::KB_32_29>(t, t, p.y);      // the fast ladder's W limbs reach 2^29
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
// load_row(0, x, y) fetches P, park(q1) stores Q1, load_row(1, x, y) / load_qz(z) fetch it back
// (the kernels park both in LDS). The two ladders are ONE copy of the ladder code, run twice
// with a wave-uniform source row: each copy is ~25 KB of straight-line doubling code, and two
// of them plus the square root's loop overflow the 64 KB instruction cache a CU pair shares.
template <typename LoadRow, typename Park, typename LoadQZ>
KZG_DEV bool in_subgroup_fast_g1(LoadRow&& load_row, Park&& park, LoadQZ&& load_qz) {
  jac<fp> q;
  int src = 0;
  auto load = [&](fp& bx, fp& bw) {  // (x, w = 2y): P's row holds y, Q1's row already holds W
    load_row(src, bx, bw);
    if (src == 0) fp_shl_nr<1>(bw, bw);
  };
#pragma unroll 1
  for (int pass = 0; pass < 2; pass++) {
    src = __builtin_amdgcn_readfirstlane(pass);
    mul_abs_u_affine(q, load);
    if (pass == 0) park(q);
  }
  {
    fp z;
    load_qz(z);
    fp_mul(q.z, q.z, z);
  }
  jac<fp>& q2 = q;
  fp x, y, beta;
  load_row(0, x, y);
  fp_set(beta, FP_BETA);
  fp_mul(x, x, beta);
  fp_neg(y, y);
  fp_shl_nr<1>(y, y);  // the ladders carry W = 2Y: compare with 2 (-y)
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
  f2_shl<1>(y, y);  // the ladder carries W = 2Y: compare with 2 (-psi(P).y)
  return jac_eq_affine(q, x, y);
}

}  // namespace kzgpot
