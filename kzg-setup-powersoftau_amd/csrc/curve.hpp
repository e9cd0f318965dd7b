// Short-Weierstrass (a = 0) Jacobian arithmetic over Fp / Fp2 and the two subgroup tests.
//
//  * jac_dbl / jac_madd restate ark-ec 0.2.0 `GroupProjective::double_in_place` (dbl-2009-l,
//    COEFF_A = 0) and `add_assign_mixed` (madd-2007-bl incl. its `self.is_zero()` and equal-point
//    branches) exactly, so `in_subgroup_ref` (= `mul_bits(r).is_zero()`, the reference's
//    `is_in_correct_subgroup_assuming_on_curve`) returns the reference's boolean for ANY input,
//    on the curve or not (read_g1/read_g2 never check the curve equation).
//  * in_subgroup_fast_g1 / _g2 are endomorphism tests, equal to the reference's boolean for every
//    point ON the curve (DESIGN.md §4 has the argument; tests/ check it on adversarial points):
//      G1: phi(P) == [-u^2] P,  phi(x, y) = (BETA x, y)       (126 doublings instead of 254)
//      G2: psi(P) == [u] P,     psi = untwist-Frobenius-twist (63 doublings instead of 254)
//
// Register pressure decides occupancy here (one point per lane, ~100+ live 32-bit limbs), so
// formulas are ordered to retire temporaries early and the affine base point is re-loaded from
// memory by a `Load` functor at each use instead of being held in registers across the loops.
#pragma once
#include "fp381.hpp"

namespace kzgpot {

template <typename F>
struct jac {
  F x, y, z;
};

// ark double_in_place (a = 0). Z = 0 stays Z = 0 (Z3 = 2 Y Z), matching ark's early return in
// everything that is observable (is_zero() reads Z only; the next add replaces X, Y).
template <typename F>
KZG_DEV void jac_dbl(jac<F>& p) {
  F a, c, d, t;
  f_sqr(a, p.x);      // A = X^2
  f_sqr(t, p.y);      // B = Y^2
  f_sqr(c, t);        // C = B^2
  f_add(t, p.x, t);   // X + B
  f_sqr(t, t);
  f_sub(t, t, a);
  f_sub(t, t, c);
  f_dbl(d, t);        // D = 2((X+B)^2 - A - C)
  f_dbl(t, a);
  f_add(a, t, a);     // E = 3A (in a)
  f_mul(p.z, p.z, p.y);
  f_dbl(p.z, p.z);    // Z3 = 2 Y Z
  f_sqr(t, a);        // F = E^2
  f_sub(t, t, d);
  f_sub(p.x, t, d);   // X3 = F - 2D
  f_sub(t, d, p.x);
  f_mul(t, t, a);     // E (D - X3)
  f_dbl(c, c);
  f_dbl(c, c);
  f_dbl(c, c);
  f_sub(p.y, t, c);   // Y3 = E (D - X3) - 8C
}

// ark add_assign_mixed: p += (x2, y2) for a finite affine (x2, y2).
template <typename F>
KZG_DEV void jac_madd(jac<F>& p, const F& x2, const F& y2) {
  F z1z1, h, r, t;
  f_sqr(z1z1, p.z);
  f_mul(h, x2, z1z1);
  f_sub(h, h, p.x);   // H = U2 - X1
  f_mul(t, y2, p.z);
  f_mul(t, t, z1z1);  // S2
  f_sub(r, t, p.y);
  f_dbl(r, r);        // r = 2 (S2 - Y1)
  const bool z1zero = f_is_zero(p.z);
  const bool same = !z1zero && f_is_zero(h) && f_is_zero(r);
  if (__builtin_expect(z1zero || same, 0)) {
    if (same) {
      jac_dbl(p);
    } else {
      p.x = x2;
      p.y = y2;
      f_one(p.z);
    }
    return;
  }
  F i, j;
  f_sqr(t, h);        // HH
  f_add(p.z, p.z, h);
  f_sqr(p.z, p.z);
  f_sub(p.z, p.z, z1z1);
  f_sub(p.z, p.z, t); // Z3 = (Z1 + H)^2 - Z1Z1 - HH
  f_dbl(i, t);
  f_dbl(i, i);        // I = 4 HH
  f_mul(j, h, i);     // J = H I
  f_mul(i, p.x, i);   // V = X1 I  (in i)
  f_sqr(t, r);
  f_sub(t, t, j);
  f_sub(t, t, i);
  f_sub(t, t, i);     // X3 = r^2 - J - 2V
  f_mul(j, j, p.y);
  f_dbl(j, j);        // 2 Y1 J
  f_sub(i, i, t);
  f_mul(i, i, r);
  f_sub(p.y, i, j);   // Y3 = r (V - X3) - 2 Y1 J
  p.x = t;
}

// p += q, both Jacobian (add-2007-bl) with the O / equal-point cases handled.
template <typename F>
KZG_DEV void jac_add(jac<F>& p, const jac<F>& q) {
  const bool pzero = f_is_zero(p.z);
  const bool qzero = f_is_zero(q.z);
  F z1z1, z2z2, u1, s1, h, r;
  f_sqr(z1z1, p.z);
  f_sqr(z2z2, q.z);
  f_mul(u1, p.x, z2z2);
  f_mul(s1, p.y, q.z);
  f_mul(s1, s1, z2z2);
  f_mul(h, q.x, z1z1);
  f_sub(h, h, u1);     // H = U2 - U1
  f_mul(r, q.y, p.z);
  f_mul(r, r, z1z1);
  f_sub(r, r, s1);
  f_dbl(r, r);         // r = 2 (S2 - S1)
  const bool same = !pzero && !qzero && f_is_zero(h) && f_is_zero(r);
  if (__builtin_expect(pzero || qzero || same, 0)) {
    if (same)
      jac_dbl(p);
    else if (pzero)
      p = q;
    return;
  }
  f_add(p.z, p.z, q.z);
  f_sqr(p.z, p.z);
  f_sub(p.z, p.z, z1z1);
  f_sub(p.z, p.z, z2z2);
  f_mul(p.z, p.z, h);  // Z3 = ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H
  f_dbl(z1z1, h);
  f_sqr(z1z1, z1z1);   // I = (2H)^2
  f_mul(z2z2, h, z1z1);  // J = H I
  f_mul(u1, u1, z1z1);   // V = U1 I
  f_sqr(h, r);
  f_sub(h, h, z2z2);
  f_sub(h, h, u1);
  f_sub(h, h, u1);       // X3 = r^2 - J - 2V
  f_mul(s1, s1, z2z2);
  f_dbl(s1, s1);         // 2 S1 J
  f_sub(u1, u1, h);
  f_mul(u1, u1, r);
  f_sub(p.y, u1, s1);    // Y3 = r (V - X3) - 2 S1 J
  p.x = h;
}

// [|u|] B for the affine finite base B delivered by load(x, y): 63 doublings, 5 mixed additions.
template <typename F, typename Load>
KZG_DEV void mul_abs_u_affine(jac<F>& acc, Load&& load) {
  load(acc.x, acc.y);
  f_one(acc.z);
#pragma unroll 1
  for (int b = BLS_ABS_U_BITS - 2; b >= 0; b--) {
    jac_dbl(acc);
    if ((BLS_ABS_U >> b) & 1) {
      F x, y;
      load(x, y);
      jac_madd(acc, x, y);
    }
  }
}
// [|u|] q for Jacobian q
template <typename F>
KZG_DEV void mul_abs_u_jac(jac<F>& acc, const jac<F>& q) {
  acc = q;
#pragma unroll 1
  for (int b = BLS_ABS_U_BITS - 2; b >= 0; b--) {
    jac_dbl(acc);
    if ((BLS_ABS_U >> b) & 1) jac_add(acc, q);
  }
}

// Jacobian (X, Y, Z) == affine (x, y)?  (X == x Z^2, Y == y Z^3, Z != 0)
template <typename F>
KZG_DEV bool jac_eq_affine(const jac<F>& p, const F& x, const F& y) {
  F z2, t;
  f_sqr(z2, p.z);
  f_mul(t, x, z2);
  f_sub(t, t, p.x);
  bool ok = f_is_zero(t);
  f_mul(z2, z2, p.z);
  f_mul(t, y, z2);
  f_sub(t, t, p.y);
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
    if ((word >> (b & 31)) & 1) {
      F x, y;
      load(x, y);
      jac_madd(acc, x, y);
    }
  }
  return f_is_zero(acc.z);
}

// G1: P in G1  <=>  [u^2] P == -phi(P) = (BETA x, -y)   (u^2 = |u|^2)
template <typename Load>
KZG_DEV bool in_subgroup_fast_g1(Load&& load) {
  jac<fp> q2;
  {
    jac<fp> q1;
    mul_abs_u_affine(q1, load);
    mul_abs_u_jac(q2, q1);
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
  fp_neg(y.c1, y.c1);
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
  fp_neg(y.c0, y.c0);
  fp_neg(y.c1, y.c1);
  return jac_eq_affine(q, x, y);
}

}  // namespace kzgpot
