"""The ladder formulas of csrc/curve.hpp restated over exact field values and checked against the
oracle's affine group law (oracle/kzgpot_oracle.py g1_mul / g2_mul, which follow ark-ec 0.2's
Jacobian formulas). tests/test_field_bounds.py proves the same functions never overflow a limb;
this file checks their algebra: each device formula returns the same point as the textbook one,
on subgroup points, on random curve points outside the subgroup and on small-order points. CPU only.

  jac_dbl (G1)            -Y3 = E (X3 - D) + 8 B^2   (fp_mul_add8sqr)
  jac_dbl (G2)            Y3 = E (D - X3) - 8 B^2 as two three-product sums per component
  jac_madd                ark add_assign_mixed with r' = S2 - Y1 (r = 2 r') and Z3 = 2 Z1 H
  tpl_g1 / tpl_g2         the Y-form tripling (EFD tpl-2007-bl with Z1 = 1; G2 as the triple
                          (X3 / 4, Y3 / 8, E), E = 12 x YY - MM): reference-only, the algebra the
                          device's W = 2Y forms jac_tpl_affine_w (tpl_g1_w / tpl_g2_w) scale
  mul_abs_u_affine        [|u|] B: the tripling, then 62 doublings and 4 mixed additions
  in_subgroup_fast_g1     [u^2] P as [|u|] of Q1 = (X : Y : Z) run on y^2 = x^3 + 4 Z^6 from the
                          affine (X, Y), mapped back by Z' -> Z' Z; compared with phi(P) = (beta x, -y)
"""
import random

import pytest

O = pytest.importorskip("kzgpot_oracle")
P = O.P
ABS_U = -O.U_PARAM


class Fp:
    zero, one = 0, 1

    @staticmethod
    def add(a, b): return (a + b) % P
    @staticmethod
    def sub(a, b): return (a - b) % P
    @staticmethod
    def mul(a, b): return a * b % P
    @staticmethod
    def sqr(a): return a * a % P
    @staticmethod
    def k(c, a): return c * a % P  # small constant times a
    @staticmethod
    def inv(a): return pow(a, P - 2, P)


class Fp2:
    zero, one = (0, 0), (1, 0)
    add = staticmethod(O.fp2_add)
    sub = staticmethod(O.fp2_sub)
    mul = staticmethod(O.fp2_mul)
    sqr = staticmethod(O.fp2_sqr)
    inv = staticmethod(O.fp2_inv)

    @staticmethod
    def k(c, a): return (c * a[0] % P, c * a[1] % P)


def affine(F, X, Y, Z):
    if Z == F.zero:
        return None
    zi = F.inv(Z)
    zi2 = F.sqr(zi)
    return F.mul(X, zi2), F.mul(F.mul(Y, zi2), zi)


def dbl_g1(X, Y, Z):
    F = Fp
    a, b = F.sqr(X), F.sqr(Y)
    d = F.mul(F.k(4, X), b)
    e = F.k(3, a)
    z3 = F.mul(F.k(2, Y), Z)
    f = F.sqr(e)
    x3 = F.sub(f, F.k(2, d))
    ny3 = F.add(F.mul(e, F.sub(x3, d)), F.k(8, F.sqr(b)))  # one reduction on the device
    return x3, F.sub(0, ny3), z3


def dbl_g2(X, Y, Z):
    F = Fp2
    b = F.sqr(Y)
    z3 = F.mul(F.k(2, Y), Z)
    a = F.sqr(X)
    d = F.mul(F.k(4, X), b)
    e = F.k(3, a)
    f = F.sqr(e)
    x3 = F.sub(f, F.k(2, d))
    t = F.sub(d, x3)
    (e0, e1), (t0, t1), (b0, b1) = e, t, b
    y0 = (e0 * t0 + e1 * (-t1) + (b0 + b1) * (-8 * (b0 - b1))) % P
    y1 = (e0 * t1 + e1 * t0 + (2 * b0) * (-8 * b1)) % P
    return x3, (y0, y1), z3


def madd(F, dbl, X, Y, Z, x2, y2):
    if Z == F.zero:
        return x2, y2, F.one
    z1z1 = F.sqr(Z)
    h = F.sub(F.mul(x2, z1z1), X)
    r = F.sub(F.mul(F.mul(y2, Z), z1z1), Y)
    if h == F.zero and r == F.zero:
        return dbl(X, Y, Z)
    hh = F.sqr(h)
    z3 = F.mul(F.k(2, Z), h)
    i = F.k(4, hh)
    j = F.mul(h, i)
    v = F.mul(X, i)
    r = F.k(2, r)
    x3 = F.sub(F.sub(F.sqr(r), j), F.k(2, v))
    y3 = F.sub(F.mul(r, F.sub(v, x3)), F.mul(F.k(2, Y), j))
    return x3, y3, z3


def tpl_g1(x, y):
    F = Fp
    xx, yy = F.sqr(x), F.sqr(y)
    yyyy = F.sqr(yy)
    m = F.k(3, xx)
    mm = F.sqr(m)
    w = F.sub(F.sub(F.sqr(F.add(x, yy)), xx), yyyy)  # 2 x YY
    e = F.sub(F.k(6, w), mm)
    ee = F.sqr(e)
    t = F.k(16, yyyy)
    u = F.sub(F.sub(F.sub(F.sqr(F.add(m, e)), mm), ee), t)
    x3 = F.k(4, F.sub(F.mul(x, ee), F.mul(F.k(4, yy), u)))
    y3 = F.k(8, F.mul(y, F.sub(F.mul(u, F.sub(t, u)), F.mul(e, ee))))
    return x3, y3, F.k(2, e)


def tpl_g2(x, y):
    F = Fp2
    xx, yy = F.sqr(x), F.sqr(y)
    m = F.k(3, xx)
    mm = F.sqr(m)
    e = F.sub(F.k(12, F.mul(x, yy)), mm)
    ee = F.sqr(e)
    t = F.k(16, F.sqr(yy))
    u = F.sub(F.sub(F.sub(F.sqr(F.add(m, e)), mm), ee), t)
    x3 = F.sub(F.mul(x, ee), F.mul(F.k(4, yy), u))
    y3 = F.mul(y, F.sub(F.mul(u, F.sub(t, u)), F.mul(e, ee)))
    return x3, y3, e


def dbl_g1_w(X, W, Z):
    F = Fp
    a, b = F.sqr(X), F.sqr(W)                       # B' = W^2
    d = F.mul(X, b)
    e = F.k(3, a)
    z3 = F.mul(W, Z)
    f = F.sqr(e)
    x3 = F.sub(f, F.k(2, d))
    nw3 = F.add(F.mul(e, F.k(2, F.sub(x3, d))), F.sqr(b))
    return x3, F.sub(0, nw3), z3


def madd_g1_w(X, W, Z, x2, w2):
    F = Fp
    if Z == 0:
        return x2, w2, 1
    z1z1 = F.sqr(Z)
    h = F.sub(F.mul(x2, z1z1), X)
    r = F.sub(F.mul(F.mul(w2, Z), z1z1), W)         # 2 S2 - W1 = ark's r
    if h == 0 and r == 0:
        return dbl_g1_w(X, W, Z)
    hh = F.sqr(h)
    z3 = F.mul(F.k(2, Z), h)
    i = F.k(4, hh)
    j = F.mul(h, i)
    v = F.mul(X, i)
    x3 = F.sub(F.sub(F.sqr(r), j), F.k(2, v))
    w3 = F.sub(F.mul(F.k(2, r), F.sub(v, x3)), F.mul(F.k(2, W), j))
    return x3, w3, z3


def tpl_g1_w(x, w):
    F = Fp
    xx, yyw = F.sqr(x), F.sqr(w)
    t = F.sqr(yyw)
    m = F.k(3, xx)
    mm = F.sqr(m)
    e = F.sub(F.k(3, F.mul(x, yyw)), mm)
    ee = F.sqr(e)
    u = F.sub(F.sub(F.sub(F.sqr(F.add(m, e)), mm), ee), t)
    x3 = F.k(4, F.sub(F.mul(x, ee), F.mul(yyw, u)))
    w3 = F.k(8, F.mul(w, F.sub(F.mul(u, F.sub(t, u)), F.mul(e, ee))))
    return x3, w3, F.k(2, e)


def mul_abs_u_w(bw):
    """mul_abs_u_affine<fp>: the W = 2Y ladder from the base (x, w = 2y); returns (X, W, Z)."""
    X, W, Z = tpl_g1_w(*bw)
    for b in range(ABS_U.bit_length() - 3, -1, -1):
        X, W, Z = dbl_g1_w(X, W, Z)
        if (ABS_U >> b) & 1:
            X, W, Z = madd_g1_w(X, W, Z, *bw)
    return X, W, Z


def test_g1_w_form_ladders():
    """in_subgroup_fast_g1's W = 2Y ladders: [|u|] P, then [|u|] of Q1 = (X, W) on the isomorphic
    curve (its base w is Q1's W), compared with (beta x, 2 (-y)) in W form."""
    rng = random.Random(6)
    for pt in _points("g1", rng):
        X, W, Z = mul_abs_u_w((pt[0], 2 * pt[1] % P))
        want = O.g1_mul(pt, ABS_U)
        got = None if Z == 0 else (X * pow(Z * Z, P - 2, P) % P, W * pow(2 * Z ** 3, P - 2, P) % P)
        assert got == want, pt
        if Z == 0:
            continue
        # second ladder: base (X, W) is (x, 2y) of the affine point (X, W / 2) on E'
        X2, W2, Z2 = mul_abs_u_w((X, W))
        z = Z2 * Z % P
        got2 = (X2 * pow(z * z, P - 2, P) % P, W2 * pow(2 * z ** 3, P - 2, P) % P)
        assert got2 == O.g1_mul(pt, ABS_U * ABS_U), pt


def mul_abs_u_jac(F, dbl, tpl, base):
    X, Y, Z = tpl(*base)
    for b in range(ABS_U.bit_length() - 3, -1, -1):
        X, Y, Z = dbl(X, Y, Z)
        if (ABS_U >> b) & 1:
            X, Y, Z = madd(F, dbl, X, Y, Z, *base)
    return X, Y, Z


def mul_abs_u(F, dbl, tpl, base):
    return affine(F, *mul_abs_u_jac(F, dbl, tpl, base))


def _points(group, rng):
    if group == "g1":
        gen, mul, rnd = O.G1_GEN, O.g1_mul, O.g1_random_on_curve
    else:
        gen, mul, rnd = O.G2_GEN, O.g2_mul, O.g2_random_on_curve
    pts = [mul(gen, rng.randrange(1, O.R_ORDER)) for _ in range(4)]
    pts += [rnd(rng) for _ in range(4)]
    # points of the cofactor part: no r component at all
    pts += [q for q in (mul(rnd(rng), O.R_ORDER) for _ in range(3)) if q is not None]
    if group == "g1":
        # the order-3 points (0, +-2): 3P = O, the tripling's Z3 = 2E must be 0
        pts += [(0, 2), (0, P - 2)]
    return pts


def test_tripling_is_3p():
    rng = random.Random(3)
    for group, F, tpl, mul in (("g1", Fp, tpl_g1, O.g1_mul), ("g2", Fp2, tpl_g2, O.g2_mul)):
        for pt in _points(group, rng):
            assert affine(F, *tpl(*pt)) == mul(pt, 3), (group, pt)


def test_doubling_and_mixed_addition():
    rng = random.Random(2)
    for group, F, dbl, mul in (("g1", Fp, dbl_g1, O.g1_mul), ("g2", Fp2, dbl_g2, O.g2_mul)):
        for pt in _points(group, rng):
            z = rng.randrange(1, P) if F is Fp else (rng.randrange(P), rng.randrange(1, P))
            z2 = F.sqr(z)
            X, Y = F.mul(pt[0], z2), F.mul(F.mul(pt[1], z2), z)  # pt with a random Z
            assert affine(F, *dbl(X, Y, z)) == mul(pt, 2)
            q = mul(pt, 5)
            if q is not None:  # pt + 5 pt, and the equal-point branch pt + pt
                assert affine(F, *madd(F, dbl, X, Y, z, *q)) == mul(pt, 6)
            assert affine(F, *madd(F, dbl, X, Y, z, *pt)) == mul(pt, 2)


def test_ladder_abs_u():
    rng = random.Random(1)
    for group, F, dbl, tpl, mul in (("g1", Fp, dbl_g1, tpl_g1, O.g1_mul), ("g2", Fp2, dbl_g2, tpl_g2, O.g2_mul)):
        for pt in _points(group, rng)[:7] + _points(group, rng)[-2:]:
            assert mul_abs_u(F, dbl, tpl, pt) == mul(pt, ABS_U), (group, pt)


def test_g1_second_ladder_on_isomorphic_curve():
    rng = random.Random(4)
    for pt in _points("g1", rng):
        X, Y, Z = mul_abs_u_jac(Fp, dbl_g1, tpl_g1, pt)
        if Z == 0:
            continue  # Q1 = O: the kernel's second ladder ends in Z' Z = 0 as well
        X2, Y2, Z2 = mul_abs_u_jac(Fp, dbl_g1, tpl_g1, (X, Y))
        got = affine(Fp, X2, Y2, Fp.mul(Z2, Z))
        assert got == O.g1_mul(pt, ABS_U * ABS_U)
        if O.g1_mul(pt, O.R_ORDER) is None:
            # on G1, [u^2] P = (beta x, -y) for one of the two primitive cube roots of unity beta
            b = next(c for c in (pow(g, (P - 1) // 3, P) for g in range(2, 20)) if c != 1)
            assert got in [((b * pt[0]) % P, (-pt[1]) % P), ((b * b * pt[0]) % P, (-pt[1]) % P)]


def dbl_g2_w(X, W, Z):
    F = Fp2
    b = F.sqr(W)
    z3 = F.mul(W, Z)
    d = F.mul(X, b)
    e = F.k(3, F.sqr(X))
    x3 = F.sub(F.sqr(e), F.k(2, d))
    t = F.sub(d, x3)
    (e0, e1), (t0, t1), (b0, b1) = F.k(2, e), t, b
    w0 = (e0 * t0 + e1 * (-t1) + (b0 + b1) * (b1 - b0)) % P
    w1 = (e0 * t1 + e1 * t0 + (2 * b0) * (-b1)) % P
    return x3, (w0, w1), z3


def madd_g2_w(X, W, Z, x2, w2):
    F = Fp2
    if Z == F.zero:
        return x2, w2, F.one
    z1z1 = F.sqr(Z)
    h = F.sub(F.mul(x2, z1z1), X)
    r = F.sub(F.mul(F.mul(w2, Z), z1z1), W)
    if h == F.zero and r == F.zero:
        return dbl_g2_w(X, W, Z)
    hh = F.sqr(h)
    z3 = F.mul(F.k(2, Z), h)
    i = F.k(4, hh)
    j = F.mul(h, i)
    v = F.mul(X, i)
    x3 = F.sub(F.sub(F.sqr(r), j), F.k(2, v))
    w3 = F.sub(F.mul(F.k(2, r), F.sub(v, x3)), F.mul(F.k(2, W), j))
    return x3, w3, z3


def tpl_g2_w(x, w):
    F = Fp2
    xx, yyw = F.sqr(x), F.sqr(w)
    t = F.sqr(yyw)
    m = F.k(3, xx)
    mm = F.sqr(m)
    e = F.sub(F.k(3, F.mul(x, yyw)), mm)
    ee = F.sqr(e)
    u = F.sub(F.sub(F.sub(F.sqr(F.add(m, e)), mm), ee), t)
    x3 = F.sub(F.mul(x, ee), F.mul(yyw, u))
    w3 = F.mul(w, F.sub(F.mul(u, F.sub(t, u)), F.mul(e, ee)))
    return x3, w3, e


def test_g2_w_form_ladder():
    """mul_abs_u_affine<fp2> in W = 2Y form: the W result over 2 Z^3 is [|u|] P's y."""
    rng = random.Random(7)
    for pt in _points("g2", rng):
        bw = (pt[0], Fp2.k(2, pt[1]))
        X, W, Z = tpl_g2_w(*bw)
        for b in range(ABS_U.bit_length() - 3, -1, -1):
            X, W, Z = dbl_g2_w(X, W, Z)
            if (ABS_U >> b) & 1:
                X, W, Z = madd_g2_w(X, W, Z, *bw)
        want = O.g2_mul(pt, ABS_U)
        if Z == Fp2.zero:
            assert want is None
            continue
        zi = Fp2.inv(Z)
        zi2 = Fp2.sqr(zi)
        got = (Fp2.mul(X, zi2), Fp2.mul(Fp2.mul(W, zi2), Fp2.mul(zi, (pow(2, P - 2, P), 0))))
        assert got == want, pt
