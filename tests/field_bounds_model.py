"""Exact interval model of the radix-2^28 field arithmetic in csrc/fp381.hpp and the formulas in
csrc/curve.hpp / codec_kernels.hip / g1_kernels.hip — used by tests/test_field_bounds.py to PROVE (for all inputs)
that no 64-bit column accumulator, 32-bit limb or borrowed-constant subtraction can overflow.

Each value is modelled by per-limb upper bounds (exact ints) and a value upper bound (in units of
p, a float nudged upward at every step). The functions mirror the device code one to one; keep
them in sync.
"""
from __future__ import annotations

import math
import os
import re
from fractions import Fraction

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
NL = 14
LB = 28
LM = (1 << LB) - 1
R = 1 << (LB * NL)
P_L = [(P >> (LB * i)) & LM for i in range(NL)]

HERE = os.path.dirname(os.path.abspath(__file__))
CONSTS = os.path.join(HERE, "..", "kzg-setup-powersoftau_amd", "csrc", "bls12_381_consts.hpp")


def _load_consts(path=CONSTS):
    text = open(path).read()
    out = {}
    for name, body in re.findall(r"static constexpr uint32_t (\w+)\[\d+\] = \{([^}]*)\}", text):
        out[name] = [int(v.strip().rstrip("u"), 16) for v in body.split(",")]
    return out


C = _load_consts()

FIELDS = {  # p, limbs, limb bits, constants header
    "bls12_381": (P, 14, 28, "bls12_381_consts.hpp"),
    "bn254": (0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47, 9, 29, "bn254_consts.hpp"),
}


def use_field(name):
    """Re-point the model at another field (the device code is generic over the traits struct)."""
    global P, NL, LB, LM, R, P_L, P_OVER_R, P_TOP, C
    P, NL, LB, hdr = FIELDS[name]
    LM = (1 << LB) - 1
    R = 1 << (LB * NL)
    P_L = [(P >> (LB * i)) & LM for i in range(NL)]
    P_OVER_R = P / R * UP
    P_TOP = P / (1 << (LB * (NL - 1))) * UP
    C = _load_consts(os.path.join(os.path.dirname(CONSTS), hdr))


class BoundError(AssertionError):
    pass


UP = 1.0 + 1e-9  # upward nudge for float value bounds
P_OVER_R = P / R * UP
P_TOP = P / (1 << (LB * (NL - 1))) * UP  # p / 2^364


class V:
    """Upper bounds: limbs[i] >= every possible limb i; val >= value / p."""

    def __init__(self, limbs, val, name=""):
        self.limbs = list(limbs)
        self.val = float(val)
        self.name = name
        for i, l in enumerate(self.limbs):
            if l >= 1 << 32:
                raise BoundError(f"{name}: limb {i} may overflow 32 bits ({l:#x})")
        if self.val * P >= R * (1 - 1e-6):
            raise BoundError(f"{name}: value {float(self.val):.1f} p does not fit 392 bits")

    def __repr__(self):
        return f"V({self.name}: bits {max(l.bit_length() for l in self.limbs)}, v {float(self.val):.3f})"


def normalized(val, name=""):
    """A normalized value: limbs 0..12 < 2^28, top limb bounded by the value."""
    top = int(float(val) * P_TOP) + 1
    return V([LM] * (NL - 1) + [min(LM, top)], val, name)


def const(limbs, name=""):
    val = sum(l << (LB * i) for i, l in enumerate(limbs)) / P * UP
    return V(limbs, val, name)


def mont_output(val):
    return normalized(val)


def mul(a: V, b: V, name="mul"):
    """fp_mul: FIPS with one 64-bit accumulator per column (+ the m*p chain merged in)."""
    carry = 0
    for i in range(2 * NL):
        j0 = 0 if i < NL else i - (NL - 1)
        j1 = i if i < NL else NL - 1
        s = sum(a.limbs[j] * b.limbs[i - j] for j in range(j0, j1 + 1))
        s += sum(LM * P_L[i - j] for j in range(j0, j1 + 1))
        s += carry
        if s >= 1 << 64:
            raise BoundError(f"{name}: column {i} may reach {s.bit_length()} bits ({a!r} x {b!r})")
        carry = s >> LB
    val = (a.val * b.val * P_OVER_R + 1) * UP  # (ab + m p) / R < ab/R + p
    out = normalized(val, name)
    return out


def mul_sum2(a: V, b: V, c: V, d: V, name="mul_sum2"):
    """fp_mul_sum2: a b + c d with one Montgomery reduction (three mad chains per column)."""
    carry = 0
    for i in range(2 * NL):
        j0 = 0 if i < NL else i - (NL - 1)
        j1 = i if i < NL else NL - 1
        s = sum(a.limbs[j] * b.limbs[i - j] + c.limbs[j] * d.limbs[i - j] for j in range(j0, j1 + 1))
        s += sum(LM * P_L[i - j] for j in range(j0, j1 + 1))
        s += carry
        if s >= 1 << 64:
            raise BoundError(f"{name}: column {i} may reach {s.bit_length()} bits")
        carry = s >> LB
    return normalized(((a.val * b.val + c.val * d.val) * P_OVER_R + 1) * UP, name)


def mul_sum3(a: V, b: V, c: V, d: V, e: V, f: V, name="mul_sum3"):
    """fp_mul_sum3: a b + c d + e f with one Montgomery reduction (four mad chains per column)."""
    carry = 0
    for i in range(2 * NL):
        j0 = 0 if i < NL else i - (NL - 1)
        j1 = i if i < NL else NL - 1
        s = sum(a.limbs[j] * b.limbs[i - j] + c.limbs[j] * d.limbs[i - j] + e.limbs[j] * f.limbs[i - j]
                for j in range(j0, j1 + 1))
        s += sum(LM * P_L[i - j] for j in range(j0, j1 + 1))
        s += carry
        if s >= 1 << 64:
            raise BoundError(f"{name}: column {i} may reach {s.bit_length()} bits")
        carry = s >> LB
    return normalized(((a.val * b.val + c.val * d.val + e.val * f.val) * P_OVER_R + 1) * UP, name)


def mul_add8sqr(a: V, b: V, c: V, name="mul_add8sqr"):
    """fp_mul_add8sqr: a b + 8 c^2 with one reduction; the c^2 half as a squaring (cross products
    c_j (16 c_k) once, squares c_j (8 c_j)), whose column sums equal those of c (8 c)."""
    if max(c.limbs) << 4 >= 1 << 32:
        raise BoundError(f"{name}: 16 c_k must fit 32 bits ({c!r})")
    c8 = V([x << 3 for x in c.limbs], c.val * 8 * UP, name + ".8c")
    carry = 0
    for i in range(2 * NL):
        j0 = 0 if i < NL else i - (NL - 1)
        j1 = i if i < NL else NL - 1
        s = sum(a.limbs[j] * b.limbs[i - j] + c.limbs[j] * c8.limbs[i - j] for j in range(j0, j1 + 1))
        s += sum(LM * P_L[i - j] for j in range(j0, j1 + 1))
        s += carry
        if s >= 1 << 64:
            raise BoundError(f"{name}: column {i} may reach {s.bit_length()} bits")
        carry = s >> LB
    return normalized(((a.val * b.val + 8 * c.val * c.val) * P_OVER_R + 1) * UP, name)


def mul_addsqr(a: V, b: V, c: V, name="mul_addsqr"):
    """fp_mul_addsqr<1>: a b + c^2 with one reduction, the c^2 half as a squaring (cross products
    c_j (2 c_k) once, squares c_j c_j): column sums equal those of a b + c c."""
    if max(c.limbs) << 1 >= 1 << 32:
        raise BoundError(f"{name}: 2 c_k must fit 32 bits ({c!r})")
    carry = 0
    for i in range(2 * NL):
        j0 = 0 if i < NL else i - (NL - 1)
        j1 = i if i < NL else NL - 1
        s = sum(a.limbs[j] * b.limbs[i - j] + c.limbs[j] * c.limbs[i - j] for j in range(j0, j1 + 1))
        s += sum(LM * P_L[i - j] for j in range(j0, j1 + 1))
        s += carry
        if s >= 1 << 64:
            raise BoundError(f"{name}: column {i} may reach {s.bit_length()} bits")
        carry = s >> LB
    return normalized(((a.val * b.val + c.val * c.val) * P_OVER_R + 1) * UP, name)


def sqr(a: V, name="sqr"):
    """fp_sqr: same column sums as mul(a, a); the doubled operand 2 a_k must fit 32 bits."""
    if max(a.limbs) >= 1 << 31:
        raise BoundError(f"{name}: squaring input limb >= 2^31 ({a!r})")
    return mul(a, a, name)


def add_nr(a, b, name="add"):
    return V([x + y for x, y in zip(a.limbs, b.limbs)], (a.val + b.val) * UP, name)


def shl(a, s, name="shl"):
    return V([x << s for x in a.limbs], a.val * (1 << s) * UP, name)


def mul3(a, name="mul3"):
    return V([3 * x for x in a.limbs], a.val * 3 * UP, name)


def subk(a, b, kname, name="subk"):
    k = C[kname]
    for i in range(NL):
        if k[i] < b.limbs[i]:
            raise BoundError(f"{name}: {kname}[{i}] = {k[i]:#x} < subtrahend limb bound {b.limbs[i]:#x} ({b!r})")
    kv = const(k).val
    return V([x + y for x, y in zip(a.limbs, k)], (a.val + kv) * UP, name)


def norm(a, name="norm"):
    for l in a.limbs:
        if l + 16 >= 1 << 32:
            raise BoundError(f"{name}: norm input limb too large")
    return normalized(a.val, name)


def half(a, name="half"):
    """fp_half: a normalized (limbs below the top < 2^28); + p if odd (the top limb absorbs the
    carry), then one right shift across the limbs: normalized, value (v + 1) / 2."""
    if any(l > LM for l in a.limbs[: NL - 1]):
        raise BoundError(f"{name}: input not normalized {a!r}")
    if a.limbs[NL - 1] + P_L[NL - 1] + 1 >= 1 << 32:
        raise BoundError(f"{name}: top limb + p may overflow {a!r}")
    return normalized((a.val + 1) / 2 * UP, name)


def canon_ok(a, name="canon"):
    """fp_canon / fp_is_zero precondition: limbs < 2^32 - 16 (fp_norm), value < 256 p."""
    if max(a.limbs) >= (1 << 32) - 16 or a.val >= 256:
        raise BoundError(f"{name}: canon precondition violated {a!r}")


def reduce_once_ok(a, name="reduce_once"):
    """fp_reduce_once precondition: normalized, value < 2 p."""
    if any(l > LM for l in a.limbs) or a.val >= 2:
        raise BoundError(f"{name}: one conditional subtraction cannot canonicalize {a!r}")


def from_mont_ok(a, name="from_mont"):
    """fp_from_mont: a must be normalized (a < R); mul(a, 1) < p + 1 then reduce_once."""
    if any(l > LM for l in a.limbs):
        raise BoundError(f"{name}: input not normalized {a!r}")
    reduce_once_ok(mul(a, normalized(Fraction(1, 10**9)), name), name)


def vmax(*vs):
    return V([max(x) for x in zip(*(v.limbs for v in vs))], max(v.val for v in vs), "join")


# ------------------------------------------------------------------------------------------
# Fp2 (components share bounds: one V per component pair, conservatively the join)
class V2:
    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    def j(self):
        return vmax(self.c0, self.c1)


def reduced(name=""):
    return normalized(2 - 1e-7, name)  # strictly below 2p (integers: at most 2p - 1)


def check_reduced(a, name):
    if a.val > 2 + 1e-6 or any(l > LM for l in a.limbs[: NL - 1]) or a.limbs[NL - 1] > reduced().limbs[NL - 1]:
        raise BoundError(f"{name}: expected a reduced (< 2p, normalized) value, got {a!r}")


def sub_red(a, b, name="sub_red"):
    """fp_sub_red: signed borrow chain a - b, + 2p if negative: reduced in, reduced out."""
    check_reduced(a, name), check_reduced(b, name)
    return reduced(name)


def add_red(a, b, name="add_red"):
    check_reduced(a, name), check_reduced(b, name)
    t = add_nr(a, b, name)
    if t.val >= 4 + 1e-6:
        raise BoundError(f"{name}: one conditional subtraction cannot reduce {t!r}")
    norm(t, name)
    return reduced(name)


def f2_mul(a: V2, b: V2, name="f2mul"):
    """f_mul(fp2): c0 = REDC(a0 b0 + a1 (4p - b1)), c1 = REDC(a0 b1 + a1 b0)."""
    for c in (a.c0, a.c1, b.c0, b.c1):
        check_reduced(c, name)
    nb1 = subk(normalized(0), b.c1, "KB_4_28", name + ".nb1")
    c0 = mul_sum2(a.c0, b.c0, a.c1, nb1, name + ".c0")
    c1 = mul_sum2(a.c0, b.c1, a.c1, b.c0, name + ".c1")
    check_reduced(c0, name), check_reduced(c1, name)
    return V2(c0, c1)


def f2_sqr(a: V2, name="f2sqr"):
    check_reduced(a.c0, name), check_reduced(a.c1, name)
    s = add_nr(a.c0, a.c1)
    d = subk(a.c0, a.c1, "KB_4_28", name + ".d")
    t = shl(a.c0, 1)
    c0, c1 = mul(s, d, name + ".c0"), mul(t, a.c1, name + ".c1")
    check_reduced(c0, name), check_reduced(c1, name)
    return V2(c0, c1)


class Field:
    """Dispatch generic formulas to the Fp (carry-free) or Fp2 (reduced) models."""

    def __init__(self, two):
        self.two = two

    def mul(self, a, b, name="mul"):
        return f2_mul(a, b, name) if self.two else mul(a, b, name)

    def sqr(self, a, name="sqr"):
        return f2_sqr(a, name) if self.two else sqr(a, name)

    def subk(self, a, b, k, name="subk"):
        if self.two:
            return V2(sub_red(a.c0, b.c0, name), sub_red(a.c1, b.c1, name))
        return subk(a, b, k, name)

    def mul_sub(self, a, b, c, d, name="mul_sub"):
        """f_mul_sub: a b - c d (Fp: mul_sum2 with d negated against KB_4_28)."""
        if self.two:
            return self.subk(self.mul(a, b, name), self.mul(c, d, name), "KB_32_28", name)
        return mul_sum2(a, b, c, subk(normalized(0), d, "KB_4_28", name + ".nd"), name)

    def shl(self, a, s, name="shl"):
        if self.two:
            for _ in range(s):
                a = V2(add_red(a.c0, a.c0, name), add_red(a.c1, a.c1, name))
            return a
        return shl(a, s, name)

    def mul3(self, a, name="mul3"):
        if self.two:
            t = V2(add_red(a.c0, a.c0, name), add_red(a.c1, a.c1, name))
            return V2(add_red(t.c0, a.c0, name), add_red(t.c1, a.c1, name))
        return mul3(a, name)

    def norm(self, a, name="norm"):
        return a if self.two else norm(a, name)

    def canon_ok(self, a, name="canon"):
        if self.two:
            canon_ok(a.c0, name), canon_ok(a.c1, name)
        else:
            canon_ok(a, name)

    def one(self):
        o = normalized(1)
        return V2(o, normalized(0)) if self.two else o


# ------------------------------------------------------------------------------------------
# formulas (mirror csrc/curve.hpp)
def jac_dbl_fp(X, Y, Z):
    """jac_dbl(jac<fp>&) — the hot path (-Y3 = E (X3 - D) + 8 B^2 in one reduction, Y3 = K - that)."""
    a = sqr(X, "A")
    b = sqr(Y, "B")
    t = shl(X, 2)
    d = mul(t, b, "D")
    e = norm(mul3(a), "E")
    t = shl(Y, 1)
    z3 = mul(t, Z, "Z3")
    f = sqr(e, "F")
    t = shl(d, 1)
    x3 = subk(f, t, "KB_8_29", "X3")
    t = subk(f, mul3(d), "KB_8_30", "F-3D")
    ny3 = mul_add8sqr(e, t, b, "-Y3")
    y3 = subk(normalized(0), ny3, "KB_2_28", "Y3")
    return x3, y3, z3


# ---- the G1 fast ladders in W = 2Y coordinates (curve.hpp jac_dbl_w / jac_madd_w / jac_tpl_affine_w)
def jac_dbl_w(X, W, Z):
    """jac_dbl_w: A = X^2, B' = W^2, D = X B', E = 3A, Z3 = W Z, X3 = F - 2D,
    -W3 = E (2 (X3 - D)) + B'^2 (one reduction), W3 = K - that."""
    a = sqr(X, "A")
    b = sqr(W, "B'")
    d = mul(X, b, "D")
    e = norm(mul3(a), "E")
    z3 = mul(W, Z, "Z3")
    f = sqr(e, "F")
    x3 = subk(f, shl(d, 1), "KB_8_29", "X3")
    t = shl(subk(f, mul3(d), "KB_8_30", "F-3D"), 1, "2(F-3D)")
    nw3 = mul_addsqr(e, t, b, "-W3")
    w3 = subk(normalized(0), nw3, "KB_2_28", "W3")
    return x3, w3, z3


def jac_madd_w(X, W, Z, x2, w2):
    """jac_madd_w: ark add_assign_mixed with r = 2 S2 - W1 (= ark's r), X3 = r^2 - J - 2V,
    W3 = 2 r (V - X3) - 2 W1 J; the equal-point branch is jac_dbl_w; base (x2, w2 = 2 y2)."""
    z1z1 = sqr(Z, "Z1Z1")
    h = norm(subk(mul(x2, z1z1, "U2"), X, "KB_128_31", "H"), "H")
    t = mul(mul(w2, Z, "w2Z"), z1z1, "2S2")
    r = norm(subk(t, W, "KB_64_31", "r"), "r")
    canon_ok(Z), canon_ok(h), canon_ok(r)
    xd, wd, zd = jac_dbl_w(X, W, Z)
    hh = sqr(h, "HH")
    z3 = mul(shl(Z, 1), h, "Z3")
    i = norm(shl(hh, 2), "I")
    j = mul(h, i, "J")
    v = mul(X, i, "V")
    t = subk(sqr(r, "r^2"), j, "KB_32_28", "X3a")
    x3 = norm(subk(t, shl(v, 1), "KB_64_29", "X3"), "X3")
    vx = norm(subk(v, x3, "KB_128_28", "V-X3"), "V-X3")
    w3 = mul_sum2(shl(r, 1), vx, shl(W, 1), subk(normalized(0), j, "KB_4_28", "-J"), "W3")
    return vmax(x3, xd, x2), vmax(w3, wd, w2), vmax(z3, zd, normalized(1))


def jac_tpl_affine_w(x, w):
    """jac_tpl_affine_w: 3P from the affine base (x, w = 2y): YYw = w^2 = 4 YY, T = YYw^2 = 16 YYYY,
    E = 3 x YYw - MM, X3 = 4 (x EE - YYw U), W3 = 8 w (U (T - U) - E EE), Z3 = 2E."""
    x = norm(x, "x")
    xx = sqr(x, "XX")
    yyw = sqr(w, "YYw")
    t = sqr(yyw, "T")
    m = norm(mul3(xx), "M")
    mm = sqr(m, "MM")
    e = norm(subk(mul3(mul(x, yyw, "x YYw")), mm, "KB_8_28", "3 x YYw - MM"), "E")
    ee = sqr(e, "EE")
    s2 = sqr(add_nr(m, e), "S2")
    u = subk(subk(subk(s2, mm, "KB_8_28", "S2-MM"), ee, "KB_16_28", "-EE"), t, "KB_8_28", "-T")
    u = norm(u, "U")
    nu = subk(normalized(0), u, "KB_128_28", "-U")
    x3 = shl(mul_sum2(x, ee, yyw, nu, "x EE - YYw U"), 2)
    tu = subk(t, u, "KB_128_28", "T-U")
    nee = subk(normalized(0), ee, "KB_16_28", "-EE")
    inner = mul_sum2(u, tu, e, nee, "U (T - U) - E EE")
    w3 = norm(shl(mul(w, inner, "w inner"), 3), "W3")
    z3 = norm(shl(e, 1), "Z3=2E")
    return x3, w3, z3


def ladder_invariant_w(base_x, base_w, rounds=12):
    """ladder_invariant for the G1 fast ladders (mul_abs_u_affine<fp>) in W = 2Y coordinates,
    including the opening tripling."""
    X, W, Z = jac_tpl_affine_w(base_x, base_w)

    def step(X, W, Z):
        x1, w1, z1 = jac_dbl_w(X, W, Z)
        x2, w2, z2 = jac_madd_w(x1, w1, z1, base_x, base_w)
        return vmax(X, x1, x2), vmax(W, w1, w2), vmax(Z, z1, z2)

    for _ in range(rounds):
        X, W, Z = step(X, W, Z)
    S = (_inflate1(X, 1.01), _inflate1(W, 1.01), _inflate1(Z, 1.01))
    for _ in range(40):
        T = step(*S)
        if all(_within(Field(False), a, b) for a, b in zip(T, S)):
            return S
        S = tuple(_inflate1(vmax(a, b), 1.01) for a, b in zip(T, S))
    raise BoundError("W-form ladder bound set is not closed")


def jac_dbl(F, X, Y, Z):
    return jac_dbl_fp2_lz(X, Y, Z) if F.two else jac_dbl_fp(X, Y, Z)


def jac_madd(F, X, Y, Z, x2, y2):
    z1z1 = F.sqr(Z, "Z1Z1")
    h = F.mul(x2, z1z1, "U2")
    h = F.norm(F.subk(h, X, "KB_128_31", "H"))
    t = F.mul(y2, Z, "y2Z")
    t = F.mul(t, z1z1, "S2")
    r = F.norm(F.subk(t, Y, "KB_64_31", "r'"))
    F.canon_ok(Z), F.canon_ok(h), F.canon_ok(r)
    xd, yd, zd = jac_dbl(F, X, Y, Z)  # the equal-point branch
    hh = F.sqr(h, "HH")
    t = F.shl(Z, 1)
    z3 = F.mul(t, h, "Z3")
    hh = F.norm(F.shl(hh, 2))
    j = F.mul(h, hh, "J")
    hh = F.mul(X, hh, "V")
    t = F.sqr(r, "r'^2")
    t = F.shl(t, 2)
    t = F.subk(t, j, "KB_32_28", "X3a")
    h2 = F.shl(hh, 1)
    t = F.norm(F.subk(t, h2, "KB_64_29", "X3"))
    hh = F.norm(F.subk(hh, t, "KB_128_28", "V-X3"))
    r = F.shl(r, 1)
    h = F.shl(Y, 1)
    y3 = F.mul_sub(r, hh, h, j, "Y3")  # r (V - X3) - 2 Y1 J
    one = F.one()
    jn = (lambda a, b: V2(vmax(a.c0, b.c0), vmax(a.c1, b.c1))) if F.two else vmax
    return jn(jn(t, xd), x2), jn(jn(y3, yd), y2), jn(jn(z3, zd), one)


def jac_eq_affine(F, X, Y, Z, x, y):
    z2 = F.sqr(Z, "z2")
    t = F.mul(x, z2, "xZ2")
    t = F.subk(t, X, "KB_128_31", "eqx")
    F.canon_ok(t)
    z2 = F.mul(z2, Z, "z3")
    t = F.mul(y, z2, "yZ3")
    t = F.subk(t, Y, "KB_128_31", "eqy")
    F.canon_ok(t)
    F.canon_ok(Z)


def join(F, a, b):
    if F.two:
        return V2(vmax(a.c0, b.c0), vmax(a.c1, b.c1))
    return vmax(a, b)


def _inflate1(a, f):
    limbs = list(a.limbs)
    limbs[NL - 1] = int(limbs[NL - 1] * f) + 2  # the top limb tracks the value
    return V(limbs, a.val * f + 0.01)


def _inflate(F, a, f=1.01):
    if F.two:  # every Fp2 op returns exactly reduced(): the joined bound is already a fixed point
        return a
    return _inflate1(a, f)


def _within(F, a, b):
    """a subset of b (all bounds of a <= those of b)."""
    pairs = ((a.c0, b.c0), (a.c1, b.c1)) if F.two else ((a, b),)
    return all(all(x <= y for x, y in zip(u.limbs, w.limbs)) and u.val <= w.val for u, w in pairs)


def ladder_invariant(F, base_x, base_y, rounds=12):
    """A bound set S for the ladder accumulator (X, Y, Z) that contains the starting point and is
    CLOSED under one ladder step (dbl, then optionally madd(base)) — hence bounds every state
    reached by in_subgroup_ref (ark's double-and-add) for any input. Found by joined iteration, then
    inflated and verified closed. (The fast ladders run in W = 2Y coordinates: ladder_invariant_w.)"""
    X, Y, Z = base_x, base_y, F.one()

    def step(X, Y, Z):
        x1, y1, z1 = jac_dbl(F, X, Y, Z)
        outs = [(x1, y1, z1), jac_madd(F, x1, y1, z1, base_x, base_y)]
        nx, ny, nz = X, Y, Z
        for ox, oy, oz in outs:
            nx, ny, nz = join(F, nx, ox), join(F, ny, oy), join(F, nz, oz)
        return nx, ny, nz

    for _ in range(rounds):
        X, Y, Z = step(X, Y, Z)
    S = (_inflate(F, X), _inflate(F, Y), _inflate(F, Z))
    for _ in range(40):
        T = step(*S)
        if all(_within(F, a, b) for a, b in zip(T, S)):
            break
        S = tuple(_inflate(F, join(F, a, b)) for a, b in zip(T, S))
    else:
        raise BoundError("ladder bound set is not closed: values keep growing")
    return S


# ------------------------------------------------------------------------------------------
# Fp2 in the carry-free ("lazy") discipline of the G1 path — the G2 ladders (curve.hpp
# jac_dbl(jac<fp2>&), jac_madd(jac<fp2>&, ..), jac_eq_affine(jac<fp2>, ..)). Each component is
# a V with its own limb / value bounds, exactly as for Fp.
def mul2(a: V2, b: V2, kname, name="mul2"):
    """f2_mul_lz: c0 = REDC(a0 b0 + a1 (K - b1)), c1 = REDC(a0 b1 + a1 b0)."""
    nb1 = subk(normalized(0), b.c1, kname, name + ".nb1")
    return V2(mul_sum2(a.c0, b.c0, a.c1, nb1, name + ".c0"), mul_sum2(a.c0, b.c1, a.c1, b.c0, name + ".c1"))


def sqr2(a: V2, kname, name="sqr2"):
    """f2_sqr_lz: c0 = REDC((a0 + a1)(a0 + K - a1)), c1 = REDC(2 a0 a1)."""
    s = add_nr(a.c0, a.c1, name + ".s")
    d = subk(a.c0, a.c1, kname, name + ".d")
    return V2(mul(s, d, name + ".c0"), mul(shl(a.c0, 1), a.c1, name + ".c1"))


def subk2(a, b, kname, name="subk2"):
    return V2(subk(a.c0, b.c0, kname, name + ".c0"), subk(a.c1, b.c1, kname, name + ".c1"))


def norm2(a, name="norm2"):
    return V2(norm(a.c0, name + ".c0"), norm(a.c1, name + ".c1"))


def shl2(a, s, name="shl2"):
    return V2(shl(a.c0, s, name), shl(a.c1, s, name))


def mul3_2(a, name="mul3_2"):
    return V2(mul3(a.c0, name), mul3(a.c1, name))


def zero_ok2(a, name):
    canon_ok(a.c0, name), canon_ok(a.c1, name)


def jac_dbl_fp2_lz(X, Y, Z):
    """curve.hpp jac_dbl(jac<fp2>&): X, Y, Z normalized in, normalized out."""
    b = sqr2(Y, "KB_32_28", "B")
    z3 = mul2(shl2(Y, 1), Z, "KB_16_28", "Z3")
    a = sqr2(X, "KB_16_28", "A")
    d = mul2(shl2(X, 2), b, "KB_2_28", "D")
    e = norm2(mul3_2(a), "E")
    f = sqr2(e, "KB_4_28", "F")
    x3 = norm2(subk2(f, shl2(d, 1), "KB_4_29", "X3"), "X3")
    t = subk2(d, x3, "KB_8_28", "D-X3")
    # Y3 = E (D - X3) - 8 B^2, one three-product reduction per component
    u = subk(normalized(0), t.c1, "KB_16_30", "-t1")
    s = add_nr(b.c0, b.c1, "b0+b1")
    n0 = norm(subk(normalized(0), shl(norm(subk(b.c0, b.c1, "KB_2_28", "b0-b1")), 3), "KB_64_31", "-8(b0-b1)"))
    y0 = mul_sum3(e.c0, t.c0, e.c1, u, s, n0, "Y3.c0")
    n1 = norm(subk(normalized(0), shl(b.c1, 3), "KB_16_31", "-8b1"))
    y1 = mul_sum3(e.c0, t.c1, e.c1, t.c0, shl(b.c0, 1), n1, "Y3.c1")
    return x3, V2(y0, y1), z3


def add2(a, b, name="add2"):
    return V2(add_nr(a.c0, b.c0, name), add_nr(a.c1, b.c1, name))


def jac_madd_fp2_lz(X, Y, Z, x2, y2):
    """curve.hpp jac_madd(jac<fp2>&, load): normalized in / out; base (x2, y2) normalized."""
    z1z1 = sqr2(Z, "KB_16_28", "Z1Z1")
    u2 = mul2(x2, z1z1, "KB_2_28", "U2")
    h = norm2(subk2(u2, X, "KB_32_28", "H"), "H")
    t = mul2(y2, Z, "KB_16_28", "y2Z")
    s2 = mul2(t, z1z1, "KB_2_28", "S2")
    r = norm2(subk2(s2, Y, "KB_32_28", "r'"), "r'")
    zero_ok2(Z, "Z"), zero_ok2(h, "H"), zero_ok2(r, "r'")
    xd, yd, zd = jac_dbl_fp2_lz(X, Y, Z)  # the equal-point branch
    hh = sqr2(h, "KB_64_28", "HH")
    z3 = mul2(shl2(Z, 1), h, "KB_64_28", "Z3m")
    i = shl2(hh, 2, "I")
    j = mul2(h, i, "KB_8_30", "J")
    v = mul2(X, i, "KB_8_30", "V")
    rr = sqr2(r, "KB_64_28", "r'^2")
    x3 = subk2(shl2(rr, 2), j, "KB_2_28", "X3a")
    x3 = norm2(subk2(x3, shl2(v, 1), "KB_4_29", "X3m"), "X3m")
    vx = subk2(v, x3, "KB_32_28", "V-X3")
    a = mul2(shl2(r, 1), vx, "KB_64_30", "r(V-X3)")
    b = mul2(shl2(Y, 1), j, "KB_2_28", "2Y1J")
    y3 = norm2(subk2(a, b, "KB_4_28", "Y3m"), "Y3m")
    return (V2(vmax(x3.c0, xd.c0, x2.c0), vmax(x3.c1, xd.c1, x2.c1)),
            V2(vmax(y3.c0, yd.c0, y2.c0), vmax(y3.c1, yd.c1, y2.c1)),
            V2(vmax(z3.c0, zd.c0, normalized(1)), vmax(z3.c1, zd.c1, normalized(1))))


def jac_eq_affine_fp2_lz(X, Y, Z, x, y):
    """curve.hpp jac_eq_affine(const jac<fp2>&, ..): x Z^2 == X, y Z^3 == Y, Z != 0."""
    z2 = sqr2(Z, "KB_16_28", "z2")
    t = subk2(mul2(x, z2, "KB_2_28", "xZ2"), X, "KB_32_28", "eqx")
    zero_ok2(t, "eqx")
    z3 = mul2(z2, Z, "KB_16_28", "z3")
    t = subk2(mul2(y, z3, "KB_2_28", "yZ3"), Y, "KB_32_29", "eqy")
    zero_ok2(t, "eqy")
    zero_ok2(Z, "Z")


def ladder_invariant_fp2_lz(base_x, base_y, rounds=12):
    """ladder_invariant for the lazy Fp2 ladder (mul_abs_u_affine / in_subgroup_ref over Fp2)."""
    def join2(a, b):
        return V2(vmax(a.c0, b.c0), vmax(a.c1, b.c1))

    def infl(a):
        return V2(_inflate1(a.c0, 1.01), _inflate1(a.c1, 1.01))

    def within(a, b):
        return all(all(x <= y for x, y in zip(u.limbs, w.limbs)) and u.val <= w.val
                   for u, w in ((a.c0, b.c0), (a.c1, b.c1)))

    def step(X, Y, Z):
        outs = [jac_dbl_fp2_lz(X, Y, Z)]
        outs.append(jac_madd_fp2_lz(*outs[0], base_x, base_y))
        nx, ny, nz = X, Y, Z
        for ox, oy, oz in outs:
            nx, ny, nz = join2(nx, ox), join2(ny, oy), join2(nz, oz)
        return nx, ny, nz

    X, Y, Z = base_x, base_y, V2(normalized(1), normalized(0))
    for _ in range(rounds):
        X, Y, Z = step(X, Y, Z)
    S = (infl(X), infl(Y), infl(Z))
    for _ in range(40):
        T = step(*S)
        if all(within(a, b) for a, b in zip(T, S)):
            return S
        S = tuple(infl(join2(a, b)) for a, b in zip(T, S))
    raise BoundError("lazy Fp2 ladder bound set is not closed")


# ---- the G2 fast ladder in W = 2Y coordinates (curve.hpp jac_dbl_w / jac_madd_w / jac_tpl_affine_w
# over Fp2): the same savings as the G1 W form
def jac_dbl_fp2_w(X, W, Z):
    """jac_dbl_w(jac<fp2>&): B' = W^2, Z3 = W Z, D = X B', E = 3A, X3 = F - 2D, t = D - X3,
    W3 = (2E) t - B'^2 as two three-product sums per component."""
    b = sqr2(W, "KB_32_29", "B'")
    z3 = mul2(W, Z, "KB_16_28", "Z3")
    a = sqr2(X, "KB_16_28", "A")
    d = mul2(X, b, "KB_2_28", "D")
    e = norm2(mul3_2(a), "E")
    f = sqr2(e, "KB_4_28", "F")
    x3 = norm2(subk2(f, shl2(d, 1), "KB_4_29", "X3"), "X3")
    t = subk2(d, x3, "KB_8_28", "D-X3")
    e2 = shl2(e, 1, "2E")
    u = subk(normalized(0), t.c1, "KB_16_30", "-t1")
    s = add_nr(b.c0, b.c1, "b0+b1")
    n0 = norm(subk(b.c1, b.c0, "KB_2_28", "b1-b0"), "b1-b0")
    w0 = mul_sum3(e2.c0, t.c0, e2.c1, u, s, n0, "W3.c0")
    n1 = subk(normalized(0), b.c1, "KB_2_28", "-b1")
    w1 = mul_sum3(e2.c0, t.c1, e2.c1, t.c0, shl(b.c0, 1), n1, "W3.c1")
    return x3, V2(w0, w1), z3


def jac_tpl_affine_fp2_w(x, w):
    """jac_tpl_affine_w(jac<fp2>&): the scaled triple (X3/4, W3/8, E) from (x, w = 2y):
    YYw = w^2, T = YYw^2, E = 3 x YYw - MM, X3/4 = x EE - YYw U, W3/8 = w (U (T - U) - E EE)."""
    xx = sqr2(x, "KB_2_28", "XX")
    yyw = sqr2(w, "KB_4_29", "YYw")
    t = sqr2(yyw, "KB_2_28", "T")
    m = norm2(mul3_2(xx), "M")
    mm = sqr2(m, "KB_4_28", "MM")
    e = norm2(subk2(mul3_2(mul2(x, yyw, "KB_2_28", "x YYw")), mm, "KB_2_28", "3 x YYw - MM"), "E")
    ee = sqr2(e, "KB_16_28", "EE")
    s2 = sqr2(norm2(add2(m, e), "M+E"), "KB_32_28", "S2")
    u = subk2(subk2(subk2(s2, mm, "KB_2_28", "S2-MM"), ee, "KB_4_28", "-EE"), t, "KB_2_28", "-T")
    u = norm2(u, "U")
    a = mul2(x, ee, "KB_2_28", "xEE")
    b = mul2(yyw, u, "KB_64_28", "YYwU")
    x3 = norm2(subk2(a, b, "KB_2_28", "xEE-YYwU"), "X3/4")
    c = mul2(u, norm2(subk2(t, u, "KB_64_28", "T-U"), "T-U"), "KB_128_28", "U(T-U)")
    d = mul2(e, ee, "KB_2_28", "E EE")
    inner = norm2(subk2(c, d, "KB_2_28", "inner"), "inner")
    w3 = mul2(w, inner, "KB_8_28", "W3/8")
    return x3, w3, e


def jac_madd_fp2_w(X, W, Z, x2, w2):
    """jac_madd_w(jac<fp2>&): r = 2 S2 - W1, X3 = r^2 - J - 2V, W3 = 2r (V - X3) - 2 W1 J."""
    z1z1 = sqr2(Z, "KB_16_28", "Z1Z1")
    u2 = mul2(x2, z1z1, "KB_2_28", "U2")
    h = norm2(subk2(u2, X, "KB_32_28", "H"), "H")
    t = mul2(w2, Z, "KB_16_28", "w2Z")
    s2 = mul2(t, z1z1, "KB_2_28", "2S2")
    r = norm2(subk2(s2, W, "KB_32_29", "r"), "r")
    zero_ok2(Z, "Z"), zero_ok2(h, "H"), zero_ok2(r, "r")
    xd, wd, zd = jac_dbl_fp2_w(X, W, Z)
    hh = sqr2(h, "KB_64_28", "HH")
    z3 = mul2(shl2(Z, 1), h, "KB_64_28", "Z3m")
    i = shl2(hh, 2, "I")
    j = mul2(h, i, "KB_8_30", "J")
    v = mul2(X, i, "KB_8_30", "V")
    rr = sqr2(r, "KB_64_28", "r^2")
    x3 = subk2(rr, j, "KB_2_28", "X3a")
    x3 = norm2(subk2(x3, shl2(v, 1), "KB_4_29", "X3m"), "X3m")
    vx = subk2(v, x3, "KB_32_28", "V-X3")
    a = mul2(shl2(r, 1), vx, "KB_64_30", "2r(V-X3)")
    b = mul2(shl2(W, 1), j, "KB_2_28", "2W1J")
    w3 = norm2(subk2(a, b, "KB_4_28", "W3m"), "W3m")
    return (V2(vmax(x3.c0, xd.c0, x2.c0), vmax(x3.c1, xd.c1, x2.c1)),
            V2(vmax(w3.c0, wd.c0, w2.c0), vmax(w3.c1, wd.c1, w2.c1)),
            V2(vmax(z3.c0, zd.c0, normalized(1)), vmax(z3.c1, zd.c1, normalized(1))))


def ladder_invariant_fp2_w(base_x, base_w, rounds=12):
    """ladder_invariant for the G2 fast ladder in W form (mul_abs_u_affine<fp2>)."""
    def join2(a, b):
        return V2(vmax(a.c0, b.c0), vmax(a.c1, b.c1))

    def infl(a):
        return V2(_inflate1(a.c0, 1.01), _inflate1(a.c1, 1.01))

    def within(a, b):
        return all(all(x <= y for x, y in zip(u.limbs, w.limbs)) and u.val <= w.val
                   for u, w in ((a.c0, b.c0), (a.c1, b.c1)))

    def step(X, W, Z):
        x1, w1, z1 = jac_dbl_fp2_w(X, W, Z)
        x2, w2, z2 = jac_madd_fp2_w(x1, w1, z1, base_x, base_w)
        return join2(join2(X, x1), x2), join2(join2(W, w1), w2), join2(join2(Z, z1), z2)

    X, W, Z = jac_tpl_affine_fp2_w(base_x, base_w)
    for _ in range(rounds):
        X, W, Z = step(X, W, Z)
    S = (infl(X), infl(W), infl(Z))
    for _ in range(40):
        T = step(*S)
        if all(within(a, b) for a, b in zip(T, S)):
            return S
        S = tuple(infl(join2(a, b)) for a, b in zip(T, S))
    raise BoundError("W-form Fp2 ladder bound set is not closed")
