"""Machine proof that the radix-2^28 arithmetic never overflows (CPU only).

tests/field_bounds_model.py mirrors csrc/fp381.hpp + csrc/curve.hpp with exact interval bounds;
every fp_mul column sum is checked < 2^64, every limb < 2^32, every borrowed constant dominates
its subtrahend limb by limb, and the ladder states are shown to live in a bound set closed under
the ladder steps (so the proof covers all 2^64 / 2^255 steps, every input point)."""
import os
import random
from fractions import Fraction

import pytest

import field_bounds_model as M


def test_ladders_closed():
    """G1 ladders (the G2 ones: test_g2_lazy_ladder_closed)."""
    two = False
    F = M.Field(two)
    base = M.normalized(Fraction(101, 100))
    S1 = M.ladder_invariant(F, base, base)                     # mul_abs_u_affine / in_subgroup_ref
    if not two:
        # G1 second ladder: Q1 = S1's (X, Y) is the affine base on the isomorphic curve; the
        # result's Z is multiplied by Q1's Z before the comparison (curve.hpp in_subgroup_fast_g1)
        S2 = M.ladder_invariant(F, S1[0], S1[1])
        z = M.mul(S2[2], S1[2], "Z'Z")
        beta_x = M.mul(base, M.normalized(1))
        ny = M.norm(M.subk(M.normalized(0), base, "KB_64_31"))
        M.jac_eq_affine(F, S2[0], S2[1], z, beta_x, ny)
    M.jac_eq_affine(F, *S1, base, base)


def test_g1_fast_ladders_w_closed():
    """The G1 fast ladders (curve.hpp in_subgroup_fast_g1: jac_tpl_affine_w / jac_dbl_w /
    jac_madd_w, W = 2Y): the base's w = 2y (a doubled normalized y), the second ladder's base is
    Q1 = (X, W) of the first, and the comparison is with (beta x, 2 (-y))."""
    base = M.normalized(Fraction(101, 100))
    w = M.shl(base, 1, "2y")
    S1 = M.ladder_invariant_w(base, w)
    S2 = M.ladder_invariant_w(S1[0], S1[1])
    z = M.mul(S2[2], S1[2], "Z'Z")
    beta_x = M.mul(base, M.normalized(1))
    nw = M.shl(M.norm(M.subk(M.normalized(0), base, "KB_64_31")), 1, "-2y")
    M.jac_eq_affine(M.Field(False), S2[0], S2[1], z, beta_x, nw)


def _pow_pm3d4(a):
    """fp_pow_pm3d4: table a, a^3, .., a^15 (via a^2), then squarings / table multiplies.
    BLS12-381 runs its own table on the radix-2^30 core (fp_pow_pm3d4_30, proven in tests/test_fp30.py for any
    input with limbs < 2^32 - 16 and value < 2^383); its output is canonical."""
    if M.NL == 14:
        assert max(a.limbs) < (1 << 32) - 16 and a.val * M.P < 2 ** 383, a
        return M.normalized(1)
    a2 = M.sqr(a, "a^2")
    t = M.mul(a, a2, "tab")
    for _ in range(8):
        t = M.vmax(t, M.mul(t, a2, "tab"))
    acc = t
    for _ in range(460):
        acc = M.vmax(M.sqr(acc, "sq"), M.mul(acc, t, "mul"))
    return acc


def test_sqrt_chain_inputs():
    # G1 decompress: x < 2^381 < 1.24 p (range check happens in parallel), a = x^3 + 4
    x = M.normalized(Fraction(124, 100))
    xm = M.mul(x, M.normalized(1), "to_mont")
    a = M.add_nr(M.mul(M.mul(xm, xm), xm), M.normalized(1))
    t = _pow_pm3d4(a)
    y = M.mul(t, a, "y")
    M.canon_ok(M.subk(M.mul(y, y), a, "KB_64_31"), "fp_eq")
    M.from_mont_ok(y)
    M.reduce_once_ok(y, "k_g1_codec: the ladder's Montgomery y")


def _fp2_mont(v):
    return M.mul(M.normalized(v), M.normalized(1), "to_mont")


def test_fp2_sqrt_and_psi():
    # G2 decompress (codec_kernels.hip k_g2_decompress / fp2_sqrt): everything reduced
    xm = M.V2(_fp2_mont(Fraction(124, 100)), _fp2_mont(Fraction(124, 100)))
    four = M.normalized(Fraction(1))
    a = M.f2_mul(M.f2_sqr(xm), xm)
    a = M.V2(M.add_red(a.c0, four), M.add_red(a.c1, four))
    nrm = M.add_nr(M.mul(a.c0, a.c0), M.mul(a.c1, a.c1))
    gam = M.mul(_pow_pm3d4(nrm), nrm, "gam")
    M.canon_ok(M.subk(M.mul(gam, gam), nrm, "KB_64_31"), "gam^2 == N")
    d = M.half(M.norm(M.add_nr(a.c0, gam)), "d")  # fp_half((a0 + gam) normalized)
    d = M.vmax(d, a.c0)
    t = _pow_pm3d4(d)
    s = M.mul(t, d, "s")
    M.canon_ok(M.subk(M.mul(s, s), d, "KB_64_31"), "s^2 == d")
    h = M.mul(M.half(a.c1, "a1/2"), t, "h")
    nh = M.sub_red(M.normalized(0), h, "-h")
    y = M.V2(M.vmax(s, nh), M.vmax(h, s))
    for c in (y.c0, y.c1):
        M.from_mont_ok(c)
        M.reduce_once_ok(c, "k_g2_codec: the ladder's Montgomery y")
    # G2 check kernel: on-curve test and psi(P) with canonical (range-checked) inputs
    pm = M.V2(_fp2_mont(1), _fp2_mont(1))
    lhs = M.f2_sqr(pm)
    rhs = M.f2_mul(M.f2_sqr(pm), pm)
    rhs = M.V2(M.add_red(rhs.c0, four), M.add_red(rhs.c1, four))
    M.canon_ok(M.sub_red(lhs.c0, rhs.c0), "on-curve")
    cx1 = M.normalized(1)
    px = M.V2(M.mul(pm.c1, cx1), M.mul(pm.c0, cx1))
    py = M.V2(pm.c0, M.sub_red(M.normalized(0), pm.c1))
    py = M.f2_mul(py, M.V2(M.normalized(1), M.normalized(1)))
    py = M.V2(M.sub_red(M.normalized(0), py.c0), M.sub_red(M.normalized(0), py.c1))
    S1 = M.ladder_invariant_fp2_lz(pm, pm)
    M.jac_eq_affine_fp2_lz(*S1, px, py)


def test_g2_lazy_ladder_closed():
    """G2 ladders (mul_abs_u_affine / in_subgroup_ref over Fp2) in the carry-free discipline:
    curve.hpp jac_dbl(jac<fp2>&) / jac_madd(jac<fp2>&, ..) / jac_eq_affine(jac<fp2>, ..)."""
    base = M.V2(M.normalized(Fraction(101, 100)), M.normalized(Fraction(101, 100)))
    S = M.ladder_invariant_fp2_lz(base, base)
    M.jac_eq_affine_fp2_lz(*S, base, base)
    # psi(P) and -y are reduced (< 2p) values from the generic Fp2 helpers: within the same bound
    red = M.V2(M.reduced(), M.reduced())
    M.jac_eq_affine_fp2_lz(*S, red, red)


def test_g2_fast_ladder_w_closed():
    """The G2 fast ladder (in_subgroup_fast_g2) in W = 2Y form: base (x, 2y), compared with
    (x', 2 y') for psi's output (x', y') reduced."""
    base = M.V2(M.normalized(Fraction(101, 100)), M.normalized(Fraction(101, 100)))
    w = M.V2(M.shl(base.c0, 1), M.shl(base.c1, 1))
    S = M.ladder_invariant_fp2_w(base, w)
    red = M.V2(M.reduced(), M.reduced())
    M.jac_eq_affine_fp2_lz(*S, red, M.V2(M.shl(red.c0, 1), M.shl(red.c1, 1)))


def test_g2_synth_madd_chain_lazy():
    """k_synth<fp2> (synth_kernels.hip): back-to-back lazy Fp2 mixed additions of table points,
    then to_affine's reduced-discipline inverse and multiplies (inputs normalized, any value)."""
    base = M.V2(M.normalized(Fraction(101, 100)), M.normalized(Fraction(101, 100)))
    S = (base, base, M.V2(M.normalized(1), M.normalized(0)))
    for _ in range(40):
        T = M.jac_madd_fp2_lz(*S, base, base)
        T = tuple(M.V2(M.vmax(a.c0, b.c0), M.vmax(a.c1, b.c1)) for a, b in zip(S, T))
        if all(M._within(M.Field(True), a, b) for a, b in zip(T, S)):
            break
        S = tuple(M.V2(M._inflate1(t.c0, 1.01), M._inflate1(t.c1, 1.01)) for t in T)
    else:
        raise AssertionError("lazy fp2 madd chain bound set not closed")
    X, Y, Z = S
    for c in (X.c0, X.c1, Y.c0, Y.c1):  # f_mul(x, p.x, z2) with z2 reduced: a mul_sum2 on normalized limbs
        M.reduce_once_ok(M.mul_sum2(c, M.reduced(), c, M.subk(M.normalized(0), M.reduced(), "KB_4_28")))
    for c in (Z.c0, Z.c1):  # f_inv: fp_sqr of each component, then a normalized sum
        M.sqr(c)


def test_bounds_model_catches_overflow():
    wide = M.V([(1 << 31) - 1] * M.NL, 100)
    with pytest.raises(M.BoundError):
        M.mul(wide, wide)
    with pytest.raises(M.BoundError):
        M.subk(M.normalized(1), wide, "KB_2_28")


def test_synth_madd_chain():
    """k_synth (synth_kernels.hip): 31 back-to-back mixed additions of table points (no doubling
    in between), then to_affine. Bound set closed under madd alone."""
    F = M.Field(False)
    base = M.normalized(Fraction(101, 100))
    S = (base, base, M.normalized(1))
    for _ in range(40):
        T = M.jac_madd(F, *S, base, base)
        T = tuple(M.join(F, a, b) for a, b in zip(S, T))
        if all(M._within(F, a, b) for a, b in zip(T, S)):
            break
        S = tuple(M._inflate(F, t) for t in T)
    else:
        raise AssertionError("madd chain bound set not closed")
    X, Y, Z = S
    zi = _pow_pm3d4(Z)
    zi = M.mul(M.mul(M.mul(zi, zi), zi), Z, "inv")
    z2 = M.mul(zi, zi)
    M.from_mont_ok(M.mul(X, z2), "x")
    M.from_mont_ok(M.mul(Y, M.mul(z2, zi)), "y")


def _ark_word_consts():
    """FP_ARK_WORD as bls12_381_consts.hpp holds it, checked against its definition."""
    import re

    text = open(os.path.join(os.path.dirname(__file__), "..", "kzg-setup-powersoftau_amd", "csrc",
                             "bls12_381_consts.hpp")).read()
    body = re.search(r"FP_ARK_WORD\[12\]\[14\] = \{(.*?)\};", text).group(1)
    rows = [[int(v.strip().rstrip("u"), 16) for v in r.split(",")] for r in re.findall(r"\{([^{}]*)\}", body)]
    p, mask = M.P, (1 << 28) - 1
    for k, row in enumerate(rows):
        assert row == [((1 << (384 + 56 + 32 * k)) % p >> (28 * j)) & mask for j in range(14)]
    return rows


def test_loader_conversion():
    """load_kernels.hip words_to_ark_mont: S = sum_k x_k C_k over the 12 input words, two
    Montgomery digit steps, one conditional subtraction. Worst case over ANY 384-bit input (every
    word 2^32 - 1, every digit m < 2^28): no 64-bit column overflows and the value stays < 2p;
    then the exact device steps on random and edge inputs reproduce x 2^384 mod p."""
    C = _ark_word_consts()
    p = M.P
    pl = [(p >> (28 * j)) & ((1 << 28) - 1) for j in range(14)]
    wmax, mmax = (1 << 32) - 1, (1 << 28) - 1
    col = [sum(wmax * C[k][j] for k in range(12)) for j in range(14)] + [0]
    for s in range(2):  # digit steps: m p added, then the column's carry (< col >> 28) moves up
        for j in range(14):
            col[s + j] += mmax * pl[j]
        col[s + 1] += col[s] >> 28
    assert max(col) < 1 << 64
    c = 0
    for k in range(13):  # normalization carries
        c += col[k + 2]
        assert c < 1 << 64
        c >>= 28
    assert c < 1 << 32
    # value: S < 12 2^32 p, so (S + m0 p + m1 p 2^28) / 2^56 < 2p for every input
    assert (12 * (1 << 32) * p + mmax * p + mmax * p * (1 << 28)) < 2 * p * (1 << 56)

    pinv = (-pow(p, -1, 1 << 28)) % (1 << 28)
    rng = random.Random(384)
    for i in range(3000):
        x = [0, 1, p - 1, p, (1 << 384) - 1][i] if i < 5 else (rng.randrange(p) if i % 4 else rng.randrange(1 << 384))
        w = [(x >> (32 * k)) & 0xFFFFFFFF for k in range(12)]
        col = [sum(w[k] * C[k][j] for k in range(12)) for j in range(14)] + [0]
        for s in range(2):
            m = ((col[s] & 0xFFFFFFFF) * pinv) & ((1 << 28) - 1)
            for j in range(14):
                col[s + j] += m * pl[j]
            assert col[s] & ((1 << 28) - 1) == 0
            col[s + 1] += col[s] >> 28
        v = sum(col[k + 2] << (28 * k) for k in range(13))
        assert v < 2 * p
        v = v - p if v >= p else v
        if x < p:
            assert v == x * (1 << 384) % p


@pytest.fixture
def bn254_model():
    M.use_field("bn254")
    yield M
    M.use_field("bls12_381")


def test_bn254_decompress_chain(bn254_model):
    """bn254_kernels.hip: x < 2^254 (< 1.33 p), a = x^3 + 3, the (p-3)/4 chain, y^2 == a
    against KB_EQ (= 8p, borrowed with 2^28 limbs), from_mont; ark Montgomery output."""
    x = M.normalized(Fraction(133, 100))
    xm = M.mul(x, M.normalized(1), "to_mont")
    a = M.norm(M.add_nr(M.mul(M.sqr(xm), xm), M.normalized(1)))
    t = _pow_pm3d4(a)
    y = M.mul(t, a, "y")
    M.canon_ok(M.subk(M.sqr(y), a, "KB_EQ"), "fp_eq")
    M.from_mont_ok(y)
    M.reduce_once_ok(M.mul(M.normalized(1), M.const(M.C["BN_ARK_R"])))
