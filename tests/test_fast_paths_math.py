"""The GPU replaces two reference algorithms by faster EQUIVALENT ones; this pins the
equivalence on the CPU, independently of the kernels.

1. Subgroup test. Reference: [r]P == O by ark double-and-add. GPU: G1 φ(P) == [-u²]P,
   G2 ψ(P) == [u]P. Both accept exactly the order-r subgroup among points ON the curve:
   * G1: on E(Fp)[ℓ] for every ℓ | h1 we have u ≡ 1 (mod ℓ), so φ + [u²] acts as φ + 1; an
     eigenvalue -1 of φ would need (-1)² + (-1) + 1 ≡ 0 (mod ℓ) — impossible.
   * G2: ψ satisfies ψ² - tψ + p = 0; an eigenvector with eigenvalue u forces
     ℓ | u² - tu + p = p - u = h1·r, but gcd(h2, h1·r) = 1.
2. Fp2 square root. Reference: Algorithm 9 (two Fp2 exponentiations, data-dependent branches).
   GPU: a norm-based root from two Fp exponentiations. Any root is fine because the sign rule
   normalises it; accept/reject must agree (a is a square in Fp2 iff N(a) is a square in Fp).
"""
import math
import random

import kzgpot_oracle as O
import pytest

P = O.P


def g1_fast(pt):
    """Restatement of in_subgroup_fast_g1 (curve.hpp) on an affine on-curve point."""
    beta = 0x5F19672FDF76CE51BA69C6076A0F77EADDB3A93BE6F89688DE17D813620A00022E01FFFFFFFEFFFE
    q = O.g1_mul(O.g1_mul(pt, -O.U_PARAM), -O.U_PARAM)  # [|u|]([|u|]P) = [u²]P
    return q == (beta * pt[0] % P, (-pt[1]) % P)


def g2_fast(pt):
    """Restatement of in_subgroup_fast_g2: [|u|]P == -ψ(P)."""
    cx = O.fp2_inv(O.fp2_pow((1, 1), (P - 1) // 3))
    cy = O.fp2_inv(O.fp2_pow((1, 1), (P - 1) // 2))
    psi = (O.fp2_mul(O.fp2_conj(pt[0]), cx), O.fp2_mul(O.fp2_conj(pt[1]), cy))
    return O.g2_mul(pt, -O.U_PARAM) == (psi[0], O.fp2_neg(psi[1]))


def g1_ref(pt):
    return O.ark_mul_bits_is_zero(O._Fp, pt[0], pt[1], False)


def g2_ref(pt):
    return O.ark_mul_bits_is_zero(O._Fp2, pt[0], pt[1], False)


def test_soundness_arguments():
    h1_primes = [3, 11, 10177, 859267, 52437899]
    assert math.prod(p ** (1 if p == 3 else 2) for p in h1_primes) == O.H1
    for ell in h1_primes:
        assert (O.U_PARAM - 1) % ell == 0             # u ≡ 1 (mod ℓ)
        assert (1 - 1 + 1) % ell != 0                 # -1 is never a root of x² + x + 1
    t = O.U_PARAM + 1
    assert O.P - O.U_PARAM == O.H1 * O.R_ORDER        # u² - t u + p = p - u
    assert math.gcd(O.H2, O.H1 * O.R_ORDER) == 1
    assert (O.U_PARAM * O.U_PARAM - t * O.U_PARAM + O.P) == O.P - O.U_PARAM


def test_endomorphisms_on_generators():
    assert g1_fast(O.G1_GEN) and g1_ref(O.G1_GEN)
    assert g2_fast(O.G2_GEN) and g2_ref(O.G2_GEN)


def test_fast_equals_ref_on_adversarial_points():
    from golden.make_golden import small_order_g1, small_order_g2

    rng = random.Random(7)
    cases1 = [O.g1_mul(O.G1_GEN, rng.randrange(1, O.R_ORDER)) for _ in range(4)]
    cases1 += [O.g1_random_on_curve(rng) for _ in range(4)]
    for ell in (3, 11, 10177):
        t = small_order_g1(rng, ell)
        cases1 += [t, O.g1_add(O.g1_mul(O.G1_GEN, rng.randrange(1, O.R_ORDER)), t)]
    for pt in cases1:
        assert g1_fast(pt) == g1_ref(pt)
    cases2 = [O.g2_mul(O.G2_GEN, rng.randrange(1, O.R_ORDER)) for _ in range(2)]
    cases2 += [O.g2_random_on_curve(rng) for _ in range(2)]
    t = small_order_g2(rng, 13)
    cases2 += [t, O.g2_add(O.g2_mul(O.G2_GEN, 5), t)]
    for pt in cases2:
        assert g2_fast(pt) == g2_ref(pt)


def _half(v):
    """fp_half: + p if odd, then >> 1 (the element v / 2)."""
    return (v + (P if v & 1 else 0)) >> 1


def fp2_sqrt_norm(a, accept_by_y2=False):
    """Restatement of fp2_sqrt (codec_kernels.hip): accepted iff gam^2 == N (accept_by_y2: the
    earlier y^2 == a test instead, for the equivalence check below)."""
    a0, a1 = a
    nrm = (a0 * a0 + a1 * a1) % P
    gam = pow(nrm, (P - 3) // 4, P) * nrm % P
    square = gam * gam % P == nrm
    d = _half((a0 + gam) % P)
    if d == 0:
        d = a0
    t = pow(d, (P - 3) // 4, P)
    s = t * d % P
    h = _half(a1) * t % P
    y = (s, h) if s * s % P == d else ((-h) % P, s)
    ok = O.fp2_sqr(y) == (a0 % P, a1 % P) if accept_by_y2 else square
    return y if ok else None


def _fp2_sqrt_cases(rng):
    cases = [(0, 0), (1, 0), (P - 1, 0), (0, 1), (0, P - 1), (4, 0), (5, 0), (0, 7), (2, 0), (P - 2, 0)]
    cases += [(rng.randrange(P), rng.randrange(P)) for _ in range(60)]
    cases += [(rng.randrange(P), 0) for _ in range(10)] + [(0, rng.randrange(P)) for _ in range(10)]
    # squares (a0 + gam = 0 happens for a = (-c^2, 0): N = c^4, gam = c^2 or -c^2)
    for _ in range(10):
        c = rng.randrange(1, P)
        cases += [((-c * c) % P, 0), (c * c % P, 0), O.fp2_sqr((rng.randrange(P), rng.randrange(P)))]
    return cases


def test_fp2_sqrt_equivalence():
    rng = random.Random(11)
    for a in _fp2_sqrt_cases(rng):
        ref = O.fq2_sqrt(a)
        got = fp2_sqrt_norm(a)
        assert (ref is None) == (got is None), a
        if ref is not None:
            assert got in (ref, O.fp2_neg(ref))


def test_fp2_sqrt_norm_test_equals_y2_test():
    """The kernel accepts a iff gam^2 == N; the y^2 == a test it replaced decides the same for
    every a (codec_kernels.hip fp2_sqrt's derivation), including d = a0 + gam = 0 and a1 = 0."""
    rng = random.Random(12)
    cases = _fp2_sqrt_cases(rng)
    for a in cases:
        assert (fp2_sqrt_norm(a) is None) == (fp2_sqrt_norm(a, accept_by_y2=True) is None), a
        got = fp2_sqrt_norm(a)
        if got is not None:
            assert O.fp2_sqr(got) == (a[0] % P, a[1] % P), a
    hits = sum(1 for a in cases if (a[0] + pow((a[0] ** 2 + a[1] ** 2) % P, (P + 1) // 4, P)) % P == 0)
    assert hits > 0  # the d = 0 fallback is exercised


def test_half_is_division_by_two():
    rng = random.Random(13)
    inv2 = pow(2, P - 2, P)
    for v in [0, 1, 2, P - 1, P, P + 1, 2 * P - 1, 3 * P - 2] + [rng.randrange(3 * P) for _ in range(200)]:
        h = _half(v)
        assert h % P == v * inv2 % P and h <= (v + P) // 2


@pytest.mark.parametrize("hdr,nl,lb", [("bls12_381_consts.hpp", 14, 28), ("bn254_consts.hpp", 9, 29)])
def test_is_zero_low_limb_filter(hdr, nl, lb):
    """fp381.hpp fp_is_zero's filter: k_c = (a.v[0] mod 2^lb) (-PINV) mod 2^lb equals k for every
    a = k p (so no zero is filtered out, whatever the unnormalized limbs above limb 0 hold), and
    random nonzero values pass it (k_c < 256) about 256 / 2^lb of the time."""
    import os
    import random
    import re

    text = open(os.path.join(os.path.dirname(__file__), "..", "kzg-setup-powersoftau_amd", "csrc", hdr)).read()
    pinv = int(re.search(r"PINV = (0x[0-9a-f]+)u;", text).group(1), 16)
    body = re.search(r"uint32_t P\[\d+\] = \{([^}]*)\}", text).group(1)
    limbs = [int(v.strip().rstrip("u"), 16) for v in body.split(",")]
    p = sum(v << (lb * i) for i, v in enumerate(limbs))
    mask = (1 << lb) - 1
    assert (p * pinv + 1) & mask == 0

    def kc(limb0):
        return ((limb0 & mask) * ((0 - pinv) & 0xFFFFFFFF) & 0xFFFFFFFF) & mask

    rng = random.Random(9)
    for k in range(256):
        a = k * p
        assert kc(a & mask) == k
        # the same value with a carry left in limb 0 (limb 0 + 2^lb, limb 1 - 1): limb 0 mod 2^lb is unchanged
        assert kc((a & mask) + (1 << lb)) == k
    hits = sum(kc(rng.randrange(1 << 32)) < 256 for _ in range(200000))
    assert hits < 200000 * 256 / (1 << lb) * 3 + 5


@pytest.mark.parametrize("hdr,nl,lb", [("bls12_381_consts.hpp", 14, 28), ("bn254_consts.hpp", 9, 29)])
def test_is_zero_quotient_estimate(hdr, nl, lb):
    """fp381.hpp fp_is_zero: for every normalized a < min(256 p, R), a == k p with
    k = trunc((top + 1) * INV_RHO) (IEEE double, as on the GPU) iff a == 0 mod p."""
    import os
    import random
    import re

    text = open(os.path.join(os.path.dirname(__file__), "..", "kzg-setup-powersoftau_amd", "csrc", hdr)).read()
    inv_rho = float(re.search(r"INV_RHO = ([0-9.e+-]+);", text).group(1))
    body = re.search(r"uint32_t P\[\d+\] = \{([^}]*)\}", text).group(1)
    limbs = [int(v.strip().rstrip("u"), 16) for v in body.split(",")]
    p = sum(v << (lb * i) for i, v in enumerate(limbs))
    sh = lb * (nl - 1)
    kmax = min(256, (1 << (lb * nl)) // p)

    def is_zero(a):
        top = a >> sh
        k = int(float(top + 1) * inv_rho)
        return a == k * p

    rng = random.Random(5)
    for k in range(kmax):
        assert is_zero(k * p)
        for d in (1, -1, 1 << lb, 1 << sh, -(1 << sh), rng.randrange(1, p)):
            a = k * p + d
            if 0 <= a < kmax * p:
                assert not is_zero(a)
    for _ in range(2000):
        a = rng.randrange(kmax * p)
        assert is_zero(a) == (a % p == 0)
