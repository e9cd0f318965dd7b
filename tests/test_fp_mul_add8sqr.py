"""csrc/fp381.hpp fp_mul_add8sqr — (a b + 8 c^2) R^-1 mod p in one column scan, the c^2 half as a
squaring (cross products c_j (16 c_k) once, squares c_j (8 c_j)) — modelled step by step on Python
integers with every 64-bit accumulator checked, against plain modular arithmetic, at the operand
bounds the G1 doubling feeds it (curve.hpp jac_dbl: a = E normalized, b = F - 3D + KB_8_30 with limbs
below 2^30 + 2^28, c = B normalized). CPU only; the column bounds for the whole ladder are proven in
tests/test_field_bounds.py (field_bounds_model.mul_add8sqr)."""
import random

import pytest

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
N, LB = 14, 28
MASK = (1 << LB) - 1
PL = [(P >> (LB * i)) & MASK for i in range(N)]
PINV = (-pow(P, -1, 1 << LB)) % (1 << LB)
R = 1 << (LB * N)


def u64(x, what):
    if not 0 <= x < 1 << 64:
        raise OverflowError(f"{what}: {x:#x} leaves uint64")
    return x


def mul_add8sqr(a, b, c, scale=8):
    c8 = [x * scale for x in c]
    c16 = [x * 2 * scale for x in c]
    assert all(x < 1 << 32 for x in c16)
    m, r, acc = [0] * N, [0] * N, 0
    for i in range(2 * N):
        j0 = 0 if i < N else i - (N - 1)
        j1 = i - 1 if i < N else N - 1
        acc2 = accp = 0
        for j in range(j0, j1 + 1):
            acc = u64(acc + a[j] * b[i - j], "acc")
            accp = u64(accp + m[j] * PL[i - j], "accp")
        for j in range(j0, i):
            if 2 * j < i and i - j < N:
                acc2 = u64(acc2 + c[j] * c16[i - j], "acc2")
        if i % 2 == 0 and i // 2 < N:
            acc2 = u64(acc2 + c[i // 2] * c8[i // 2], "acc2")
        if i < N:
            acc = u64(acc + a[i] * b[0], "acc")
            acc = u64(acc + acc2 + accp, "acc")
            m[i] = ((acc & 0xFFFFFFFF) * PINV) & MASK
            acc = u64(acc + m[i] * PL[0], "acc")
            assert acc & MASK == 0
        else:
            acc = u64(acc + acc2 + accp, "acc")
            r[i - N] = acc & MASK
        acc >>= LB
    return r


def val(limbs):
    return sum(x << (LB * k) for k, x in enumerate(limbs))


def rand_limbs(rng, limb_max, top_max):
    return [rng.randrange(limb_max + 1) for _ in range(N - 1)] + [rng.randrange(top_max + 1)]


@pytest.mark.parametrize("scale", [8, 1])
def test_mul_add8sqr_exact(scale):
    """scale 8: fp_mul_addsqr<8> (the Y-form doubling); scale 1: fp_mul_addsqr<1> (jac_dbl_w, whose
    b = 2 (X3 - D) has limbs below 2^31 + 2^29)."""
    rng = random.Random(8 + scale)
    top_n = (3 * P) >> (LB * (N - 1))          # normalized operands: values below ~3 p
    a_max, b_max = MASK, (1 << 30) + (1 << 28)  # E normalized; F - 3D + KB_8_30 lazy
    if scale == 1:
        b_max = 2 * b_max  # doubled
    cases = [([MASK] * (N - 1) + [top_n], [b_max] * (N - 1) + [top_n << 3], [MASK] * (N - 1) + [top_n])]
    for _ in range(400):
        cases.append((rand_limbs(rng, a_max, top_n), rand_limbs(rng, b_max, top_n << 3), rand_limbs(rng, MASK, top_n)))
    for a, b, c in cases:
        r = mul_add8sqr(a, b, c, scale)
        assert all(x <= MASK for x in r)
        assert (val(r) * R - (val(a) * val(b) + scale * val(c) ** 2)) % P == 0
