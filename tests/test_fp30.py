"""The radix-2^30 balanced core of csrc/fp381.hpp (f30_mul, f30_sqr, f30_from_fp, fp_from_f30,
fp_pow_pm3d4_30: BLS12-381's square-root exponentiation), CPU only.

1. Worst-case column bounds: with the ACTUAL balanced digits of p, every column sum of f30_mul /
   f30_sqr stays inside int64 for every input whose digits are balanced (|d| <= 2^29) and whose top
   digit is < 2^23 (f30_from_fp of any value < 2^383, and every f30 product output).
2. An exact model: the device functions step by step on Python integers, with every 64-bit
   accumulator checked against the int64 range, against plain modular arithmetic — the
   exponentiation (same schedule as the header) on random and edge inputs, and the conversions.
"""
import os
import random
import re

import pytest

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
HERE = os.path.dirname(os.path.abspath(__file__))
HDR = os.path.join(HERE, "..", "kzg-setup-powersoftau_amd", "csrc", "bls12_381_consts.hpp")
N = 13
M30 = (1 << 30) - 1
R30 = 1 << 390
R28 = 1 << 392
E = (P - 3) // 4
TOP_IN = (1 << 23) + 1  # |top digit| < TOP_IN for every f30 operand (see test_top_digit_bounds)


def _consts():
    text = open(HDR).read()
    s32 = {n: [int(v) for v in b.split(",")]
           for n, b in re.findall(r"static constexpr int32_t (\w+)\[\d+\] = \{([^}]*)\}", text)}
    pinv = int(re.search(r"PINV30 = 0x([0-9a-f]+)u", text).group(1), 16)
    steps_sq = [int(v) for v in re.search(r"SQRT_STEP_SQ\[SQRT_STEPS\] = \{([^}]*)\}", text).group(1).split(",")]
    steps_idx = [int(v) for v in re.search(r"SQRT_STEP_IDX\[SQRT_STEPS\] = \{([^}]*)\}", text).group(1).split(",")]
    table = [int(v) for v in re.search(r"SQRT_TABLE_EXP\[SQRT_TABLE\] = \{([^}]*)\}", text).group(1).split(",")]
    return s32["P30"], pinv, s32["POW30_OUT"], steps_sq, steps_idx, table


P30, PINV30, POW30_OUT, STEP_SQ, STEP_IDX, TABLE_EXP = _consts()


def val(d):
    return sum(v << (30 * k) for k, v in enumerate(d))


def s64(x, what):
    if not -(1 << 63) <= x < (1 << 63):
        raise OverflowError(f"{what}: {x:#x} leaves int64")
    return x


def sext30(x):
    x &= M30
    return x - (1 << 30) if x >= 1 << 29 else x


def f30_mul(a, b, sq=False):
    """fp381.hpp f30_mul / f30_sqr, column by column (the compiler may re-associate the sums of
    one column; every partial sum is bounded by the sum of absolute values checked in
    test_worst_case_columns)."""
    m = [0] * N
    r = [0] * N
    acc = 0
    for i in range(2 * N - 1):
        j0 = 0 if i < N else i - (N - 1)
        j1 = i - 1 if i < N else N - 1
        accab = 0 if i < N else 1 << 29
        if sq:
            d = [2 * x for x in a]
            for j in range(j0, i):
                if 2 * j < i:
                    accab = s64(accab + a[j] * d[i - j], "ab")
            if i % 2 == 0:
                accab = s64(accab + a[i // 2] * a[i // 2], "ab")
        else:
            for j in range(j0, j1 + 1):
                accab = s64(accab + a[j] * b[i - j], "ab")
        accp = 0
        for j in range(j0, j1 + 1):
            accp = s64(accp + m[j] * P30[i - j], "mp")
        acc = s64(acc + accab, "acc")
        if i < N:
            if not sq:
                acc = s64(acc + a[i] * b[0], "acc")
            acc = s64(acc + accp, "acc")
            m[i] = sext30((acc & 0xFFFFFFFF) * PINV30)
            acc = s64(acc + m[i] * P30[0], "acc")
            assert acc % (1 << 30) == 0
        else:
            acc = s64(acc + accp, "acc")
            r[i - N] = (acc & M30) - (1 << 29)
        acc >>= 30
    r[N - 1] = acc
    return r


def f30_from_fp(limbs28):
    """fp_norm (carry to 28-bit limbs, top keeps the excess), then 30-bit digits, balanced."""
    n, c = [], 0
    for k in range(13):
        t = limbs28[k] + c
        n.append(t & ((1 << 28) - 1))
        c = t >> 28
    n.append(limbs28[13] + c)
    assert all(x < 1 << 32 for x in n)
    r, c = [], 0
    for k in range(N):
        bit = 30 * k
        i, off = bit // 28, bit % 28
        u = (n[i] >> off) | ((n[i + 1] << (28 - off)) & 0xFFFFFFFF if i + 1 < 14 else 0)
        u &= 0xFFFFFFFF
        if k < N - 1:
            t = (u & M30) + c
            c = (t + (1 << 29)) >> 30
            r.append(sext30(t))
        else:
            r.append(u + c)
    return r


def fp_from_f30(z):
    u, c = [], 0
    for k in range(N):
        t = z[k] + P30[k] + c
        assert -(1 << 31) <= t < (1 << 31)
        if k < N - 1:
            u.append(t & M30)
            c = t >> 30
        else:
            assert t >= 0
            u.append(t)
    limbs = []
    for j in range(14):
        bit = 28 * j
        i, off = bit // 30, bit % 30
        v = u[i] >> off
        if off > 2 and i + 1 < N:
            v |= (u[i + 1] << (30 - off)) & 0xFFFFFFFF
        limbs.append(v & ((1 << 28) - 1) if j < 13 else v)
    x = sum(l << (28 * j) for j, l in enumerate(limbs))
    assert x < 2 * P
    return x - P if x >= P else x


def pow_pm3d4_30(limbs28):
    """fp_pow_pm3d4_30 step by step: the table chain (a, a^3, a^7, a^9, a^11, a^13, a^21, a^255), the
    header's windows over it, and the radix conversion."""
    a = f30_from_fp(limbs28)
    a2 = f30_mul(a, a, sq=True)
    t = f30_mul(a, a2)                 # a^3
    tab = [a, t]
    a4 = f30_mul(a2, a2, sq=True)
    t = f30_mul(t, a4)                 # a^7
    tab.append(t)
    for _ in range(3):                 # a^9, a^11, a^13
        t = f30_mul(t, a2)
        tab.append(t)
    a8 = f30_mul(a4, a4, sq=True)
    tab.append(f30_mul(t, a8))         # a^21
    t = f30_mul(t, a2)                 # a^15
    u = t
    for _ in range(4):
        u = f30_mul(u, u, sq=True)     # a^240
    tab.append(f30_mul(u, t))          # a^255
    acc = tab[STEP_IDX[0]]
    for nsq, idx in zip(STEP_SQ[1:], STEP_IDX[1:]):
        for _ in range(nsq):
            acc = f30_mul(acc, acc, sq=True)
        if idx >= 0:
            acc = f30_mul(acc, tab[idx])
    return fp_from_f30(f30_mul(acc, POW30_OUT))


def limbs28(x, loose=False, rng=None):
    """x as 14 limbs of 28 bits; loose: push random multiples of 2^28 down into lower limbs
    (limbs up to 2^30, same value), as the kernels' lazy sums produce."""
    lim = [(x >> (28 * k)) & ((1 << 28) - 1) for k in range(13)] + [x >> 364]
    if loose:
        for k in range(13, 0, -1):
            take = min(lim[k], rng.randrange(4))
            lim[k] -= take
            lim[k - 1] += take << 28
    return lim


def test_constants():
    assert val(P30) == P and all(-(1 << 29) <= d < (1 << 29) for d in P30)
    assert (PINV30 * P) % (1 << 30) == (1 << 30) - 1
    assert val(POW30_OUT) == R28 * pow(4, -E, P) % P
    # the header's table is the one pow_pm3d4_30 (and fp_pow_pm3d4_30) builds, and its windows
    # spell (p-3)/4
    assert TABLE_EXP == [1, 3, 7, 9, 11, 13, 21, 255]
    acc = TABLE_EXP[STEP_IDX[0]]
    for nsq, idx in zip(STEP_SQ[1:], STEP_IDX[1:]):
        acc = (acc << nsq) + (TABLE_EXP[idx] if idx >= 0 else 0)
    assert acc == E


def test_worst_case_columns():
    """|column| < 2^63 for every balanced input with top digits < TOP_IN: sum of |products| over
    the column, |m| <= 2^29 against the actual digits of p, the incoming carry, the bias."""
    dig = [1 << 29] * (N - 1) + [TOP_IN]
    worst, carry = 0, 0
    for i in range(2 * N - 1):
        j0 = 0 if i < N else i - (N - 1)
        j1 = i if i < N else N - 1
        ab = sum(dig[j] * dig[i - j] for j in range(j0, j1 + 1))
        mp = sum((1 << 29) * abs(P30[i - j]) for j in range(j0, j1 + 1))
        tot = carry + ab + mp + (1 << 29)
        worst = max(worst, tot)
        carry = (tot >> 30) + 1
    assert worst < 1 << 63, f"2^{worst.bit_length()}"
    # margin for the record: the tightest column uses about 2^62.x
    assert worst.bit_length() <= 63


def test_top_digit_bounds():
    """Every f30 operand has |top digit| <= 2^23: f30_from_fp of a value < 2^383 (fp_pow's inputs:
    x^3 + 4 < 2.01 p, the Fp2 norm < 2.01 p, d < 1.01 p, synth's Z < 1.01 p, all < 2^383), and
    products (|value| < p/2 + |a||b|/R30 < 0.51 p)."""
    lower = sum((1 << 29) << (30 * k) for k in range(N - 1))  # largest |lower-digit part|
    assert ((1 << 383) + lower) >> 360 < TOP_IN
    assert (int(0.51 * P) + lower) >> 360 < TOP_IN
    # product value bound with operands up to 2^383: |a||b| / R30 + p/2 stays < 2^383
    assert (1 << 383) * (1 << 383) // R30 + P < (1 << 383)


def test_mul_exact_random_and_extreme():
    rng = random.Random(30)
    cases = []
    for t in range(600):
        if t < 8:
            a = [((1 << 29) - 1 if (t + k) & 1 else -(1 << 29)) for k in range(N - 1)] + [TOP_IN - 1 if t & 2 else -(TOP_IN - 1)]
            b = [((1 << 29) - 1 if (t >> 1) & 1 else -(1 << 29))] * (N - 1) + [TOP_IN - 1]
        else:
            a = [rng.randrange(-(1 << 29), 1 << 29) for _ in range(N - 1)] + [rng.randrange(-(1 << 22), 1 << 22)]
            b = [rng.randrange(-(1 << 29), 1 << 29) for _ in range(N - 1)] + [rng.randrange(-(1 << 22), 1 << 22)]
        cases.append((a, b))
    for a, b in cases:
        for r, want in ((f30_mul(a, b), val(a) * val(b)), (f30_mul(a, a, sq=True), val(a) * val(a))):
            assert (val(r) * R30 - want) % P == 0
            assert all(-(1 << 29) <= d < (1 << 29) for d in r[:-1])
            assert abs(val(r)) < P // 2 + abs(want) // R30 + 1


def test_conversions_exact():
    rng = random.Random(31)
    for t in range(2000):
        x = [0, 1, P - 1, P, 2 * P + 5, (1 << 383) - 1][t] if t < 6 else rng.randrange(1 << 383)
        a = f30_from_fp(limbs28(x, loose=bool(t & 1), rng=rng))
        assert val(a) == x and all(-(1 << 29) <= d < (1 << 29) for d in a[:-1]) and abs(a[-1]) < TOP_IN
        z = rng.randrange(-(P - 1), P) if t >= 6 else [0, 1, -1, P - 1, -(P - 1), P // 2][t]
        zd, rest = [], z
        for k in range(N - 1):
            d = sext30(rest)
            zd.append(d)
            rest = (rest - d) >> 30
        zd.append(rest)
        assert fp_from_f30(zd) == z % P


def test_pow_exact():
    """The whole exponentiation: canonical (a 2^-392)^e 2^392 for Montgomery inputs a."""
    rng = random.Random(32)
    xs = [0, 1, P - 1, 4, P + 7, 2 * P - 1] + [rng.randrange(2 * P) for _ in range(14)]
    for t, x in enumerate(xs):
        got = pow_pm3d4_30(limbs28(x, loose=bool(t & 1), rng=rng))
        want = pow(x * pow(2, -392, P) % P, E, P) * R28 % P
        assert got == want, t


def test_model_catches_overflow():
    with pytest.raises(OverflowError):
        big = [1 << 31] * N
        f30_mul(big, big)
