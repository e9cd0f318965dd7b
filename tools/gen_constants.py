"""Emit kzg-setup-powersoftau_amd/csrc/bls12_381_consts.hpp (device constants for the HIP codec).

    python tools/gen_constants.py

Field representation (csrc/fp381.hpp): 14 limbs of 28 bits in 32-bit registers, Montgomery form
with R = 2^392. Everything here is derived from p, r and u (BLS12-381) and re-checked:
  * Montgomery constants (P, -p^-1 mod 2^28, R^2, and R*c for c = 1, 4, 1/2);
  * BETA: the cube root of unity for which phi(x, y) = (BETA x, y) acts as [-u^2] on G1;
  * PSI_CX1 / PSI_CY: psi(x, y) = (conj(x) (0 + CX1 u), conj(y) CY) acting as [u] on G2;
  * KB_c_L: c*p in a "borrowed" limb form whose limbs 0..12 are all >= 2^L - 2^(L-28), so that
    a + KB - b is a carry-free limb-wise subtraction for any b with limbs <= 2^L - 2^(L-28) and
    value < (c - 0.001) p;
  * the window schedule for a^((p-3)/4) (Fp square root and inverse square root): BLS12-381 over
    an 8-entry table chosen for its exponent, BN254 a w = 4 sliding window;
  * 32-bit words of p for byte-level range checks; generator points (synthetic data).
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import kzgpot_oracle as O  # noqa: E402

P, R, U = O.P, O.R_ORDER, O.U_PARAM
LB = 28                 # limb bits
NL = 14                 # limbs (BLS12-381)
RM = 1 << (LB * NL)     # Montgomery R = 2^392
W = 4                   # sqrt sliding window (BN254)
# BLS12-381's square-root table (fp381.hpp fp_pow_pm3d4_30 builds it): 8 odd powers in registers,
# chosen for (p-3)/4 (tools/sqrt_chain_search.py): 67 windows where the w = 4 sliding window takes
# 79, for 6 more squarings and 2 more multiplies to build the table
BLS_SQRT_TABLE = (1, 3, 7, 9, 11, 13, 21, 255)
# (c, L) borrowed multiples used by the formulas in csrc/curve.hpp / fp381.hpp
KB = [(2, 28), (4, 28), (8, 28), (8, 29), (16, 28), (32, 28), (32, 29), (64, 28), (64, 29), (64, 31), (128, 28), (128, 31),
      (4, 29), (8, 30), (16, 30), (64, 30), (16, 31)]  # the last five: the G2 ladders (curve.hpp, fp2)

# BN254 base field (config 5; ark-bn254 0.2 Fq): 10 x 28-bit limbs, R = 2^280
BN_P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
BN_R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
BN_NL = 9   # 9 x 29-bit limbs (261 bits for a 254-bit p): 81 products per multiply, not 100
BN_LB = 29


def limbs28(x, n=NL, lb=LB):
    return [(x >> (lb * i)) & ((1 << lb) - 1) for i in range(n)]


def words32(x, n=12):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def arr(name, vals, comment=""):
    s = f"static constexpr uint32_t {name}[{len(vals)}] = {{" + ", ".join(f"0x{v:08x}u" for v in vals) + "};"
    return s + (f"  // {comment}" if comment else "")


def balanced30(x, n=13):
    """x as n signed 30-bit digits in [-2^29, 2^29) (the last one takes the rest)."""
    d = []
    for k in range(n - 1):
        r = x & ((1 << 30) - 1)
        r -= (1 << 30) if r >= (1 << 29) else 0
        d.append(r)
        x = (x - r) >> 30
    d.append(x)
    assert -(1 << 29) <= x < (1 << 29)
    return d


def arr_s32(name, vals, comment=""):
    c = f"  // {comment}" if comment else ""
    return f"static constexpr int32_t {name}[{len(vals)}] = {{" + ", ".join(str(v) for v in vals) + "};" + c


def mont(x):
    return x * RM % P


def borrowed(c, L, p=None, nl=NL, vmax=None, lb=LB):
    """c p in the borrowed limb form; its top limb must dominate the top limb of any normalized
    subtrahend of value < vmax p (default c - 0.001)."""
    p = P if p is None else p
    vmax = c - 0.001 if vmax is None else vmax
    k = limbs28(c * p, nl, lb)
    assert sum(v << (lb * i) for i, v in enumerate(k)) == c * p
    hi, lo = 1 << L, 1 << (L - lb)
    out = list(k)
    out[0] += hi
    for i in range(1, nl - 1):
        out[i] += hi - lo
    out[nl - 1] -= lo
    assert sum(v << (lb * i) for i, v in enumerate(out)) == c * p
    assert all(0 <= v < (1 << 32) for v in out)
    assert min(out[: nl - 1]) >= hi - lo
    assert out[nl - 1] >= int(vmax * 1000) * p // 1000 >> (lb * (nl - 1)), (c, L)
    return out


def sliding_window(e, w):
    bits = bin(e)[2:]
    steps = []
    i = 0
    pending_sq = 0
    first = True
    while i < len(bits):
        if bits[i] == "0":
            pending_sq += 1
            i += 1
            continue
        j = min(i + w, len(bits))
        while bits[j - 1] == "0":
            j -= 1
        val = int(bits[i:j], 2)
        if first:
            assert pending_sq == 0
            steps.append((0, (val - 1) // 2))
            first = False
        else:
            steps.append((pending_sq + (j - i), (val - 1) // 2))
        pending_sq = 0
        i = j
    if pending_sq:
        steps.append((pending_sq, -1))
    acc = None
    for nsq, idx in steps:
        if acc is None:
            acc = 2 * idx + 1
            continue
        acc <<= nsq
        if idx >= 0:
            acc += 2 * idx + 1
    assert acc == e, (acc, e)
    return steps


def table_windows(e, table, maxw=8):
    """Fewest-multiplies window partition of e's bits over a table of odd exponents: a window starts
    and ends on a 1 and its value is in `table`; the zeros between windows are free squarings.
    Same step format as sliding_window, with indices into `table`."""
    bits = bin(e)[2:]
    n = len(bits)
    INF = 1 << 30
    f, pick = [0] * (n + 1), [0] * (n + 1)
    for i in range(n - 1, -1, -1):
        if bits[i] == "0":
            f[i], pick[i] = f[i + 1], 0
            continue
        f[i] = INF
        for w in range(1, maxw + 1):
            if i + w <= n and bits[i + w - 1] == "1" and int(bits[i:i + w], 2) in table and 1 + f[i + w] < f[i]:
                f[i], pick[i] = 1 + f[i + w], w
        assert f[i] < INF, "the table cannot cover e"
    steps, i, pending = [], 0, 0
    while i < n:
        if bits[i] == "0":
            pending += 1
            i += 1
            continue
        w = pick[i]
        idx = table.index(int(bits[i:i + w], 2))
        steps.append((0, idx) if not steps else (pending + w, idx))
        pending, i = 0, i + w
    if pending:
        steps.append((pending, -1))
    acc = None
    for nsq, idx in steps:
        acc = table[idx] if acc is None else (acc << nsq) + (table[idx] if idx >= 0 else 0)
    assert acc == e, (acc, e)
    return steps


def field_struct(name, p, nl, nw, kb, comment, lb=LB, headroom=2048, table=None):
    """Field parameters as a traits struct consumed by the generic field core (csrc/fp381.hpp).
    lb = limb bits; headroom = the value bound (in units of p) that must fit below R."""
    rm = 1 << (lb * nl)
    assert p % 4 == 3 and p < rm // headroom
    pinv = (-pow(p, -1, 1 << lb)) % (1 << lb)
    L28 = lambda x: limbs28(x, nl, lb)  # noqa: E731
    if table is None:  # sliding window: the odd powers 1, 3, .., 2^W - 1
        table = tuple(range(1, 2 ** W, 2))
        steps = sliding_window((p - 3) // 4, W)
        how = f"sliding window w={W}"
    else:
        steps = table_windows((p - 3) // 4, list(table))
        how = "optimal windows over the table (tools/sqrt_chain_search.py)"
    nmul = sum(1 for st in steps if st[1] >= 0) - 1
    nsq = sum(st[0] for st in steps)
    L = [f"// {comment}: {nl} x {lb}-bit limbs, Montgomery R = 2^{lb * nl}.",
         f"struct {name} {{",
         f"  static constexpr int NL = {nl};  // limbs",
         f"  static constexpr int LB = {lb};  // bits per limb (each held in a 32-bit register)",
         f"  static constexpr uint32_t MASK = 0x{(1 << lb) - 1:08x}u;",
         f"  static constexpr int NW = {nw};  // 32-bit words of a serialized coordinate",
         "  " + arr("P", L28(p)),
         f"  static constexpr uint32_t PINV = 0x{pinv:08x}u;  // -p^-1 mod 2^{lb}",
         "  " + arr("R2", L28(rm * rm % p), "R^2 mod p"),
         "  " + arr("ONE", L28(rm % p), "R mod p (Montgomery 1)"),
         f"  static constexpr double INV_RHO = {float((1 << (lb * (nl - 1))) / p)!r};  "
         f"// 2^{lb * (nl - 1)} / p (fp_is_zero quotient estimate)"]
    for c in (1, 2, 4, 8, 16, 32, 64, 128):
        L.append("  " + arr(f"P_X{c}", L28(c * p), f"{c} p, normalized (canonical reduction)"))
    for c, Lb, vmax, alias in kb:
        nm = alias or f"KB_{c}_{Lb}"
        L.append("  " + arr(nm, borrowed(c, Lb, p, nl, vmax, lb),
                            f"{c} p, limbs >= 2^{Lb} - 2^{Lb - lb}, dominates values < {vmax if vmax else c - 0.001} p"))
    L += ["  " + arr("P_WORDS", words32(p, nw), f"p as {nw} x 32-bit words (byte-level range checks)"),
          f"  // a^((p-3)/4): {how}; {nsq} squarings + {nmul} multiplications after the table of "
          f"{len(table)} odd powers a^SQRT_TABLE_EXP[k].",
          f"  static constexpr int SQRT_TABLE = {len(table)};",
          "  static constexpr int16_t SQRT_TABLE_EXP[SQRT_TABLE] = {" + ", ".join(str(t) for t in table) + "};",
          f"  static constexpr int SQRT_STEPS = {len(steps)};",
          "  static constexpr int8_t SQRT_STEP_SQ[SQRT_STEPS] = {" + ", ".join(str(st[0]) for st in steps) + "};",
          "  static constexpr int8_t SQRT_STEP_IDX[SQRT_STEPS] = {" + ", ".join(str(st[1]) for st in steps) + "};",
          "};"]
    return L, nsq, nmul


def write(fname, lines):
    out = os.path.join(HERE, "..", "kzg-setup-powersoftau_amd", "csrc", fname)
    with open(out, "w") as f:
        f.write("\n".join(lines))
    print("wrote", out)


def main():
    lam = (-U * U) % R
    q = O.g1_mul(O.G1_GEN, lam)
    beta = None
    for g in range(2, 100):
        c = pow(g, (P - 1) // 3, P)
        if c == 1:
            continue
        for cand in (c, c * c % P):
            if (cand * O.G1_GEN[0] % P, O.G1_GEN[1]) == q:
                beta = cand
        if beta:
            break
    assert beta is not None
    xi = (1, 1)
    cx = O.fp2_inv(O.fp2_pow(xi, (P - 1) // 3))
    cy = O.fp2_inv(O.fp2_pow(xi, (P - 1) // 2))
    psi = (O.fp2_mul(O.fp2_conj(O.G2_GEN[0]), cx), O.fp2_mul(O.fp2_conj(O.G2_GEN[1]), cy))
    assert psi == O.g2_mul(O.G2_GEN, U)
    assert cx[0] == 0  # purely imaginary: conj(x) * (0 + c u) = (x1 c, x0 c)
    inv2 = pow(2, P - 2, P)
    absu = -U
    bls_kb = [(c, Lb, None, None) for c, Lb in KB] + [(64, 31, None, "KB_EQ")]
    pow30_out = (1 << 392) * pow(4, -((P - 3) // 4), P) % P
    fs, nsq, nmul = field_struct("BlsFp", P, NL, 12, bls_kb, "BLS12-381 Fq", table=BLS_SQRT_TABLE)
    lines = [
        "// GENERATED by tools/gen_constants.py — do not edit by hand.",
        "#pragma once",
        "#include <stdint.h>",
        "namespace kzgpot {",
    ] + fs + [
        "// BLS12-381 curve constants (Montgomery form of BlsFp unless noted)",
        arr("FP_FOUR", limbs28(mont(4))),
        arr("FP_ARK_R", limbs28((1 << 384) * RM % P), "2^384 R mod p: fp_mul(x, .) = x 2^384 (ark-ff Montgomery form)"),
        "// 2^(384 + 56 + 32 k) mod p, k = 0..11: x 2^384 mod p = (sum_k x_k FP_ARK_WORD[k]) 2^-56 for the",
        "// 32-bit words x_k of x (the loader's canonical -> ark Montgomery conversion, load_kernels.hip)",
        "static constexpr uint32_t FP_ARK_WORD[12][14] = {"
        + ", ".join("{" + ", ".join(f"0x{v:08x}u" for v in limbs28((1 << (384 + 56 + 32 * k)) % P)) + "}"
                    for k in range(12)) + "};",
        arr("FP_INV2", limbs28(mont(inv2))),
        arr("FP_BETA", limbs28(mont(beta))),
        arr("FP_PSI_CX1", limbs28(mont(cx[1]))),
        arr("FP_PSI_CY0", limbs28(mont(cy[0]))),
        arr("FP_PSI_CY1", limbs28(mont(cy[1]))),
        arr("G1_GEN_X", limbs28(mont(O.G1_GEN[0])), "Montgomery form (synthetic-data generator)"),
        arr("G1_GEN_Y", limbs28(mont(O.G1_GEN[1]))),
        arr("G2_GEN_X0", limbs28(mont(O.G2_GEN[0][0]))),
        arr("G2_GEN_X1", limbs28(mont(O.G2_GEN[0][1]))),
        arr("G2_GEN_Y0", limbs28(mont(O.G2_GEN[1][0]))),
        arr("G2_GEN_Y1", limbs28(mont(O.G2_GEN[1][1]))),
        "// radix-2^30 balanced core (fp381.hpp f30_*): 13 signed limbs in [-2^29, 2^29), R30 = 2^390;",
        "// the square-root exponentiation runs there (fp_pow_pm3d4 for BlsFp)",
        arr_s32("P30", balanced30(P), "p, balanced 30-bit digits"),
        f"static constexpr uint32_t PINV30 = 0x{(-pow(P, -1, 1 << 30)) % (1 << 30):08x}u;  // -p^-1 mod 2^30",
        arr_s32("POW30_OUT", balanced30(pow30_out), "2^392 4^-e mod p, e = (p-3)/4: R30-domain (4a)^e -> R = 2^392 a^e"),
        f"static constexpr uint64_t BLS_ABS_U = 0x{absu:016x}ull;  // |u|, u < 0",
        "static constexpr int BLS_ABS_U_BITS = %d;" % absu.bit_length(),
        arr("FR_R", words32(R, 8), "group order r (ref-mode double-and-add)"),
        "static constexpr int FR_R_BITS = %d;" % R.bit_length(),
        "}  // namespace kzgpot",
        "",
    ]
    write("bls12_381_consts.hpp", lines)
    print(f"  BLS12-381 sqrt chain: {nsq} sq + {nmul} mul after the table {BLS_SQRT_TABLE}")

    # BN254 (config 5): only the decompress chain runs here; fp_eq compares against normalized
    # values < 4p, which KB_8_28 dominates even with the small top limb of a 254-bit p
    bn_rm = 1 << (BN_LB * BN_NL)
    fs, nsq, nmul = field_struct("Bn254Fp", BN_P, BN_NL, 8, [(8, 29, 4, "KB_EQ")], "BN254 Fq (ark-bn254 0.2)",
                                 lb=BN_LB, headroom=64)
    lines = [
        "// GENERATED by tools/gen_constants.py — do not edit by hand.",
        "#pragma once",
        "#include <stdint.h>",
        "namespace kzgpot {",
    ] + fs + [
        "// BN254 G1: y^2 = x^3 + 3, cofactor 1",
        arr("BN_THREE", limbs28(3 * bn_rm % BN_P, BN_NL, BN_LB), "3 R mod p"),
        arr("BN_ARK_R", limbs28((1 << 256) * bn_rm % BN_P, BN_NL, BN_LB),
            "2^256 R mod p (ark-ff Fp256 Montgomery form)"),
        arr("BN_FR_R", words32(BN_R, 8), "group order r"),
        "}  // namespace kzgpot",
        "",
    ]
    write("bn254_consts.hpp", lines)
    print(f"  BN254 sqrt chain: {nsq} sq + {nmul} mul")


if __name__ == "__main__":
    main()
