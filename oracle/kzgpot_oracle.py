"""CPU ORACLE (test infrastructure only) — pure-Python restatement of the reference's hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker. The product path (the HIP kernels behind the C ABI) never
calls it.

What it restates (reference = heliaxdev/kzg-setup-powersoftau, Rust):

* `src/bin/preprocess-kgz.rs:105-110` → `powersoftau::Accumulator::deserialize(.., UseCompression::Yes,
  CheckForCorrectness::No)` → pairing 0.14.2 `G1Compressed/G2Compressed::into_affine_unchecked`
  (flag byte, x < p, `get_point_from_x`, `Fq::sqrt` = a^((p-3)/4) form, `Fq2::sqrt` = Algorithm 9 of
  eprint 2012/685, lexicographic sign rule).                              → `pairing_g1_decompress`,
                                                                             `pairing_g2_decompress`
* `src/bin/preprocess-kgz.rs:122-125` → `Accumulator::serialize(UseCompression::No)` →
  pairing `into_uncompressed` (x‖y big-endian; G2 c1 before c0; infinity = 0x40‖0…).
                                                                           → `pairing_g1_uncompressed`, …
* `src/lib.rs:41-54` `read_g1` and `src/lib.rs:56-80` `read_g2` (byte reversal / c0,c1 reorder) →
  ark-ec 0.2.0 `GroupAffine::deserialize_uncompressed` = `deserialize_unchecked` (Fp384 read, x<p,
  SWFlags on y's top byte, `GroupAffine::new(x, y, inf)`, NO on-curve check) followed by
  `is_in_correct_subgroup_assuming_on_curve` = `mul_bits(r).is_zero()` with ark's Jacobian
  `double_in_place` (dbl-2009-l, a = 0) and `add_assign_mixed` (madd-2007-bl) formulas, restated
  operation by operation so the boolean matches the reference even for off-curve inputs.
                                                                           → `read_g1`, `read_g2`
* `src/bin/preprocess-kgz.rs:188-194`, `preprocess-fastkgz.rs:193-208` → ark
  `CanonicalSerialize::serialize_uncompressed` (x LE, y LE + SWFlags in y's top byte; G2 = c0, c1).
                                                                           → `ark_g1_serialize`, …
* the file pipelines `preprocess-kgz.rs:69-199` / `preprocess-fastkgz.rs:70-213`
                                                                           → `preprocess_kgz`,
                                                                             `preprocess_fastkgz`

The third-party crates (pairing 0.14.2, ark-* 0.2.0, powersoftau@e3318303) are NOT in this
container; their algorithms are restated from their published sources as pinned in
`/root/reference/Cargo.lock`.

PARITY PINNING: the reference ships no test vectors for this path and cannot be built here
(Rust toolchain absent). This oracle is pinned by the published BLS12-381 spec constants
(generator encodings, which every real transcript's τG1[0]/τG2[0] must equal), by internal
identities (ark bytes = per-coordinate byte reversal of pairing bytes), by cross-agreement with
the independent C restatement in `oracle/kzgpot_ref.c`, and — only when the real Zcash transcript
is supplied offline — by the reference's own BLAKE2b-512 output digests (`src/lib.rs:21-22`).
Without that file, bit-exactness against the reference binary itself is "parity unpinned".
"""
from __future__ import annotations

import hashlib
import random

# ----------------------------------------------------------------------------------------------
# BLS12-381 constants (ark-bls12-381 0.2 / pairing 0.14.2 parameters)
# ----------------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
U_PARAM = -0xD201000000010000  # BLS parameter u (x in the pairing crate)
H1 = 0x396C8C005555E1568C00AAAB0000AAAB
H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5
B1 = 4
B2 = (4, 4)  # 4(1 + u)

G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)

# Reference-layout constants (src/lib.rs:23-24, src/bin/preprocess-kgz.rs:22-23)
TAU_POWERS_LENGTH = 1 << 21
G1_COMPRESSED = 48
G2_COMPRESSED = 96
G1_UNCOMPRESSED = 96
G2_UNCOMPRESSED = 192
PUBLIC_KEY_SIZE = 3 * G2_UNCOMPRESSED + 6 * G1_UNCOMPRESSED  # powersoftau PublicKey, uncompressed
HASH_SIZE = 64
VK_SIZE = 2 * G1_UNCOMPRESSED + 2 * G2_UNCOMPRESSED  # ark-poly-commit VerifierKey, uncompressed

# Error classes (the reference's reject set). Accept/reject is graded, not class.
OK = 0
E_COMPRESSION_MODE = 1      # pairing UnexpectedCompressionMode (bit7 clear)
E_UNEXPECTED_INFO = 2       # pairing UnexpectedInformation (infinity with stray bits)
E_NOT_IN_FIELD = 3          # pairing CoordinateDecodingError / ark InvalidData (coordinate >= p)
E_NOT_ON_CURVE = 4          # pairing NotOnCurve (x^3+b non-residue)
E_NOT_IN_SUBGROUP = 5       # ark InvalidData from is_in_correct_subgroup_assuming_on_curve
E_UNEXPECTED_FLAGS = 6      # ark UnexpectedFlags (both SW flag bits set)
E_INFINITY = 7              # infinity reached read_g1/read_g2: the reference panics (x >= p)

ERROR_NAMES = {
    OK: "ok", E_COMPRESSION_MODE: "UnexpectedCompressionMode", E_UNEXPECTED_INFO: "UnexpectedInformation",
    E_NOT_IN_FIELD: "NotInField", E_NOT_ON_CURVE: "NotOnCurve", E_NOT_IN_SUBGROUP: "NotInSubgroup",
    E_UNEXPECTED_FLAGS: "UnexpectedFlags", E_INFINITY: "Infinity",
}


def powersoftau_contribution_size(n: int) -> int:
    """powersoftau `CONTRIBUTION_BYTE_SIZE` generalised to N powers (checked at preprocess-kgz.rs:83)."""
    return ((2 * n - 1) * G1_COMPRESSED + n * G2_COMPRESSED + 2 * n * G1_COMPRESSED + G2_COMPRESSED
            + PUBLIC_KEY_SIZE + HASH_SIZE)


# ----------------------------------------------------------------------------------------------
# Field arithmetic. Fp = python int mod P; Fp2 = (c0, c1) with u^2 = -1.
# ----------------------------------------------------------------------------------------------
class _Fp:
    zero = 0
    one = 1

    @staticmethod
    def add(a, b): return (a + b) % P
    @staticmethod
    def sub(a, b): return (a - b) % P
    @staticmethod
    def mul(a, b): return a * b % P
    @staticmethod
    def sqr(a): return a * a % P
    @staticmethod
    def dbl(a): return 2 * a % P
    @staticmethod
    def neg(a): return (-a) % P
    @staticmethod
    def is_zero(a): return a == 0


def fp2_add(a, b): return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)
def fp2_sub(a, b): return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)
def fp2_neg(a): return ((-a[0]) % P, (-a[1]) % P)
def fp2_mul(a, b): return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)
def fp2_sqr(a): return fp2_mul(a, a)
def fp2_conj(a): return (a[0], (-a[1]) % P)


def fp2_pow(a, e):
    r = (1, 0)
    for bit in bin(e)[2:]:
        r = fp2_sqr(r)
        if bit == "1":
            r = fp2_mul(r, a)
    return r


def fp2_inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = pow(n, P - 2, P)
    return (a[0] * ni % P, (-a[1]) * ni % P)


class _Fp2:
    zero = (0, 0)
    one = (1, 0)
    add = staticmethod(fp2_add)
    sub = staticmethod(fp2_sub)
    mul = staticmethod(fp2_mul)
    sqr = staticmethod(fp2_sqr)
    neg = staticmethod(fp2_neg)

    @staticmethod
    def dbl(a): return fp2_add(a, a)
    @staticmethod
    def is_zero(a): return a == (0, 0)


def fq_sqrt(a):
    """pairing 0.14.2 `impl SqrtField for Fq` (p = 3 mod 4, eprint 2012/685 Alg. 2)."""
    a1 = pow(a, (P - 3) // 4, P)
    a0 = a1 * a1 % P * a % P
    if a0 == P - 1:
        return None
    return a1 * a % P


def fq2_sqrt(a):
    """pairing 0.14.2 `impl SqrtField for Fq2` — Algorithm 9 of eprint 2012/685."""
    if a == (0, 0):
        return (0, 0)
    a1 = fp2_pow(a, (P - 3) // 4)
    alpha = fp2_mul(fp2_sqr(a1), a)
    a0 = fp2_mul(fp2_conj(alpha), alpha)  # frobenius_map(1) = conjugation
    neg1 = (P - 1, 0)
    if a0 == neg1:
        return None
    a1 = fp2_mul(a1, a)
    if alpha == neg1:
        return fp2_mul(a1, (0, 1))
    b = fp2_pow(fp2_add(alpha, (1, 0)), (P - 1) // 2)
    return fp2_mul(a1, b)


def fq_lt(a, b):
    """pairing `Ord for Fq`: canonical integer order."""
    return a < b


def fq2_lt(a, b):
    """pairing `Ord for Fq2`: lexicographic, c1 first then c0."""
    if a[1] != b[1]:
        return a[1] < b[1]
    return a[0] < b[0]


# ----------------------------------------------------------------------------------------------
# pairing 0.14.2 encodings
# ----------------------------------------------------------------------------------------------
def _be48(b: bytes) -> int:
    return int.from_bytes(b, "big")


def pairing_g1_decompress(enc: bytes):
    """`G1Compressed::into_affine_unchecked` → (OK, (x, y)) | (OK, None)=infinity | (err, None)."""
    assert len(enc) == 48
    copy = bytearray(enc)
    if copy[0] & 0x80 == 0:
        return E_COMPRESSION_MODE, None
    if copy[0] & 0x40:
        copy[0] &= 0x3F
        if any(copy):
            return E_UNEXPECTED_INFO, None
        return OK, None
    greatest = bool(copy[0] & 0x20)
    copy[0] &= 0x1F
    x = _be48(copy)
    if x >= P:
        return E_NOT_IN_FIELD, None
    # G1Affine::get_point_from_x
    x3b = (x * x % P * x + B1) % P
    y = fq_sqrt(x3b)
    if y is None:
        return E_NOT_ON_CURVE, None
    negy = (-y) % P
    y = y if (fq_lt(y, negy) ^ greatest) else negy
    return OK, (x, y)


def pairing_g2_decompress(enc: bytes):
    """`G2Compressed::into_affine_unchecked`: x.c1 ‖ x.c0 big-endian, flags in x.c1's top byte."""
    assert len(enc) == 96
    copy = bytearray(enc)
    if copy[0] & 0x80 == 0:
        return E_COMPRESSION_MODE, None
    if copy[0] & 0x40:
        copy[0] &= 0x3F
        if any(copy):
            return E_UNEXPECTED_INFO, None
        return OK, None
    greatest = bool(copy[0] & 0x20)
    copy[0] &= 0x1F
    x_c1 = _be48(copy[0:48])
    x_c0 = _be48(copy[48:96])
    if x_c0 >= P or x_c1 >= P:
        return E_NOT_IN_FIELD, None
    x = (x_c0, x_c1)
    x3b = fp2_add(fp2_mul(fp2_sqr(x), x), B2)
    y = fq2_sqrt(x3b)
    if y is None:
        return E_NOT_ON_CURVE, None
    negy = fp2_neg(y)
    y = y if (fq2_lt(y, negy) ^ greatest) else negy
    return OK, (x, y)


def pairing_g1_uncompressed(pt) -> bytes:
    """`G1Uncompressed::from_affine` (powersoftau Accumulator::serialize(UseCompression::No))."""
    if pt is None:
        return bytes([0x40]) + bytes(95)
    return pt[0].to_bytes(48, "big") + pt[1].to_bytes(48, "big")


def pairing_g2_uncompressed(pt) -> bytes:
    if pt is None:
        return bytes([0x40]) + bytes(191)
    (x0, x1), (y0, y1) = pt
    return b"".join(v.to_bytes(48, "big") for v in (x1, x0, y1, y0))


def pairing_g1_compress(pt) -> bytes:
    """`G1Compressed::from_affine` — used only to build synthetic transcripts."""
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    b = bytearray(x.to_bytes(48, "big"))
    negy = (-y) % P
    if y > negy:
        b[0] |= 0x20
    b[0] |= 0x80
    return bytes(b)


def pairing_g2_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    (x0, x1), y = pt
    b = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
    if fq2_lt(fp2_neg(y), y):
        b[0] |= 0x20
    b[0] |= 0x80
    return bytes(b)


# ----------------------------------------------------------------------------------------------
# ark 0.2 side: read_g1 / read_g2 (src/lib.rs:41-80) + deserialize_uncompressed + serialize
# ----------------------------------------------------------------------------------------------
def _jac_double(F, X, Y, Z):
    """ark-ec 0.2 `GroupProjective::double_in_place`, COEFF_A = 0 branch (dbl-2009-l)."""
    if F.is_zero(Z):
        return X, Y, Z
    a = F.sqr(X)
    b = F.sqr(Y)
    c = F.sqr(b)
    d = F.dbl(F.sub(F.sub(F.sqr(F.add(X, b)), a), c))
    e = F.add(a, F.dbl(a))
    f = F.sqr(e)
    Z3 = F.dbl(F.mul(Z, Y))
    X3 = F.sub(F.sub(f, d), d)
    c8 = F.dbl(F.dbl(F.dbl(c)))
    Y3 = F.sub(F.mul(F.sub(d, X3), e), c8)
    return X3, Y3, Z3


def _jac_add_mixed(F, X1, Y1, Z1, x2, y2, inf2):
    """ark-ec 0.2 `GroupProjective::add_assign_mixed` (madd-2007-bl with the equal-point branch)."""
    if inf2:
        return X1, Y1, Z1
    if F.is_zero(Z1):
        return x2, y2, F.one
    z1z1 = F.sqr(Z1)
    u2 = F.mul(x2, z1z1)
    s2 = F.mul(F.mul(y2, Z1), z1z1)
    if X1 == u2 and Y1 == s2:
        return _jac_double(F, X1, Y1, Z1)
    h = F.sub(u2, X1)
    hh = F.sqr(h)
    i = F.dbl(F.dbl(hh))
    j = F.mul(h, i)
    r = F.dbl(F.sub(s2, Y1))
    v = F.mul(X1, i)
    X3 = F.sub(F.sub(F.sub(F.sqr(r), j), v), v)
    j2 = F.dbl(F.mul(j, Y1))
    Y3 = F.sub(F.mul(F.sub(v, X3), r), j2)
    Z3 = F.sub(F.sub(F.sqr(F.add(Z1, h)), z1z1), hh)
    return X3, Y3, Z3


def ark_mul_bits_is_zero(F, x, y, inf, scalar=R_ORDER):
    """`GroupAffine::mul_bits(BitIteratorBE(r))` then `.is_zero()` (= Z == 0)."""
    X, Y, Z = F.zero, F.one, F.zero  # GroupProjective::zero()
    for bit in bin(scalar)[2:]:  # BitIteratorBE skip_while(!b): bin() has no leading zeros
        X, Y, Z = _jac_double(F, X, Y, Z)
        if bit == "1":
            X, Y, Z = _jac_add_mixed(F, X, Y, Z, x, y, inf)
    return F.is_zero(Z)


def _ark_fp_read_with_flags(le48: bytes, with_flags: bool):
    """ark-ff 0.2 Fp384 `deserialize_with_flags` / `deserialize` (EmptyFlags)."""
    b = bytearray(le48)
    flags_inf = False
    if with_flags:
        top = b[47]
        pos = bool(top >> 7 & 1)
        inf = bool(top >> 6 & 1)
        if pos and inf:
            return E_UNEXPECTED_FLAGS, None, False
        flags_inf = inf
        b[47] &= 0x3F
    v = int.from_bytes(b, "little")
    if v >= P:
        return E_NOT_IN_FIELD, None, False
    return OK, v, flags_inf


def ark_g1_deserialize_uncompressed(ark96: bytes, subgroup_check: bool = True):
    """ark-ec 0.2 `GroupAffine::<g1>::deserialize_uncompressed` → (status, (x, y, infinity))."""
    st, x, _ = _ark_fp_read_with_flags(ark96[0:48], False)
    if st:
        return st, None
    st, y, inf = _ark_fp_read_with_flags(ark96[48:96], True)
    if st:
        return st, None
    if subgroup_check and not ark_mul_bits_is_zero(_Fp, x, y, inf):
        return E_NOT_IN_SUBGROUP, None
    return OK, (x, y, inf)


def ark_g2_deserialize_uncompressed(ark192: bytes, subgroup_check: bool = True):
    """ark-ec 0.2 `GroupAffine::<g2>::deserialize_uncompressed`: x.c0, x.c1, y.c0, y.c1 (flags on y.c1)."""
    st, x0, _ = _ark_fp_read_with_flags(ark192[0:48], False)
    if st:
        return st, None
    st, x1, _ = _ark_fp_read_with_flags(ark192[48:96], False)
    if st:
        return st, None
    st, y0, _ = _ark_fp_read_with_flags(ark192[96:144], False)
    if st:
        return st, None
    st, y1, inf = _ark_fp_read_with_flags(ark192[144:192], True)
    if st:
        return st, None
    x, y = (x0, x1), (y0, y1)
    if subgroup_check and not ark_mul_bits_is_zero(_Fp2, x, y, inf):
        return E_NOT_IN_SUBGROUP, None
    return OK, (x, y, inf)


def ark_g1_serialize(pt) -> bytes:
    """ark-ec 0.2 `serialize_uncompressed`: x LE, y LE with SWFlags (infinity → bit 6 of byte 95)."""
    x, y, inf = pt
    b = bytearray(x.to_bytes(48, "little") + y.to_bytes(48, "little"))
    if inf:
        b[95] |= 0x40
    return bytes(b)


def ark_g2_serialize(pt) -> bytes:
    (x0, x1), (y0, y1), inf = pt
    b = bytearray(b"".join(v.to_bytes(48, "little") for v in (x0, x1, y0, y1)))
    if inf:
        b[191] |= 0x40
    return bytes(b)


ARK_G1_ZERO = (0, 1, True)          # ark-ec 0.2 GroupAffine::zero() = (0, 1, infinity)
ARK_G2_ZERO = ((0, 0), (1, 0), True)


def read_g1_bytes(pairing96: bytes):
    """`src/lib.rs:41-54` read_g1 on an in-memory 96-byte record: reverse [0..48) and [48..96)."""
    b = pairing96[0:48][::-1] + pairing96[48:96][::-1]
    return ark_g1_deserialize_uncompressed(b)


def read_g2_bytes(pairing192: bytes):
    """`src/lib.rs:56-80` read_g2: ark order = [48..96) [0..48) [144..192) [96..144), each reversed."""
    parts = (pairing192[48:96], pairing192[0:48], pairing192[144:192], pairing192[96:144])
    b = b"".join(q[::-1] for q in parts)
    return ark_g2_deserialize_uncompressed(b)


# ----------------------------------------------------------------------------------------------
# Fused per-point semantics of the reference pipeline (the kernel contract)
# ----------------------------------------------------------------------------------------------
def g1_decompress_point(enc48: bytes, check: bool = True):
    """One compressed G1 point through decompress → uncompressed file → read_g1 → serialize.

    check=True: the path of every point the reference reads back with read_g1 (τG1, ατG1; βτG1
    in fastkgz). check=False: decompression only (βτG1 in kgz), where infinity is legal.
    Returns (status, ark96 | None).
    """
    st, pt = pairing_g1_decompress(enc48)
    if st:
        return st, None
    if not check:
        return OK, ark_g1_serialize(ARK_G1_ZERO if pt is None else (pt[0], pt[1], False))
    st, apt = read_g1_bytes(pairing_g1_uncompressed(pt))
    if st:
        return (E_INFINITY if pt is None else st), None
    return OK, ark_g1_serialize(apt)


def g2_decompress_point(enc96: bytes, check: bool = True):
    st, pt = pairing_g2_decompress(enc96)
    if st:
        return st, None
    if not check:
        return OK, ark_g2_serialize(ARK_G2_ZERO if pt is None else (pt[0], pt[1], False))
    st, apt = read_g2_bytes(pairing_g2_uncompressed(pt))
    if st:
        return (E_INFINITY if pt is None else st), None
    return OK, ark_g2_serialize(apt)


def g1_transcode_point(pairing96: bytes):
    """read_g1 alone (uncompressed input, e.g. powersoftau_uncompressed / phase1radix2m)."""
    st, apt = read_g1_bytes(pairing96)
    return (st, None) if st else (OK, ark_g1_serialize(apt))


def g2_transcode_point(pairing192: bytes):
    st, apt = read_g2_bytes(pairing192)
    return (st, None) if st else (OK, ark_g2_serialize(apt))


# ----------------------------------------------------------------------------------------------
# Loader mirror: load_kzg_setup / load_fastkzg_setup, src/lib.rs:174-228
# ----------------------------------------------------------------------------------------------
ARK_R = 1 << 384          # ark-ff 0.2 Fp384 Montgomery radix
G1_ARK_MONT = 104         # GroupAffine<g1> in memory: x[6 x u64] y[6 x u64] infinity(u8) pad[7]
G2_ARK_MONT = 200         # GroupAffine<g2>: x.c0 x.c1 y.c0 y.c1, infinity, pad


def _ark_mont_bytes(v: int) -> bytes:
    return (v * ARK_R % P).to_bytes(48, "little")


def g1_deserialize_unchecked_point(ark96: bytes):
    """ark-ec 0.2 `GroupAffine::<g1>::deserialize_unchecked` (src/lib.rs:180,183): coordinates < p
    and SWFlags only — no curve, no subgroup check. Returns (status, in-memory 104-B record)."""
    st, pt = ark_g1_deserialize_uncompressed(ark96, subgroup_check=False)
    if st:
        return st, None
    x, y, inf = pt
    return OK, _ark_mont_bytes(x) + _ark_mont_bytes(y) + bytes([1 if inf else 0]) + bytes(7)


def g2_deserialize_unchecked_point(ark192: bytes):
    """ark-ec 0.2 `GroupAffine::<g2>::deserialize_unchecked` (src/lib.rs:209-215)."""
    st, pt = ark_g2_deserialize_uncompressed(ark192, subgroup_check=False)
    if st:
        return st, None
    (x0, x1), (y0, y1), inf = pt
    body = b"".join(_ark_mont_bytes(v) for v in (x0, x1, y0, y1))
    return OK, body + bytes([1 if inf else 0]) + bytes(7)


def _load_sections(data: bytes, plan):
    """Sequential deserialize_unchecked over `plan` = [(g2?, count)] → (status, [section bytes]).
    Raises on a short file (the reference's reader hits UnexpectedEof and unwraps)."""
    off, outs = 0, []
    for g2, count in plan:
        rec = G2_UNCOMPRESSED if g2 else G1_UNCOMPRESSED
        if off + count * rec > len(data):
            raise ValueError("setup file too short")
        fn = g2_deserialize_unchecked_point if g2 else g1_deserialize_unchecked_point
        out, sts, bad = batch(fn, data[off:off + count * rec], rec, G2_ARK_MONT if g2 else G1_ARK_MONT)
        if bad >= 0:
            return sts[bad], outs
        outs.append(out)
        off += count * rec
    return OK, outs


def load_kzg_setup(data: bytes, n: int):
    """src/lib.rs:174-195 → (status, (powers_of_g, powers_of_gamma_g, vk)) as in-memory records;
    vk = g ‖ gamma_g ‖ h ‖ beta_h (VerifierKey::deserialize_unchecked)."""
    st, outs = _load_sections(data, [(False, 2 * n - 1), (False, n), (False, 2), (True, 2)])
    if st:
        return st, None
    return OK, (outs[0], outs[1], outs[2] + outs[3])


def load_fastkzg_setup(data: bytes, n: int):
    """src/lib.rs:197-228 → (status, (powers_of_g, powers_of_gamma_g, h ‖ beta_h, powers_of_h))."""
    st, outs = _load_sections(data, [(False, 2 * n - 1), (False, n), (True, 2), (True, n)])
    if st:
        return st, None
    return OK, tuple(outs)


def g1_read_to_mont(pairing96: bytes):
    """read_g1 (src/lib.rs:41-54) → the in-memory GroupAffine it returns (104 B)."""
    st, apt = read_g1_bytes(pairing96)
    if st:
        return st, None
    x, y, inf = apt
    return OK, _ark_mont_bytes(x) + _ark_mont_bytes(y) + bytes([1 if inf else 0]) + bytes(7)


def g2_read_to_mont(pairing192: bytes):
    """read_g2 (src/lib.rs:56-80) → in-memory GroupAffine<g2> (200 B)."""
    st, apt = read_g2_bytes(pairing192)
    if st:
        return st, None
    (x0, x1), (y0, y1), inf = apt
    return OK, b"".join(_ark_mont_bytes(v) for v in (x0, x1, y0, y1)) + bytes([1 if inf else 0]) + bytes(7)


def load_phase1(data: bytes, exp: int):
    """src/lib.rs:82-121: alpha, beta_g1, beta_g2, then coeffs_g1, coeffs_g2, alpha_coeffs_g1,
    beta_coeffs_g1 (2^exp each), all through read_g1 / read_g2. → (status, section, index, [7 outs])."""
    m = 1 << exp
    plan = [(False, 1), (False, 1), (True, 1), (False, m), (True, m), (False, m), (False, m)]
    off, outs = 0, []
    for sec, (g2, count) in enumerate(plan):
        rec = G2_UNCOMPRESSED if g2 else G1_UNCOMPRESSED
        if off + count * rec > len(data):
            raise ValueError("phase1 file too short")
        fn = g2_read_to_mont if g2 else g1_read_to_mont
        out, sts, bad = batch(fn, data[off:off + count * rec], rec, G2_ARK_MONT if g2 else G1_ARK_MONT)
        if bad >= 0:
            return sts[bad], sec, bad, outs
        outs.append(out)
        off += count * rec
    return OK, -1, -1, outs


# ----------------------------------------------------------------------------------------------
# BN254 G1 (config 5, SURVEY §8f 4 — no reference counterpart): ark-bn254 0.2 compressed G1
# → ark-ec 0.2 GroupAffine::deserialize → serialize_uncompressed. Same ark rules as the BLS12-381
# read path above (SWFlags, Fp < p), plus ark's compressed branch: Infinity → zero(); else
# get_point_from_x(x, PositiveY) with the `(y < -y) ^ greatest` rule; cofactor 1.
# ----------------------------------------------------------------------------------------------
BN_P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
BN_R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
BN_B = 3
BN_G1_GEN = (1, 2)


def bn_sqrt(a):
    a %= BN_P
    y = pow(a, (BN_P + 1) // 4, BN_P)
    return y if y * y % BN_P == a else None


def bn_on_curve(pt):
    x, y = pt
    return (y * y - x * x * x - BN_B) % BN_P == 0


def bn_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    (x1, y1), (x2, y2) = a, b
    if x1 == x2:
        if (y1 + y2) % BN_P == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, -1, BN_P) % BN_P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, BN_P) % BN_P
    x3 = (lam * lam - x1 - x2) % BN_P
    return (x3, (lam * (x1 - x3) - y1) % BN_P)


def bn_mul(pt, k):
    acc = None
    for bit in bin(k)[2:] if k > 0 else "":
        acc = bn_add(acc, acc)
        if bit == "1":
            acc = bn_add(acc, pt)
    return acc


def bn254_g1_compress(pt) -> bytes:
    """ark-ec 0.2 `serialize` (compressed): x LE + SWFlags (PositiveY iff y > -y; zero → Infinity)."""
    if pt is None:
        return bytes(31) + b"\x40"
    x, y = pt
    b = bytearray(x.to_bytes(32, "little"))
    if y > (BN_P - y) % BN_P:
        b[31] |= 0x80
    return bytes(b)


def bn254_g1_decompress_point(enc32: bytes):
    """ark-bn254 G1Affine::deserialize (compressed) → serialize_uncompressed. (status, 64 B | None)."""
    b = bytearray(enc32)
    top = b[31]
    pos, inf = bool(top >> 7 & 1), bool(top >> 6 & 1)
    if pos and inf:
        return E_UNEXPECTED_FLAGS, None
    b[31] &= 0x3F
    x = int.from_bytes(b, "little")
    if x >= BN_P:
        return E_NOT_IN_FIELD, None
    if inf:
        out = bytearray(bytes(32) + (1).to_bytes(32, "little"))
        out[63] |= 0x40
        return OK, bytes(out)
    y = bn_sqrt(x * x * x + BN_B)
    if y is None:
        return E_NOT_ON_CURVE, None
    negy = (BN_P - y) % BN_P
    y = y if (y < negy) ^ pos else negy
    return OK, x.to_bytes(32, "little") + y.to_bytes(32, "little")


def batch(fn, data: bytes, rec: int, out_rec: int, **kw):
    """Apply a per-point function over a packed stream → (out bytes, statuses, first_bad)."""
    n = len(data) // rec
    out = bytearray(n * out_rec)
    statuses = []
    first_bad = -1
    for i in range(n):
        st, o = fn(data[i * rec:(i + 1) * rec], **kw)
        statuses.append(st)
        if st == OK:
            out[i * out_rec:(i + 1) * out_rec] = o
        elif first_bad < 0:
            first_bad = i
    return bytes(out), statuses, first_bad


# ----------------------------------------------------------------------------------------------
# Curve arithmetic for synthetic data (affine, straightforward)
# ----------------------------------------------------------------------------------------------
def g1_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    (x1, y1), (x2, y2) = a, b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, P - 2, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, P - 2, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def g1_mul(pt, k):
    """Scalar multiplication via Jacobian double-and-add, then one inversion."""
    if k < 0:
        pt = None if pt is None else (pt[0], (-pt[1]) % P)
        k = -k
    if pt is None or k == 0:
        return None
    X, Y, Z = 0, 1, 0
    for bit in bin(k)[2:]:
        X, Y, Z = _jac_double(_Fp, X, Y, Z)
        if bit == "1":
            X, Y, Z = _jac_add_mixed(_Fp, X, Y, Z, pt[0], pt[1], False)
    if Z == 0:
        return None
    zi = pow(Z, P - 2, P)
    zi2 = zi * zi % P
    return (X * zi2 % P, Y * zi2 % P * zi % P)


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    (x1, y1), (x2, y2) = a, b
    if x1 == x2:
        if fp2_add(y1, y2) == (0, 0):
            return None
        lam = fp2_mul(fp2_mul((3, 0), fp2_sqr(x1)), fp2_inv(fp2_add(y1, y1)))
    else:
        lam = fp2_mul(fp2_sub(y2, y1), fp2_inv(fp2_sub(x2, x1)))
    x3 = fp2_sub(fp2_sub(fp2_sqr(lam), x1), x2)
    return (x3, fp2_sub(fp2_mul(lam, fp2_sub(x1, x3)), y1))


def g2_mul(pt, k):
    if k < 0:
        pt = None if pt is None else (pt[0], fp2_neg(pt[1]))
        k = -k
    if pt is None or k == 0:
        return None
    X, Y, Z = (0, 0), (1, 0), (0, 0)
    for bit in bin(k)[2:]:
        X, Y, Z = _jac_double(_Fp2, X, Y, Z)
        if bit == "1":
            X, Y, Z = _jac_add_mixed(_Fp2, X, Y, Z, pt[0], pt[1], False)
    if Z == (0, 0):
        return None
    zi = fp2_inv(Z)
    zi2 = fp2_sqr(zi)
    return (fp2_mul(X, zi2), fp2_mul(fp2_mul(Y, zi2), zi))


def g1_on_curve(pt):
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g2_on_curve(pt):
    x, y = pt
    return fp2_sub(fp2_sqr(y), fp2_add(fp2_mul(fp2_sqr(x), x), B2)) == (0, 0)


def g1_random_on_curve(rng: random.Random):
    """A random point of E(Fp) with NO cofactor clearing (almost surely outside G1)."""
    while True:
        x = rng.randrange(P)
        y = fq_sqrt((x * x * x + B1) % P)
        if y is not None:
            return (x, y if rng.random() < 0.5 else (-y) % P)


def g2_random_on_curve(rng: random.Random):
    while True:
        x = (rng.randrange(P), rng.randrange(P))
        y = fq2_sqrt(fp2_add(fp2_mul(fp2_sqr(x), x), B2))
        if y is not None:
            return (x, y if rng.random() < 0.5 else fp2_neg(y))


# ----------------------------------------------------------------------------------------------
# Synthetic Powers-of-Tau response transcript + the two reference pipelines
# ----------------------------------------------------------------------------------------------
def make_response_transcript(n: int, seed: int) -> bytes:
    """A response file in powersoftau's layout for N powers: hash(64) ‖ τG1×(2N−1) ‖ τG2×N ‖
    ατG1×N ‖ βτG1×N ‖ βG2 ‖ pubkey(1152), all points compressed. τ, α, β from `seed`."""
    rng = random.Random(seed)
    tau = rng.randrange(1, R_ORDER)
    alpha = rng.randrange(1, R_ORDER)
    beta = rng.randrange(1, R_ORDER)
    out = bytearray(rng.randbytes(HASH_SIZE))
    g1 = [None] * (2 * n - 1)
    cur = G1_GEN
    for i in range(2 * n - 1):
        g1[i] = cur
        cur = g1_mul(cur, tau)
    out += b"".join(pairing_g1_compress(q) for q in g1)
    g2cur = G2_GEN
    g2 = []
    for i in range(n):
        g2.append(g2cur)
        g2cur = g2_mul(g2cur, tau)
    out += b"".join(pairing_g2_compress(q) for q in g2)
    out += b"".join(pairing_g1_compress(g1_mul(q, alpha)) for q in g1[:n])
    out += b"".join(pairing_g1_compress(g1_mul(q, beta)) for q in g1[:n])
    out += pairing_g2_compress(g2_mul(G2_GEN, beta))
    out += rng.randbytes(PUBLIC_KEY_SIZE)
    assert len(out) == powersoftau_contribution_size(n)
    return bytes(out)


def make_phase1_file(exp: int, seed: int) -> bytes:
    """A phase1radix2m{exp}-layout file (src/lib.rs:82-121): alpha, beta_g1, beta_g2, then
    coeffs_g1, coeffs_g2, alpha_coeffs_g1, beta_coeffs_g1 (2^exp each), pairing-uncompressed.
    Synthetic: [a]G1, [b]G1, [b]G2, [c_i]G1, [c_i]G2, [a c_i]G1, [b c_i]G1 for random a, b, c_i."""
    rng = random.Random(seed)
    a, b = rng.randrange(1, R_ORDER), rng.randrange(1, R_ORDER)
    cs = [rng.randrange(1, R_ORDER) for _ in range(1 << exp)]
    e1 = lambda k: pairing_g1_uncompressed(g1_mul(G1_GEN, k % R_ORDER))  # noqa: E731
    e2 = lambda k: pairing_g2_uncompressed(g2_mul(G2_GEN, k % R_ORDER))  # noqa: E731
    parts = [e1(a), e1(b), e2(b)] + [e1(c) for c in cs] + [e2(c) for c in cs] + [e1(a * c) for c in cs] + \
        [e1(b * c) for c in cs]
    return b"".join(parts)


def _sections(n: int):
    off = HASH_SIZE
    sec = {}
    for name, count, rec in (("tau_g1", 2 * n - 1, 48), ("tau_g2", n, 96), ("alpha_g1", n, 48),
                             ("beta_g1", n, 48), ("beta_g2", 1, 96)):
        sec[name] = (off, count, rec)
        off += count * rec
    return sec


class ReferencePanic(Exception):
    """The reference binary would panic (`unwrap`/`expect`) on this transcript."""


def _load(transcript: bytes, n: int, fast: bool):
    """preprocess-{kgz,fastkgz} `powersoftau_uncompress` + `load_powersoftau_accumulator`."""
    if len(transcript) != powersoftau_contribution_size(n):
        raise ReferencePanic("size mismatch (preprocess-kgz.rs:83-91)")
    sec = _sections(n)
    res = {}
    for name, (off, count, rec) in sec.items():
        check = name in ("tau_g1", "tau_g2", "alpha_g1") or (fast and name == "beta_g1")
        fn = g1_decompress_point if rec == 48 else g2_decompress_point
        outs = []
        for i in range(count):
            st, o = fn(transcript[off + i * rec: off + (i + 1) * rec], check=check)
            if st:
                raise ReferencePanic(f"{name}[{i}]: {ERROR_NAMES[st]}")
            outs.append(o)
        res[name] = outs
    return res


def preprocess_kgz(transcript: bytes, n: int) -> bytes:
    """preprocess-kgz.rs main (`:162-199`): [τG1 ×(2N−1)][ατG1 ×N][vk: g, gamma_g, h, beta_h]."""
    r = _load(transcript, n, fast=False)
    vk = r["tau_g1"][0] + r["alpha_g1"][0] + r["tau_g2"][0] + r["tau_g2"][1]
    return b"".join(r["tau_g1"]) + b"".join(r["alpha_g1"]) + vk


def preprocess_fastkgz(transcript: bytes, n: int) -> bytes:
    """preprocess-fastkgz.rs main (`:180-213`): [τG1][ατG1 (BTreeMap order)][h][beta_h][τG2 ×N]."""
    r = _load(transcript, n, fast=True)
    return (b"".join(r["tau_g1"]) + b"".join(r["alpha_g1"]) + r["tau_g2"][0] + r["tau_g2"][1]
            + b"".join(r["tau_g2"]))


def blake2b_hex(data: bytes) -> str:
    """`blake2b_simd::State::new().update(data).finalize().to_hex()` (64-byte digest)."""
    return hashlib.blake2b(data).hexdigest()
