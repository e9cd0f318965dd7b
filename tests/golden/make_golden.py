"""Generate the committed golden fixtures from the pure-Python oracle (oracle/kzgpot_oracle.py).

    python tests/golden/make_golden.py            # writes tests/golden/*.json, transcript fixture

Vectors (all seeded, deterministic):
  g1_decompress.json   compressed G1 → ark uncompressed, positive + negative (+ NO_SUBGROUP_CHECK mode)
  g2_decompress.json   compressed G2 → ark uncompressed, positive + negative
  g1_transcode.json    pairing-uncompressed G1 → ark (read_g1, src/lib.rs:41-54), incl. off-curve
  g2_transcode.json    pairing-uncompressed G2 → ark (read_g2, src/lib.rs:56-80)
  g1_load.json         ark uncompressed G1 → in-memory GroupAffine (deserialize_unchecked, the
  g2_load.json         load_kzg_setup / load_fastkzg_setup loaders, src/lib.rs:174-228)
  bn254_g1_decompress.json  config 5: ark-bn254 compressed G1 → ark uncompressed (no reference
                       counterpart; pinned by the BN254 spec constants and the ark format rules)
  transcript_n1024.bin a powersoftau response file for N = 2^10 (config 1), + expected digests of
                       the kgz / fastkgz outputs in transcript_n1024.json

The reference ships no vectors for this path; these pin our implementations to
one another and to the BLS12-381 spec constants (see the oracle header for what that does and
does not prove).
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import kzgpot_oracle as O  # noqa: E402

P = O.P


def _order_ell(rnd_point, mul, n, ell):
    """A point of order exactly ell: strip ell from n (the Sylow-ell part may be Z/ell x Z/ell,
    so [n/ell]R can be O for every R), then multiply by ell until the next step would give O."""
    m = n
    while m % ell == 0:
        m //= ell
    while True:
        t = mul(rnd_point(), m)
        if t is None:
            continue
        while True:
            t2 = mul(t, ell)
            if t2 is None:
                return t
            t = t2


def small_order_g1(rng, ell):
    return _order_ell(lambda: O.g1_random_on_curve(rng), O.g1_mul, O.H1 * O.R_ORDER, ell)


def small_order_g2(rng, ell):
    return _order_ell(lambda: O.g2_random_on_curve(rng), O.g2_mul, O.H2 * O.R_ORDER, ell)


def vec(kind, inp: bytes, status, out, note, check=True):
    return {"in": inp.hex(), "check": check, "status": status, "out": out.hex() if out else None, "note": note}


def g1_vectors(rng):
    V = []

    def add(enc, note, check=True):
        st, out = O.g1_decompress_point(enc, check=check)
        V.append(vec("g1", enc, st, out, note, check))

    add(O.pairing_g1_compress(O.G1_GEN), "generator")
    for i in range(96):
        add(O.pairing_g1_compress(O.g1_mul(O.G1_GEN, rng.randrange(1, O.R_ORDER))), f"random subgroup point {i}")
    q = O.g1_mul(O.G1_GEN, 12345)
    enc = bytearray(O.pairing_g1_compress(q))
    enc[0] ^= 0x20
    add(bytes(enc), "greatest bit flipped (= -P, still valid)")
    enc = bytearray(O.pairing_g1_compress(q))
    enc[0] &= 0x7F
    add(bytes(enc), "bit7 clear: UnexpectedCompressionMode")
    add(bytes([0xC0]) + bytes(47), "infinity: reference panics in read_g1")
    add(bytes([0xC0]) + bytes(47), "infinity, decompress-only section", check=False)
    add(bytes([0xE0]) + bytes(47), "infinity + greatest: UnexpectedInformation")
    add(bytes([0xC0]) + bytes(46) + b"\x01", "infinity with stray low bit")
    add(bytes([0xC1]) + bytes(47), "infinity with stray bit in byte 0")
    add(O.pairing_g1_compress(q), "valid point, decompress-only section", check=False)
    for note, x in (("x = p", P), ("x = p + 1", P + 1), ("x = 2^381 - 1", (1 << 381) - 1)):
        b = bytearray(x.to_bytes(48, "big"))
        b[0] |= 0x80
        add(bytes(b), note + ": not in field")
    nres = 0
    while nres < 6:
        x = rng.randrange(P)
        if O.fq_sqrt((x * x * x + 4) % P) is None:
            b = bytearray(x.to_bytes(48, "big"))
            b[0] |= 0x80 | (0x20 if nres % 2 else 0)
            add(bytes(b), "x^3+4 non-residue: NotOnCurve")
            nres += 1
    for i in range(16):
        add(O.pairing_g1_compress(O.g1_random_on_curve(rng)), f"on-curve, no cofactor clearing {i}")
    for i, ell in enumerate((3, 11, 10177, 859267, 52437899)):
        t = small_order_g1(rng, ell)
        add(O.pairing_g1_compress(t), f"order-{ell} point")
        pt = O.g1_add(O.g1_mul(O.G1_GEN, rng.randrange(1, O.R_ORDER)), t)
        add(O.pairing_g1_compress(pt), f"subgroup point + order-{ell} point")
        add(O.pairing_g1_compress(t), f"order-{ell} point, decompress-only", check=False)
    # a point with y = 0 would need x^3 = -4: check whether one exists and include it
    cube = pow((-4) % P, (2 * P - 1) // 9, P)
    if (cube ** 3 + 4) % P == 0:
        add(O.pairing_g1_compress((cube, 0)), "2-torsion point (y = 0)")
    return V


def g2_vectors(rng):
    V = []

    def add(enc, note, check=True):
        st, out = O.g2_decompress_point(enc, check=check)
        V.append(vec("g2", enc, st, out, note, check))

    add(O.pairing_g2_compress(O.G2_GEN), "generator")
    for i in range(32):
        add(O.pairing_g2_compress(O.g2_mul(O.G2_GEN, rng.randrange(1, O.R_ORDER))), f"random subgroup point {i}")
    q = O.g2_mul(O.G2_GEN, 777)
    enc = bytearray(O.pairing_g2_compress(q))
    enc[0] ^= 0x20
    add(bytes(enc), "greatest bit flipped")
    enc = bytearray(O.pairing_g2_compress(q))
    enc[0] &= 0x7F
    add(bytes(enc), "bit7 clear")
    add(bytes([0xC0]) + bytes(95), "infinity: reference panics in read_g2")
    add(bytes([0xC0]) + bytes(95), "infinity, decompress-only", check=False)
    add(bytes([0xE0]) + bytes(95), "infinity + greatest")
    add(bytes([0xC0]) + bytes(94) + b"\x01", "infinity with stray bit")
    for note, c1, c0 in (("x.c1 = p", P, 5), ("x.c0 = p", 5, P), ("x.c0 = p + 3", 1, P + 3)):
        b = bytearray(c1.to_bytes(48, "big") + c0.to_bytes(48, "big"))
        b[0] |= 0x80
        add(bytes(b), note + ": not in field")
    # x with c1 = 0 (exercises the Fp2 sqrt special cases)
    found = 0
    for x0 in range(1, 400):
        x = (x0, 0)
        rhs = O.fp2_add(O.fp2_mul(O.fp2_sqr(x), x), O.B2)
        if O.fq2_sqrt(rhs) is not None:
            b = bytearray((0).to_bytes(48, "big") + x0.to_bytes(48, "big"))
            b[0] |= 0x80 | (0x20 if found % 2 else 0)
            add(bytes(b), f"x.c1 = 0, x.c0 = {x0}")
            found += 1
            if found == 3:
                break
    nres = 0
    while nres < 4:
        x = (rng.randrange(P), rng.randrange(P))
        if O.fq2_sqrt(O.fp2_add(O.fp2_mul(O.fp2_sqr(x), x), O.B2)) is None:
            b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
            b[0] |= 0x80 | (0x20 if nres % 2 else 0)
            add(bytes(b), "non-residue: NotOnCurve")
            nres += 1
    for i in range(8):
        add(O.pairing_g2_compress(O.g2_random_on_curve(rng)), f"on-curve, no cofactor clearing {i}")
    for ell in (13, 23, 2713):
        t = small_order_g2(rng, ell)
        add(O.pairing_g2_compress(t), f"order-{ell} point")
        add(O.pairing_g2_compress(O.g2_add(O.g2_mul(O.G2_GEN, rng.randrange(1, O.R_ORDER)), t)),
            f"subgroup point + order-{ell} point")
    return V


def g1_transcode_vectors(rng):
    V = []

    def add(b, note):
        st, out = O.g1_transcode_point(b)
        V.append(vec("g1t", b, st, out, note))

    for i in range(24):
        add(O.pairing_g1_uncompressed(O.g1_mul(O.G1_GEN, rng.randrange(1, O.R_ORDER))), f"subgroup point {i}")
    add(O.pairing_g1_uncompressed(None), "pairing infinity encoding: x >= p after reversal")
    q = O.g1_mul(O.G1_GEN, 99)
    b = bytearray(O.pairing_g1_uncompressed(q))
    b[48] |= 0x80
    add(bytes(b), "PositiveY flag set on y (ignored for uncompressed)")
    b = bytearray(O.pairing_g1_uncompressed(q))
    b[48] |= 0x40
    add(bytes(b), "ark infinity flag set: accepted as infinity, x/y kept")
    b = bytearray(O.pairing_g1_uncompressed(q))
    b[48] |= 0xC0
    add(bytes(b), "both SW flags: UnexpectedFlags")
    b = bytearray(O.pairing_g1_uncompressed(q))
    b[48] |= 0x20
    add(bytes(b), "y >= p after flag removal")
    for i in range(4):
        x, y = rng.randrange(P), rng.randrange(P)
        add(x.to_bytes(48, "big") + y.to_bytes(48, "big"), f"random off-curve (x, y) {i}")
    # points on the isomorphic curve y^2 = x^3 + 4c^6 with order r: the reference (no on-curve
    # check) ACCEPTS them
    for i in range(4):
        c = rng.randrange(2, P)
        g = O.g1_mul(O.G1_GEN, rng.randrange(1, O.R_ORDER))
        pt = (g[0] * c * c % P, g[1] * c * c * c % P)
        add(O.pairing_g1_uncompressed(pt), f"order-r point on isomorphic off-curve twist {i}")
    add(bytes(48) + bytes(48), "(0, 0): singular off-curve point")
    add(bytes(47) + b"\x05" + bytes(48), "(5, 0): off-curve y = 0")
    for ell in (3, 11):
        add(O.pairing_g1_uncompressed(small_order_g1(rng, ell)), f"order-{ell} point")
    return V


def g2_transcode_vectors(rng):
    V = []

    def add(b, note):
        st, out = O.g2_transcode_point(b)
        V.append(vec("g2t", b, st, out, note))

    for i in range(8):
        add(O.pairing_g2_uncompressed(O.g2_mul(O.G2_GEN, rng.randrange(1, O.R_ORDER))), f"subgroup point {i}")
    add(O.pairing_g2_uncompressed(None), "pairing infinity encoding")
    q = O.g2_mul(O.G2_GEN, 5)
    b = bytearray(O.pairing_g2_uncompressed(q))
    b[96] |= 0x40
    add(bytes(b), "ark infinity flag on y.c1")
    b = bytearray(O.pairing_g2_uncompressed(q))
    b[96] |= 0xC0
    add(bytes(b), "both SW flags")
    b = bytearray(O.pairing_g2_uncompressed(q))
    b[144] |= 0x80
    add(bytes(b), "top bit of y.c0 set: y.c0 >= p")
    for i in range(2):
        add(bytes(rng.randrange(256) & (0x0F if k % 48 == 0 else 0xFF) for k in range(192)), f"random off-curve {i}")
    for ell in (13,):
        add(O.pairing_g2_uncompressed(small_order_g2(rng, ell)), f"order-{ell} point")
    return V


def g1_load_vectors(rng):
    V = []

    def add(b, note):
        st, out = O.g1_deserialize_unchecked_point(b)
        V.append(vec("g1l", b, st, out, note))

    for i in range(16):
        add(O.ark_g1_serialize((*O.g1_mul(O.G1_GEN, rng.randrange(1, O.R_ORDER)), False)), f"subgroup point {i}")
    add(O.ark_g1_serialize(O.ARK_G1_ZERO), "ark zero (0, 1, infinity)")
    q = O.g1_mul(O.G1_GEN, 7)
    b = bytearray(O.ark_g1_serialize((*q, False)))
    b[95] |= 0x40
    add(bytes(b), "infinity flag with finite coordinates: kept as read")
    b = bytearray(O.ark_g1_serialize((*q, False)))
    b[95] |= 0x80
    add(bytes(b), "PositiveY flag: ignored")
    b = bytearray(O.ark_g1_serialize((*q, False)))
    b[95] |= 0xC0
    add(bytes(b), "both SW flags: UnexpectedFlags")
    b = bytearray(O.ark_g1_serialize((*q, False)))
    b[95] |= 0x20
    add(bytes(b), "y >= p after flag removal")
    for note, x in (("x = p", P), ("x = p - 1", P - 1), ("x = 2^384 - 1", (1 << 384) - 1)):
        add(x.to_bytes(48, "little") + (3).to_bytes(48, "little"), note)
    add(bytes(96), "(0, 0) unchecked: accepted")
    for i in range(4):
        add(rng.randrange(P).to_bytes(48, "little") + rng.randrange(P).to_bytes(48, "little"),
            f"random off-curve (x, y) {i}: accepted (no curve check)")
    add(O.ark_g1_serialize((*small_order_g1(rng, 11), False)), "order-11 point: accepted (no subgroup check)")
    return V


def g2_load_vectors(rng):
    V = []

    def add(b, note):
        st, out = O.g2_deserialize_unchecked_point(b)
        V.append(vec("g2l", b, st, out, note))

    for i in range(8):
        add(O.ark_g2_serialize((*O.g2_mul(O.G2_GEN, rng.randrange(1, O.R_ORDER)), False)), f"subgroup point {i}")
    add(O.ark_g2_serialize(O.ARK_G2_ZERO), "ark zero")
    q = O.g2_mul(O.G2_GEN, 3)
    for note, byte, bit in (("infinity flag on y.c1", 191, 0x40), ("both SW flags", 191, 0xC0),
                            ("PositiveY flag", 191, 0x80), ("top bit of y.c0: y.c0 >= p", 143, 0x80),
                            ("top bit of x.c1: x.c1 >= p", 95, 0x80), ("bit 5 of y.c1: >= p", 191, 0x20)):
        b = bytearray(O.ark_g2_serialize((*q, False)))
        b[byte] |= bit
        add(bytes(b), note)
    add(b"".join(rng.randrange(P).to_bytes(48, "little") for _ in range(4)), "random off-curve: accepted")
    return V


def bn254_vectors(rng):
    V = []

    def add(b, note):
        st, out = O.bn254_g1_decompress_point(b)
        V.append(vec("bn", b, st, out, note))

    BP = O.BN_P
    add(O.bn254_g1_compress(O.BN_G1_GEN), "generator (1, 2)")
    for i in range(40):
        add(O.bn254_g1_compress(O.bn_mul(O.BN_G1_GEN, rng.randrange(1, O.BN_R))), f"random point {i}")
    q = O.bn_mul(O.BN_G1_GEN, 4242)
    b = bytearray(O.bn254_g1_compress(q))
    b[31] ^= 0x80
    add(bytes(b), "PositiveY flipped (= -P)")
    add(O.bn254_g1_compress(None), "infinity (ark zero)")
    add((5).to_bytes(32, "little")[:31] + b"\x40", "infinity flag with x = 5: zero()")
    b = bytearray((BP - 1).to_bytes(32, "little"))
    b[31] |= 0x40
    add(bytes(b), "infinity flag with x = p - 1: zero()")
    b = bytearray(BP.to_bytes(32, "little"))
    b[31] |= 0x40
    add(bytes(b), "infinity flag with x = p: InvalidData")
    b = bytearray(O.bn254_g1_compress(q))
    b[31] |= 0xC0
    add(bytes(b), "both SW flags: UnexpectedFlags")
    for note, x in (("x = p", BP), ("x = p + 1", BP + 1), ("x = 2^254 - 1", (1 << 254) - 1)):
        add(x.to_bytes(32, "little"), note + ": not in field")
    nres = 0
    while nres < 6:
        x = rng.randrange(BP)
        if O.bn_sqrt(x ** 3 + 3) is None:
            b = bytearray(x.to_bytes(32, "little"))
            b[31] |= 0x80 if nres % 2 else 0
            add(bytes(b), "x^3+3 non-residue: NotOnCurve")
            nres += 1
    return V


def main():
    rng = random.Random(20261015)
    for name, fn in (("g1_decompress", g1_vectors), ("g2_decompress", g2_vectors),
                     ("g1_transcode", g1_transcode_vectors), ("g2_transcode", g2_transcode_vectors)):
        V = fn(rng)
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump({"generator": "tests/golden/make_golden.py", "oracle": "oracle/kzgpot_oracle.py",
                       "vectors": V}, f, indent=0)
        print(name, len(V), "vectors;", sum(v["status"] == 0 for v in V), "accepted")
    rng = random.Random(20261016)  # separate stream: the loader vectors came later
    for name, fn in (("g1_load", g1_load_vectors), ("g2_load", g2_load_vectors),
                     ("bn254_g1_decompress", bn254_vectors)):
        V = fn(rng)
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump({"generator": "tests/golden/make_golden.py", "oracle": "oracle/kzgpot_oracle.py",
                       "vectors": V}, f, indent=0)
        print(name, len(V), "vectors;", sum(v["status"] == 0 for v in V), "accepted")
    n = 1 << 10
    tr = O.make_response_transcript(n, seed=1)
    with open(os.path.join(HERE, "transcript_n1024.bin"), "wb") as f:
        f.write(tr)
    kgz = O.preprocess_kgz(tr, n)
    fast = O.preprocess_fastkgz(tr, n)
    meta = {
        "n": n, "seed": 1, "transcript_blake2b": O.blake2b_hex(tr), "transcript_size": len(tr),
        "kgz_size": len(kgz), "kgz_blake2b": O.blake2b_hex(kgz),
        "fastkgz_size": len(fast), "fastkgz_blake2b": O.blake2b_hex(fast),
        "kgz_head_hex": kgz[:192].hex(), "kgz_tail_hex": kgz[-576:].hex(),
        "fastkgz_tail_hex": fast[-192:].hex(),
    }
    st, loaded = O.load_kzg_setup(kgz, n)
    assert st == 0
    meta["load_kzg_blake2b"] = O.blake2b_hex(b"".join(loaded))
    st, loaded = O.load_fastkzg_setup(fast, n)
    assert st == 0
    meta["load_fastkzg_blake2b"] = O.blake2b_hex(b"".join(loaded))
    with open(os.path.join(HERE, "transcript_n1024.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("transcript", len(tr), "kgz", len(kgz), "fastkgz", len(fast))


if __name__ == "__main__":
    main()
