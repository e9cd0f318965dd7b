"""Randomized parity: streams of random records through the HIP codec (C ABI) and the C oracle
(oracle/kzgpot_ref.c: the reference's own algorithms — pairing sqrt + sign rule, ark
deserialize_uncompressed with the subgroup check by double-and-add by r).

Random x values land on the curve about half the time, and such a point is essentially never in
the r-subgroup (the cofactor is ~2^126 for G1 and ~2^256 for G2). These streams therefore hit the
NotInSubgroup verdict thousands of times with distinct points, next to non-residues, x >= p,
flag damage and valid subgroup points. That is the equivalence the endomorphism tests (phi/psi)
must keep with the reference's multiplication by r (src/lib.rs:41-80). The transcode streams add
random OFF-curve (x, y), which the reference accepts or rejects by ark's double-and-add with no
curve check. Bytes, per-point status and first_bad must all match."""
import ctypes
import random

import pytest

from conftest import golden, oracle_run

pytestmark = pytest.mark.gpu

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def _rand_fp(rng):
    return rng.randrange(P)


def _compressed_fp(rng, x, kind):
    """48-B pairing compressed encoding of x with random flag damage (kind picks the class)."""
    b = bytearray(x.to_bytes(48, "big"))
    if kind < 80:
        b[0] |= 0x80 | (0x20 if rng.random() < 0.5 else 0)  # well-formed, either sign
    elif kind < 85:
        pass  # compression bit clear -> UnexpectedCompressionMode
    elif kind < 90:
        b = bytearray(48)
        b[0] = 0xC0 if rng.random() < 0.5 else 0xE0  # infinity (rejected on a checked stream)
    elif kind < 95:
        b[0] |= 0xC0  # infinity flag with garbage -> UnexpectedInformation
    else:
        b = bytearray((P + rng.randrange(1 << 32)).to_bytes(48, "big"))  # x >= p
        b[0] |= 0x80
    return bytes(b)


def _subgroup_g1(oracle_lib, n, seed):
    rng = random.Random(seed)
    scal = b"".join(rng.randrange(1, 1 << 255).to_bytes(32, "big") for _ in range(n))
    comp = ctypes.create_string_buffer(n * 48)
    ark = ctypes.create_string_buffer(n * 96)
    oracle_lib.oracle_g1_scalar_mul_encode(scal, ctypes.c_size_t(n), comp, ark)
    return [comp.raw[i * 48:(i + 1) * 48] for i in range(n)]


@pytest.mark.parametrize("mode", [0, 4], ids=["fused", "split"])
def test_fuzz_g1_decompress(gpu, oracle_lib, mode):
    rng = random.Random(1234 + mode)
    n = 4000
    valid = _subgroup_g1(oracle_lib, 64, seed=77)
    recs = []
    for _ in range(n):
        k = rng.randrange(100)
        recs.append(rng.choice(valid) if k < 10 else _compressed_fp(rng, _rand_fp(rng), k))
    data = b"".join(recs)
    r = gpu.run_codec("g1_decompress", data, mode, want_status=True)
    out, st, fb, ret = oracle_run(oracle_lib, "g1_decompress", data, n, threads=8)
    assert r.status == st
    assert r.out == out
    assert (r.ret, r.first_bad) == (ret, fb)
    assert st.count(5) > 1000  # thousands of distinct on-curve, off-subgroup points


@pytest.mark.parametrize("mode", [0, 4], ids=["fused", "split"])
def test_fuzz_g2_decompress(gpu, oracle_lib, mode):
    rng = random.Random(4321 + mode)
    n = 1500
    valid = [bytes.fromhex(v["in"]) for v in golden("g2_decompress") if v["check"] and v["status"] == 0]
    recs = []
    for _ in range(n):
        k = rng.randrange(100)
        if k < 10:
            recs.append(rng.choice(valid))
            continue
        c1 = _compressed_fp(rng, _rand_fp(rng), k)  # flags live on x.c1 (sent first)
        c0 = _rand_fp(rng).to_bytes(48, "big") if rng.random() < 0.97 else (P + 1).to_bytes(48, "big")
        recs.append(c1 + c0)
    data = b"".join(recs)
    r = gpu.run_codec("g2_decompress", data, mode, want_status=True)
    out, st, fb, ret = oracle_run(oracle_lib, "g2_decompress", data, n, threads=8)
    assert r.status == st
    assert r.out == out
    assert (r.ret, r.first_bad) == (ret, fb)
    assert st.count(5) > 300


def _pairing_uncompressed_g1(ark_rec):
    """ark G1 record (x LE ‖ y LE) -> pairing uncompressed (x BE ‖ y BE): the A6 identity."""
    return ark_rec[:48][::-1] + ark_rec[48:96][::-1]


def _pairing_uncompressed_g2(ark_rec):
    """ark G2 (x.c0, x.c1, y.c0, y.c1 LE) -> pairing (x.c1, x.c0, y.c1, y.c0 BE)."""
    c = [ark_rec[i * 48:(i + 1) * 48][::-1] for i in range(4)]
    return c[1] + c[0] + c[3] + c[2]


def test_fuzz_g1_transcode(gpu, oracle_lib):
    """read_g1 on: on-curve off-subgroup points (random x decompressed without the subgroup
    check), random off-curve (x, y) (the reference's ark double-and-add decides them), valid
    subgroup points, y >= p and flag damage."""
    rng = random.Random(99)
    m = 1200
    comp = b"".join(_compressed_fp(rng, _rand_fp(rng), 0) for _ in range(m))
    oc, ost, _, _ = oracle_run(oracle_lib, "g1_decompress", comp, m, flags=1, threads=8)
    on_curve = [_pairing_uncompressed_g1(oc[i * 96:(i + 1) * 96]) for i in range(m) if ost[i] == 0]
    valid = [bytes.fromhex(v["in"]) for v in golden("g1_transcode") if v["status"] == 0]
    recs = []
    for i in range(2000):
        k = rng.randrange(100)
        if k < 40:
            recs.append(rng.choice(on_curve))
        elif k < 50:
            recs.append(rng.choice(valid))
        elif k < 90:
            recs.append(_rand_fp(rng).to_bytes(48, "big") + _rand_fp(rng).to_bytes(48, "big"))
        elif k < 95:
            recs.append(_rand_fp(rng).to_bytes(48, "big") + (P + rng.randrange(1 << 20)).to_bytes(48, "big"))
        else:
            b = bytearray(rng.choice(on_curve))
            b[0] |= rng.choice([0x80, 0x40, 0xC0, 0x20])
            recs.append(bytes(b))
    data = b"".join(recs)
    n = len(recs)
    r = gpu.run_codec("g1_transcode", data, 0, want_status=True)
    out, st, fb, ret = oracle_run(oracle_lib, "g1_transcode", data, n, threads=8)
    assert r.status == st
    assert r.out == out
    assert (r.ret, r.first_bad) == (ret, fb)


def test_fuzz_g2_transcode(gpu, oracle_lib):
    rng = random.Random(7)
    m = 400
    comp = b"".join(_compressed_fp(rng, _rand_fp(rng), 0) + _rand_fp(rng).to_bytes(48, "big") for _ in range(m))
    oc, ost, _, _ = oracle_run(oracle_lib, "g2_decompress", comp, m, flags=1, threads=8)
    on_curve = [_pairing_uncompressed_g2(oc[i * 192:(i + 1) * 192]) for i in range(m) if ost[i] == 0]
    valid = [bytes.fromhex(v["in"]) for v in golden("g2_transcode") if v["status"] == 0]
    recs = []
    for _ in range(600):
        k = rng.randrange(100)
        if k < 45:
            recs.append(rng.choice(on_curve))
        elif k < 55:
            recs.append(rng.choice(valid))
        else:
            recs.append(b"".join(_rand_fp(rng).to_bytes(48, "big") for _ in range(4)))
    data = b"".join(recs)
    n = len(recs)
    r = gpu.run_codec("g2_transcode", data, 0, want_status=True)
    out, st, fb, ret = oracle_run(oracle_lib, "g2_transcode", data, n, threads=8)
    assert r.status == st
    assert r.out == out
    assert (r.ret, r.first_bad) == (ret, fb)


P_BN = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47


def test_fuzz_bn254_decompress(gpu):
    """Config 5's codec on random ark-compressed BN254 records (x LE, SWFlags in byte 31): random
    x (about half on the curve; cofactor 1, so every curve point is accepted), x >= p, both
    flags, infinity. Checked point by point against the Python oracle (ark-bn254 0.2
    deserialize -> serialize_uncompressed)."""
    O = pytest.importorskip("kzgpot_oracle")
    rng = random.Random(254)
    recs = []
    for _ in range(1500):
        k = rng.randrange(100)
        if k < 85:
            x = rng.randrange(P_BN)
        elif k < 90:
            x = P_BN + rng.randrange(1 << 20)
        else:
            x = 0
        if k >= 90 or rng.random() < 0.05:
            flags = rng.choice([0x00, 0x40, 0x80, 0xC0])  # Infinity / both set / plain
        else:
            flags = rng.choice([0x00, 0x80])  # PositiveY clear or set
        b = bytearray(x.to_bytes(32, "little"))
        b[31] |= flags
        recs.append(bytes(b))
    data = b"".join(recs)
    r = gpu.bn254_g1_decompress(data, want_status=True)
    want_st, want_out = [], []
    for rec in recs:
        st, out = O.bn254_g1_decompress_point(rec)
        want_st.append(st)
        want_out.append(out if st == 0 else bytes(64))
    assert list(r.status) == want_st
    assert r.out == b"".join(want_out)
    bad = [i for i, s in enumerate(want_st) if s]
    assert r.first_bad == (bad[0] if bad else -1)
    assert 300 < want_st.count(0) and want_st.count(4) > 300


@pytest.mark.parametrize("g2", [False, True], ids=["g1", "g2"])
def test_fuzz_loader(gpu, g2):
    """load_kzg_setup's per-point work (ark deserialize_unchecked: coordinates < p, SWFlags, x 2^384
    into ark Montgomery form) on random records — random canonical coordinates (no curve needed),
    coordinates >= p and every flag combination on y's top byte — against the Python oracle."""
    O = pytest.importorskip("kzgpot_oracle")
    rng = random.Random(200 + g2)
    nc = 4 if g2 else 2
    recs = []
    for i in range(3000 if not g2 else 1500):
        k = rng.randrange(100)
        coords = [_rand_fp(rng) for _ in range(nc)]
        if i < 4:
            coords = [[0, 1, P - 1, (1 << 381) - 1][i]] * nc
        elif k < 5:
            coords[rng.randrange(nc)] = P + rng.randrange(1 << 40)
        b = bytearray(b"".join(c.to_bytes(48, "little") for c in coords))
        if k >= 90 or (i >= 4 and i % 13 == 0):
            b[-1] |= rng.choice([0x40, 0x80, 0xC0])  # Infinity / PositiveY / both (UnexpectedFlags)
        recs.append(bytes(b))
    data = b"".join(recs)
    r = gpu.deserialize_unchecked(data, g2=g2, want_status=True)
    fn = O.g2_deserialize_unchecked_point if g2 else O.g1_deserialize_unchecked_point
    rout = 200 if g2 else 104
    want_st, want_out = [], []
    for rec in recs:
        st, out = fn(rec)
        want_st.append(st)
        want_out.append(out if st == 0 else bytes(rout))
    assert list(r.status) == want_st
    assert r.out == b"".join(want_out)
    assert want_st.count(0) > 1000 if not g2 else want_st.count(0) > 500


@pytest.mark.parametrize("g2", [False, True], ids=["g1", "g2"])
def test_loader_fault_precedence_and_tails(gpu, g2):
    """Records with several faults at once (coordinates >= p in any subset, with and without flag
    damage on y's top byte), so the per-record status must be the FIRST fault in ark's read order
    (x[.c0, .c1], then y[.c0], the flags, y[.c1]) — the direct loader merges its lanes' statuses by
    lane order — at stream lengths around the kernels' 128- / 32-point blocks (ragged tails, single
    records) and the first_bad of each stream, against the Python oracle."""
    O = pytest.importorskip("kzgpot_oracle")
    rng = random.Random(900 + g2)
    nc = 4 if g2 else 2
    fn = O.g2_deserialize_unchecked_point if g2 else O.g1_deserialize_unchecked_point
    rout = 200 if g2 else 104
    recs = []
    for mask in range(1 << nc):
        for flags in (0x00, 0x40, 0x80, 0xC0):
            coords = [P + rng.randrange(1 << 40) if mask >> c & 1 else _rand_fp(rng) for c in range(nc)]
            b = bytearray(b"".join(c.to_bytes(48, "little") for c in coords))
            b[-1] |= flags
            recs.append(bytes(b))
    ok = [rec for rec in recs if fn(rec)[0] == 0]
    assert ok and len({fn(rec)[0] for rec in recs}) >= 3  # accepted, InvalidData and UnexpectedFlags all occur
    block = 32 if g2 else 128
    for n in (1, 2, block - 1, block, block + 1, 2 * block + 3, len(recs)):
        stream = [recs[(7 * i + n) % len(recs)] if i % 3 == 0 else ok[i % len(ok)] for i in range(n)]
        r = gpu.deserialize_unchecked(b"".join(stream), g2=g2, want_status=True)
        want = [fn(rec) for rec in stream]
        want_st = [st for st, _ in want]
        assert list(r.status) == want_st, n
        assert r.out == b"".join(out if st == 0 else bytes(rout) for st, out in want), n
        bad = [i for i, s in enumerate(want_st) if s]
        assert r.first_bad == (bad[0] if bad else -1), n
