"""Full-population independent parity at the BASELINE sizes (the 2^27 round
trip compared the codec with a generator built from the same fp381.hpp / curve.hpp; only 16,640
points of it were re-decoded by the C oracle).

tests/gpu_oracle/oracle_gpu.hip restates the C oracle's per-point functions (oracle/kzgpot_ref.c:
6 x 64-bit ark-ff CIOS, pairing's Fq::sqrt / Fq2::sqrt Algorithm 9, ark mul_bits(r), byte-level
parsing) and the Python oracle's BN254 decompression as device code, sharing nothing with csrc/.
First it is pinned to the oracles themselves — every golden vector and mixed random streams (valid,
off-subgroup, non-residue, x >= p, flag damage) must give the C / Python oracle's bytes and
statuses — then it re-derives EVERY point of config 4 (2^27 G1 + 2^16 G2), config 3's 2^20 G2,
2^24 transcoded G1 records and config 5 (2^28 BN254), which the product kernels' output must equal
byte for byte. Reference anchors: src/bin/preprocess-kgz.rs:105-110 (decompression),
src/lib.rs:41-80 (read_g1 / read_g2), preprocess-kgz.rs:188-194 (serialize_uncompressed)."""
import ctypes
import os
import random
import subprocess

import pytest

from conftest import ROOT, golden, oracle_run

pytestmark = pytest.mark.gpu

PORT = os.path.join(ROOT, "tests", "gpu_oracle", "build", "liboracle_gpu.so")
OPS = {"g1_decompress": (0, 48, 96), "g2_decompress": (1, 96, 192), "g1_transcode": (2, 96, 96),
       "g2_transcode": (3, 192, 192), "bn254_g1_decompress": (4, 32, 64), "g1_load": (5, 96, 104),
       "g2_load": (6, 192, 200)}


@pytest.fixture(scope="module")
def port(gpu):
    if not os.path.exists(PORT):
        subprocess.run(["make", "-C", os.path.dirname(os.path.dirname(PORT))], check=True)
    lib = ctypes.CDLL(PORT)
    lib.oracle_gpu_run.restype = ctypes.c_int
    lib.oracle_gpu_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_uint32, ctypes.c_void_p]
    return lib


def run_port(port, op, d_in, flags=0):
    """The port over device bytes d_in: (out, status) device tensors."""
    import torch

    code, rin, rout = OPS[op]
    n = d_in.numel() // rin
    out = torch.full((max(1, n * rout),), 0x5A, dtype=torch.uint8, device=d_in.device)
    st = torch.full((max(1, n),), 0xEE, dtype=torch.uint8, device=d_in.device)
    rc = port.oracle_gpu_run(code, d_in.data_ptr(), n, out.data_ptr(), st.data_ptr(), flags,
                             torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
    torch.cuda.synchronize()
    return out[:n * rout], st[:n]


def port_host(port, op, data: bytes, flags=0):
    import torch

    d = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    out, st = run_port(port, op, d, flags)
    return bytes(out.cpu().numpy()), bytes(st.cpu().numpy())


# ------------------------------------------------------------------ the port against the oracles
@pytest.mark.parametrize("op", ["g1_decompress", "g2_decompress", "g1_transcode", "g2_transcode"])
@pytest.mark.parametrize("flags", [0, 1], ids=["checked", "unchecked"])
def test_port_matches_c_oracle_on_golden_vectors(port, oracle_lib, op, flags):
    if flags and "transcode" in op:
        pytest.skip("the transcode path has no unchecked mode")
    vecs = golden(op)  # every vector in both modes: the oracle defines the answer for any input
    data = b"".join(bytes.fromhex(v["in"]) for v in vecs)
    n = len(vecs)
    out, st, _, _ = oracle_run(oracle_lib, op, data, n, flags=flags)
    pout, pst = port_host(port, op, data, flags)
    assert pst == st and pout == out


def _mixed_g1(oracle_lib, n, seed):
    """n compressed G1 points: multiples [k]G from the C oracle, with every 7th replaced by a
    golden negative (off-subgroup, non-residue, x >= p, flags) and every 11th by random bytes with
    the compression bit set (mostly non-residues or x >= p; on-curve ones are off-subgroup)."""
    rng = random.Random(seed)
    scal = b"".join(rng.randrange(1, 1 << 255).to_bytes(32, "big") for _ in range(n))
    comp = ctypes.create_string_buffer(n * 48)
    ark = ctypes.create_string_buffer(n * 96)
    oracle_lib.oracle_g1_scalar_mul_encode(scal, ctypes.c_size_t(n), comp, ark)
    data = bytearray(comp.raw)
    negs = [bytes.fromhex(v["in"]) for v in golden("g1_decompress") if v["status"]]
    for i in range(3, n, 7):
        data[i * 48:(i + 1) * 48] = rng.choice(negs)
    for i in range(5, n, 11):
        r = bytearray(rng.randbytes(48))
        r[0] = 0x80 | (r[0] & 0x3F)
        data[i * 48:(i + 1) * 48] = r
    return bytes(data)


@pytest.mark.parametrize("flags", [0, 1], ids=["checked", "unchecked"])
def test_port_matches_c_oracle_on_mixed_g1_stream(port, oracle_lib, flags):
    n = 1500
    data = _mixed_g1(oracle_lib, n, seed=17 + flags)
    out, st, _, _ = oracle_run(oracle_lib, "g1_decompress", data, n, flags=flags)
    pout, pst = port_host(port, "g1_decompress", data, flags)
    assert sum(s != 0 for s in st) > 100  # the stream exercises the reject paths
    assert pst == st and pout == out


def test_port_matches_c_oracle_on_mixed_g2_stream(port, oracle_lib):
    vecs = [bytes.fromhex(v["in"]) for v in golden("g2_decompress")]
    rng = random.Random(23)
    n = 400
    data = b"".join(rng.choice(vecs) for _ in range(n))
    out, st, _, _ = oracle_run(oracle_lib, "g2_decompress", data, n)
    pout, pst = port_host(port, "g2_decompress", data)
    assert pst == st and pout == out


def test_port_matches_python_oracle_on_bn254(port):
    """BN254 has no C restatement: the port follows kzgpot_oracle.bn254_g1_decompress_point, whose
    golden vectors (valid, infinity, flag and range rejects, non-residues) it must reproduce."""
    import kzgpot_oracle as O

    vecs = golden("bn254_g1_decompress")
    data = b"".join(bytes.fromhex(v["in"]) for v in vecs)
    pout, pst = port_host(port, "bn254_g1_decompress", data)
    for i, v in enumerate(vecs):
        status, want = O.bn254_g1_decompress_point(bytes.fromhex(v["in"]))
        assert pst[i] == status, v.get("note")
        assert pout[i * 64:(i + 1) * 64] == (want if want is not None else bytes(64)), v.get("note")


@pytest.mark.parametrize("op,name,g2", [("g1_load", "g1_load", False), ("g2_load", "g2_load", True)])
def test_port_matches_python_oracle_on_loader_vectors(port, op, name, g2):
    """The loader (ark deserialize_unchecked into the in-memory GroupAffine) against the Python
    oracle's g1/g2_deserialize_unchecked_point on the loader golden vectors."""
    import kzgpot_oracle as O

    rin, rout = (192, 200) if g2 else (96, 104)
    fn = O.g2_deserialize_unchecked_point if g2 else O.g1_deserialize_unchecked_point
    vecs = golden(name)
    data = b"".join(bytes.fromhex(v["in"]) for v in vecs)
    pout, pst = port_host(port, op, data)
    for i, v in enumerate(vecs):
        status, want = fn(bytes.fromhex(v["in"]))
        assert pst[i] == status, v.get("note")
        assert pout[i * rout:(i + 1) * rout] == (want if want is not None else bytes(rout)), v.get("note")


# ------------------------------------------------------------------ full populations
@pytest.fixture(scope="module")
def dev(gpu):
    import torch

    from kzgpot import device as D

    return torch, D, torch.device("cuda", 0)


def _product(D, torch, op, comp, rout, flags=0):
    n = comp.numel() // OPS[op][1]
    out = torch.empty(n * rout, dtype=torch.uint8, device=comp.device)
    key = torch.empty(1, dtype=torch.int64, device=comp.device)
    D.codec_dev(op, comp, out, key, flags)
    return out, D.read_key(key)


def test_config4_every_point_matches_the_port(port, dev):
    """BASELINE config 4 at its size: all 2^27 G1 and 2^16 G2 records of the product codec equal
    the oracle port's, and the port accepts every point."""
    torch, D, cuda = dev
    for kind, op, n, seed in (("g2", "g2_decompress", 1 << 16, 11), ("g1", "g1_decompress", 1 << 27, 10)):
        comp, _ = D.synth(kind, seed, 0, n, cuda, with_expected=False)
        out, key = _product(D, torch, op, comp, OPS[op][2])
        assert key == (1 << 64) - 1
        pout, pst = run_port(port, op, comp)
        assert int(pst.count_nonzero()) == 0, op
        assert torch.equal(out, pout), op
        del comp, out, pout, pst
        torch.cuda.empty_cache()


def test_config3_g2_every_point_matches_the_port(port, dev):
    torch, D, cuda = dev
    comp, _ = D.synth("g2", 5, 0, 1 << 20, cuda, with_expected=False)
    out, key = _product(D, torch, "g2_decompress", comp, 192)
    pout, pst = run_port(port, "g2_decompress", comp)
    assert key == (1 << 64) - 1 and int(pst.count_nonzero()) == 0
    assert torch.equal(out, pout)


def test_transcode_2e24_every_record_matches_the_port(port, dev):
    """The uncompressed-input mode (read_g1 loop) on bench.py's 2^24 records."""
    torch, D, cuda = dev
    n = 1 << 24
    _, ark = D.synth("g1", 12, 0, n, cuda)
    pin = ark.view(n, 2, 48).flip(-1).contiguous().view(-1)  # pairing-uncompressed = byte-reversed coords
    del ark
    out, key = _product(D, torch, "g1_transcode", pin, 96)
    pout, pst = run_port(port, "g1_transcode", pin)
    assert key == (1 << 64) - 1 and int(pst.count_nonzero()) == 0
    assert torch.equal(out, pout)


def test_loaders_every_record_matches_the_port(port, dev):
    """The load_kzg_setup / load_fastkzg_setup per-point work at bench.py's sizes: 2^27 G1 ark
    records -> 104-B GroupAffine and 2^26 G2 -> 200-B, product loader against the port."""
    torch, D, cuda = dev
    n = 1 << 27
    _, ark = D.synth("g1", 13, 0, n, cuda)  # the generator's ark bytes (every record valid)
    for op, recs, rin, rout in (("g1_load", n, 96, 104), ("g2_load", n // 2, 192, 200)):
        src = ark[:recs * rin]
        out, key = _product(D, torch, op, src, rout)
        assert key == (1 << 64) - 1
        pout, pst = run_port(port, op, src)
        assert int(pst.count_nonzero()) == 0, op
        assert torch.equal(out, pout), op
        del out, pout, pst
        torch.cuda.empty_cache()


def test_config5_every_point_matches_the_port(port, dev):
    """BASELINE config 5 at its size: all 2^28 BN254 records (16 GiB) against the port of the
    Python oracle's decompression."""
    torch, D, cuda = dev
    n = 1 << 28
    comp, _ = D.synth("bn254", 9, 0, n, cuda, with_expected=False)
    out, key = _product(D, torch, "bn254_g1_decompress", comp, 64)
    assert key == (1 << 64) - 1
    pout, pst = run_port(port, "bn254_g1_decompress", comp)
    assert int(pst.count_nonzero()) == 0
    assert torch.equal(out, pout)


# ------------------------------------------------------------------ random streams at scale
def _random_records(torch, n, rec, seed, fix):
    """n random records of `rec` bytes on the GPU, shaped by fix(view) in place."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    r = torch.randint(0, 256, (n, rec), dtype=torch.uint8, device="cuda", generator=g)
    fix(r)
    return r.view(-1)


def _compare_random(port, dev, op, d_in, flags=0):
    """Product (fast subgroup test) vs the oracle port on the same random records: bytes and every
    per-point status. Returns the port's status histogram."""
    torch, D, _ = dev
    _, rin, rout = OPS[op]
    n = d_in.numel() // rin
    out = torch.empty(n * rout, dtype=torch.uint8, device=d_in.device)
    st = torch.empty(n, dtype=torch.uint8, device=d_in.device)
    key = torch.empty(1, dtype=torch.int64, device=d_in.device)
    D.codec_dev(op, d_in, out, key, flags, d_status=st)
    pout, pst = run_port(port, op, d_in, flags)
    assert torch.equal(st, pst), (op, (st != pst).nonzero()[:8].flatten().tolist())
    assert torch.equal(out, pout), op
    return {int(k): int(v) for k, v in zip(*torch.unique(pst, return_counts=True))}


def test_random_g1_x_at_scale(port, dev):
    """2^22 random G1 encodings (compression bit set, random infinity / greatest bits, random x):
    about half are on the curve and, being random, outside G1 — every one of those ~2^21 points is
    decided by the product's endomorphism test and by ark's mul_bits(r) in the port, identically."""
    torch = dev[0]

    def fix(r):
        r[:, 0] = 0x80 | (r[:, 0] & 0x7F)

    hist = _compare_random(port, dev, "g1_decompress", _random_records(torch, 1 << 22, 48, 1, fix))
    assert hist.get(5, 0) > (1 << 19)  # NotInSubgroup: the off-subgroup on-curve points
    assert hist.get(4, 0) > (1 << 19) and hist.get(3, 0) > 0 and hist.get(2, 0) > 0


def test_random_g2_x_at_scale(port, dev):
    torch = dev[0]

    def fix(r):
        r[:, 0] = 0x80 | (r[:, 0] & 0x3F)  # no infinity bit: every record reaches the square root
        r[:, 48] &= 0x1F                      # x.c0 < 2^381: mostly < p

    hist = _compare_random(port, dev, "g2_decompress", _random_records(torch, 1 << 18, 96, 2, fix))
    assert hist.get(5, 0) > (1 << 15) and hist.get(4, 0) > (1 << 15)


def test_random_uncompressed_at_scale(port, dev):
    """read_g1 / read_g2 on random (x, y): almost all OFF the curve, which the reference never
    checks — the product decides those with ark's exact double-and-add, the port with its own —
    and SWFlags on y at random (both set: UnexpectedFlags; infinity: ark accepts any x, y)."""
    torch = dev[0]

    def fix1(r):
        r[:, 0] &= 0x1F   # x < 2^381
        r[:, 48] &= 0xDF  # y's top byte: random SWFlags, value bits mostly < p

    def fix2(r):  # pairing G2 uncompressed: x.c1 | x.c0 | y.c1 | y.c0; the flags ride on y.c1's top byte
        for k in (0, 48, 144):
            r[:, k] &= 0x1F
        r[:, 96] &= 0xDF

    h1 = _compare_random(port, dev, "g1_transcode", _random_records(torch, 1 << 17, 96, 3, fix1))
    h2 = _compare_random(port, dev, "g2_transcode", _random_records(torch, 1 << 15, 192, 4, fix2))
    for h in (h1, h2):
        assert h.get(6, 0) > 0 and h.get(5, 0) > 0 and h.get(0, 0) > 0, h  # flags / off-curve / infinity


def test_random_loader_records_at_scale(port, dev):
    """deserialize_unchecked on random records: x / y ranges and random SWFlags on the last
    coordinate, no curve check (most records are accepted as they are)."""
    torch = dev[0]

    def fix1(r):
        r[:, 47] &= 0x1F  # x < 2^381 (LE: the top byte is the last)
        r[:, 95] &= 0xDF  # y: random SWFlags

    def fix2(r):
        for k in (47, 95, 143):
            r[:, k] &= 0x1F
        r[:, 191] &= 0xDF

    for op, rec, fix in (("g1_load", 96, fix1), ("g2_load", 192, fix2)):
        h = _compare_random(port, dev, op, _random_records(torch, 1 << 20, rec, 6, fix))
        assert h.get(0, 0) > 0 and h.get(3, 0) > 0 and h.get(6, 0) > 0, (op, h)


def test_random_bn254_at_scale(port, dev):
    torch = dev[0]

    def fix(r):
        r[:, 31] &= 0xDF  # random PositiveY / Infinity flags, x mostly < p

    hist = _compare_random(port, dev, "bn254_g1_decompress", _random_records(torch, 1 << 22, 32, 5, fix))
    assert hist.get(0, 0) > (1 << 19) and hist.get(4, 0) > (1 << 19) and hist.get(6, 0) > 0


def test_preprocess_2e21_output_matches_the_port(port, dev, kzgpot_mod):
    """The reference's own size, N = 2^21 (preprocess-kgz.rs:162-199, preprocess-fastkgz.rs:180-214):
    a full response-layout transcript of GPU-generated points through kzgpot_preprocess_buffer, and
    the expected kgz / fastkzg files assembled from the port's decode of every section (τG1, ατG1
    and τG2 checked, βτG1 checked in fastkzg only, βG2 decompress-only): byte-equal files."""
    torch, D, cuda = dev
    n = 1 << 21
    cnt = [("g1", 2 * n - 1), ("g2", n), ("g1", n), ("g1", n), ("g2", 1)]
    parts = [torch.zeros(64, dtype=torch.uint8, device=cuda)]
    for k, (kind, c) in enumerate(cnt):
        parts.append(D.synth(kind, 90 + k, 0, c, cuda, with_expected=False)[0])
    parts.append(torch.zeros(3 * 192 + 6 * 96, dtype=torch.uint8, device=cuda))
    tr = torch.cat(parts)
    del parts
    secs, off = [], 64
    for kind, c in cnt:
        rin = 48 if kind == "g1" else 96
        secs.append(tr[off:off + c * rin])
        off += c * rin
    host_tr = tr.cpu().numpy().tobytes()
    for mode in (kzgpot_mod.MODE_KZG, kzgpot_mod.MODE_FASTKZG):
        got = kzgpot_mod.preprocess_buffer(host_tr, 21, mode, n_gpus=1)
        checked = [True, True, True, mode == kzgpot_mod.MODE_FASTKZG, False]
        dec = []
        for (kind, c), sec, chk in zip(cnt, secs, checked):
            out, st = run_port(port, f"{kind}_decompress", sec, 0 if chk else 1)
            assert int(st.count_nonzero()) == 0
            dec.append(out)
        tau_g1, tau_g2, alpha_g1 = dec[0], dec[1], dec[2]
        if mode == kzgpot_mod.MODE_KZG:  # Powers + VerifierKey{g, gamma_g, h, beta_h}
            want = torch.cat([tau_g1, alpha_g1, tau_g1[:96], alpha_g1[:96], tau_g2[:384]])
        else:  # UniversalParams (powers_of_g, powers_of_gamma_g, h, beta_h) + powers_of_h
            want = torch.cat([tau_g1, alpha_g1, tau_g2[:384], tau_g2])
        assert len(got) == want.numel() == kzgpot_mod.output_size(21, mode)
        assert got == want.cpu().numpy().tobytes(), mode
