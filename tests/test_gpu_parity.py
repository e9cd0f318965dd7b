"""GPU parity: the HIP codec (through the C ABI) against the oracle — bit-exact bytes and
identical accept/reject on every vector, in both subgroup modes."""
import ctypes
import hashlib
import json
import os
import random

import pytest

from conftest import GOLDEN, golden, oracle_run

pytestmark = pytest.mark.gpu

OPS = [("g1_decompress", 48, 96), ("g2_decompress", 96, 192), ("g1_transcode", 96, 96), ("g2_transcode", 192, 192)]


@pytest.mark.parametrize("op,rin,rout", OPS)
@pytest.mark.parametrize("mode", [0, 2, 4], ids=["fast", "ref", "split"])
def test_golden_vectors_one_by_one(gpu, op, rin, rout, mode):
    for v in golden(op):
        flags = mode | (0 if v["check"] else gpu.NO_SUBGROUP_CHECK)
        r = gpu.run_codec(op, bytes.fromhex(v["in"]), flags, want_status=True)
        assert r.status[0] == v["status"], v["note"]
        want = bytes.fromhex(v["out"]) if v["out"] else bytes(rout)
        assert r.out == want, v["note"]
        assert r.ret == -v["status"] and r.first_bad == (0 if v["status"] else -1)


@pytest.mark.parametrize("op,rin,rout", OPS)
def test_golden_vectors_batched(gpu, oracle_lib, op, rin, rout):
    vecs = [v for v in golden(op) if v["check"]]
    data = b"".join(bytes.fromhex(v["in"]) for v in vecs)
    n = len(vecs)
    r = gpu.run_codec(op, data, 0, want_status=True)
    out, st, fb, ret = oracle_run(oracle_lib, op, data, n)
    assert r.out == out and r.status == st and r.first_bad == fb and r.ret == ret


def _random_stream(oracle_lib, n, seed, neg_every=0):
    """n compressed G1 points [k]G (C oracle) with optional negatives sprinkled in."""
    rng = random.Random(seed)
    scal = b"".join(rng.randrange(1, 1 << 255).to_bytes(32, "big") for _ in range(n))
    comp = ctypes.create_string_buffer(n * 48)
    ark = ctypes.create_string_buffer(n * 96)
    oracle_lib.oracle_g1_scalar_mul_encode(scal, ctypes.c_size_t(n), comp, ark)
    data = bytearray(comp.raw)
    if neg_every:
        negs = [bytes.fromhex(v["in"]) for v in golden("g1_decompress") if v["status"] and v["check"]]
        for i in range(neg_every // 2, n, neg_every):
            data[i * 48:(i + 1) * 48] = negs[rng.randrange(len(negs))]
    return bytes(data), ark.raw


@pytest.mark.parametrize("n", [1, 63, 255, 256, 257, 1000, 4099])
def test_random_g1_ragged_sizes(gpu, oracle_lib, n):
    data, ark = _random_stream(oracle_lib, n, seed=n)
    r = gpu.g1_decompress(data, want_status=True)
    assert r.ret == 0 and r.first_bad == -1
    assert r.out == ark


def test_empty_input(gpu):
    for op, rin, _ in OPS:
        r = gpu.run_codec(op, b"", 0, want_status=True)
        assert r.ret == 0 and r.out == b"" and r.first_bad == -1


# modes: fused one-pass kernel (default) / split decompress + check launches (SPLIT_PHASES), each
# with the endomorphism subgroup test or the reference's double-and-add by r (SUBGROUP_REF)
@pytest.mark.parametrize("mode", [0, 2, 4, 6], ids=["fast", "ref", "fast-split", "ref-split"])
def test_mixed_stream_matches_oracle(gpu, oracle_lib, mode):
    n = 3000
    data, _ = _random_stream(oracle_lib, n, seed=99 + mode, neg_every=37)
    r = gpu.g1_decompress(data, flags=mode, want_status=True)
    out, st, fb, ret = oracle_run(oracle_lib, "g1_decompress", data, n)
    assert r.status == st
    assert r.out == out
    assert (r.ret, r.first_bad) == (ret, fb)


@pytest.mark.parametrize("mode", [0, 2, 4, 6], ids=["fast", "ref", "fast-split", "ref-split"])
def test_g2_mixed_stream_matches_oracle(gpu, oracle_lib, mode):
    """G2 through the fused codec and the split pair: every checked golden vector class (valid,
    non-residue, x >= p, infinity, bad flags, off-subgroup) shuffled into one 700-point stream."""
    vecs = [bytes.fromhex(v["in"]) for v in golden("g2_decompress") if v["check"]]
    rng = random.Random(7 + mode)
    n = 700
    data = b"".join(rng.choice(vecs) for _ in range(n))
    r = gpu.run_codec("g2_decompress", data, mode, want_status=True)
    out, st, fb, ret = oracle_run(oracle_lib, "g2_decompress", data, n)
    assert r.status == st and r.out == out and (r.ret, r.first_bad) == (ret, fb)


def test_no_subgroup_check_mode(gpu, oracle_lib):
    n = 2000
    data, _ = _random_stream(oracle_lib, n, seed=5, neg_every=41)
    r = gpu.g1_decompress(data, flags=gpu.NO_SUBGROUP_CHECK, want_status=True)
    out, st, fb, ret = oracle_run(oracle_lib, "g1_decompress", data, n, flags=1)
    assert r.status == st and r.out == out and (r.ret, r.first_bad) == (ret, fb)


def test_chunked_host_path_first_bad(gpu, oracle_lib):
    """> 2^22 points run the host API's two-stream chunk pipeline (8 chunks of 524,800 points, so
    both slots are reused); bad points in the fourth and the last chunk: the smallest global index
    is reported, every status lands at its global index."""
    base, ark = _random_stream(oracle_lib, 4096, seed=3)
    n = (1 << 22) + 4096
    reps = n // 4096
    data = bytearray(base * reps)
    first = (1 << 21) + 5
    bad_at = (1 << 22) + 17
    data[bad_at * 48] &= 0x7F
    data[first * 48] &= 0x7F
    r = gpu.g1_decompress(bytes(data), want_status=True)
    assert r.ret == -1 and r.first_bad == first
    assert r.status[bad_at] == 1 and r.status[first] == 1 and r.status.count(0) == n - 2
    assert r.out[:4096 * 96] == ark and r.out[bad_at * 96:(bad_at + 1) * 96] == bytes(96)


@pytest.mark.parametrize("n", [(1 << 18), (1 << 18) + 1, 3 * (1 << 17) + 5, (1 << 21) + 777, (1 << 24) + 3])
def test_host_chunk_schedule_boundaries(gpu, oracle_lib, n):
    """run_host's chunk plan (csrc/capi.hip ChunkPlan; its tiling is checked on the CPU by
    tests/test_host.py): up to 2^18 points one chunk; above, equal chunks of >= 2^17 points — here
    1, 3 and 4 chunks, the last a ragged 1 / 5 points — and from ~2^21 points a ramp: 2^17 points
    growing x4 to the chunk size, then halving back to 2^17, the ragged remainder in the middle
    (2^21 + 777 and 2^24 + 3 points: 10 and 21 chunks). A bad point in the middle and one in the
    very last record: first_bad is the middle one, each status lands at its global index, every
    other record is the oracle's."""
    base, ark = _random_stream(oracle_lib, 4096, seed=11)
    reps = -(-n // 4096)
    data = bytearray((base * reps)[:n * 48])
    mid, last = n // 2 + 3, n - 1
    data[mid * 48] &= 0x7F
    data[last * 48] &= 0x7F
    r = gpu.g1_decompress(bytes(data), want_status=True)
    assert r.ret == -1 and r.first_bad == mid
    assert r.status[mid] == 1 and r.status[last] == 1 and r.status.count(0) == n - 2
    want = bytearray((ark * reps)[:n * 96])
    want[mid * 96:(mid + 1) * 96] = bytes(96)
    want[last * 96:(last + 1) * 96] = bytes(96)
    assert r.out == bytes(want)


def test_transcript_config1(gpu):
    meta = json.load(open(os.path.join(GOLDEN, "transcript_n1024.json")))
    tr = open(os.path.join(GOLDEN, "transcript_n1024.bin"), "rb").read()
    kgz = gpu.preprocess_buffer(tr, 10, gpu.MODE_KZG)
    fast = gpu.preprocess_buffer(tr, 10, gpu.MODE_FASTKZG)
    assert hashlib.blake2b(kgz).hexdigest() == meta["kgz_blake2b"]
    assert hashlib.blake2b(fast).hexdigest() == meta["fastkgz_blake2b"]


def test_transcript_file_api_and_rejections(gpu, tmp_path):
    meta = json.load(open(os.path.join(GOLDEN, "transcript_n1024.json")))
    src = os.path.join(GOLDEN, "transcript_n1024.bin")
    out = tmp_path / "kzg_setup"
    gpu.preprocess_kgz(src, str(out), n_log2=10)
    assert hashlib.blake2b(out.read_bytes()).hexdigest() == meta["kgz_blake2b"]
    tr = bytearray(open(src, "rb").read())
    n = 1024
    # τG2[7] with x.c0 >= p (section 1)
    off = 64 + (2 * n - 1) * 48 + 7 * 96
    tr[off + 48:off + 96] = b"\xff" * 48
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.preprocess_buffer(bytes(tr), 10)
    assert e.value.code == -3 and e.value.section == 1 and e.value.first_bad == 7
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.preprocess_buffer(bytes(tr[:-5]), 10)
    assert e.value.code == -103
    # βτG1 infinity: legal in kgz (decompress-only section), rejected by fastkgz (read_g1 panics)
    tr = bytearray(open(src, "rb").read())
    off = 64 + (2 * n - 1) * 48 + n * 96 + n * 48 + 3 * 48
    tr[off:off + 48] = bytes([0xC0]) + bytes(47)
    kgz = gpu.preprocess_buffer(bytes(tr), 10, gpu.MODE_KZG)
    assert hashlib.blake2b(kgz).hexdigest() == meta["kgz_blake2b"]
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.preprocess_buffer(bytes(tr), 10, gpu.MODE_FASTKZG)
    assert e.value.code == -7 and e.value.section == 3 and e.value.first_bad == 3


def test_read_g1_read_g2_mirror(gpu):
    import io

    v1 = [v for v in golden("g1_transcode") if v["status"] == 0]
    stream = io.BytesIO(b"".join(bytes.fromhex(v["in"]) for v in v1))
    assert gpu.read_g1(stream, count=len(v1)) == b"".join(bytes.fromhex(v["out"]) for v in v1)
    v2 = [v for v in golden("g2_transcode") if v["status"] == 0]
    stream = io.BytesIO(b"".join(bytes.fromhex(v["in"]) for v in v2))
    assert gpu.read_g2(stream, count=len(v2)) == b"".join(bytes.fromhex(v["out"]) for v in v2)
    bad = next(v for v in golden("g1_transcode") if v["status"] == 5)
    with pytest.raises(gpu.KzgPotError):
        gpu.read_g1(io.BytesIO(bytes.fromhex(bad["in"])))


# ------------------------------------------------------------------ loader mirror (§8f 2)
@pytest.mark.parametrize("name,g2,rin,rout", [("g1_load", False, 96, 104), ("g2_load", True, 192, 200)])
def test_load_golden_vectors(gpu, name, g2, rin, rout):
    vecs = golden(name)
    for v in vecs:  # one by one: status class and bytes
        r = gpu.deserialize_unchecked(bytes.fromhex(v["in"]), g2=g2, want_status=True)
        assert r.status[0] == v["status"], v["note"]
        assert r.out == (bytes.fromhex(v["out"]) if v["out"] else bytes(rout)), v["note"]
    r = gpu.deserialize_unchecked(b"".join(bytes.fromhex(v["in"]) for v in vecs), g2=g2, want_status=True)
    first = next(i for i, v in enumerate(vecs) if v["status"])
    assert r.first_bad == first and r.ret == -vecs[first]["status"]
    assert r.out == b"".join(bytes.fromhex(v["out"]) if v["out"] else bytes(rout) for v in vecs)


def test_load_setup_config1(gpu, tmp_path):
    meta = json.load(open(os.path.join(GOLDEN, "transcript_n1024.json")))
    tr = open(os.path.join(GOLDEN, "transcript_n1024.bin"), "rb").read()
    kgz = gpu.preprocess_buffer(tr, 10, gpu.MODE_KZG)
    powers, vk = gpu.load_kzg_setup_buffer(kgz, 10)
    assert powers.powers_of_g.shape == (2047, 104) and powers.powers_of_gamma_g.shape == (1024, 104)
    blob = powers.powers_of_g.tobytes() + powers.powers_of_gamma_g.tobytes() + vk.g + vk.gamma_g + vk.h + vk.beta_h
    assert hashlib.blake2b(blob).hexdigest() == meta["load_kzg_blake2b"]
    assert vk.g == powers.powers_of_g[0].tobytes()  # g = τG1[0]
    path = tmp_path / "kzg_setup"
    path.write_bytes(kgz + b"trailing bytes are ignored")
    p2, vk2 = gpu.load_kzg_setup(str(path), 10)
    assert p2.powers_of_g.tobytes() == powers.powers_of_g.tobytes() and vk2 == vk

    fast = gpu.preprocess_buffer(tr, 10, gpu.MODE_FASTKZG)
    params, powers_of_h = gpu.load_fastkzg_setup_buffer(fast, 10)
    blob = (params.powers_of_g.tobytes() + params.powers_of_gamma_g.tobytes() + params.h + params.beta_h_read
            + powers_of_h.tobytes())
    assert hashlib.blake2b(blob).hexdigest() == meta["load_fastkzg_blake2b"]
    assert params.beta_h == powers_of_h[1].tobytes() and params.h == powers_of_h[0].tobytes()


def test_load_setup_rejections(gpu):
    tr = open(os.path.join(GOLDEN, "transcript_n1024.bin"), "rb").read()
    kgz = bytearray(gpu.preprocess_buffer(tr, 10, gpu.MODE_KZG))
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.load_kzg_setup_buffer(bytes(kgz[:-1]), 10)
    assert e.value.code == -103
    off = 2047 * 96 + 5 * 96  # powers_of_gamma_g[5].y top byte: both SW flags
    kgz[off + 95] |= 0xC0
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.load_kzg_setup_buffer(bytes(kgz), 10)
    assert e.value.code == -6 and e.value.section == 1 and e.value.first_bad == 5
    kgz[off + 95] &= 0x3F
    kgz[12 * 96:12 * 96 + 48] = b"\xff" * 48  # powers_of_g[12].x >= p
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.load_kzg_setup_buffer(bytes(kgz), 10)
    assert e.value.code == -3 and e.value.section == 0 and e.value.first_bad == 12


def test_load_dev_api(gpu):
    import torch

    from kzgpot import device

    vecs = [v for v in golden("g1_load")]
    data = b"".join(bytes.fromhex(v["in"]) for v in vecs)
    d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    d_out = torch.empty(len(vecs) * 104, dtype=torch.uint8, device="cuda")
    key = torch.empty(1, dtype=torch.int64, device="cuda")
    device.codec_dev("g1_load", d_in, d_out, key)
    torch.cuda.synchronize()
    first = next(i for i, v in enumerate(vecs) if v["status"])
    assert device.read_key(key) == (first << 8) | vecs[first]["status"]
    assert d_out.cpu().numpy().tobytes() == b"".join(bytes.fromhex(v["out"]) if v["out"] else bytes(104) for v in vecs)


def test_preprocess_digests(gpu, tmp_path):
    """kzgpot_preprocess_ex: BLAKE2b of transcript and output computed beside the GPU pass."""
    meta = json.load(open(os.path.join(GOLDEN, "transcript_n1024.json")))
    src = os.path.join(GOLDEN, "transcript_n1024.bin")
    tr = open(src, "rb").read()
    for mode, key in ((gpu.MODE_KZG, "kgz_blake2b"), (gpu.MODE_FASTKZG, "fastkgz_blake2b")):
        res = gpu.preprocess_buffer(tr, 10, mode, with_digests=True)
        assert res.transcript_digest == meta["transcript_blake2b"]
        assert res.output_digest == meta[key] == hashlib.blake2b(res.out).hexdigest()
    out = gpu.preprocess_buffer(tr, 10, expect_transcript_digest=meta["transcript_blake2b"])
    assert hashlib.blake2b(out).hexdigest() == meta["kgz_blake2b"]
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.preprocess_buffer(tr, 10, expect_transcript_digest=gpu.POWERSOFTAU_DIGEST)
    assert e.value.code == -104
    res = gpu.preprocess_fastkgz(src, str(tmp_path / "fast"), n_log2=10)
    assert res.output_digest == meta["fastkgz_blake2b"] and res.transcript_digest == meta["transcript_blake2b"]
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.preprocess_kgz(src, str(tmp_path / "kgz"), n_log2=10, check_digest=True)
    assert e.value.code == -104 and not (tmp_path / "kgz").exists()


# ------------------------------------------------------------------ BN254 (config 5, §8f 4)
def test_bn254_golden_vectors(gpu):
    vecs = golden("bn254_g1_decompress")
    for v in vecs:
        r = gpu.bn254_g1_decompress(bytes.fromhex(v["in"]), want_status=True)
        assert r.status[0] == v["status"], v["note"]
        assert r.out == (bytes.fromhex(v["out"]) if v["out"] else bytes(64)), v["note"]
    r = gpu.bn254_g1_decompress(b"".join(bytes.fromhex(v["in"]) for v in vecs), want_status=True)
    first = next(i for i, v in enumerate(vecs) if v["status"])
    assert r.first_bad == first and r.ret == -vecs[first]["status"]
    assert r.out == b"".join(bytes.fromhex(v["out"]) if v["out"] else bytes(64) for v in vecs)


def test_bn254_synth_round_trip(gpu):
    """GPU-generated BN254 points (the bench's config-5 data) decode to the generator's expected
    bytes; a sample is re-derived by the Python oracle independently."""
    import torch

    from kzgpot import device

    O = pytest.importorskip("kzgpot_oracle")
    n = (1 << 16) + 77
    comp, exp = device.synth("bn254", 11, 0, n, "cuda")
    out = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    key = torch.empty(1, dtype=torch.int64, device="cuda")
    device.codec_dev("bn254_g1_decompress", comp, out, key)
    torch.cuda.synchronize()
    assert device.read_key(key) == (1 << 64) - 1
    assert torch.equal(out, exp)
    c, o = comp.cpu().numpy().tobytes(), out.cpu().numpy().tobytes()
    for i in random.Random(3).sample(range(n), 64):
        st, want = O.bn254_g1_decompress_point(c[32 * i:32 * i + 32])
        assert st == 0 and want == o[64 * i:64 * i + 64]



@pytest.mark.gpu
def test_load_phase1_matches_oracle(gpu):
    """load_phase1 (src/lib.rs:82-121) on a synthetic phase1radix2m3 file: all seven sections
    equal the oracle's in-memory GroupAffine records; a non-subgroup point planted in coeffs_g2
    and one in beta_coeffs_g1 are reported at the first (section 4) with its index."""
    import kzgpot_oracle as O

    data = bytearray(O.make_phase1_file(3, seed=11))
    st, _, _, want = O.load_phase1(bytes(data), 3)
    assert st == O.OK
    got = gpu.load_phase1_buffer(bytes(data), 3)
    fields = [got.alpha, got.beta_g1, got.beta_g2, got.coeffs_g1, got.coeffs_g2, got.alpha_coeffs_g1,
              got.beta_coeffs_g1]
    for f, w in zip(fields, want):
        assert bytes(f if isinstance(f, bytes) else f.tobytes()) == w
    bad2 = next(v for v in golden("g2_transcode") if v["status"] == 5)
    bad1 = next(v for v in golden("g1_transcode") if v["status"] == 5)
    off_c2 = 2 * 96 + 192 + 8 * 96
    data[off_c2 + 5 * 192: off_c2 + 6 * 192] = bytes.fromhex(bad2["in"])
    off_b1 = off_c2 + 8 * 192 + 8 * 96
    data[off_b1 + 2 * 96: off_b1 + 3 * 96] = bytes.fromhex(bad1["in"])
    st, sec, idx, _ = O.load_phase1(bytes(data), 3)
    assert (st, sec, idx) == (5, 4, 5)
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.load_phase1_buffer(bytes(data), 3)
    assert (e.value.code, e.value.section, e.value.first_bad) == (-5, 4, 5)
