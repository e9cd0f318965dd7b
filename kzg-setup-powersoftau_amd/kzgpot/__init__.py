"""kzgpot — MI355X-native Powers-of-Tau → arkworks KZG preprocessor (Python host side).

Mirrors the reference crate's surface (heliaxdev/kzg-setup-powersoftau, `src/lib.rs`) above the
C ABI in `include/kzgpot.h`:

  read_g1 / read_g2            src/lib.rs:41-80     (batched: whole record streams per call)
  load_kzg_setup               src/lib.rs:174-195
  load_fastkzg_setup           src/lib.rs:197-228
  load_phase1                  src/lib.rs:82-121
  download_kzg_setup /
  download_fastkzg_setup       src/lib.rs:166-172   (no network in this build: local file + digest)
  preprocess_kgz /
  preprocess_fastkgz           src/bin/preprocess-{kgz,fastkgz}.rs main

Every compute call runs the HIP kernels; errors raise `KzgPotError` (the reference `unwrap()`s
and panics on the first bad point — preprocess-kgz.rs:110,142).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

from . import _lib

KZG_SETUP_FILE = "kzg_setup"                               # src/lib.rs:20
KZG_SETUP_FILE_DIGEST = (                                  # src/lib.rs:21
    "87932f626204ab9a5d4be67ef2ee479471baf942364ada2f89840a2afec8925911fb88cb77024e66d759b4970b25cf2a7b03d1fc8c15768e021220b8ba21efcf")
FASTKZG_SETUP_FILE_DIGEST = (                              # src/lib.rs:22
    "d177841ad145c0d526e56a8d2cde473f09e85944f5c5d6b72d8063e4a199f8a6fca0b0f6ee91ef79df48518b5edd8165bbdecf0fe4eb0d29809032878f8b17ce")
POWERSOFTAU_DIGEST = (                                     # src/bin/preprocess-kgz.rs:19
    "88dc1dc6914e44568e8511eace177e6ecd9da9a9bd8f67e4c0c9f215b517db4d1d54a755d051978dbb85ef947918193c93cd4cf4c99c0dc5a767d4eeb10047a4")
TAU_POWERS_LOG2 = 21                                       # src/lib.rs:23
TAU_POWERS_LENGTH = 1 << TAU_POWERS_LOG2
TAU_POWERS_G1_LENGTH = (TAU_POWERS_LENGTH << 1) - 1        # src/lib.rs:24

NO_SUBGROUP_CHECK = 0x1
SUBGROUP_REF = 0x2
SPLIT_PHASES = 0x4  # checked G1: decompress and check as two launches (A/B of the fused kernel)
MODE_KZG = 0
MODE_FASTKZG = 1

ST_OK, ST_COMPRESSION_MODE, ST_UNEXPECTED_INFO, ST_NOT_IN_FIELD = 0, 1, 2, 3
ST_NOT_ON_CURVE, ST_NOT_IN_SUBGROUP, ST_UNEXPECTED_FLAGS, ST_INFINITY = 4, 5, 6, 7
SECTIONS = ("tau_g1", "tau_g2", "alpha_g1", "beta_g1", "beta_g2")
LOAD_SECTIONS = ("powers_of_g", "powers_of_gamma_g", "vk / h, beta_h", "powers_of_h")
PHASE1_SECTIONS = ("alpha", "beta_g1", "beta_g2", "coeffs_g1", "coeffs_g2", "alpha_coeffs_g1", "beta_coeffs_g1")


class KzgPotError(RuntimeError):
    def __init__(self, code: int, first_bad: int = -1, section: int = -1, section_names=SECTIONS):
        self.code = code
        self.first_bad = first_bad
        self.section = section
        name = status_name(code)
        where = f" at index {first_bad}" if first_bad >= 0 else ""
        if section >= 0:
            where += f" in section {section_names[section]}"
        super().__init__(f"kzgpot error {code} ({name}){where}")


def status_name(code: int) -> str:
    return _lib.load().kzgpot_status_name(code).decode()


def device_count() -> int:
    return _lib.load().kzgpot_device_count()


def version() -> str:
    return _lib.load().kzgpot_version().decode()


@dataclass
class CodecResult:
    out: bytes
    ret: int
    first_bad: int
    status: bytes | None


def _buf(data) -> tuple[ctypes.c_void_p, int, object]:
    if isinstance(data, (bytes, bytearray, memoryview)):
        b = bytes(data)
        return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p), len(b), b
    import numpy as np  # numpy arrays (uint8, C-contiguous)
    arr = np.ascontiguousarray(data, dtype=np.uint8)
    return ctypes.c_void_p(arr.ctypes.data), arr.nbytes, arr


_OPS = {
    "g1_decompress": ("kzgpot_g1_decompress_ex", 48, 96),
    "g2_decompress": ("kzgpot_g2_decompress_ex", 96, 192),
    "g1_transcode": ("kzgpot_g1_transcode_uncompressed_ex", 96, 96),
    "g2_transcode": ("kzgpot_g2_transcode_uncompressed_ex", 192, 192),
}


def run_codec(op: str, data, flags: int = 0, want_status: bool = False) -> CodecResult:
    """Run one batched codec op over a packed record stream on the current GPU."""
    fname, rin, rout = _OPS[op]
    ptr, nbytes, keep = _buf(data)
    if nbytes % rin:
        raise ValueError(f"{op}: input length {nbytes} is not a multiple of {rin}")
    n = nbytes // rin
    out = ctypes.create_string_buffer(max(1, n * rout))
    st = ctypes.create_string_buffer(max(1, n)) if want_status else None
    fb = ctypes.c_int64(-1)
    ret = getattr(_lib.load(), fname)(ptr, n, out, flags, ctypes.byref(fb), st)
    del keep
    if ret <= -100:
        raise KzgPotError(ret)
    return CodecResult(out.raw[: n * rout], ret, fb.value, st.raw[:n] if st is not None else None)


def g1_decompress(data, flags: int = 0, want_status: bool = False) -> CodecResult:
    return run_codec("g1_decompress", data, flags, want_status)


def g2_decompress(data, flags: int = 0, want_status: bool = False) -> CodecResult:
    return run_codec("g2_decompress", data, flags, want_status)


def _checked(res: CodecResult) -> bytes:
    if res.ret != 0:
        raise KzgPotError(res.ret, res.first_bad)
    return res.out


def read_g1(reader, count: int = 1, flags: int = 0) -> bytes:
    """src/lib.rs:41-54 read_g1, batched: reads `count` 96-B pairing-uncompressed G1 records from
    `reader` and returns their ark `serialize_uncompressed` bytes (subgroup-checked). Raises on the
    first invalid point, as the reference's callers `unwrap()`."""
    data = reader.read(96 * count)
    if len(data) != 96 * count:
        raise EOFError("read_g1: short read")  # reference: read_exact(..).unwrap()
    return _checked(run_codec("g1_transcode", data, flags))


def read_g2(reader, count: int = 1, flags: int = 0) -> bytes:
    """src/lib.rs:56-80 read_g2, batched (192-B records, x.c1‖x.c0‖y.c1‖y.c0 → ark c0,c1 order)."""
    data = reader.read(192 * count)
    if len(data) != 192 * count:
        raise EOFError("read_g2: short read")
    return _checked(run_codec("g2_transcode", data, flags))


def contribution_size(n_log2: int = TAU_POWERS_LOG2) -> int:
    return _lib.load().kzgpot_contribution_size(n_log2)


def output_size(n_log2: int = TAU_POWERS_LOG2, mode: int = MODE_KZG) -> int:
    return _lib.load().kzgpot_output_size(n_log2, mode)


@dataclass
class PreprocessResult:
    out: bytes | None
    transcript_digest: str
    output_digest: str


def preprocess_buffer(transcript, n_log2: int, mode: int = MODE_KZG, n_gpus: int = 0,
                      expect_transcript_digest: str | None = None, with_digests: bool = False):
    """preprocess-{kgz,fastkgz} main on an in-memory response transcript → output file bytes
    (or a PreprocessResult with the BLAKE2b-512 digests, computed beside the GPU pass)."""
    ptr, nbytes, keep = _buf(transcript)
    out = ctypes.create_string_buffer(output_size(n_log2, mode))
    sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
    din, dout = ctypes.create_string_buffer(129), ctypes.create_string_buffer(129)
    exp = expect_transcript_digest.encode() if expect_transcript_digest else None
    r = _lib.load().kzgpot_preprocess_buffer_ex(ptr, nbytes, out, mode, n_log2, n_gpus, exp,
                                                din if (with_digests or exp) else None,
                                                dout if with_digests else None, ctypes.byref(sec),
                                                ctypes.byref(idx))
    del keep
    if r:
        raise KzgPotError(r, idx.value, sec.value)
    if with_digests:
        return PreprocessResult(out.raw, din.value.decode(), dout.value.decode())
    return out.raw


def preprocess(transcript_path: str, out_path: str = KZG_SETUP_FILE, mode: int = MODE_KZG,
               n_log2: int = TAU_POWERS_LOG2, n_gpus: int = 0, check_digest: bool | None = None) -> PreprocessResult:
    """`preprocess-kgz` / `preprocess-fastkgz` main (preprocess-kgz.rs:162-199) without the network:
    download_parameters' transcript check (BLAKE2b == POWERSOFTAU_DIGEST, preprocess-kgz.rs:32-67)
    runs when check_digest is True (default: only for the real 2^21 configuration); on a mismatch
    the reference would re-download — here it raises KzgPotError(-104). Returns both digests."""
    if check_digest is None:
        check_digest = n_log2 == TAU_POWERS_LOG2
    sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
    din, dout = ctypes.create_string_buffer(129), ctypes.create_string_buffer(129)
    exp = POWERSOFTAU_DIGEST.encode() if check_digest else None
    r = _lib.load().kzgpot_preprocess_ex(transcript_path.encode(), out_path.encode(), mode, n_log2, n_gpus, exp,
                                         din, dout, ctypes.byref(sec), ctypes.byref(idx))
    if r:
        raise KzgPotError(r, idx.value, sec.value)
    return PreprocessResult(None, din.value.decode(), dout.value.decode())


def preprocess_kgz(transcript_path: str = "powersoftau", out_path: str = KZG_SETUP_FILE, **kw) -> PreprocessResult:
    return preprocess(transcript_path, out_path, MODE_KZG, **kw)


def preprocess_fastkgz(transcript_path: str = "powersoftau", out_path: str = KZG_SETUP_FILE, **kw) -> PreprocessResult:
    return preprocess(transcript_path, out_path, MODE_FASTKZG, **kw)


# ------------------------------------------------------------------ loader mirror (src/lib.rs:174-228)
G1_ARK_MONT_BYTES = 104  # in-memory GroupAffine<g1>: x, y as 6 LE u64 Montgomery (R = 2^384), infinity, pad
G2_ARK_MONT_BYTES = 200


def deserialize_unchecked(data, g2: bool = False, want_status: bool = False) -> CodecResult:
    """ark-ec 0.2 `GroupAffine::deserialize_unchecked` over packed ark-uncompressed records
    (96 B G1 / 192 B G2) → in-memory GroupAffine records (104 / 200 B). Coordinates < p and
    SWFlags are checked; no curve or subgroup check (that is what "unchecked" means)."""
    rin, rout = (192, G2_ARK_MONT_BYTES) if g2 else (96, G1_ARK_MONT_BYTES)
    fname = "kzgpot_g2_deserialize_unchecked_ex" if g2 else "kzgpot_g1_deserialize_unchecked_ex"
    ptr, nbytes, keep = _buf(data)
    if nbytes % rin:
        raise ValueError(f"deserialize_unchecked: input length {nbytes} is not a multiple of {rin}")
    n = nbytes // rin
    out = ctypes.create_string_buffer(max(1, n * rout))
    st = ctypes.create_string_buffer(max(1, n)) if want_status else None
    fb = ctypes.c_int64(-1)
    ret = getattr(_lib.load(), fname)(ptr, n, out, ctypes.byref(fb), st)
    del keep
    if ret <= -100:
        raise KzgPotError(ret)
    return CodecResult(out.raw[: n * rout], ret, fb.value, st.raw[:n] if st is not None else None)


def bn254_g1_decompress(data, want_status: bool = False) -> CodecResult:
    """BN254 G1 (config 5): ark-bn254 compressed (32 B) → ark uncompressed (64 B) on the GPU."""
    ptr, nbytes, keep = _buf(data)
    if nbytes % 32:
        raise ValueError(f"bn254_g1_decompress: input length {nbytes} is not a multiple of 32")
    n = nbytes // 32
    out = ctypes.create_string_buffer(max(1, n * 64))
    st = ctypes.create_string_buffer(max(1, n)) if want_status else None
    fb = ctypes.c_int64(-1)
    ret = _lib.load().kzgpot_bn254_g1_decompress_ex(ptr, n, out, ctypes.byref(fb), st)
    del keep
    if ret <= -100:
        raise KzgPotError(ret)
    return CodecResult(out.raw[: n * 64], ret, fb.value, st.raw[:n] if st is not None else None)


def _records(buf, rec: int):
    import numpy as np
    return np.frombuffer(buf, dtype=np.uint8).reshape(-1, rec)


@dataclass
class Powers:
    """ark-poly-commit 0.2 `kzg10::Powers` (Cow::Owned): rows are in-memory GroupAffine<g1>."""
    powers_of_g: object        # (2N-1, 104) uint8
    powers_of_gamma_g: object  # (N, 104) uint8


@dataclass
class VerifierKey:
    """ark-poly-commit 0.2 `kzg10::VerifierKey`. prepared_h / prepared_beta_h are the pairing
    precomputations `h.into()` / `beta_h.into()` the consumer builds from these two points."""
    g: bytes
    gamma_g: bytes
    h: bytes
    beta_h: bytes


@dataclass
class UniversalParams:
    """ark-poly-commit 0.2 `kzg10::UniversalParams` as built by load_fastkzg_setup (src/lib.rs:219-227).
    powers_of_gamma_g row i is the BTreeMap entry with key i. beta_h = powers_of_h[1] (lib.rs:221);
    prepared_beta_h is built from `beta_h_read`, the point stored after h in the file."""
    powers_of_g: object
    powers_of_gamma_g: object
    h: bytes
    beta_h: bytes
    beta_h_read: bytes


def _load_err(r, sec, idx):
    if r:
        raise KzgPotError(r, idx.value, sec.value, LOAD_SECTIONS)


def load_kzg_setup_buffer(data, n_log2: int = TAU_POWERS_LOG2):
    n = 1 << n_log2
    ptr, nbytes, keep = _buf(data)
    pg = ctypes.create_string_buffer((2 * n - 1) * G1_ARK_MONT_BYTES)
    pgg = ctypes.create_string_buffer(n * G1_ARK_MONT_BYTES)
    vk = ctypes.create_string_buffer(2 * G1_ARK_MONT_BYTES + 2 * G2_ARK_MONT_BYTES)
    sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
    r = _lib.load().kzgpot_load_kzg_setup_buffer(ptr, nbytes, n_log2, pg, pgg, vk, ctypes.byref(sec),
                                                 ctypes.byref(idx))
    del keep
    _load_err(r, sec, idx)
    v, a = vk.raw, G1_ARK_MONT_BYTES
    return (Powers(_records(pg.raw, a), _records(pgg.raw, a)),
            VerifierKey(v[:a], v[a:2 * a], v[2 * a:2 * a + G2_ARK_MONT_BYTES], v[2 * a + G2_ARK_MONT_BYTES:]))


def load_kzg_setup(path: str = KZG_SETUP_FILE, n_log2: int = TAU_POWERS_LOG2):
    """src/lib.rs:174-195 `load_kzg_setup() -> (Powers, VerifierKey)`; the per-point
    deserialize_unchecked runs on the GPU. Raises KzgPotError where the reference unwrap()s."""
    with open(path, "rb") as f:
        return load_kzg_setup_buffer(f.read(), n_log2)


def load_fastkzg_setup_buffer(data, n_log2: int = TAU_POWERS_LOG2):
    n = 1 << n_log2
    ptr, nbytes, keep = _buf(data)
    pg = ctypes.create_string_buffer((2 * n - 1) * G1_ARK_MONT_BYTES)
    pgg = ctypes.create_string_buffer(n * G1_ARK_MONT_BYTES)
    hb = ctypes.create_string_buffer(2 * G2_ARK_MONT_BYTES)
    ph = ctypes.create_string_buffer(n * G2_ARK_MONT_BYTES)
    sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
    r = _lib.load().kzgpot_load_fastkzg_setup_buffer(ptr, nbytes, n_log2, pg, pgg, hb, ph, ctypes.byref(sec),
                                                     ctypes.byref(idx))
    del keep
    _load_err(r, sec, idx)
    b = G2_ARK_MONT_BYTES
    powers_of_h = _records(ph.raw, b)
    params = UniversalParams(_records(pg.raw, G1_ARK_MONT_BYTES), _records(pgg.raw, G1_ARK_MONT_BYTES),
                             hb.raw[:b], ph.raw[b:2 * b], hb.raw[b:])
    return params, powers_of_h


def load_fastkzg_setup(path: str = KZG_SETUP_FILE, n_log2: int = TAU_POWERS_LOG2):
    """src/lib.rs:197-228 `load_fastkzg_setup() -> (UniversalParams, Vec<G2Affine>)`. The default
    path is KZG_SETUP_FILE because that is the file the reference opens here (lib.rs:198)."""
    with open(path, "rb") as f:
        return load_fastkzg_setup_buffer(f.read(), n_log2)


def blake2b_hex(data) -> str:
    """blake2b_simd::State::new().update(data).finalize().to_hex() (src/lib.rs:129), computed by
    the library's host BLAKE2b (the one kzgpot_preprocess_ex runs beside the GPU)."""
    ptr, nbytes, keep = _buf(data)
    d = ctypes.create_string_buffer(64)
    r = _lib.load().kzgpot_blake2b(ptr, nbytes, d)
    del keep
    if r:
        raise KzgPotError(r)
    return d.raw.hex()


def _download_setup(file_digest: str, check_digest: bool, path: str = KZG_SETUP_FILE) -> None:
    """src/lib.rs:123-164 without the HTTPS fetch (no network in this build). A local file is
    accepted as the reference does; with check_digest a mismatch RAISES (the reference silently
    returns Ok on mismatch, lib.rs:133-143 — a bug not reproduced)."""
    if not os.path.exists(path):
        raise KzgPotError(-105)
    if check_digest:
        with open(path, "rb") as f:
            if blake2b_hex(f.read()) != file_digest:
                raise KzgPotError(-104)


def download_kzg_setup(check_digest: bool, path: str = KZG_SETUP_FILE) -> None:
    _download_setup(KZG_SETUP_FILE_DIGEST, check_digest, path)


def download_fastkzg_setup(check_digest: bool, path: str = KZG_SETUP_FILE) -> None:
    _download_setup(FASTKZG_SETUP_FILE_DIGEST, check_digest, path)


@dataclass
class Phase1Parameters:
    """src/lib.rs:30-39 `Phase1Parameters`: rows / fields are in-memory GroupAffine records
    (G1 104 B, G2 200 B; include/kzgpot.h)."""
    alpha: bytes
    beta_g1: bytes
    beta_g2: bytes
    coeffs_g1: object        # (m, 104) uint8
    coeffs_g2: object        # (m, 200) uint8
    alpha_coeffs_g1: object  # (m, 104) uint8
    beta_coeffs_g1: object   # (m, 104) uint8


def phase1_size(exp: int) -> int:
    return int(_lib.load().kzgpot_phase1_size(exp))


def load_phase1_buffer(data, exp: int) -> Phase1Parameters:
    m = 1 << exp
    ptr, nbytes, keep = _buf(data)
    g1, g2 = G1_ARK_MONT_BYTES, G2_ARK_MONT_BYTES
    bufs = [ctypes.create_string_buffer(k) for k in (g1, g1, g2, m * g1, m * g2, m * g1, m * g1)]
    sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
    r = _lib.load().kzgpot_load_phase1_buffer(ptr, nbytes, exp, *bufs, ctypes.byref(sec), ctypes.byref(idx))
    del keep
    if r:
        raise KzgPotError(r, idx.value, sec.value, PHASE1_SECTIONS)
    return Phase1Parameters(bufs[0].raw, bufs[1].raw, bufs[2].raw, _records(bufs[3].raw, g1),
                            _records(bufs[4].raw, g2), _records(bufs[5].raw, g1), _records(bufs[6].raw, g1))


def load_phase1(exp: int, path: str | None = None) -> Phase1Parameters:
    """src/lib.rs:82-121 `load_phase1(exp)`: every point through read_g1 / read_g2 (subgroup
    check included) on the GPU. The reference opens "../phase1radix2m{exp}" (lib.rs:84): that is
    the default path here too."""
    with open(path or f"../phase1radix2m{exp}", "rb") as f:
        return load_phase1_buffer(f.read(), exp)
