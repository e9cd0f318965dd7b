"""Host-side checks that need no GPU: the C ABI library loads and exports every symbol the
public header declares, host-only helpers return the reference's sizes, the constants header is
reproducible, and compute calls FAIL LOUDLY without a GPU (no CPU fallback on the product path)."""
import ctypes
import os
import subprocess
import sys

import pytest

from conftest import PKG, ROOT


def test_library_exports_header_symbols(kzgpot_mod):
    from kzgpot import _lib

    lib = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(_lib.SIGNATURES) == set(syms)


def test_test_hooks_only_in_test_build(kzgpot_mod):
    """Failure injection and the KZGPOT_RCCL_LIB override live in libkzgpot_test.so only
    (-DKZGPOT_TEST_HOOKS, tests/kzgpot_test_hooks.h): the product library exports no inject symbol
    and binds nothing but librccl.so.1."""
    from kzgpot import _lib

    prod = open(_lib.LIB_PATH, "rb").read()
    assert b"kzgpot_comm_inject_fault" not in prod and b"KZGPOT_RCCL_LIB" not in prod
    if not os.path.exists(_lib.TEST_LIB_PATH):
        subprocess.run(["make", "-C", PKG, "-j", "8"], check=True)
    test_lib = ctypes.CDLL(_lib.TEST_LIB_PATH)
    assert hasattr(test_lib, "kzgpot_comm_inject_fault") and hasattr(test_lib, "kzgpot_comm_size")
    assert b"KZGPOT_RCCL_LIB" in open(_lib.TEST_LIB_PATH, "rb").read()


def test_product_library_needs_no_profiler(kzgpot_mod):
    """the roctx stage ranges are bound with dlopen at first use (csrc/trace.hpp), so
    libkzgpot.so and the CLI drop-ins load on a host without rocprofiler-sdk: no DT_NEEDED entry
    names roctx or rocprofiler, and the library still names the roctx soname it dlopens."""
    from kzgpot import _lib

    for path in (_lib.LIB_PATH, os.path.join(PKG, "build", "kzgpot-preprocess-kgz")):
        dyn = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
        needed = [ln for ln in dyn.splitlines() if "(NEEDED)" in ln]
        assert needed and not any("roctx" in ln or "rocprofiler" in ln for ln in needed), needed
    assert b"librocprofiler-sdk-roctx.so.1" in open(_lib.LIB_PATH, "rb").read()


def test_rank_failed_key_never_decodes_as_success(kzgpot_mod):
    """KZGPOT_KEY_RANK_FAILED (0), the all-reduced key when a peer could not decode its share,
    decodes to KZGPOT_E_RANK_FAILED — not to 'every point accepted' (ADVICE r03)."""
    from kzgpot import _lib

    lib = _lib.load()
    fb = ctypes.c_int64(123)
    assert lib.kzgpot_decode_bad_key(0, ctypes.byref(fb)) == -106 and fb.value == -1
    assert lib.kzgpot_decode_bad_key((1 << 64) - 1, ctypes.byref(fb)) == 0 and fb.value == -1
    assert lib.kzgpot_decode_bad_key((5 << 8) | 3, ctypes.byref(fb)) == -3 and fb.value == 5
    assert lib.kzgpot_decode_bad_key(1, ctypes.byref(fb)) == -1 and fb.value == 0


def test_synth_library_exports():
    from kzgpot import device

    if not os.path.exists(device.SYNTH_PATH):
        subprocess.run(["make", "-C", PKG, "-j", "8"], check=True)
    lib = ctypes.CDLL(device.SYNTH_PATH)
    assert hasattr(lib, "kzgpot_synth_g1_dev") and hasattr(lib, "kzgpot_synth_g2_dev")


def test_fake_rccl_exports_what_the_library_binds():
    """tests/fake_rccl stands in for librccl.so.1 in tests/test_gpu_multirank.py: it must export
    every RCCL symbol csrc/comm.hip binds (dlsym in rccl())."""
    path = os.path.join(ROOT, "tests", "fake_rccl", "build", "libfake_rccl.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-C", os.path.dirname(path)], check=True)
    src = open(os.path.join(PKG, "csrc", "comm.hip")).read()
    import re

    bound = set(re.findall(r'dlsym\(h, "(nccl[A-Za-z]+)"\)', src))
    assert {"ncclAllGather", "ncclAllReduce", "ncclCommAbort", "ncclCommInitRank"} <= bound
    lib = ctypes.CDLL(path)
    assert all(hasattr(lib, s) for s in bound), bound
    uid = ctypes.create_string_buffer(128)
    assert lib.ncclGetUniqueId(uid) == 0 and uid.raw.startswith(b"fake_rccl:")


def test_sizes_match_reference(kzgpot_mod):
    k = kzgpot_mod
    assert k.contribution_size(21) == 603_981_040          # preprocess-kgz.rs:83
    assert k.output_size(21, k.MODE_KZG) == 603_980_256     # preprocess-kgz.rs:187-194
    assert k.output_size(21, k.MODE_FASTKZG) == 1_006_633_248
    assert k.TAU_POWERS_G1_LENGTH == (1 << 22) - 1


def test_status_names(kzgpot_mod):
    k = kzgpot_mod
    assert k.status_name(-5) == "NotInSubgroup"
    assert k.status_name(-101) == "DeviceError"
    assert k.status_name(-106) == "RankFailed" and k.status_name(-107) == "Timeout"
    assert k.status_name(0) == "ok"
    assert "gfx950" in k.version()


def test_constants_header_is_reproducible(tmp_path):
    hdr = os.path.join(PKG, "csrc", "bls12_381_consts.hpp")
    before = open(hdr).read()
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_constants.py")], check=True,
                   capture_output=True)
    assert open(hdr).read() == before


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="a GPU is present")
def test_no_cpu_fallback_without_gpu(kzgpot_mod):
    k = kzgpot_mod
    assert k.device_count() == 0
    enc = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
    with pytest.raises(k.KzgPotError) as e:
        k.g1_decompress(enc)
    assert e.value.code == -101
    with pytest.raises(k.KzgPotError):
        k.preprocess_buffer(bytes(k.contribution_size(2)), 2)


def test_download_stub_has_no_network(kzgpot_mod, tmp_path):
    k = kzgpot_mod
    with pytest.raises(k.KzgPotError) as e:
        k.download_kzg_setup(True, path=str(tmp_path / "absent"))
    assert e.value.code == -105
    p = tmp_path / "kzg_setup"
    p.write_bytes(b"not the setup")
    k.download_kzg_setup(False, path=str(p))  # existing file, no digest check: accepted (lib.rs:133)
    with pytest.raises(k.KzgPotError) as e:
        k.download_kzg_setup(True, path=str(p))
    assert e.value.code == -104


def test_blake2b_matches_hashlib(kzgpot_mod):
    """The library's host BLAKE2b-512 (used by kzgpot_preprocess_ex beside the GPU pass) against
    hashlib, across block-boundary lengths. Host-only: no GPU needed."""
    import hashlib
    import random

    rng = random.Random(7)
    for n in (0, 1, 63, 64, 127, 128, 129, 255, 256, 257, 1023, 4096, 100_003):
        data = bytes(rng.randrange(256) for _ in range(n))
        assert kzgpot_mod.blake2b_hex(data) == hashlib.blake2b(data).hexdigest(), n


def test_python_mirror_api_surface(kzgpot_mod):
    """The crate's public API (src/lib.rs) and the two binaries' mains, by their reference names."""
    for name in ("read_g1", "read_g2", "load_kzg_setup", "load_fastkzg_setup", "download_kzg_setup",
                 "download_fastkzg_setup", "preprocess_kgz", "preprocess_fastkgz", "deserialize_unchecked",
                 "g1_decompress", "g2_decompress", "blake2b_hex", "KZG_SETUP_FILE", "KZG_SETUP_FILE_DIGEST",
                 "FASTKZG_SETUP_FILE_DIGEST", "POWERSOFTAU_DIGEST", "TAU_POWERS_LENGTH"):
        assert hasattr(kzgpot_mod, name), name


CLI = {m: os.path.join(PKG, "build", f"kzgpot-preprocess-{m}") for m in ("kgz", "fastkgz")}


@pytest.mark.parametrize("mode", ["kgz", "fastkgz"])
def test_cli_reference_failure_paths(mode, tmp_path):
    """The native drop-ins for src/bin/preprocess-{kgz,fastkgz}: --help, and the reference's
    panics (exit 101) for a missing ./powersoftau (no download here) and a wrong-size transcript
    (preprocess-kgz.rs:83-91) — both decided before any GPU work."""
    exe = CLI[mode]
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", PKG, "-j", "8"], check=True)
    r = subprocess.run([exe, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--transcript" in r.stdout
    r = subprocess.run([exe], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 101 and "`powersoftau` not found" in r.stderr
    bad = tmp_path / "powersoftau"
    bad.write_bytes(b"\0" * 1000)
    r = subprocess.run([exe, "--n-log2", "10"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 101
    assert "The size of `powersoftau` should be 296176, but it's 1000, so something isn't right." in r.stderr
    assert not (tmp_path / "kzg_setup").exists()
    # --expect-digest takes a full BLAKE2b-512 hex digest; anything else is refused up front
    r = subprocess.run([exe, "--n-log2", "10", "--expect-digest", "abc"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 101 and "128 hex characters" in r.stderr
    r = subprocess.run([exe, "--bogus"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 2 and "--output-digest" in r.stdout and "--timing" in r.stdout


def test_load_phase1_short_file_is_size_error(kzgpot_mod):
    """A short phase1 file is KZGPOT_E_SIZE (the reference's read_exact hits EOF and panics),
    decided before any GPU work."""
    assert kzgpot_mod.phase1_size(3) == 2 * 96 + 192 + 8 * (3 * 96 + 192)
    with pytest.raises(kzgpot_mod.KzgPotError) as e:
        kzgpot_mod.load_phase1_buffer(b"\0" * 100, 3)
    assert e.value.code == -103


@pytest.mark.parametrize("streaming", [0, 1], ids=["plain", "digest_consumer"])
def test_host_chunk_plan_tiles_the_call(kzgpot_mod, streaming):
    """run_host's chunk plan (csrc/capi.hip ChunkPlan, through the test build's
    kzgpot_test_chunk_plan): the chunks tile [0, n) in order with no gap or overlap, none exceeds
    the staging size (2^21 points), calls of 2^20 to 2^24 points get at least 8 chunks, and a long
    call starts and ends on 2^17-point chunks (so only those chunks' copies are exposed), ramping
    x4 up and /2 down."""
    from kzgpot import _lib

    if not os.path.exists(_lib.TEST_LIB_PATH):
        subprocess.run(["make", "-C", PKG, "-j", "8"], check=True)
    lib = ctypes.CDLL(_lib.TEST_LIB_PATH)
    fn = lib.kzgpot_test_chunk_plan
    fn.restype = ctypes.c_long
    fn.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_long]
    kmin, cmax_all = 1 << 17, 1 << 21
    sizes = [1, 255, 256, 1 << 16, (1 << 17) + 1, 1 << 18, (1 << 18) + 1, (1 << 20) + 12345, 1 << 21,
             (1 << 21) + 7, 3 << 20, (1 << 22) + 999, 1 << 23, (1 << 24) + 3, 1 << 25, (1 << 27) + 5, 1 << 28]
    for n in sizes:
        cap = 4096
        buf = (ctypes.c_uint64 * (2 * cap))()
        k = fn(n, streaming, buf, cap)
        assert 0 < k <= cap, (n, k)
        spans = [(buf[2 * j], buf[2 * j + 1]) for j in range(k)]
        off = 0
        for o, m in spans:
            assert o == off and 0 < m <= cmax_all, (n, spans)
            off += m
        assert off == n, (n, off)
        ms = [m for _, m in spans]
        if 1 << 20 <= n <= 1 << 24:
            assert k >= 8, (n, k)
        if n >= 1 << 23:  # long enough for both ramps
            assert ms[0] == kmin and ms[-1] == kmin and ms[1] == 4 * kmin, (n, ms[:3], ms[-3:])
            assert ms[-2] == 2 * kmin, (n, ms[-3:])
            assert max(ms) == min(cmax_all, max(kmin, ((n + 7) // 8 + 255) & ~255)), (n, max(ms))
        if streaming and k > 1 and n < 1 << 21:  # equal-chunk calls: a small first chunk for the digest
            assert ms[0] <= 1 << 16, (n, ms[0])
        if 2 * kmin < n <= 8 * kmin:  # equal 2^17-point chunks between 2^16-point end chunks
            assert ms[0] == ms[-1] == 1 << 16 and max(ms) == kmin, (n, ms)
