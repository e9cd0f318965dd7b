"""GPU, C ABI only (no torch in the process): the end-to-end preprocess at sizes where every shard
runs several host chunks with the output digest streaming from them, and the file path's buffer
release across back-to-back calls. tools/asan_gpu_tests.sh runs this file under the host-ASan
build of the library (torch does not initialise under the ASan runtime, so these tests build
their transcript on the host).

The transcript tiles the config-1 transcript's sections (tests/golden/transcript_n1024.bin) up to
N = 2^18 / 2^19; the expected τG1 / ατG1 records are the C oracle's decode of the 2047 / 1024
golden points, tiled the same way. Reference: preprocess-kgz.rs:69-199 (the `main` these calls
replace), :187-194 (its writer owns its buffers synchronously)."""
import ctypes
import hashlib
import os
import time

import pytest

from conftest import GOLDEN, oracle_run

pytestmark = pytest.mark.gpu

N0 = 1024
E_IO = -102  # KZGPOT_E_IO (include/kzgpot.h)
SRC = os.path.join(GOLDEN, "transcript_n1024.bin")


@pytest.fixture(scope="session")
def capi(kzgpot_mod):
    """The library through ctypes alone (no torch import)."""
    if kzgpot_mod.device_count() < 1:
        pytest.fail("GPU test on a machine without a visible GPU")
    return kzgpot_mod


def _sections(tr, n):
    out, o = [], 64
    for cnt, rec in ((2 * n - 1, 48), (n, 96), (n, 48), (n, 48), (1, 96)):
        out.append(tr[o:o + cnt * rec])
        o += cnt * rec
    out.append(tr[o:])  # the public key (never read)
    return out


def _tile(b, rec, cnt):
    k = len(b) // rec
    return (b * ((cnt + k - 1) // k))[:cnt * rec]


_CACHE = {}


def _tiled(oracle_lib, n_log2):
    """(transcript, expected τG1 ark records, expected ατG1 ark records) at N = 2^n_log2."""
    if n_log2 not in _CACHE:
        n = 1 << n_log2
        s = _sections(open(SRC, "rb").read(), N0)
        tr = b"\0" * 64 + _tile(s[0], 48, 2 * n - 1) + _tile(s[1], 96, n) + _tile(s[2], 48, n) + \
            _tile(s[3], 48, n) + s[4] + s[5]
        tau, st, _, r = oracle_run(oracle_lib, "g1_decompress", s[0], 2 * N0 - 1)
        alpha, st2, _, r2 = oracle_run(oracle_lib, "g1_decompress", s[2], N0)
        assert r == 0 and r2 == 0
        _CACHE[n_log2] = (tr, _tile(tau, 96, 2 * n - 1), _tile(alpha, 96, n))
    return _CACHE[n_log2]


@pytest.mark.parametrize("mode", [0, 1], ids=["kgz", "fastkgz"])
@pytest.mark.parametrize("n_log2,shards", [(18, 3), (19, 2)], ids=["2e18x3", "2e19x2"])
def test_streamed_digests_multi_shard_capi(capi, oracle_lib, mode, n_log2, shards):
    """Several chunks per shard, the small first chunk of each, and the cursor that hands records
    to the digest and writer threads in file order across shards: τG1 / ατG1 equal the oracle's,
    both digests equal hashlib's, and a bad point in a later chunk of the LAST shard is reported with
    its global index (a second one in a later section does not mask it)."""
    n = 1 << n_log2
    tr, tau, alpha = _tiled(oracle_lib, n_log2)
    assert len(tr) == capi.contribution_size(n_log2)
    res = capi.preprocess_buffer(tr, n_log2, mode, n_gpus=shards, with_digests=True)
    g1n = (2 * n - 1) * 96
    assert res.out[:g1n] == tau and res.out[g1n:g1n + n * 96] == alpha
    assert res.transcript_digest == hashlib.blake2b(tr).hexdigest()
    assert res.output_digest == hashlib.blake2b(res.out).hexdigest()
    per = (2 * n - 1 + shards - 1) // shards
    last = 2 * n - 1 - (shards - 1) * per  # the last shard's size
    # past the shard's small first chunk (2^16 points) and, where the shard has one, a second chunk
    bad = (shards - 1) * per + min(last - 7, (1 << 16) + (1 << 17) + 5)
    t = bytearray(tr)
    t[64 + bad * 48] &= 0x7F
    t[64 + (2 * n - 1) * 48 + n * 96 + 3 * 48] &= 0x7F  # ατG1[3]: a later section
    with pytest.raises(capi.KzgPotError) as e:
        capi.preprocess_buffer(bytes(t), n_log2, mode, n_gpus=shards, with_digests=True)
    assert (e.value.code, e.value.section, e.value.first_bad) == (-1, 0, bad)


def _rss():
    with open("/proc/self/statm") as f:
        return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")


def test_file_calls_back_to_back_release_buffers(capi, oracle_lib, tmp_path):
    """kzgpot_preprocess_ex unmaps its 2 x ~150 MB file buffers on a helper thread after it
    returns, with at most one release outstanding (the next call joins the previous helper when it
    hands over its own buffers). Five calls in a row therefore never hold more than one call's
    buffers beyond the baseline when they return, and once the last helper has run the RSS is
    back at the baseline."""
    n_log2 = 19
    tr, tau, _ = _tiled(oracle_lib, n_log2)
    src = tmp_path / "powersoftau"
    src.write_bytes(tr)
    dst = tmp_path / "kzg_setup"
    lib = capi._lib.load()
    sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
    call = lambda path: lib.kzgpot_preprocess_ex(str(path).encode(), str(dst).encode(), 0, n_log2, 1, None, None,
                                                 None, ctypes.byref(sec), ctypes.byref(idx))
    assert call(src) == 0  # warm-up: staging buffers, HIP state
    assert call(tmp_path / "missing") == E_IO  # fails at open, before any mapping
    time.sleep(1.0)  # the warm-up call's release (~10 ms of munmap at this size) has run
    base = _rss()
    bufs = len(tr) + capi.output_size(n_log2, 0)
    peaks = []
    for _ in range(5):
        assert call(src) == 0
        peaks.append(_rss() - base)
    assert max(peaks) < bufs + (64 << 20), peaks  # never two calls' buffers at once
    with open(dst, "rb") as f:
        assert f.read(len(tau)) == tau
    time.sleep(1.0)
    assert _rss() - base < (64 << 20), (_rss() - base, peaks)
