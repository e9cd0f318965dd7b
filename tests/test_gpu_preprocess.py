"""GPU: the C ABI's end-to-end preprocess (the reference's two `main`s, preprocess-kgz.rs:162-199 /
preprocess-fastkgz.rs:180-213) on the config-1 transcript, through its multi-shard path and its
streaming file path.

`n_gpus` is the shard count: shards map round-robin onto the visible devices from the current
one, so on a one-GPU box n_gpus = 3 or 5 runs the multi-GPU host code (one thread per shard,
per-shard first-bad offsets merged to the global minimum, output handed to the digest and writer
in file order as far as every shard has landed) on a single device. Expected digests and sizes are the oracle's
(tests/golden/transcript_n1024.json)."""
import hashlib
import json
import os

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

N = 1024
META = json.load(open(os.path.join(GOLDEN, "transcript_n1024.json")))
SRC = os.path.join(GOLDEN, "transcript_n1024.bin")


def _tr():
    return bytearray(open(SRC, "rb").read())


def _off_g1(section, i):
    """Byte offset of point i of a G1 section of the response transcript (64-B hash header)."""
    base = {0: 64, 2: 64 + (2 * N - 1) * 48 + N * 96, 3: 64 + (2 * N - 1) * 48 + N * 96 + N * 48}[section]
    return base + i * 48


@pytest.mark.parametrize("shards", [1, 2, 3, 5])
def test_shards_digest_exact(gpu, shards):
    for mode, key in ((gpu.MODE_KZG, "kgz_blake2b"), (gpu.MODE_FASTKZG, "fastkgz_blake2b")):
        res = gpu.preprocess_buffer(bytes(_tr()), 10, mode, n_gpus=shards, with_digests=True)
        assert res.transcript_digest == META["transcript_blake2b"]
        assert res.output_digest == META[key] == hashlib.blake2b(res.out).hexdigest()


@pytest.mark.parametrize("shards", [3, 5])
def test_shards_first_bad_is_global_minimum(gpu, shards):
    """A bad point in the third shard is reported with its global index; with a second bad point
    in an earlier shard that one wins; a bad point in a later section never masks an earlier one."""
    per = (2 * N - 1 + shards - 1) // shards          # τG1 shard size (contiguous shards)
    in_shard2 = 2 * per + 17
    tr = _tr()
    tr[_off_g1(0, in_shard2)] &= 0x7F                 # bit 7 clear: UnexpectedCompressionMode (-1)
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.preprocess_buffer(bytes(tr), 10, gpu.MODE_KZG, n_gpus=shards)
    assert (e.value.code, e.value.section, e.value.first_bad) == (-1, 0, in_shard2)
    in_shard1 = per + 5
    o = _off_g1(0, in_shard1)
    tr[o:o + 48] = b"\x9f" + b"\xff" * 47           # flags 100 (compressed, finite), x >= p: NotInField (-3)
    for mode in (gpu.MODE_KZG, gpu.MODE_FASTKZG):
        with pytest.raises(gpu.KzgPotError) as e:
            gpu.preprocess_buffer(bytes(tr), 10, mode, n_gpus=shards)
        assert (e.value.code, e.value.section, e.value.first_bad) == (-3, 0, in_shard1)
    # only ατG1 (section 2) bad, in its last shard, plus βτG1 (section 3, checked in fastkgz only)
    tr = _tr()
    last = N - 3
    tr[_off_g1(2, last)] &= 0x7F
    tr[_off_g1(3, 1)] &= 0x7F
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.preprocess_buffer(bytes(tr), 10, gpu.MODE_FASTKZG, n_gpus=shards)
    assert (e.value.code, e.value.section, e.value.first_bad) == (-1, 2, last)


def test_digest_mismatch_takes_precedence(gpu):
    """The reference checks the transcript digest before decoding anything (download_parameters,
    preprocess-kgz.rs:51-61): a wrong transcript that also holds a bad point is a digest error."""
    tr = _tr()
    tr[_off_g1(0, 9)] &= 0x7F
    for shards in (1, 3):
        with pytest.raises(gpu.KzgPotError) as e:
            gpu.preprocess_buffer(bytes(tr), 10, n_gpus=shards, expect_transcript_digest=META["transcript_blake2b"])
        assert e.value.code == -104 and e.value.section == -1 and e.value.first_bad == -1


@pytest.mark.parametrize("shards", [1, 3])
def test_file_path_streams_and_writes_atomically(gpu, tmp_path, shards):
    """kzgpot_preprocess_ex: the transcript is pread() in chunks behind the GPU and the output
    pwrite()n as it lands, into a temporary file renamed into place only on success."""
    out = tmp_path / "kzg_setup"
    res = gpu.preprocess_kgz(SRC, str(out), n_log2=10, n_gpus=shards)
    assert res.transcript_digest == META["transcript_blake2b"] and res.output_digest == META["kgz_blake2b"]
    assert out.stat().st_size == META["kgz_size"]
    assert hashlib.blake2b(out.read_bytes()).hexdigest() == META["kgz_blake2b"]
    fast = tmp_path / "fast"
    res = gpu.preprocess_fastkgz(SRC, str(fast), n_log2=10, n_gpus=shards)
    assert hashlib.blake2b(fast.read_bytes()).hexdigest() == META["fastkgz_blake2b"] == res.output_digest
    # a rejected point: error, no output file and no temporary file left behind
    bad = tmp_path / "bad_transcript"
    tr = _tr()
    tr[_off_g1(2, 100)] &= 0x7F
    bad.write_bytes(bytes(tr))
    dst = tmp_path / "never"
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.preprocess_kgz(str(bad), str(dst), n_log2=10, n_gpus=shards)
    assert (e.value.code, e.value.section, e.value.first_bad) == (-1, 2, 100)
    assert not dst.exists()
    assert sorted(p.name for p in tmp_path.iterdir()) == ["bad_transcript", "fast", "kzg_setup"]
    # an existing output file is replaced only on success
    out.write_bytes(b"old")
    with pytest.raises(gpu.KzgPotError):
        gpu.preprocess_kgz(str(bad), str(out), n_log2=10, n_gpus=shards)
    assert out.read_bytes() == b"old"


def test_current_device_is_restored(gpu):
    """The library switches devices per shard; the caller's current device is unchanged after."""
    import torch

    before = torch.cuda.current_device()
    gpu.preprocess_buffer(bytes(_tr()), 10, n_gpus=3)
    assert gpu.g1_decompress(bytes(48)).ret == -1  # a rejected point: the error path through run_host
    assert torch.cuda.current_device() == before


def _synth_transcript(n_log2, seed):
    """A response-layout transcript of GPU-generated valid points (as bench.py's e2e rows) plus the
    generator's expected ark bytes of τG1 and ατG1."""
    import torch
    from kzgpot import device as D

    dev = torch.device("cuda", 0)
    n = 1 << n_log2
    parts, expect = [torch.zeros(64, dtype=torch.uint8, device=dev)], {}
    for k, (name, kind, cnt) in enumerate((("tau_g1", "g1", 2 * n - 1), ("tau_g2", "g2", n), ("alpha_g1", "g1", n),
                                           ("beta_g1", "g1", n), ("beta_g2", "g2", 1))):
        c, e = D.synth(kind, seed + k, 0, cnt, dev, with_expected=name in ("tau_g1", "alpha_g1"))
        parts.append(c)
        if e is not None:
            expect[name] = bytes(e.cpu().numpy())
    parts.append(torch.zeros(3 * 192 + 6 * 96, dtype=torch.uint8, device=dev))
    return bytearray(torch.cat(parts).cpu().numpy()), expect


@pytest.mark.parametrize("mode", [0, 1], ids=["kgz", "fastkgz"])
@pytest.mark.parametrize("n_log2,shards", [(18, 1), (19, 2)], ids=["2e18x1", "2e19x2"])
def test_streamed_digest_with_small_first_chunk(gpu, mode, n_log2, shards):
    """τG1 (2N - 1 points) and ατG1 run in several host chunks per shard, and with the output
    digest streaming from them each shard's first chunk is the small 2^16-point one (csrc/capi.hip
    run_host); with 2 shards the records reach the digest in file order only as far as both shards
    have landed (preprocess_impl's cursor). Both digests equal hashlib's over the same bytes,
    τG1 / ατG1 equal the generator's; then bad points in the first chunk and in a later one: the
    first chunk's is reported."""
    n = 1 << n_log2
    tr, expect = _synth_transcript(n_log2, seed=71 + mode + 2 * shards)
    res = gpu.preprocess_buffer(bytes(tr), n_log2, mode, n_gpus=shards, with_digests=True)
    g1n = (2 * n - 1) * 96
    assert res.out[:g1n] == expect["tau_g1"] and res.out[g1n:g1n + n * 96] == expect["alpha_g1"]
    assert res.transcript_digest == hashlib.blake2b(bytes(tr)).hexdigest()
    assert res.output_digest == hashlib.blake2b(res.out).hexdigest()
    for i in ((1 << 16) - 1, 3 * (1 << 17) + 9):
        tr[64 + i * 48] &= 0x7F  # compression bit cleared: UnexpectedCompressionMode
    with pytest.raises(gpu.KzgPotError) as e:
        gpu.preprocess_buffer(bytes(tr), n_log2, mode, n_gpus=shards, with_digests=True)
    assert (e.value.code, e.value.section, e.value.first_bad) == (-1, 0, (1 << 16) - 1)
