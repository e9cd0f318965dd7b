"""N > 1 path on CPU: world_size-2 gloo processes shard a G1 stream, decode their shards (with the
C oracle standing in for the GPU kernels), reduce the first-bad key and all-gather one contiguous
arkworks buffer — the same kzgpot.dist code bench.py runs over RCCL."""
import ctypes
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, data, n, bad_index, q):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))
    from kzgpot import dist as KD

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libkzgpot_oracle.so"))
    lo, hi = KD.shard_bounds(n, rank, world)
    m = hi - lo
    out = ctypes.create_string_buffer(m * 96)
    fb = ctypes.c_int64(-1)
    r = lib.oracle_g1_decompress(data[lo * 48: hi * 48], ctypes.c_size_t(m), out, 0, ctypes.byref(fb), None, 1, 1)
    key = KD.NO_BAD if r == 0 else ((fb.value << 8) | (-r))
    gkey = KD.allreduce_min_key(KD.key_with_offset(key, lo), "cpu")
    local = torch.frombuffer(bytearray(out.raw), dtype=torch.uint8)
    full = KD.gather_shards(local, world)
    if rank == 0:
        q.put((bytes(full.numpy()), gkey))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_decode_and_gather(oracle_lib, world):
    vecs = [v for v in golden("g1_decompress") if v["check"] and v["status"] == 0][:32]
    assert len(vecs) == 32
    bad = golden("g1_decompress")
    bad_vec = next(v for v in bad if v["status"] == 5)
    data = bytearray(b"".join(bytes.fromhex(v["in"]) for v in vecs))
    bad_index = 21  # in rank 1's shard
    data[bad_index * 48:(bad_index + 1) * 48] = bytes.fromhex(bad_vec["in"])
    n = len(vecs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bytes(data), n, bad_index, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, gkey = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference
    out = ctypes.create_string_buffer(n * 96)
    fb = ctypes.c_int64(-1)
    r = oracle_lib.oracle_g1_decompress(bytes(data), ctypes.c_size_t(n), out, 0, ctypes.byref(fb), None, 1, 1)
    assert full == out.raw
    assert r == -5 and fb.value == bad_index
    assert gkey == (bad_index << 8) | 5


def test_shard_bounds_cover():
    from kzgpot import dist as KD

    for n in (0, 1, 7, 1 << 16, (1 << 22) - 1):
        for world in (1, 2, 4, 8):
            spans = [KD.shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
    assert KD.key_with_offset(KD.NO_BAD, 5) == KD.NO_BAD
    assert KD.key_with_offset((3 << 8) | 5, 100) == (103 << 8) | 5


def _worker_pipelined(rank, world, port, data, n, chunks, q):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))
    from kzgpot import dist as KD

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libkzgpot_oracle.so"))
    full = torch.zeros(n * 96, dtype=torch.uint8)
    keys = []

    def decode(c, g0, dst):  # the C oracle stands in for the chunk-c kernel launch
        b = dst.numel() // 96
        out = ctypes.create_string_buffer(b * 96)
        fb = ctypes.c_int64(-1)
        r = lib.oracle_g1_decompress(data[g0 * 48:(g0 + b) * 48], ctypes.c_size_t(b), out, 0, ctypes.byref(fb),
                                     None, 1, 1)
        dst.copy_(torch.frombuffer(bytearray(out.raw), dtype=torch.uint8))
        keys.append(KD.key_with_offset(KD.NO_BAD if r == 0 else ((fb.value << 8) | (-r)), g0))

    works = KD.decode_gather_pipelined(decode, full, 96, n, rank, world, chunks)
    for w in works:
        w.wait()
    gkey = KD.allreduce_min_key(min(keys), "cpu")
    q.put((rank, bytes(full.numpy()), gkey))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks", [(2, 4), (4, 2)])
def test_block_cyclic_pipelined_gather(oracle_lib, world, chunks):
    """bench.py's N > 1 layout: rank r decodes blocks c N + r and all-gathers each chunk in place
    as soon as it is decoded; every rank ends with the single-process buffer and the global
    first-bad key (a bad point planted in a block of the last rank)."""
    vecs = [v for v in golden("g1_decompress") if v["check"] and v["status"] == 0][:32]
    bad_vec = next(v for v in golden("g1_decompress") if v["status"] == 5)
    n = 32
    data = bytearray(b"".join(bytes.fromhex(v["in"]) for v in vecs))
    from kzgpot import dist as KD

    b = KD.cyclic_block(n, world, chunks)
    bad_index = KD.owned_block_starts(n, world - 1, world, chunks)[1] + b - 1
    data[bad_index * 48:(bad_index + 1) * 48] = bytes.fromhex(bad_vec["in"])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pipelined, args=(r, world, port, bytes(data), n, chunks, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out = ctypes.create_string_buffer(n * 96)
    fb = ctypes.c_int64(-1)
    r = oracle_lib.oracle_g1_decompress(bytes(data), ctypes.c_size_t(n), out, 0, ctypes.byref(fb), None, 1, 1)
    assert r == -5 and fb.value == bad_index
    for _, full, gkey in got:
        assert full == out.raw
        assert gkey == (bad_index << 8) | 5


def test_cyclic_layout():
    from kzgpot import dist as KD

    n, world, chunks = 1 << 12, 8, 4
    b = KD.cyclic_block(n, world, chunks)
    starts = sorted(s for r in range(world) for s in KD.owned_block_starts(n, r, world, chunks))
    assert starts == list(range(0, n, b))
    with pytest.raises(ValueError):
        KD.cyclic_block(100, 8, 4)


@pytest.mark.parametrize("n,world,chunks", [((1 << 22) - 1, 8, 8), (1 << 27, 8, 8), (100, 8, 4), (3, 2, 8), (0, 4, 2)])
def test_library_layout_covers_every_point(kzgpot_mod, n, world, chunks):
    """kzgpot_shard_layout (the C ABI's block-cyclic layout for kzgpot_decode_allgather_dev) and its
    Python mirror agree; the owned blocks over all ranks plus the tail cover [0, n) exactly once,
    and each chunk's world blocks are adjacent (one contiguous in-place all-gather per chunk)."""
    from kzgpot import _lib
    from kzgpot import dist as KD

    blk, tl = ctypes.c_uint64(), ctypes.c_uint64()
    assert _lib.load().kzgpot_shard_layout(n, world, chunks, ctypes.byref(blk), ctypes.byref(tl)) == 0
    b, tail = KD.shard_layout(n, world, chunks)
    assert (blk.value, tl.value) == (b, tail)
    assert tail < world * chunks
    covered = []
    for r in range(world):
        rng = KD.lib_local_ranges(n, r, world, chunks)
        owned = rng[:-1] if tail else rng
        covered += [i for g0, c in owned for i in range(g0, g0 + c)] if n < 5000 else [g0 for g0, _ in owned]
        if tail:
            assert rng[-1] == (n - tail, tail)  # every rank decodes the tail itself
    if n < 5000:
        assert sorted(covered) == list(range(n - tail))
    else:
        assert sorted(covered) == list(range(0, n - tail, b))
    for c in range(chunks):  # chunk c = blocks c*world .. c*world + world - 1, contiguous
        starts = sorted(KD.lib_local_ranges(n, r, world, chunks)[c][0] for r in range(world)) if b else []
        assert starts == [(c * world + r) * b for r in range(world)] if b else True


def test_bench_lib_gather_fallback():
    """bench.py's warm-up insurance: a failing library decode_allgather switches every stream to
    the torch.distributed gathers over the same block-cyclic layout — only when the blocks are
    identical (n splits into world x chunks equal blocks)."""
    import types

    import bench

    mk = lambda n, world, chunks: types.SimpleNamespace(n=n, world=world, chunks=chunks, comm=object())
    streams = [mk(1 << 27, 8, 8), mk(1 << 16, 8, 1)]
    bench.FALLBACKS.clear()
    assert bench.lib_to_torch_gather(streams, RuntimeError("x"))
    assert all(s.comm is None for s in streams) and len(bench.FALLBACKS) == 1
    assert not bench.lib_to_torch_gather(streams, RuntimeError("again"))  # nothing left to switch
    ragged = [mk((1 << 20) + 3, 4, 8)]
    assert not bench.lib_to_torch_gather(ragged, RuntimeError("x")) and ragged[0].comm is not None
    bench.FALLBACKS.clear()


def _agree_worker(rank, world, port, cases, q):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))
    from kzgpot import dist as KD

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = [KD.agree_on_failure(*case[rank], device="cpu") for case in cases]
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_warmup_failure_decision_is_collective():
    """bench.py's warm-up fallback: a failure injected on ONE rank must lead every
    rank to the same decision — switch gather paths together after an in-band failure, stop
    together after an aborted communicator — so no rank runs collectives its peers do not."""
    world = 2
    # per case: (failed, aborted) for rank 0, rank 1
    cases = [((False, False), (False, False)),
             ((False, False), (True, False)),    # rank 1's decode failed in-band
             ((True, False), (False, False)),
             ((False, True), (True, False)),     # rank 0's communicator aborted
             ((False, False), (False, True))]
    want = ["ok", "fallback", "fallback", "abort", "abort"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    assert res == {0: want, 1: want}
