"""The library's own multi-GPU entry (kzgpot_decode_allgather_dev: block-cyclic decode + in-place
RCCL all-gathers + all-reduce(min) of the first bad key, include/kzgpot.h §8e) with the REAL RCCL
at one rank (RCCL refuses two ranks on one device): every code path of the call runs (chunk loop,
per-chunk events into the comm stream, the in-place ncclAllGather, the ragged tail, the key merge
kernel and the ncclAllReduce). The multi-rank arithmetic (rank > 0 offsets, failure paths) runs in
tests/test_gpu_multirank.py through the test-only RCCL stand-in. Outputs are compared with the
single-launch codec (itself parity-tested against the oracle) and the generator's expected bytes;
bad points are planted and must come back at their global index."""
import pytest

pytestmark = pytest.mark.gpu

NO_BAD = (1 << 64) - 1


@pytest.fixture(scope="module")
def env(gpu):
    import torch

    from kzgpot import device as D
    from kzgpot import dist as KD

    comm = KD.LibComm(0, 1)
    yield torch, D, KD, comm
    comm.close()


REC = {"g1_decompress": ("g1", 48, 96), "g2_decompress": ("g2", 96, 192), "bn254_g1_decompress": ("bn254", 32, 64)}


def local_input(torch, D, KD, kind, seed, n, chunks, cuda):
    comp, exp = D.synth(kind, seed, 0, n, cuda)
    rin = {"g1": 48, "g2": 96, "bn254": 32}[kind]
    parts = [comp[g0 * rin:(g0 + c) * rin] for g0, c in KD.lib_local_ranges(n, 0, 1, chunks)]
    return comp, exp, (torch.cat(parts) if parts else comp[:0].clone())


@pytest.mark.parametrize("op,n,chunks", [
    ("g1_decompress", (1 << 14) + 5, 4),   # ragged: 5-point tail every rank decodes
    ("g1_decompress", 1 << 14, 8),
    ("g2_decompress", 1000, 3),
    ("bn254_g1_decompress", (1 << 15) + 1, 8),
    ("g1_decompress", 3, 8),                # fewer points than blocks: all tail
])
def test_decode_allgather_matches_expected(env, op, n, chunks):
    torch, D, KD, comm = env
    cuda = torch.device("cuda", 0)
    kind, rin, rout = REC[op]
    _, exp, loc = local_input(torch, D, KD, kind, 7 + n, n, chunks, cuda)
    out = torch.full((n * rout,), 0x5A, dtype=torch.uint8, device=cuda)
    key = torch.empty(1, dtype=torch.int64, device=cuda)
    comm.decode_allgather(op, loc, n, chunks, out, key)
    torch.cuda.synchronize()
    assert D.read_key(key) == NO_BAD
    assert torch.equal(out, exp)


def test_decode_allgather_first_bad_is_global(env):
    """Bad points in a later block and in the tail: the key is the smallest GLOBAL index, the
    records are zero-filled, everything else is decoded."""
    torch, D, KD, comm = env
    cuda = torch.device("cuda", 0)
    n, chunks = (1 << 12) + 3, 4
    comp, exp = D.synth("g1", 21, 0, n, cuda)
    comp = comp.clone()
    b, tail = KD.shard_layout(n, 1, chunks)
    bad = [2 * b + 17, n - 1]                 # block 2 and the tail
    for i in bad:
        comp[i * 48] &= 0x7F                    # clear the compression bit: UnexpectedCompressionMode
    parts = [comp[g0 * 48:(g0 + c) * 48] for g0, c in KD.lib_local_ranges(n, 0, 1, chunks)]
    out = torch.empty(n * 96, dtype=torch.uint8, device=cuda)
    key = torch.empty(1, dtype=torch.int64, device=cuda)
    comm.decode_allgather("g1_decompress", torch.cat(parts), n, chunks, out, key)
    torch.cuda.synchronize()
    k = D.read_key(key)
    assert k >> 8 == bad[0] and k & 0xFF == 1
    o, e = out.view(n, 96), exp.view(n, 96)
    for i in bad:
        assert int(o[i].count_nonzero()) == 0
    keep = torch.ones(n, dtype=torch.bool, device=cuda)
    keep[bad] = False
    assert torch.equal(o[keep], e[keep])


def test_decode_allgather_rejects_bad_args(env):
    torch, D, KD, comm = env
    lib = comm.lib
    import ctypes

    assert lib.kzgpot_decode_allgather_dev(None, 0, None, 0, 1, None, 0, None, None) < 0
    assert lib.kzgpot_decode_allgather_dev(comm.handle, 99, None, 0, 1, None, 0, None, None) < 0
    key = torch.empty(1, dtype=torch.int64, device="cuda")
    assert lib.kzgpot_decode_allgather_dev(comm.handle, 0, None, 0, 0, None, 0, key.data_ptr(), None) < 0  # 0 chunks
    # n = 0 is a valid empty stream
    assert lib.kzgpot_decode_allgather_dev(comm.handle, 0, None, 0, 4, None, 0, key.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert D.read_key(key) == NO_BAD
    blk, tl = ctypes.c_uint64(), ctypes.c_uint64()
    assert lib.kzgpot_shard_layout((1 << 22) - 1, 8, 8, ctypes.byref(blk), ctypes.byref(tl)) == 0
    assert (blk.value, tl.value) == KD.shard_layout((1 << 22) - 1, 8, 8)
