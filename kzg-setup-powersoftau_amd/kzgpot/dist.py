"""Multi-GPU sharding for the point codec: one process per GPU (torch.distributed over RCCL).

The τ^i arrays shard trivially (every point is independent); the only exchange is the all-gather
that assembles one contiguous arkworks buffer on every rank (the north_star's "final RCCL
all-gather over xGMI"), plus an 8-byte all-reduce(min) of the first-bad key.

Two layouts:
  * contiguous shards (`shard_bounds` + `gather_shards`): rank r decodes [r n/N, (r+1) n/N), one
    all-gather at the end;
  * block-cyclic, pipelined (`cyclic_block` + `decode_gather_pipelined`): the n points are cut
    into N x C equal blocks and rank r owns blocks c N + r (c < C). Chunk c's N blocks are
    adjacent in the output, so its all-gather is ONE in-place `all_gather_into_tensor` into a
    contiguous slice of the final buffer — issued asynchronously right after the rank's chunk-c
    launch, so the xGMI transfer of chunk c overlaps the decoding of chunk c + 1 and only the
    last chunk's gather is exposed.

These helpers are backend-agnostic so the same code is exercised with `gloo` on CPU tensors in
tests/test_dist.py and with `nccl` (= RCCL on ROCm) on HBM tensors in bench.py.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

NO_BAD = (1 << 64) - 1


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of n points for `rank`; equal sizes when world divides n."""
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def gather_shards(local: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """All-gather equal-sized 1-D byte shards into one contiguous buffer (rank order)."""
    if world == 1:
        return local
    out = torch.empty(local.numel() * world, dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "gloo":  # gloo has no all_gather_into_tensor
        dist.all_gather(list(out.chunk(world)), local, group=group)  # chunks are views of out
        return out
    dist.all_gather_into_tensor(out, local, group=group)
    return out


def cyclic_block(n: int, world: int, chunks: int) -> int:
    """Block size of the block-cyclic layout (n must split into world x chunks equal blocks)."""
    if n % (world * chunks):
        raise ValueError(f"{n} points do not split into {world} x {chunks} equal blocks")
    return n // (world * chunks)


def owned_block_starts(n: int, rank: int, world: int, chunks: int) -> list[int]:
    """First global point index of each block rank owns, in chunk order (block c N + rank)."""
    b = cyclic_block(n, world, chunks)
    return [(c * world + rank) * b for c in range(chunks)]


def decode_gather_pipelined(decode, full: torch.Tensor, rec_out: int, n: int, rank: int, world: int,
                            chunks: int, group=None) -> list:
    """For c = 0..chunks-1: `decode(c, g0, dst)` writes the rank's chunk-c block (global points
    [g0, g0 + B)) into its final place `dst` inside `full` (n records of rec_out bytes), then the
    chunk's N blocks are all-gathered in place, asynchronously. Returns the work handles: wait on
    them (on GPU this orders the current stream after the collectives) before reading `full`."""
    b = cyclic_block(n, world, chunks)
    works = []
    for c in range(chunks):
        g0 = (c * world + rank) * b
        mine = full[g0 * rec_out:(g0 + b) * rec_out]
        decode(c, g0, mine)
        if world == 1:
            continue
        region = full[c * world * b * rec_out:(c + 1) * world * b * rec_out]
        if dist.get_backend(group) == "gloo":  # no all_gather_into_tensor; output views alias `full`
            works.append(dist.all_gather(list(region.chunk(world)), mine.clone(), group=group, async_op=True))
        else:
            works.append(dist.all_gather_into_tensor(region, mine, group=group, async_op=True))
    return works


def shard_layout(n: int, world: int, chunks: int) -> tuple[int, int]:
    """(block, tail) of the library's block-cyclic layout (kzgpot_shard_layout, include/kzgpot.h):
    world x chunks blocks of floor(n / (world chunks)) points, then a tail every rank decodes."""
    b = n // (world * chunks)
    return b, n - b * world * chunks


def lib_local_ranges(n: int, rank: int, world: int, chunks: int) -> list[tuple[int, int]]:
    """Global (first point, count) ranges whose inputs rank's d_in_local holds, in order: its
    owned blocks c world + rank, then the tail."""
    b, tail = shard_layout(n, world, chunks)
    rng = [((c * world + rank) * b, b) for c in range(chunks)] if b else []
    if tail:
        rng.append((b * world * chunks, tail))
    return rng


LIB_OPS = {"g1_decompress": 0, "g2_decompress": 1, "g1_transcode": 2, "g2_transcode": 3, "bn254_g1_decompress": 4}


class LibComm:
    """A kzgpot communicator: RCCL inside libkzgpot.so (kzgpot_comm_init), so the decode and the
    all-gather that assembles the contiguous arkworks buffer are one library call
    (kzgpot_decode_allgather_dev). The 128-byte RCCL id travels over torch.distributed."""

    def __init__(self, rank: int, world: int, group=None):
        import ctypes

        from . import _lib

        self._ct, self.lib = ctypes, _lib.load()
        self.rank, self.world = rank, world
        uid = ctypes.create_string_buffer(128)
        if rank == 0:
            rc = self.lib.kzgpot_comm_unique_id(uid)
            if rc:
                raise RuntimeError(f"kzgpot_comm_unique_id failed ({rc})")
        if world > 1:
            obj = [uid.raw]
            dist.broadcast_object_list(obj, src=0, group=group)
            uid = ctypes.create_string_buffer(obj[0], 128)
        self.handle = ctypes.c_void_p()
        rc = self.lib.kzgpot_comm_init(ctypes.byref(self.handle), uid, world, rank)
        if rc:
            raise RuntimeError(f"kzgpot_comm_init({rank} of {world}) failed ({rc})")

    def decode_allgather(self, op: str, d_in_local: torch.Tensor, n: int, chunks: int, d_out: torch.Tensor,
                         key: torch.Tensor, flags: int = 0) -> None:
        """Asynchronous on torch's current stream: this rank's blocks decoded, every block
        all-gathered into d_out (n records on every rank), key = global first bad point."""
        from .device import _DEV_FNS

        _, rin, rout = _DEV_FNS[op]
        need_in = sum(c for _, c in lib_local_ranges(n, self.rank, self.world, chunks)) * rin
        if d_in_local.numel() < need_in or d_out.numel() < n * rout:
            raise ValueError(f"{op}: bad buffer sizes {d_in_local.numel()} / {d_out.numel()}")
        rc = self.lib.kzgpot_decode_allgather_dev(self.handle, LIB_OPS[op], d_in_local.data_ptr(), n, chunks,
                                                  d_out.data_ptr(), flags, key.data_ptr(),
                                                  torch.cuda.current_stream().cuda_stream)
        if rc:
            raise RuntimeError(f"kzgpot_decode_allgather_dev({op}) failed ({rc})")

    def wait(self, key: torch.Tensor, timeout_ms: int = 0) -> tuple[int, int]:
        """kzgpot_comm_wait on torch's current stream: (rc, first_bad). rc 0 = all accepted,
        -(status) = a rejected point at global index first_bad, KZGPOT_E_RANK_FAILED (-106) = a
        rank could not decode its share, KZGPOT_E_TIMEOUT (-107) / KZGPOT_E_DEVICE (-101) = the
        communicator was aborted."""
        fb = self._ct.c_int64(-1)
        rc = self.lib.kzgpot_comm_wait(self.handle, key.data_ptr(), self._ct.byref(fb), timeout_ms,
                                       torch.cuda.current_stream().cuda_stream)
        return rc, fb.value

    def size(self) -> dict:
        """What RCCL reports for this communicator (kzgpot_comm_size: ncclCommCount,
        ncclCommUserRank, ncclCommCuDevice)."""
        n, r, d = self._ct.c_int(-1), self._ct.c_int(-1), self._ct.c_int(-1)
        rc = self.lib.kzgpot_comm_size(self.handle, self._ct.byref(n), self._ct.byref(r), self._ct.byref(d))
        if rc:
            raise RuntimeError(f"kzgpot_comm_size failed ({rc})")
        return {"nranks": n.value, "rank": r.value, "device": d.value}

    def close(self) -> None:
        if self.handle:
            self.lib.kzgpot_comm_destroy(self.handle)
            self.handle = self._ct.c_void_p()


def agree_on_failure(failed: bool, aborted: bool, device, group=None) -> str:
    """One decision every rank takes together after a library decode + gather that may have
    failed somewhere: "ok" (no rank failed), "fallback" (some rank's decode failed in-band — the
    library still issued every collective, so the ranks are in step and may all switch to another
    gather path), or "abort" (some rank's communicator was aborted: collectives may be out of step,
    nothing collective may follow on it). Deciding per rank instead would let ranks run different
    collectives and hang."""
    t = torch.tensor([int(bool(failed)), int(bool(aborted))], dtype=torch.int64, device=device)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    f, a = (int(x) for x in t.tolist())
    return "abort" if a else ("fallback" if f else "ok")


def key_with_offset(key: int, offset: int) -> int:
    """Shift a shard-local bad key ((index << 8) | status) to global indices."""
    if key == NO_BAD:
        return NO_BAD
    return (((key >> 8) + offset) << 8) | (key & 0xFF)


def allreduce_min_key(key: int, device, group=None) -> int:
    """Global first bad point across ranks (keys are unsigned; carried as signed int64)."""
    signed = key - (1 << 64) if key >= (1 << 63) else key
    # NO_BAD (all ones) is -1 as int64: map it above every real key for the min
    t = torch.tensor([signed if key != NO_BAD else (1 << 63) - 1], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    v = int(t.item())
    return NO_BAD if v == (1 << 63) - 1 else v & NO_BAD
