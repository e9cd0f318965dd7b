"""Device-resident (HBM) codec calls and the synthetic-transcript generator, via torch tensors.

torch is plumbing here (HBM allocation, streams, RCCL); the compute is the C ABI's `_dev` entry
points, launched on torch's current stream so torch events and collectives order against them.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib

SYNTH_PATH = os.path.join(_lib.PKG_ROOT, "build", "libkzgpot_synth.so")
_synth = None


def synth_lib() -> ctypes.CDLL:
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise OSError(f"{SYNTH_PATH} not built")
        lib = ctypes.CDLL(SYNTH_PATH, mode=ctypes.RTLD_GLOBAL)
        for name in ("kzgpot_synth_g1_dev", "kzgpot_synth_g2_dev", "kzgpot_synth_bn254_dev"):
            fn = getattr(lib, name)
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p]
        lib.kzgpot_synth_clock_probe.restype = ctypes.c_int
        lib.kzgpot_synth_clock_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _synth = lib
    return _synth


def clock_probe(device) -> torch.Tensor:
    """Launch the clock probe on the current stream; returns its (64, 3) int64 device tensor
    (xcc id, shader-clock counter, 100 MHz real-time counter per block)."""
    t = torch.empty((64, 3), dtype=torch.int64, device=device)
    if synth_lib().kzgpot_synth_clock_probe(t.data_ptr(), _stream()):
        raise RuntimeError("kzgpot_synth_clock_probe failed")
    return t


def clock_mhz(before: torch.Tensor, after: torch.Tensor):
    """Average shader clock (MHz) between two probes, per XCD (paired by XCC id: each XCD has its
    own counters), and their mean. None if no XCD appears in both."""
    b, a = before.cpu().tolist(), after.cpu().tolist()
    first = {int(x): (t, r) for x, t, r in b}
    last = {int(x): (t, r) for x, t, r in a}
    per = {x: (last[x][0] - first[x][0]) / max(1, last[x][1] - first[x][1]) * 100.0
           for x in sorted(first) if x in last and last[x][1] > first[x][1]}
    if not per:
        return None
    return {"mean": sum(per.values()) / len(per), "per_xcd": per}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def synth(kind: str, seed: int, start: int, n: int, device, with_expected: bool = True):
    """Points start..start+n-1 of synthetic stream `seed`: (compressed, expected ark bytes)."""
    rin, rout = {"g1": (48, 96), "g2": (96, 192), "bn254": (32, 64)}[kind]
    comp = torch.empty(max(1, n * rin), dtype=torch.uint8, device=device)
    ark = torch.empty(max(1, n * rout), dtype=torch.uint8, device=device) if with_expected else None
    fn = getattr(synth_lib(), f"kzgpot_synth_{kind}_dev")
    rc = fn(seed, start, n, comp.data_ptr(), ark.data_ptr() if ark is not None else None, _stream())
    if rc:
        raise RuntimeError(f"synth {kind} failed: {rc}")
    return comp[: n * rin], (ark[: n * rout] if ark is not None else None)


_DEV_FNS = {
    "g1_decompress": ("kzgpot_g1_decompress_dev", 48, 96),
    "g2_decompress": ("kzgpot_g2_decompress_dev", 96, 192),
    "g1_transcode": ("kzgpot_g1_transcode_uncompressed_dev", 96, 96),
    "g2_transcode": ("kzgpot_g2_transcode_uncompressed_dev", 192, 192),
    "g1_load": ("kzgpot_g1_deserialize_unchecked_dev", 96, 104),   # no flags argument
    "g2_load": ("kzgpot_g2_deserialize_unchecked_dev", 192, 200),
    "bn254_g1_decompress": ("kzgpot_bn254_g1_decompress_dev", 32, 64),  # no flags argument
}


def codec_dev(op: str, d_in: torch.Tensor, d_out: torch.Tensor, key: torch.Tensor, flags: int = 0,
              d_status: torch.Tensor | None = None) -> None:
    """Asynchronous codec launch on device tensors (torch's current stream). `key` is one int64
    device word that receives min((index << 8) | status) of rejected points (all ones if none)."""
    fname, rin, rout = _DEV_FNS[op]
    n = d_in.numel() // rin
    if d_in.numel() != n * rin or d_out.numel() < n * rout:
        raise ValueError(f"{op}: bad buffer sizes {d_in.numel()} / {d_out.numel()}")
    if not (d_in.is_cuda and d_out.is_cuda and key.is_cuda):
        raise ValueError("codec_dev needs device tensors")
    st = d_status.data_ptr() if d_status is not None else None
    fn = getattr(_lib.load(), fname)
    if op.endswith("_load") or op.startswith("bn254"):
        rc = fn(d_in.data_ptr(), n, d_out.data_ptr(), key.data_ptr(), st, _stream())
    else:
        rc = fn(d_in.data_ptr(), n, d_out.data_ptr(), flags, key.data_ptr(), st, _stream())
    if rc:
        raise RuntimeError(f"{op}: launch failed ({rc})")


def read_key(key: torch.Tensor) -> int:
    return int(key.item()) & ((1 << 64) - 1)
