"""ctypes binding of the C ABI in include/kzgpot.h (build/libkzgpot.so).

The shared library is the product: HIP kernels for gfx950 plus the host driver. There is no
CPU fallback — if the library or a GPU is missing, calls raise instead of computing elsewhere.
"""
from __future__ import annotations

import ctypes
import os
import re

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("KZGPOT_LIB", os.path.join(PKG_ROOT, "build", "libkzgpot.so"))
# test build (-DKZGPOT_TEST_HOOKS): + kzgpot_comm_inject_fault and the KZGPOT_RCCL_LIB override
# (tests/kzgpot_test_hooks.h); tests select it through KZGPOT_LIB
TEST_LIB_PATH = os.path.join(PKG_ROOT, "build", "libkzgpot_test.so")
HEADER_PATH = os.path.join(REPO_ROOT, "include", "kzgpot.h")

u8p = ctypes.POINTER(ctypes.c_uint8)
i64p = ctypes.POINTER(ctypes.c_int64)
u64p = ctypes.POINTER(ctypes.c_uint64)
intp = ctypes.POINTER(ctypes.c_int)

# name -> (restype, argtypes)
SIGNATURES = {
    "kzgpot_g1_decompress": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, i64p]),
    "kzgpot_g2_decompress": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, i64p]),
    "kzgpot_g1_transcode_uncompressed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, i64p]),
    "kzgpot_g2_transcode_uncompressed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, i64p]),
    "kzgpot_g1_decompress_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, i64p, ctypes.c_void_p]),
    "kzgpot_g2_decompress_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, i64p, ctypes.c_void_p]),
    "kzgpot_g1_transcode_uncompressed_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, i64p, ctypes.c_void_p]),
    "kzgpot_g2_transcode_uncompressed_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, i64p, ctypes.c_void_p]),
    "kzgpot_g1_decompress_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kzgpot_g2_decompress_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kzgpot_g1_transcode_uncompressed_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kzgpot_g2_transcode_uncompressed_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kzgpot_decode_bad_key": (ctypes.c_int, [ctypes.c_uint64, i64p]),
    "kzgpot_contribution_size": (ctypes.c_uint64, [ctypes.c_uint32]),
    "kzgpot_output_size": (ctypes.c_uint64, [ctypes.c_uint32, ctypes.c_int]),
    "kzgpot_preprocess": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, intp, i64p]),
    "kzgpot_preprocess_buffer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, intp, i64p]),
    "kzgpot_g1_deserialize_unchecked": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, i64p]),
    "kzgpot_g2_deserialize_unchecked": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, i64p]),
    "kzgpot_g1_deserialize_unchecked_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, i64p, ctypes.c_void_p]),
    "kzgpot_g2_deserialize_unchecked_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, i64p, ctypes.c_void_p]),
    "kzgpot_g1_deserialize_unchecked_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kzgpot_g2_deserialize_unchecked_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kzgpot_load_kzg_setup": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, intp, i64p]),
    "kzgpot_load_kzg_setup_buffer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, intp, i64p]),
    "kzgpot_load_fastkzg_setup": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, intp, i64p]),
    "kzgpot_load_fastkzg_setup_buffer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, intp, i64p]),
    "kzgpot_phase1_size": (ctypes.c_uint64, [ctypes.c_uint32]),
    "kzgpot_load_phase1": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32] + [ctypes.c_void_p] * 7 + [intp, i64p]),
    "kzgpot_load_phase1_buffer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32] + [ctypes.c_void_p] * 7 + [intp, i64p]),
    "kzgpot_preprocess_ex": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, intp, i64p]),
    "kzgpot_preprocess_buffer_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, intp, i64p]),
    "kzgpot_blake2b": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "kzgpot_bn254_g1_decompress": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, i64p]),
    "kzgpot_bn254_g1_decompress_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, i64p, ctypes.c_void_p]),
    "kzgpot_bn254_g1_decompress_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kzgpot_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "kzgpot_comm_init": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "kzgpot_comm_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "kzgpot_shard_layout": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, u64p, u64p]),
    "kzgpot_decode_allgather_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "kzgpot_comm_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, i64p, ctypes.c_uint32, ctypes.c_void_p]),
    "kzgpot_comm_size": (ctypes.c_int, [ctypes.c_void_p, intp, intp, intp]),
    "kzgpot_status_name": (ctypes.c_char_p, [ctypes.c_int]),
    "kzgpot_device_count": (ctypes.c_int, []),
    "kzgpot_version": (ctypes.c_char_p, []),
}


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function the public header declares (used by the export test)."""
    text = open(path).read()
    return sorted(set(re.findall(r"\b(kzgpot_[a-z0-9_]+)\s*\(", text)))


_lib = None


def load() -> ctypes.CDLL:
    """Load build/libkzgpot.so (once). Raises OSError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not built: run `make -C kzg-setup-powersoftau_amd` or __graft_entry__.build()")
    # If torch is already loaded it brought its own libamdhip64.so.7 (same SONAME): the loader
    # reuses it, so device pointers from torch tensors are valid here.
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
