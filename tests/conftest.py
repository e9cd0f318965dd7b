import ctypes
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kzg-setup-powersoftau_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def golden(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)["vectors"]


@pytest.fixture(scope="session")
def oracle_lib():
    """The C restatement of the reference (test infrastructure only)."""
    path = os.environ.get("KZGPOT_ORACLE_LIB", os.path.join(ROOT, "oracle", "_build", "libkzgpot_oracle.so"))
    if not os.path.exists(path):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(path)
    lib.oracle_contribution_size.restype = ctypes.c_size_t
    lib.oracle_output_size.restype = ctypes.c_size_t
    return lib


@pytest.fixture(scope="session")
def kzgpot_mod():
    import kzgpot
    from kzgpot import _lib

    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", PKG, "-j", "8"], check=True)
    return kzgpot


@pytest.fixture(scope="session")
def gpu(kzgpot_mod):
    import torch  # noqa: F401  (HIP runtime shared with the library)

    if kzgpot_mod.device_count() < 1:
        pytest.fail("GPU test on a machine without a visible GPU")
    return kzgpot_mod


def oracle_run(lib, op, data: bytes, n: int, flags: int = 0, threads: int = 4):
    """Run the C oracle over n packed records → (out bytes, status bytes, first_bad, ret)."""
    rout = {"g1_decompress": 96, "g2_decompress": 192, "g1_transcode": 96, "g2_transcode": 192}[op]
    out = ctypes.create_string_buffer(max(1, n * rout))
    st = ctypes.create_string_buffer(max(1, n))
    fb = ctypes.c_int64(-1)
    if op == "g1_decompress":
        r = lib.oracle_g1_decompress(data, ctypes.c_size_t(n), out, ctypes.c_uint32(flags), ctypes.byref(fb), st,
                                     threads, threads)
    elif op == "g2_decompress":
        r = lib.oracle_g2_decompress(data, ctypes.c_size_t(n), out, ctypes.c_uint32(flags), ctypes.byref(fb), st,
                                     threads, threads)
    elif op == "g1_transcode":
        r = lib.oracle_g1_transcode(data, ctypes.c_size_t(n), out, ctypes.byref(fb), st, threads)
    else:
        r = lib.oracle_g2_transcode(data, ctypes.c_size_t(n), out, ctypes.byref(fb), st, threads)
    return out.raw[: n * rout], st.raw[:n], fb.value, r
