"""Host-resource failures at the C ABI: a host thread that cannot start
(std::system_error EAGAIN, as under a process limit), a host buffer mapping that fails, or a
std::bad_alloc must come back as KZGPOT_E_OUT_OF_MEMORY (-108) — never as an exception crossing
an extern "C" function (std::terminate, SIGABRT) — with every thread the call started joined and
no "<out>.kzgpot-tmp-*" file left behind. The reference returns a Result at this boundary
(Accumulator::deserialize, /root/reference/src/bin/preprocess-kgz.rs:105-110) and panics only at
its own expect().

The faults are injected by the test build (libkzgpot_test.so, kzgpot_test_inject_host_fault,
tests/kzgpot_test_hooks.h); the driver runs in a child process so that an abort is seen as its
exit status. tools/asan_gpu_tests.sh runs the GPU case under the host-ASan build."""
import json
import os
import subprocess
import sys

import pytest

from conftest import PKG, ROOT

E_DEVICE, E_OOM = -101, -108
DRIVER = os.path.join(ROOT, "tests", "host_fault_driver.py")
TEST_LIB = os.path.join(PKG, "build", "libkzgpot_test.so")


def _run(what, timeout=240):
    if not os.path.exists(TEST_LIB):
        subprocess.run(["make", "-C", PKG, "-j", "8"], check=True)
    env = dict(os.environ)
    env.setdefault("KZGPOT_LIB", TEST_LIB)
    p = subprocess.run([sys.executable, DRIVER, what], capture_output=True, text=True, timeout=timeout, env=env)
    # an exception across the C ABI would have ended the child with SIGABRT (-6); 3 = the driver's
    # own check of the results failed (host_fault_driver.problems)
    assert p.returncode in (0, 3), (p.returncode, p.stderr[-3000:])
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert not res["problems"], res["problems"]
    return res


def test_status_name_out_of_memory(kzgpot_mod):
    assert kzgpot_mod.status_name(E_OOM) == "OutOfMemory"


def test_host_faults_before_device_work():
    """Runs without a GPU: the transcript hasher, the two file-buffer mappings and the reader
    thread, each failing in turn, return -108 with no temporary file and no output
    (host_fault_driver.problems holds the requirements); with no fault, a machine without a GPU
    is a device error (the hasher joined first)."""
    res = _run("cpu")
    assert [c["ret"] for c in res["cases"]] == [E_OOM] * 5


@pytest.fixture(scope="module")
def capi(kzgpot_mod):
    """No torch in the process (the host-ASan run cannot initialise it)."""
    if kzgpot_mod.device_count() < 1:
        pytest.fail("GPU test on a machine without a visible GPU")
    return kzgpot_mod


@pytest.mark.gpu
def test_every_thread_start_failing_returns_out_of_memory(capi):
    """A 3-shard file call starts 19 threads (reader, transcript hasher, output hasher, writer,
    3 shards x 5 sections) and a 20th that releases its buffers. Failing every start from the
    (k + 1)-th on, for each k: -108 with nothing left behind while a pipeline thread failed; once
    only the release fails, the call succeeds (the buffers go on the calling thread) and the file
    is the reference file. Afterwards a clean call still writes it."""
    res = _run("gpu", timeout=600)
    assert sum(c["ret"] == E_OOM for c in res["cases"]) == 2 * 19
