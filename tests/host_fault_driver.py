"""Child process of tests/test_host_faults.py: drives the file / buffer pipeline of the test build
(libkzgpot_test.so, or KZGPOT_LIB) with host-resource faults injected through
kzgpot_test_inject_host_fault (tests/kzgpot_test_hooks.h), and prints one JSON line.

It runs in its own process so that an exception escaping the C ABI (std::terminate → SIGABRT)
shows up as the child's exit status instead of killing pytest.

  host_fault_driver.py cpu   — the paths before any device work (runs without a GPU)
  host_fault_driver.py gpu   — every thread start of a 3-shard file call in turn (needs a GPU)

It checks its own results (problems(), the test's requirements) and exits 3 on a violation, so
tools/asan_gpu_tests.sh can run it as a top-level process under the host-ASan build.

The transcript is the config-1 fixture (tests/golden/transcript_n1024.bin, N = 2^10)."""
import ctypes
import glob
import hashlib
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kzg-setup-powersoftau_amd")
LIB = os.environ.get("KZGPOT_LIB", os.path.join(PKG, "build", "libkzgpot_test.so"))
GOLDEN = os.path.join(ROOT, "tests", "golden")
THREAD, HOSTBUF = 1, 2  # KZGPOT_HOST_FAULT_* (tests/kzgpot_test_hooks.h)
MODE_KZG, MODE_FASTKZG = 0, 1


def main():
    what = sys.argv[1]
    lib = ctypes.CDLL(LIB, mode=ctypes.RTLD_GLOBAL)  # as kzgpot._lib.load() binds it
    lib.kzgpot_test_inject_host_fault.argtypes = [ctypes.c_int, ctypes.c_long]
    lib.kzgpot_status_name.restype = ctypes.c_char_p
    # put the GPU to work on this (main) thread first, as every other test process has by the time
    # it reaches the file pipeline: under the host-ASan runtime (tools/asan_gpu_tests.sh) a process
    # whose first device allocation came from one of the library's shard threads aborted in HSA's
    # pool allocation ("AddressSanitizer: out of memory", profiles/r06a_asan_fault_child.txt); one
    # generator point decoded here (the G1 generator's published encoding) avoids that
    res_devices = lib.kzgpot_device_count()
    if res_devices > 0:
        gen = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
        o96, fb = ctypes.create_string_buffer(96), ctypes.c_int64(0)
        if lib.kzgpot_g1_decompress(gen, ctypes.c_size_t(1), o96, 0, ctypes.byref(fb)) != 0:
            raise SystemExit("the G1 generator did not decode")
    meta = json.load(open(os.path.join(GOLDEN, "transcript_n1024.json")))
    src = os.path.join(GOLDEN, "transcript_n1024.bin")
    tr = open(src, "rb").read()
    work = tempfile.mkdtemp(prefix="kzgpot_fault_")
    out_path = os.path.join(work, "kzg_setup")
    res = {"lib": LIB, "devices": res_devices, "cases": []}

    def leftovers():
        return sorted(os.path.basename(p) for p in glob.glob(out_path + ".kzgpot-tmp-*"))

    def file_call(mode, expect, shards):
        sec, idx = ctypes.c_int(7), ctypes.c_int64(7)
        tdig, odig = ctypes.create_string_buffer(129), ctypes.create_string_buffer(129)
        r = lib.kzgpot_preprocess_ex(src.encode(), out_path.encode(), mode, 10, shards,
                                     expect.encode() if expect else None, tdig, odig,
                                     ctypes.byref(sec), ctypes.byref(idx))
        return r, sec.value, idx.value, odig.value.decode()

    def buffer_call(expect):
        out = ctypes.create_string_buffer(meta["kgz_size"])
        sec, idx = ctypes.c_int(7), ctypes.c_int64(7)
        tdig = ctypes.create_string_buffer(129)
        r = lib.kzgpot_preprocess_buffer_ex(tr, len(tr), out, MODE_KZG, 10, 1, expect.encode(), tdig, None,
                                            ctypes.byref(sec), ctypes.byref(idx))
        return r, sec.value, idx.value

    if what == "cpu":
        # no GPU needed: each fault hits before the first device call
        for name, site, skip, call in (
                ("buffer: transcript hasher", THREAD, 0, lambda: buffer_call(meta["transcript_blake2b"])),
                ("file: host buffer mapping", HOSTBUF, 0, lambda: file_call(MODE_KZG, meta["transcript_blake2b"], 1)),
                ("file: second host buffer mapping", HOSTBUF, 1,
                 lambda: file_call(MODE_FASTKZG, meta["transcript_blake2b"], 1)),
                ("file: reader thread", THREAD, 0, lambda: file_call(MODE_KZG, meta["transcript_blake2b"], 1)),
                ("file: transcript hasher after the reader", THREAD, 1,
                 lambda: file_call(MODE_KZG, meta["transcript_blake2b"], 1))):
            lib.kzgpot_test_inject_host_fault(site, skip)
            r = call()
            lib.kzgpot_test_inject_host_fault(0, 0)
            res["cases"].append({"name": name, "ret": r[0], "status": lib.kzgpot_status_name(r[0]).decode(),
                                 "bad_section": r[1], "bad_index": r[2], "tmp_left": leftovers(),
                                 "out_exists": os.path.exists(out_path)})
        # without a fault and without a GPU the same call is a device error, after joining the hasher
        r = buffer_call(meta["transcript_blake2b"])
        res["no_fault_no_gpu"] = r[0]
    else:
        want = {MODE_KZG: meta["kgz_blake2b"], MODE_FASTKZG: meta["fastkgz_blake2b"]}
        for mode in (MODE_KZG, MODE_FASTKZG):
            # thread starts of one 3-shard file call: reader, transcript hasher, output hasher,
            # writer, then 3 shards per section (5 sections), then the buffer release. Failing
            # every start from the (skip + 1)-th on covers each in turn; the last skip fails only
            # the release, whose buffers then go on the calling thread.
            for skip in range(0, 4 + 5 * 3 + 1):
                if os.path.exists(out_path):
                    os.unlink(out_path)
                lib.kzgpot_test_inject_host_fault(THREAD, skip)
                r, sec, idx, odig = file_call(mode, meta["transcript_blake2b"], 3)
                lib.kzgpot_test_inject_host_fault(0, 0)
                ok_file = os.path.exists(out_path) and \
                    hashlib.blake2b(open(out_path, "rb").read()).hexdigest() == want[mode]
                res["cases"].append({"mode": mode, "skip": skip, "ret": r, "bad_section": sec, "bad_index": idx,
                                     "tmp_left": leftovers(), "out_exists": os.path.exists(out_path),
                                     "file_ok": ok_file, "output_digest_ok": odig == want[mode]})
            # the library is still usable: a clean call writes the reference file
            if os.path.exists(out_path):
                os.unlink(out_path)
            r, sec, idx, odig = file_call(mode, meta["transcript_blake2b"], 3)
            res.setdefault("after", []).append({"mode": mode, "ret": r, "output_digest_ok": odig == want[mode],
                                                "tmp_left": leftovers()})
    for p in glob.glob(os.path.join(work, "*")):
        os.unlink(p)
    os.rmdir(work)
    res["problems"] = problems(what, res)
    print(json.dumps(res))
    return 3 if res["problems"] else 0


E_DEVICE, E_OOM = -101, -108


def problems(what, res):
    """What tests/test_host_faults.py requires of a run, as a list of violations (empty = pass)."""
    bad = []
    if what == "cpu":
        if len(res["cases"]) != 5:
            bad.append("expected 5 cases")
        for c in res["cases"]:
            if c["ret"] != E_OOM or c["status"] != "OutOfMemory":
                bad.append(f"{c['name']}: returned {c['ret']}")
            if c["tmp_left"] or c["out_exists"]:
                bad.append(f"{c['name']}: left {c['tmp_left']} / output {c['out_exists']}")
            if c["bad_section"] != -1 or c["bad_index"] != -1:
                bad.append(f"{c['name']}: bad_section / bad_index set")
        if res.get("no_fault_no_gpu") not in (0, E_DEVICE):
            bad.append(f"no fault: returned {res.get('no_fault_no_gpu')}")
    else:
        if len(res["cases"]) != 2 * 20:
            bad.append("expected 40 cases")
        for c in res["cases"]:
            tag = f"mode {c['mode']} skip {c['skip']}"
            if c["tmp_left"]:
                bad.append(f"{tag}: left {c['tmp_left']}")
            if c["skip"] < 19:
                if c["ret"] != E_OOM or c["out_exists"] or c["bad_section"] != -1 or c["bad_index"] != -1:
                    bad.append(f"{tag}: returned {c['ret']}, output {c['out_exists']}")
            elif not (c["ret"] == 0 and c["file_ok"] and c["output_digest_ok"]):
                bad.append(f"{tag}: the release-only fault must still write the reference file ({c['ret']})")
        for a in res.get("after", []):
            if not (a["ret"] == 0 and a["output_digest_ok"] and not a["tmp_left"]):
                bad.append(f"mode {a['mode']}: the clean call afterwards failed ({a['ret']})")
    return bad


if __name__ == "__main__":
    sys.exit(main())
