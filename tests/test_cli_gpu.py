"""The native drop-ins for the reference's binaries (build/kzgpot-preprocess-{kgz,fastkgz},
csrc/preprocess_main.cpp) run end to end on the GPU.

This module sorts before every other GPU test on purpose: it starts the CLI as a child process
while the pytest process itself has not touched the GPU yet (no `gpu` fixture here), so no child
is ever started from a process that holds a HIP context."""
import hashlib
import json
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN, PKG


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["kgz", "fastkgz"])
def test_cli_preprocess_config1(mode, tmp_path):
    """Config 1 (N = 2^10 transcript) through the CLI: the kzg_setup file's BLAKE2b-512 equals the
    oracle pipeline's (tests/golden/transcript_n1024.json); with the default POWERSOFTAU_DIGEST
    check the synthetic transcript fails validation (exit 101, no output file)."""
    meta = json.load(open(os.path.join(GOLDEN, "transcript_n1024.json")))
    shutil.copy(os.path.join(GOLDEN, "transcript_n1024.bin"), tmp_path / "powersoftau")
    exe = os.path.join(PKG, "build", f"kzgpot-preprocess-{mode}")
    r = subprocess.run([exe, "--n-log2", "10", "--no-digest-check", "--output-digest"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = (tmp_path / "kzg_setup").read_bytes()
    assert len(out) == meta[f"{mode}_size"]
    assert hashlib.blake2b(out).hexdigest() == meta[f"{mode}_blake2b"]
    assert f"output BLAKE2b-512: {meta[f'{mode}_blake2b']}" in r.stdout
    assert f"transcript BLAKE2b-512: {meta['transcript_blake2b']}" in r.stdout
    (tmp_path / "kzg_setup").unlink()
    # the reference's own work: the transcript checked against a given digest, the output not hashed
    r = subprocess.run([exe, "--n-log2", "10", "--expect-digest", meta["transcript_blake2b"]], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "output BLAKE2b-512" not in r.stdout and "Checking passed" in r.stdout
    assert hashlib.blake2b((tmp_path / "kzg_setup").read_bytes()).hexdigest() == meta[f"{mode}_blake2b"]
    (tmp_path / "kzg_setup").unlink()
    r = subprocess.run([exe, "--n-log2", "10", "--expect-digest", "0" * 128], cwd=tmp_path, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 101 and "failed validation" in r.stderr and not (tmp_path / "kzg_setup").exists()
    r = subprocess.run([exe, "--n-log2", "10"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 101 and "failed validation" in r.stderr
    assert not (tmp_path / "kzg_setup").exists()
