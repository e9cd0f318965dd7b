#!/usr/bin/env bash
# The checker under AddressSanitizer + UBSan while the GPU parity / fuzz tests lean on it hardest
# (oracle/_build/asan: make -C oracle asan on the CPU first). torch-driven tests are left out (its
# GPU initialisation does not survive the preloaded runtime); the library itself is the normal one.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
export KZGPOT_ORACLE_LIB=$ROOT/oracle/_build/asan/libkzgpot_oracle.so
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:log_path=$ROOT/gpurun_out/asan_oracle
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
LD_PRELOAD=$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so) timeout -k 10 600 \
  python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread \
  -k "not load_dev_api and not bn254_synth_round_trip" > "$ROOT/gpurun_out/asan_oracle_pytest.txt" 2>&1
