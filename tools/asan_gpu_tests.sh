#!/usr/bin/env bash
# Host-side AddressSanitizer pass over the library's host code (C ABI, chunk pipelines, preprocess
# threads, file streaming, BLAKE2b, loaders, communicator) while the GPU tests drive it.
# Build first on the CPU: make -C kzg-setup-powersoftau_amd asan. Device code is not instrumented.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
ASANRT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export KZGPOT_LIB=$ROOT/kzg-setup-powersoftau_amd/build/asan/libkzgpot.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1:log_path=$ROOT/gpurun_out/asan
# torch's GPU initialisation does not survive the preloaded runtime (its dlopen of
# libcaffe2_nvrtc fails), so the tests that drive the library through torch tensors are left out:
# everything here goes through the C ABI's host-buffer entry points, the CLI binaries aside.
# The host-resource fault injection first (tests/test_host_faults.py's driver; the ASan build
# carries the test hooks, Makefile), as top-level processes that check their own results (exit 3
# on a violated requirement, 134 on an abort): started from the ASan pytest process, and after it,
# the driver aborted in HSA's pool allocation under the ASan runtime
# (profiles/r06a_asan_fault_child.txt), before any library call had returned.
rc=0
for what in cpu gpu; do
  LD_PRELOAD=$ASANRT timeout -k 10 300 python -u tests/host_fault_driver.py $what \
    > "$ROOT/gpurun_out/asan_host_faults_$what.json" 2> "$ROOT/gpurun_out/asan_host_faults_$what.err"
  r=$?
  echo "host_fault_driver.py $what (ASan): exit $r" >> "$ROOT/gpurun_out/asan_host_faults.txt"
  [ $rc -eq 0 ] && rc=$r
done
# (-k names whole test functions: "streamed_digest_with_small_first_chunk" is the torch-based one;
# test_streamed_digests_multi_shard_capi is C-ABI only and runs here.)
LD_PRELOAD=$ASANRT timeout -k 10 600 python -u -m pytest tests/test_gpu_preprocess.py tests/test_gpu_capi_stream.py tests/test_gpu_parity.py \
  tests/test_gpu_fuzz.py -v --timeout 300 --timeout-method thread \
  -k "not current_device_is_restored and not load_dev_api and not bn254_synth_round_trip and not streamed_digest_with_small_first_chunk" \
  > "$ROOT/gpurun_out/asan_pytest.txt" 2>&1
r=$?
[ $rc -eq 0 ] && rc=$r
ls "$ROOT"/gpurun_out/asan* >/dev/null 2>&1
exit $rc
