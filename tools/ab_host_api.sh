#!/usr/bin/env bash
# Same-box A/B of the host-buffer entry point (kzgpot_g1_decompress on 2^25 and kzgpot_g2_decompress
# on 2^20 pageable points, against
# the same points device-resident): the previous build (build_exp_old/libkzgpot.so, from the parent
# commit: make OUT=../build_exp_old) and this tree, alternating, three rounds.
# Results: gpurun_out/ab_host/{old,new}_<round>.json
set -e
mkdir -p gpurun_out/ab_host
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export KZGPOT_LIB=$PWD/build_exp_old/libkzgpot.so; else unset KZGPOT_LIB; fi
    timeout -k 10 120 python3 tools/host_api_trace.py > gpurun_out/ab_host/${v}_$r.json
    timeout -k 10 120 python3 tools/host_api_trace.py --kind g2 --log2 20 > gpurun_out/ab_host/${v}_g2_$r.json
  done
done
