#!/usr/bin/env bash
# Same-box comparison of host-buffer pipelines (csrc/capi.hip run_host / ChunkPlan): the product
# build (A) against variant libraries build_exp_<V>/libkzgpot.so, alternating, two rounds, on G1 / G2
# calls of several sizes (tools/host_api_trace.py). Variants measured: `old` = equal chunks (before
# r06x); B / D / E = -DKZGPOT_CHUNK_END_LOG2 / -DKZGPOT_CHUNK_FLOOR_LOG2 = 17/18, 16/18, 17/19
# (profiles/r06za_ab_plans); `two` = the product's two-slot pipeline beside a three-slot A
# (profiles/r06zb_ab_slots). Build a variant by copying build/*.o to build_exp_<V>/ and rebuilding
# capi.o there with the knobs.
# Results: gpurun_out/ab_plans/<variant>_<kind><log2>_<round>.json
set -e
V=${VARIANTS:-A old}
mkdir -p gpurun_out/ab_plans
for r in 1 2; do
  for v in $V; do
    if [ $v = A ]; then unset KZGPOT_LIB; else export KZGPOT_LIB=$PWD/build_exp_$v/libkzgpot.so; fi
    for c in g2:20 g2:21 g1:20 g1:22 g1:25; do
      k=${c%%:*}; l=${c##*:}
      timeout -k 10 120 python3 tools/host_api_trace.py --kind $k --log2 $l > gpurun_out/ab_plans/${v}_${k}${l}_$r.json
    done
  done
done
