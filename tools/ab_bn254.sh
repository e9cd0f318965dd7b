set -e
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in def bn; do
    export KZGPOT_LIB=$PWD/build_exp_$v/libkzgpot.so
    timeout -k 10 200 python bench.py --steps 3 --g1-log2 20 --no-cpu-baseline --no-verify --e2e-log2 0 > gpurun_out/ab/bnrow_${v}_$r.json 2>/dev/null
  done
done
