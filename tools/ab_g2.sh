# Same-box A/B of the config-3 row (2^20 G1 + 2^20 G2): previous build (build_exp_old/) vs this tree.
set -e
mkdir -p gpurun_out/ab
B="python bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline --bn254-log2 0 --e2e-log2 0 --g1-log2 22"
for r in 1 2; do
  KZGPOT_LIB=$PWD/build_exp_old/libkzgpot.so timeout -k 10 150 $B > gpurun_out/ab/g2old_$r.json 2>/dev/null
  timeout -k 10 150 $B > gpurun_out/ab/g2new_$r.json 2>/dev/null
done
