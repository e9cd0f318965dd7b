set -e
mkdir -p gpurun_out/ab
B="python bench.py --steps 3 --no-next-rows --no-cpu-baseline --no-verify"
for r in 1 2; do
  KZGPOT_LIB=$PWD/build_exp_old/libkzgpot.so timeout -k 10 150 $B > gpurun_out/ab/old_$r.json 2>/dev/null
  timeout -k 10 150 $B > gpurun_out/ab/fused_$r.json 2>/dev/null
  timeout -k 10 150 $B --split-phases > gpurun_out/ab/split_$r.json 2>/dev/null
done
