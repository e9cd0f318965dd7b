# Same-box A/B of the headline G1 codec: previous build (build_exp_old/) vs this tree, alternating.
set -e
mkdir -p gpurun_out/ab
B="python bench.py --steps 3 --no-next-rows --no-cpu-baseline --no-verify"
for r in 1 2; do
  KZGPOT_LIB=$PWD/build_exp_old/libkzgpot.so timeout -k 10 150 $B > gpurun_out/ab/g1old_$r.json 2>/dev/null
  timeout -k 10 150 $B > gpurun_out/ab/g1new_$r.json 2>/dev/null
done
