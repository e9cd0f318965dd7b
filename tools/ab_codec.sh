# Same-box A/B of the checked codecs: the previous build (build_exp_old/libkzgpot.so, built from the
# parent commit with `make OUT=../build_exp_old`) against this tree, alternating, three rounds:
#   tools/codec_phases.py (2^20 G1 and G2: fused / phase 1 / split, event-timed)
#   bench.py headline only (2^27 G1 + 2^16 G2, 3 steps)
# Results: gpurun_out/ab/{old,new}_{phases,bench}_<round>.json
set -e
mkdir -p gpurun_out/ab
B="python bench.py --steps 3 --no-next-rows --no-cpu-baseline --no-verify"
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export KZGPOT_LIB=$PWD/build_exp_old/libkzgpot.so; else unset KZGPOT_LIB; fi
    timeout -k 10 120 python tools/codec_phases.py > gpurun_out/ab/${v}_phases_$r.json
    timeout -k 10 150 $B > gpurun_out/ab/${v}_bench_$r.json 2>/dev/null
  done
done
