# Same-box A/B of several builds of the library, alternating, three rounds:
#   bash tools/ab_libs.sh name1=path/libkzgpot.so name2=path/libkzgpot.so ...   ("-" = this tree's build)
# Per build and round: tools/codec_phases.py (2^20 G1 and G2) and the headline bench line.
# Results: gpurun_out/ab/<name>_{phases,bench}_<round>.json; PHASES_ONLY=1 skips the bench line.
set -e
mkdir -p gpurun_out/ab
B="python bench.py --steps 3 --no-next-rows --no-cpu-baseline --no-verify"
for r in 1 2 3; do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = "-" ]; then unset KZGPOT_LIB; else export KZGPOT_LIB=$PWD/$lib; fi
    timeout -k 10 120 python tools/codec_phases.py > gpurun_out/ab/${name}_phases_$r.json
    if [ -z "$PHASES_ONLY" ]; then timeout -k 10 150 $B > gpurun_out/ab/${name}_bench_$r.json 2>/dev/null; fi
  done
done
