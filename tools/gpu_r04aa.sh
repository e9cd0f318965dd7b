set -o pipefail
mkdir -p gpurun_out
for v in default v3 bmi2 default v3 bmi2; do echo "== $v"; timeout -k 10 60 tools/microbench/bin/blake2b_$v; done > gpurun_out/r04aa_blake2b_flags.txt 2>&1 || exit 11
lscpu | grep -i "model name\|flags" | cut -c1-200 >> gpurun_out/r04aa_blake2b_flags.txt
