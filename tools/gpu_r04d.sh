set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile_round.sh r04d || exit 11
