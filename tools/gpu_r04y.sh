set -o pipefail
mkdir -p gpurun_out
timeout -k 10 660 python3 -u tools/random_campaign.py --budget 540 > gpurun_out/r04y_random_campaign.json 2> gpurun_out/r04y_random_campaign.err || exit 11
