set -o pipefail
mkdir -p gpurun_out
timeout -k 10 660 python3 -u tools/random_campaign.py --budget 540 --seed0 100000 --ops g1_decompress,g2_decompress,g1_transcode,g2_transcode > gpurun_out/r04z_random_campaign.json 2> gpurun_out/r04z_random_campaign.err || exit 11
