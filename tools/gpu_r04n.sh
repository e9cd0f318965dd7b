set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/loader_timing.py --launches 24 --idle 1.0 --order g2,g1 > gpurun_out/r04n2_loader_timing.json 2> gpurun_out/r04n2_loader_timing.err
