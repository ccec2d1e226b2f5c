#!/bin/bash
# C4 pyramid stage under k_pyramid_linear_chain band / thread variants (experiment)
set -e
O=gpurun_out/pyrab
mkdir -p $O
B="python3 bench.py --frames 512 --steps 5 --warmup 1 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-a11"
for v in libygzfe.so libygzfe_pyr_1_1024.so libygzfe_pyr_2_1024.so libygzfe_pyr_4_512.so libygzfe_pyr_4_256.so libygzfe_pyr_8_256.so libygzfe_pyr_8_512.so; do
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$v timeout -k 10 200 $B > $O/$v.json 2> $O/$v.err
done
