#!/bin/bash
# Latency leg under align-stream variants (experiment): reduced bench, then the full default bench
set -e
O=gpurun_out/latab2
mkdir -p $O
B="python3 bench.py --frames 512 --steps 2 --warmup 1 --cpu-sample 0 --latency-frames 100 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-stage-timing"
for v in 0 3; do
  YGZFE_ALIGN_PRIO=$v timeout -k 10 200 $B > $O/r_$v.json 2> $O/r_$v.err
done
for v in 0 3; do
  YGZFE_ALIGN_PRIO=$v timeout -k 10 300 python3 bench.py --cpu-sample 0 > $O/f_$v.json 2> $O/f_$v.err
done
