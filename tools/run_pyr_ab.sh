#!/bin/bash
# C4 pyramid stage under library variants (experiment): bash tools/run_pyr_ab.sh lib1.so lib2.so ...
set -e
O=gpurun_out/pyrab
mkdir -p $O
rm -f $O/summary.txt
B="python3 bench.py --frames 512 --steps 5 --warmup 1 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-a11"
for v in "$@"; do
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$v timeout -k 10 200 $B > $O/$v.json 2> $O/$v.err
  python3 -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); c=d['c4_batched']; print('$v', c['ms_per_step'], c['stages_ms']['pyramid'])" >> $O/summary.txt
done
