#!/bin/bash
# C5 step + stage times under library variants (YGZFE_LIB), alternating (experiment)
set -e
O=gpurun_out/libab
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11"
for v in "$@"; do
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$v timeout -k 10 200 $B > $O/$v.json 2> $O/$v.err
  python3 -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); r=d['roofline']['stages_ms']; print('$v', d['value'], json.dumps(r))" >> $O/summary.txt
done
