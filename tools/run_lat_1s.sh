#!/bin/bash
# Single-frame latency: extraction DAG on side streams vs one stream (A/B)
set -e
O=gpurun_out/lat1s
mkdir -p $O
B="python3 bench.py --frames 512 --steps 2 --warmup 1 --cpu-sample 0 --latency-frames 100 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-stage-timing"
for v in dag one dag one; do
  if [ $v = one ]; then export YGZFE_SF_ONESTREAM=1; else unset YGZFE_SF_ONESTREAM; fi
  timeout -k 10 200 $B > $O/$v.json 2> $O/$v.err
  python3 -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); l=d['latency']; print('$v', l['median_ms'], l['median_extract_ms'], l['median_align_wait_ms'], l['serial']['median_ms'], l['serial']['median_extract_ms'])" >> $O/summary.txt
done
