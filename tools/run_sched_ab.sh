#!/bin/bash
# C5 step under the three stage schedules (A/B; main line only)
set -e
O=gpurun_out/sched
mkdir -p $O
B="python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-stage-timing"
for s in tail serial tail serial overlap; do
  timeout -k 10 200 $B --schedule $s > $O/$s.json 2> $O/$s.err
  python3 -c "import json; d=json.loads(open('$O/$s.json').read().strip().splitlines()[-1]); print('$s', d['value'], d['ms_per_step'])" >> $O/summary.txt
done
