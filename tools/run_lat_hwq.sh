#!/bin/bash
# Single-frame latency under GPU_MAX_HW_QUEUES 4 (HIP's default) vs 8 (experiment)
set -e
O=gpurun_out/lathwq
mkdir -p $O
B="python3 bench.py --frames 512 --steps 2 --warmup 1 --cpu-sample 0 --latency-frames 100 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-stage-timing"
for q in 4 8 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 $B > $O/q$q.json 2> $O/q$q.err
  python3 -c "import json; d=json.loads(open('$O/q$q.json').read().strip().splitlines()[-1]); l=d['latency']; print('$q', d['value'], l['median_ms'], l['median_extract_ms'], l['median_align_wait_ms'], l['serial']['median_ms'])" >> $O/summary.txt
done
