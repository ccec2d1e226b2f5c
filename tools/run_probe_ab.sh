#!/bin/bash
# FAST phase split / compaction variant (mb_fast, FAST stage only), then the latency leg
# with and without the align-stream placement probe, alternating (experiment)
set -e
O=gpurun_out/${1:-probeab}
mkdir -p $O
L=$PWD/orb-ygz-slam_amd/lib
YGZ_MB_STAGES=0 timeout -k 10 300 python3 tools/mb_fast.py 1024 $L/libygzfe_base.so $L/libygzfe_c3.so \
  $L/libygzfe_stop1.so $L/libygzfe_stop3.so $L/libygzfe_base.so $L/libygzfe_c3.so > $O/mb_fast.txt 2>&1
B="python3 bench.py --frames 512 --steps 2 --warmup 1 --cpu-sample 0 --latency-frames 100 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-stage-timing"
for i in 1 2 3; do
  for v in 1 0; do
    YGZFE_ALIGN_PROBE=$v timeout -k 10 200 $B > $O/lat_${v}_$i.json 2> $O/lat_${v}_$i.err
    python3 -c "import json; d=json.loads(open('$O/lat_${v}_$i.json').read().strip().splitlines()[-1]); print('probe=$v run $i', json.dumps(d.get('latency', {}).get('median_ms')), json.dumps(d.get('latency', {}).get('median_align_wait_ms')))" >> $O/lat_summary.txt
  done
done
if [ -n "$FULL" ]; then
  timeout -k 10 400 python3 bench.py > $O/bench_full.json 2> $O/bench_full.err
fi
