#!/bin/bash
# kernel-alone durations for the roofline's dominant kernel: the bench's own command in the
# serial schedule over the same 4 chunk batches (no kernel overlaps another), under rocprofv3
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05prof}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --schedule serial --chunks 4 --steps 5 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin > $O/prof_bench.json 2> $O/prof_bench.err
python tools/prof_summary.py $(find $O/prof -name '*kernel_stats.csv') > $O/kernel_summary.txt 2>&1 || true
