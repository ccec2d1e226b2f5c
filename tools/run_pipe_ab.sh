#!/bin/bash
# pipe schedule: staggered chunk starts (default) vs none, 4 and 3 chunks
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_pipeab}
mkdir -p $O
Q="--steps 10 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin --no-stage-timing"
for r in 1 2; do
  timeout -k 10 300 python bench.py $Q >> $O/stagger4.jsonl 2>> $O/err.log
  YGZ_PIPE_STAGGER=0 timeout -k 10 300 python bench.py $Q >> $O/nostagger4.jsonl 2>> $O/err.log
  timeout -k 10 300 python bench.py $Q --chunks 3 >> $O/stagger3.jsonl 2>> $O/err.log
  timeout -k 10 300 python bench.py $Q --chunks 6 >> $O/stagger6.jsonl 2>> $O/err.log
done
