#!/bin/bash
# pipe schedule chunk count re-check after this round's kernel changes: headline legs, alternating
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_chunks}
mkdir -p $O
A="--steps 10 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin"
for r in 1 2; do
  for k in 3 4 5 6 8; do
    timeout -k 10 200 python bench.py $A --chunks $k >> $O/chunks_$k.jsonl 2>> $O/err.log
  done
done
