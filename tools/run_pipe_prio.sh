#!/bin/bash
# pipe schedule: SparseImgAlign on its own stream at high / low priority vs on the chunk's stream
# (record of a measured-negative experiment: the YGZFE_PIPE_ALIGN_PRIO knob was removed after it)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_prio}
mkdir -p $O
A="--steps 10 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin"
for rep in 1 2; do
  for p in none high low; do
    YGZFE_PIPE_ALIGN_PRIO=$p timeout -k 10 300 python bench.py $A >> $O/$p.jsonl 2>> $O/err.log
  done
done
