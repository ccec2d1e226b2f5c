#!/bin/bash
# the pipe schedule: C5 byte-equality tests, then bench A/B against overlap (headline legs only)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_pipe}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_c5.py -k "schedules" > $O/tests.txt 2>&1
Q="--steps 10 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin"
for r in 1 2; do
  timeout -k 10 300 python bench.py $Q --schedule overlap >> $O/overlap.jsonl 2>> $O/err.log
  timeout -k 10 300 python bench.py $Q --schedule pipe --chunks 2 >> $O/pipe2.jsonl 2>> $O/err.log
  timeout -k 10 300 python bench.py $Q --schedule pipe --chunks 4 >> $O/pipe4.jsonl 2>> $O/err.log
done
