#!/bin/bash
# single-frame ComputeBoW through pinned staging (one DMA each way) and the norm's batched LDS reads:
# parity (BoW + drop-in tests), the bench's DBoW2 leg and drop-in timing, a rocprof summary of the leg
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_bow}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bow.py tests/test_gpu_dropin.py > $O/tests.txt 2>&1
A="--steps 2 --warmup 1 --cpu-sample 1 --latency-frames 0 --no-direct --no-stereo --no-undistort --no-c4 --no-a11"
timeout -k 10 400 python bench.py $A > $O/bench.json 2> $O/bench.err
