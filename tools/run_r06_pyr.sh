#!/bin/bash
# pyramid levels formed by the level-0 blur strips (batch path): parity tests, then the bench
# A/B against YGZFE_PYR_UNFUSED=1 (the separate pyramid pass), alternating
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_pyr}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_extract_split.py tests/test_gpu_c5.py > $O/tests.txt 2>&1
A="--steps 10 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin"
for r in 1 2; do
timeout -k 10 300 python bench.py $A >> $O/fused.jsonl 2>> $O/err.log
YGZFE_PYR_UNFUSED=1 timeout -k 10 300 python bench.py $A >> $O/unfused.jsonl 2>> $O/err.log
done
