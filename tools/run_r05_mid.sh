#!/bin/bash
# mid-round check: C5 / align / extract GPU tests, then the default bench line (pipe, 4 chunks)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_mid}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c5.py tests/test_gpu_align.py tests/test_gpu_align_lm.py tests/test_gpu_extract.py > $O/tests.txt 2>&1
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin > $O/bench.json 2> $O/bench.err
