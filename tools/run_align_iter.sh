#!/bin/bash
# SparseImgAlign iteration: batch/single parity tests, microbench, drop-in timing + kernel profile
set -e
O=gpurun_out/${1:-align}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_align.py tests/test_gpu_align_batch.py > $O/tests.log 2>&1
timeout -k 10 200 python tools/mb_align.py --reps 10 > $O/mb_align.txt 2>&1
PROF=1 bash tools/run_dropin_time.sh ${1:-align}/dropin
