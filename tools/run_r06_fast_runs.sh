#!/bin/bash
# FAST (2-wave workgroups) XCD runs of 16 cells (libygzfe.so) against 8 (libygzfe_r8.so, the run length that
# 2-wave blocks got from the 4-block runs) and 32 (libygzfe_r32.so): parity, FAST traffic alone, bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_fast_runs}
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_extract.py -k "sampled or batch or orbslam or dense" > $O/tests.txt 2>&1
LIBS="libygzfe_r8.so libygzfe_r32.so" bash tools/run_r06_fast_traffic.sh ${1:-r06_fast_runs}
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_r8.so libygzfe_r32.so
