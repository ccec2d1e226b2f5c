#!/bin/bash
# FAST staging only the ROI's rows (libygzfe_fr.so, YGZ_FAST_ROWS_ROI=1): parity, traffic, time, bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_fast_rows}
mkdir -p $O
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_fr.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_c5.py -k "sampled or batch or orbslam or dense" > $O/tests.txt 2>&1
LIBS=libygzfe_fr.so bash tools/run_r06_fast_traffic.sh ${1:-r06_fast_rows}
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_fr.so
