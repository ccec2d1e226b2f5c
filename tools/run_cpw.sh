#!/bin/bash
# FAST cells-per-wave (pipelined ROI staging) experiment: bit-exactness, the FAST stage alone, the bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_cpw}
mkdir -p $O
for v in cpw2 cpw4; do
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py > $O/tests_$v.txt 2>&1 || echo "tests failed" >> $O/tests_$v.txt
done
YGZ_MB_STAGES=0 timeout -k 10 300 python3 tools/mb_fast.py 1024 libygzfe.so libygzfe_cpw2.so libygzfe_cpw4.so libygzfe.so libygzfe_cpw2.so libygzfe_cpw4.so > $O/times.txt 2>&1
BENCH_ARGS="--schedule pipe --chunks 4" bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_octrad.so libygzfe_cpw2.so
BENCH_ARGS="--schedule pipe --chunks 8" bash tools/ab_bench_lib.sh $O/c8 libygzfe.so
