#!/bin/bash
# Hamming experiment: two tiles per barrier; parity through the build, then the bench A/B (stage times)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_ham}
mkdir -p $O
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_hdual.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_c5.py -k "best2 or hamming or sampled or schedules" > $O/tests.txt 2>&1 || echo "tests failed" >> $O/tests.txt
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_hdual.so
