#!/bin/bash
# blur experiment: halo dwords loaded by the two edge lanes only; bit-exactness + the blur stage alone
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_blur}
mkdir -p $O
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_bhalo.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py -k "blur or bitexact" > $O/tests.txt 2>&1 || echo "tests failed" >> $O/tests.txt
YGZ_MB_STAGES=2 timeout -k 10 300 python3 tools/mb_fast.py 1024 libygzfe.so libygzfe_bhalo.so libygzfe.so libygzfe_bhalo.so > $O/times.txt 2>&1
