#!/bin/bash
# octree final rounds with per-thread contiguous scans: bit-exact order through the build, then the bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_segscan}
mkdir -p $O
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_segscan.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_extract_split.py tests/test_gpu_c5.py -k "not rccl and not pipe" > $O/tests.txt 2>&1 || echo "tests failed" >> $O/tests.txt
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_segscan.so
