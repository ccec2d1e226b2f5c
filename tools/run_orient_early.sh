#!/bin/bash
# orientation: both windows' loads issued at the start (one load latency fewer per workgroup); parity + bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_oearly}
mkdir -p $O
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_oearly.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_extract_split.py > $O/tests.txt 2>&1
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_oearly.so
