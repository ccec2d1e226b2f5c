#!/bin/bash
# octree candidate-sort experiment: bit-exact extraction through the variant, then the bench A/B (stage times)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_octrad}
mkdir -p $O
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_octrad.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py > $O/tests.txt 2>&1 || echo "tests failed" >> $O/tests.txt
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_octrad.so
