#!/bin/bash
# octree first-stage shapes: parity of each variant (C5 sampled frames + extraction tests), then the
# bench A/B (product, o1: 512-class 2,048 keys / 256 threads, o2: 2,048 / 512, o3: 1024-class 1,024 threads)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_oct}
mkdir -p $O
for lib in libygzfe_o1.so libygzfe_o2.so libygzfe_o3.so; do
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_c5.py -k "sampled or batch or orbslam or dense" > $O/tests_$lib.txt 2>&1 || echo FAIL >> $O/tests_$lib.txt
done
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_o1.so libygzfe_o2.so libygzfe_o3.so
