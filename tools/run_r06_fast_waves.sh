#!/bin/bash
# FAST waves per workgroup 2 / 8 (cells per block; the XCD run then covers 8 / 32 neighbouring cells)
# against the product's 4: parity subset, bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_fast_waves}
mkdir -p $O
for v in libygzfe_fw2.so libygzfe_fw8.so; do
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$v timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_extract.py -k "sampled or batch or orbslam or dense" > $O/tests_$v.txt 2>&1
done
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_fw2.so libygzfe_fw8.so
