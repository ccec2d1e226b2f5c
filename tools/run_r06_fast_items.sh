#!/bin/bash
# FAST: K cells per wave with the next cell's ROI loads in flight (extract.hip YGZ_FAST_ITEMS,
# YGZ_FAST_WPE): parity of every variant, the stage alone (tools/mb_fast.py), bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_fast_items}
mkdir -p $O
V="libygzfe_k2.so libygzfe_k4.so libygzfe_k8.so libygzfe_k2w7.so libygzfe_k4w7.so"
for v in $V; do
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$v timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_extract.py -k "sampled or batch or orbslam or dense" > $O/tests_$v.txt 2>&1
done
YGZ_MB_STAGES=0 timeout -k 10 400 python tools/mb_fast.py 1024 libygzfe.so $V libygzfe.so > $O/mb.txt 2>&1
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_k4.so libygzfe_k4w7.so
