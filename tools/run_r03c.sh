#!/bin/bash
# tests + default bench + octree block stamps (diag builds, STAMPK 3 / 4)
set -e
O=gpurun_out/${1:-r03c}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
for k in 3 4; do
  STAMPK=$k YGZ_DIAG_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_diag$k.so timeout -k 10 120 python tools/diag_blocks.py 1024 > $O/diag$k.log 2>&1
done
