#!/bin/bash
# align A/B of an experiment lib: parity tests through it, then the batch microbench interleaved with the product lib
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; X=$2
mkdir -p $O
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$X timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_align.py tests/test_gpu_c5.py > $O/tests_$X.txt 2>&1 || echo "tests failed" >> $O/tests_$X.txt
for r in 1 2; do
  for lib in libygzfe.so $X; do
    YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$lib timeout -k 10 120 python tools/mb_align.py --reps 10 >> $O/mb_$lib.txt 2>&1
  done
done
