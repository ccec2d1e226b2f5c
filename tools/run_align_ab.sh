#!/bin/bash
# align A/B: parity tests on the product lib, then batch microbench (product vs base lib, interleaved) and stamps
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_alignab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_align.py tests/test_gpu_align_lm.py tests/test_gpu_c5.py > $O/tests.txt 2>&1
for r in 1 2; do
  for lib in libygzfe.so libygzfe_base.so; do
    YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$lib timeout -k 10 120 python tools/mb_align.py --reps 10 >> $O/mb_$lib.txt 2>&1
  done
done
timeout -k 10 120 python tools/diag_align.py > $O/diag_pair.txt 2>&1
