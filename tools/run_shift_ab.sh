#!/bin/bash
# FAST with the ROI rows staged one byte right (YGZ_FAST_SHIFT) vs the default and the
# 40-byte level-0 stride alone: parity of the variant, then alternating stage timings
set -e
O=gpurun_out/${1:-shiftab}
mkdir -p $O
L=$PWD/orb-ygz-slam_amd/lib
YGZFE_LIB=$L/libygzfe_shift.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_shift.log 2>&1
YGZ_MB_STAGES=0 timeout -k 10 300 python3 tools/mb_fast.py 1024 $L/libygzfe_base.so $L/libygzfe_shift.so \
  $L/libygzfe_base.so $L/libygzfe_shift.so $L/libygzfe_base.so $L/libygzfe_shift.so > $O/mb_fast.txt 2>&1
