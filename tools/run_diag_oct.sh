#!/bin/bash
# octree block stamps (diag build, STAMPK 3) at batch 1024
set -e
O=gpurun_out/${1:-diag_oct}
mkdir -p $O
STAMPK=3 YGZ_DIAG_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_diag3.so timeout -k 10 120 python tools/diag_blocks.py 1024 > $O/diag3.log 2>&1
