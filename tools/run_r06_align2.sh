#!/bin/bash
# SparseImgAlign residency probe: reg vs x2 kernel time at 256 / 512 / 1023 pairs per launch
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_align2}
mkdir -p $O
for P in 256 512 1023; do
YGZFE_ALIGN_X2_MIN=1000000 timeout -k 10 180 python tools/mb_align.py --reps 10 --pairs $P > $O/mb_reg_$P.txt 2>&1
timeout -k 10 180 python tools/mb_align.py --reps 10 --pairs $P > $O/mb_x2_$P.txt 2>&1
done
