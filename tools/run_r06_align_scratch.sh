#!/bin/bash
# SparseImgAlign register kernel without the generic path's device call (libygzfe_nogen.so: no private
# segment; every C2 job has <= 960 features so the results are the same) against the product: does the
# 2,612 B/lane scratch the call brings cost the kernel anything?  Stage alone (tools/mb_align.py) + bench A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_align_scratch}
mkdir -p $O
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_nogen.so
