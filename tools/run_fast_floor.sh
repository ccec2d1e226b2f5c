#!/bin/bash
# FAST per-level LDS floor re-checked after the round's FAST changes (bench A/B, pipe schedule)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_floor2}
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_fl0.so libygzfe_fl20000.so libygzfe_fl26800.so
