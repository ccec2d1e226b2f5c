#!/bin/bash
# FAST 2 waves per workgroup (libygzfe_fw2.so) against 4 (libygzfe.so): three more alternating pass pairs
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_fast_waves2}
mkdir -p $O
bash tools/ab_bench_lib.sh $O libygzfe_fw2.so libygzfe.so
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_fw2.so
