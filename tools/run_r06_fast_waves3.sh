#!/bin/bash
# FAST 4-wave workgroups (libygzfe_fw4.so) against 2 (libygzfe.so), both in 32-cell XCD runs: two alternating pass pairs
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_fast_waves3}
mkdir -p $O
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_fw4.so
bash tools/ab_bench_lib.sh $O libygzfe_fw4.so libygzfe.so
