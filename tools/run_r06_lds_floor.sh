#!/bin/bash
# FAST LDS floor 0 (libygzfe_lds0.so) against the product's 23,000 B (libygzfe.so): three alternating passes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_lds_floor}
mkdir -p $O
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_lds0.so
bash tools/ab_bench_lib.sh $O libygzfe_lds0.so libygzfe.so
