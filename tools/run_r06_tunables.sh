#!/bin/bash
# tunables re-checked on the closing code (headline legs, two alternating passes): FAST LDS floor 0 / 20,000
# (product 23,000), blur rows in flight 8 / 12 (product 10)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_tunables}
mkdir -p $O
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_lds0.so libygzfe_lds20k.so libygzfe_ah8.so libygzfe_ah12.so
