#!/bin/bash
# tunables re-checked on the closing code (headline legs, two alternating passes): Hamming one query group per
# wave (69 VGPRs, 7 waves/SIMD) and 8-wave workgroups, blur at 6 waves/SIMD
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_tunables2}
mkdir -p $O
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_hg1.so libygzfe_hw8.so libygzfe_beu6.so
