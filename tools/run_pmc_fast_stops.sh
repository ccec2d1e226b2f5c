#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pmcstops}
mkdir -p $OUT
for v in stop0 stop1 stop2 stop3; do
B="python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/libygzfe_$v.so"
timeout -s KILL 120 rocprofv3 --output-format csv --kernel-include-regex k_fast_cells --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d $OUT/$v -o run -- $B > $OUT/$v.log 2>&1
done
