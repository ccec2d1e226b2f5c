#!/bin/bash
# PMC passes over the FAST-only microbench (tools/mb_fast.py), one counter group per pass.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pmcfast}
LIBN=${2:-libygzfe.so}
mkdir -p $OUT
B="python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/$LIBN"
R="rocprofv3 --output-format csv --kernel-include-regex k_fast_"
timeout -s KILL 120 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1
timeout -s KILL 120 $R --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1
python3 tools/pmc_summary.py $(find $OUT/p1 $OUT/p2 -name '*counter_collection.csv') > $OUT/summary.txt
