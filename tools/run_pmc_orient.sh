#!/bin/bash
# PMC passes over the orientation + rBRIEF stage alone (tools/mb_fast.py, stage 1)
# usage: run_pmc_orient.sh OUTDIR [libname]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pmcorient}
LIBN=${2:-libygzfe.so}
mkdir -p $OUT
B="python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/$LIBN"
export YGZ_MB_STAGES=1
R="rocprofv3 --output-format csv --kernel-include-regex k_orient_desc"
timeout -s KILL 120 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1
timeout -s KILL 120 $R --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1
