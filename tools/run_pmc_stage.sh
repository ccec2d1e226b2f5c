#!/bin/bash
# PMC passes over one stage alone (tools/mb_fast.py): run_pmc_stage.sh OUTDIR KERNEL_REGEX STAGE [libname]
# (stage 0: FAST, 1: orientation + rBRIEF, 2: blur)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
KRE=$2
export YGZ_MB_STAGES=$3
LIBN=${4:-libygzfe.so}
mkdir -p $OUT
B="python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/$LIBN"
R="rocprofv3 --output-format csv --kernel-include-regex $KRE"
timeout -s KILL 120 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1
timeout -s KILL 120 $R --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE SQ_WAIT_ANY -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1
timeout -s KILL 120 $R --pmc FETCH_SIZE -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1
timeout -s KILL 120 $R --pmc WRITE_SIZE -d $OUT/p4 -o run -- $B > $OUT/p4.log 2>&1
