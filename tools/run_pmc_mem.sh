#!/bin/bash
# Memory-path counters (TA / TD / TCP / TCC) of one kernel of the stage microbench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pmcmem}
KRE=${2:-k_orient_desc}
export YGZ_MB_STAGES=${3:-1}
mkdir -p $OUT
B="python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/libygzfe.so"
R="rocprofv3 --output-format csv --kernel-include-regex $KRE"
timeout -s KILL 120 $R --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d $OUT/m1 -o run -- $B > $OUT/m1.log 2>&1
timeout -s KILL 120 $R --pmc TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum -d $OUT/m2 -o run -- $B > $OUT/m2.log 2>&1
