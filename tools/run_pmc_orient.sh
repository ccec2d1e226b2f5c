#!/bin/bash
# PMC pass over the orientation + rBRIEF stage alone (tools/mb_fast.py, stage 1)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pmcorient}
mkdir -p $OUT
B="python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/libygzfe.so"
export YGZ_MB_STAGES=1
timeout -s KILL 120 rocprofv3 --output-format csv --kernel-include-regex k_orient_desc --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1
