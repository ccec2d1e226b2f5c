#!/bin/bash
# PMC passes over a short bench run, each counter group in its own pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; no trace domains mixed in).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-x}/pmc
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11"
R="rocprofv3 --output-format csv"
timeout -k 10 150 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1
timeout -k 10 150 $R --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAVES -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1
timeout -k 10 150 $R --pmc FETCH_SIZE -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1
timeout -k 10 150 $R --pmc WRITE_SIZE -d $OUT/p4 -o run -- $B > $OUT/p4.log 2>&1
