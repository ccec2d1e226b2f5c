#!/bin/bash
# PMC passes (one counter group per pass, no trace domains) plus a kernel
# trace over an arbitrary python command: tools/run_pmc_cmd.sh TAG script.py args...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
R="rocprofv3 --output-format csv"
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 "$@" > $OUT/kt.log 2>&1
timeout -k 10 150 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/p1 -o run -- python3 "$@" > $OUT/p1.log 2>&1
timeout -k 10 150 $R --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAVES -d $OUT/p2 -o run -- python3 "$@" > $OUT/p2.log 2>&1
timeout -k 10 150 $R --pmc FETCH_SIZE -d $OUT/p3 -o run -- python3 "$@" > $OUT/p3.log 2>&1
timeout -k 10 150 $R --pmc WRITE_SIZE -d $OUT/p4 -o run -- python3 "$@" > $OUT/p4.log 2>&1
python3 tools/prof_summary.py $(find $OUT/kt -name '*kernel_stats.csv') > $OUT/kt_summary.txt 2>&1 || true
python3 tools/pmc_summary.py $(find $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 -name '*counter_collection.csv') > $OUT/summary.txt
cat $OUT/kt_summary.txt $OUT/summary.txt
