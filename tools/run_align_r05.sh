#!/bin/bash
# Align diagnostics: batch microbench (product + stamp builds), one-pair phase stamps, PMC pass on the batch
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_align}
mkdir -p $O
timeout -k 10 180 python tools/mb_align.py --reps 10 > $O/mb.txt 2>&1
timeout -k 10 180 python tools/mb_align.py --reps 3 --diag > $O/mb_diag.txt 2>&1
timeout -k 10 120 python tools/diag_align.py > $O/diag_pair.txt 2>&1
if [ -n "$PMC" ]; then
R="rocprofv3 --output-format csv --kernel-include-regex k_sparse_align"
timeout -s KILL 90 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/p1 -o run -- python3 tools/mb_align.py --reps 3 > $O/p1.log 2>&1
timeout -s KILL 90 $R --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/p2 -o run -- python3 tools/mb_align.py --reps 3 > $O/p2.log 2>&1
fi
