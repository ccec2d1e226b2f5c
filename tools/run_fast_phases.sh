#!/bin/bash
# FAST phase knock-outs (YGZ_FAST_KO 1..4 builds) beside the product: stage time and one PMC pass each
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_fastko}
mkdir -p $O
export YGZ_MB_STAGES=0
timeout -k 10 300 python3 tools/mb_fast.py 1024 libygzfe.so libygzfe_ko1.so libygzfe_ko2.so libygzfe_ko3.so libygzfe_ko4.so > $O/times.txt 2>&1
for v in libygzfe libygzfe_ko1 libygzfe_ko2 libygzfe_ko3 libygzfe_ko4; do
timeout -s KILL 90 rocprofv3 --output-format csv --kernel-include-regex k_fast_cells --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d $O/$v -o run -- python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/$v.so > $O/$v.log 2>&1
done
