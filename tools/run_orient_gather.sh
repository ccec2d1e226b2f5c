#!/bin/bash
# orientation experiment: bit-exactness of the gather build through the extraction tests, then the orient stage alone
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_ogather}
mkdir -p $O
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_ogather.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py > $O/tests.txt 2>&1 || echo "tests failed" >> $O/tests.txt
export YGZ_MB_STAGES=1
timeout -k 10 300 python3 tools/mb_fast.py 1024 libygzfe.so libygzfe_ogather.so libygzfe.so libygzfe_ogather.so > $O/times.txt 2>&1
R="rocprofv3 --output-format csv --kernel-include-regex k_orient_desc"
for v in libygzfe libygzfe_ogather; do
timeout -s KILL 90 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES -d $O/$v -o run -- python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/$v.so > $O/$v.log 2>&1
timeout -s KILL 90 $R --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT -d $O/${v}_ta -o run -- python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/$v.so > $O/${v}_ta.log 2>&1
done
