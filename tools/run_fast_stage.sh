#!/bin/bash
# FAST ROI staging: unconditional loads at uniform row offsets (immediate LDS offsets) vs per-row predicated loads
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_stage}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_extract_split.py tests/test_gpu_c5.py -k "not rccl" > $O/tests.txt 2>&1
YGZ_MB_STAGES=0 timeout -k 10 300 python3 tools/mb_fast.py 1024 libygzfe.so libygzfe_prev.so libygzfe.so libygzfe_prev.so > $O/mb.txt 2>&1
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_prev.so
