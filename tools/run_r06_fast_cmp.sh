#!/bin/bash
# FAST phase A A/B: libygzfe.so (working tree) against libygzfe_base.so (HEAD): parity, stage alone, bench A/B
# (r06_fast_cmp: shared sign compares + lane-pointer list writes; r06_fast_chunk: full chunks without the row test, incremental row addresses)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_fast_cmp}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_initializer.py tests/test_gpu_fast10_golden.py > $O/tests.txt 2>&1
YGZ_MB_STAGES=0 timeout -k 10 300 python tools/mb_fast.py 1024 libygzfe_base.so libygzfe.so libygzfe_base.so libygzfe.so > $O/mb.txt 2>&1
bash tools/ab_bench_lib.sh $O libygzfe_base.so libygzfe.so
