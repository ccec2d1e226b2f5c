#!/bin/bash
# orientation + rBRIEF: one-path sincosf (each polynomial once) and aligned-row tap addresses;
# parity (extract, split, C5 sampled, drop-in sites) then the stage microbenchmark and bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_orab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_extract_split.py tests/test_gpu_c5.py tests/test_gpu_dropin.py -k "not rccl" > $O/tests.txt 2>&1
YGZ_MB_STAGES=1 timeout -k 10 300 python3 tools/mb_fast.py 1024 libygzfe.so libygzfe_sc.so libygzfe_prev.so libygzfe.so libygzfe_sc.so libygzfe_prev.so > $O/mb.txt 2>&1
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_prev.so
