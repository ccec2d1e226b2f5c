#!/bin/bash
# orientation + rBRIEF: the pattern as FP8 pairs (one v_cvt_pk_f32_fp8 per point) against the int8
# form (libygzfe_base.so): parity, stage alone (tools/mb_fast.py stage 1), bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_orient_f8}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_initializer.py tests/test_gpu_dropin.py > $O/tests.txt 2>&1
YGZ_MB_STAGES=1 timeout -k 10 300 python tools/mb_fast.py 1024 libygzfe_base.so libygzfe.so libygzfe_base.so libygzfe.so > $O/mb.txt 2>&1
bash tools/ab_bench_lib.sh $O libygzfe_base.so libygzfe.so
