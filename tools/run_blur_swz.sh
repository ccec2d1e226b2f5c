#!/bin/bash
# blur: one frame's strips per XCD (halo rows from L2) and the strip height; parity then stage + bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_bswz}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_extract_split.py tests/test_gpu_c5.py -k "not rccl" > $O/tests.txt 2>&1
for v in b48 b64; do
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py > $O/tests_$v.txt 2>&1
done
YGZ_MB_STAGES=2 timeout -k 10 300 python3 tools/mb_fast.py 1024 libygzfe.so libygzfe_bnoswz.so libygzfe_b48.so libygzfe_b64.so libygzfe.so libygzfe_bnoswz.so libygzfe_b48.so libygzfe_b64.so > $O/mb.txt 2>&1
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_bnoswz.so libygzfe_b48.so
