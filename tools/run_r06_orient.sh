#!/bin/bash
# orientation + rBRIEF with 32 lanes per keypoint (k_orient_desc32, product) vs 16 (YGZFE_ORIENT16=1):
# parity, the stage microbenchmark, the bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_orient}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_extract_split.py tests/test_gpu_initializer.py tests/test_gpu_c5.py > $O/tests.txt 2>&1
YGZ_MB_STAGES=1 timeout -k 10 200 python tools/mb_fast.py 1024 $PWD/orb-ygz-slam_amd/lib/libygzfe.so > $O/mb32.txt 2>&1 || true
YGZFE_ORIENT16=1 YGZ_MB_STAGES=1 timeout -k 10 200 python tools/mb_fast.py 1024 $PWD/orb-ygz-slam_amd/lib/libygzfe.so > $O/mb16.txt 2>&1 || true
YGZFE_ORIENT16=1 YGZ_MB_STAGES=1 timeout -k 10 200 python tools/mb_fast.py 1024 $PWD/orb-ygz-slam_amd/lib/libygzfe.so > $O/mb16b.txt 2>&1 || true
YGZ_MB_STAGES=1 timeout -k 10 200 python tools/mb_fast.py 1024 $PWD/orb-ygz-slam_amd/lib/libygzfe_oe8.so > $O/mb32e8.txt 2>&1 || true
A="--steps 10 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin"
for r in 1 2; do
timeout -k 10 300 python bench.py $A >> $O/o32.jsonl 2>> $O/err.log
YGZFE_ORIENT16=1 timeout -k 10 300 python bench.py $A >> $O/o16.jsonl 2>> $O/err.log
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_oe8.so timeout -k 10 300 python bench.py $A >> $O/o32e8.jsonl 2>> $O/err.log
done
