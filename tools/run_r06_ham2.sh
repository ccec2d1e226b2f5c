#!/bin/bash
# Hamming FP4 variants: fused accumulator keys (product) / per-element keys (hnf) / 4 groups (hg4) /
# 8 waves (hw8) / the i8 form (hi8): parity tests on the product, stage microbench, bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_ham2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_c5.py -k "best2 or hamming or sampled or match" > $O/tests.txt 2>&1
for lib in libygzfe.so libygzfe_hnf.so libygzfe_hg4.so libygzfe_hw8.so libygzfe_hi8.so; do
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$lib timeout -k 10 200 python tools/mb_hamming.py --n 936 9000 --check > $O/mb_$lib.txt 2>&1
YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$lib timeout -k 10 200 python tools/mb_hamming.py --real > $O/mb_real_$lib.txt 2>&1
done
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_hnf.so
