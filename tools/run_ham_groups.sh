#!/bin/bash
# Hamming: query groups per wave (A operand LDS reads shared by G MFMAs); parity, stage microbench, bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_hamg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_c5.py > $O/tests.txt 2>&1
for lib in libygzfe.so libygzfe_h24p1.so libygzfe_h18p1.so libygzfe_h18.so libygzfe.so libygzfe_h24p1.so; do
  echo "== $lib" >> $O/mb.txt
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$lib timeout -k 10 120 python tools/mb_hamming.py --n 415 936 1000 --check >> $O/mb.txt 2>&1
done
bash tools/ab_bench_lib.sh $O libygzfe.so libygzfe_h24p1.so libygzfe_h18p1.so
