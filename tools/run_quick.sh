#!/bin/bash
# Quick GPU iteration: parity tests (optionally a -k filter), the C2 batch bench
# line without side legs, and the per-phase block stamps of FAST / orientation.
set -e
O=gpurun_out/${1:-quick}
K=${2:-}
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/tests.log 2>&1
else
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
fi
timeout -k 10 200 python bench.py --workload c2batch --steps 20 --warmup 3 --cpu-sample 0 --latency-frames 0 --no-c4 --no-undistort --no-bow --no-stereo --no-direct > $O/bench.json 2> $O/bench.err
for k in 2 1; do
  if [ -f orb-ygz-slam_amd/lib/libygzfe_diag$k.so ]; then
    STAMPK=$k YGZ_DIAG_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_diag$k.so timeout -k 10 120 python tools/diag_blocks.py 1024 > $O/diag$k.log 2>&1
  fi
done
