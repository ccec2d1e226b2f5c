#!/bin/bash
# Round-5 full GPU check: every -m gpu test, the drop-in parity + timing, smoke, quick bench.
set -e
O=gpurun_out/${1:-r05full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 200 compat/build/dropin_calls > $O/parity.txt 2>&1
timeout -k 10 300 compat/build/dropin_calls --time > $O/time.txt 2>&1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-undistort --no-bow --no-stereo \
  --no-a11 --no-dropin --no-direct --no-c4 > $O/bench.json 2> $O/bench.err
