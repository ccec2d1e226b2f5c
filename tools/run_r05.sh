#!/bin/bash
# Round-5 iteration on the GPU box: align + drop-in parity, the drop-in timing lines,
# the align stamp breakdown (diag build) and a short bench (stage times + latency).
# Usage: tools/run_r05.sh OUTDIR [pytest files...]
set -e
O=gpurun_out/${1:-r05}
shift || true
mkdir -p $O
T=${*:-tests/test_gpu_align.py tests/test_gpu_align_batch.py}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > $O/tests.txt 2>&1
timeout -k 10 200 compat/build/dropin_calls > $O/parity.txt 2>&1
timeout -k 10 300 compat/build/dropin_calls --time > $O/time.txt 2>&1
if [ -n "$DIAG" ]; then timeout -k 10 120 python tools/diag_align.py > $O/diag_align.txt 2>&1; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-undistort --no-bow --no-stereo \
  --no-a11 --no-dropin --no-direct --no-c4 > $O/bench.json 2> $O/bench.err
