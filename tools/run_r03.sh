#!/bin/bash
# Round-3 GPU iteration: parity tests (optional -k filter), smoke, optional bench.
set -e
O=gpurun_out/${1:-r03}
K=${2:-}
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $O/tests.log 2>&1
else
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py $BENCH > $O/bench.json 2> $O/bench.err
fi
