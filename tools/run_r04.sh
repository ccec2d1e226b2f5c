#!/bin/bash
# Round-4 GPU iteration: parity tests (optional -k filter), smoke, bench, optional
# rocprofv3 kernel summary of a short bench (PROF=1).
set -e
O=gpurun_out/${1:-r04}
K=${2:-}
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "$K" > $O/tests.log 2>&1
else
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py $BENCH > $O/bench.json 2> $O/bench.err
fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 5 --warmup 2 > $O/prof_bench.json 2> $O/prof_bench.err
  python tools/prof_summary.py $(find $O/prof -name '*kernel_stats.csv') > $O/kernel_summary.txt 2>&1 || true
fi
