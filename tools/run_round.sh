#!/bin/bash
# One GPU session for a round's evidence: parity tests, the default bench line,
# a rocprofv3 kernel-trace/stats profile of the same bench command, PMC passes.
set -e
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 > $O/ktrace.log 2>&1
bash tools/run_pmc.sh $TAG
