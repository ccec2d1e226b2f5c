#!/bin/bash
# round 6 first check: round 5's crash order (C5, align, align LM) then the initialiser
# extractor's tests with the graph path on; the whole GPU suite; the default bench line
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:randomly \
  tests/test_gpu_c5.py tests/test_gpu_align.py tests/test_gpu_align_lm.py tests/test_gpu_initializer.py > $O/repro.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
