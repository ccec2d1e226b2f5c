#!/bin/bash
# round 6 mid-round check: the whole GPU suite, smoke, the default bench line
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_mid}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
