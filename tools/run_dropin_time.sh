#!/bin/bash
# drop-in call sites: parity + --time lines (tests/dropin/dropin_calls)
set -e
O=gpurun_out/${1:-dropin}
mkdir -p $O
make -s -C compat dropin
timeout -k 10 200 compat/build/dropin_calls > $O/parity.txt 2>&1
timeout -k 10 200 compat/build/dropin_calls --time > $O/time.txt 2>&1
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- compat/build/dropin_calls --time > $O/prof_time.txt 2>&1
  python tools/prof_summary.py $(find $O/prof -name '*kernel_stats.csv') > $O/kernel_summary.txt 2>&1 || true
fi
