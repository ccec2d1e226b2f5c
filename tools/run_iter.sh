#!/bin/bash
# one GPU iteration: full parity suite, smoke, FAST / align microbenches, drop-in timing
set -e
O=gpurun_out/${1:-iter}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python tools/mb_fast.py 1024 libygzfe.so > $O/mb_fast.txt 2>&1
timeout -k 10 200 python tools/mb_align.py --reps 10 > $O/mb_align.txt 2>&1
bash tools/run_dropin_time.sh ${1:-iter}/dropin
