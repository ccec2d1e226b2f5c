#!/bin/bash
# the order-dependent crash (C5 then align then LM) after the extractor-lifetime fix, and the lifetime test
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_dbg3; mkdir -p $O
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 200 $P tests/test_gpu_lifetime.py > $O/lifetime.txt 2>&1; echo "rc $?" >> $O/lifetime.txt
timeout -k 10 500 $P tests/test_gpu_c5.py tests/test_gpu_align.py tests/test_gpu_align_lm.py > $O/repro.txt 2>&1; echo "rc $?" >> $O/repro.txt
