#!/bin/bash
# the hipGraphLaunch crash repro after taking the octree fork out of the extract graph
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_dbg7; mkdir -p $O
export YGZFE_SEGV_TRACE=$PWD/tools/segv/libsegv_trace.so
P="python -u -m pytest -s -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 500 $P tests/test_gpu_c5.py tests/test_gpu_align.py tests/test_gpu_align_lm.py tests/test_gpu_extract.py > $O/repro.txt 2>&1; echo "rc $?" >> $O/repro.txt
