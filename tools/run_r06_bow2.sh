#!/bin/bash
# k_bow_vectors as two workgroups per frame (BowVector | FeatureVector) with the folded values
# kept in LDS: parity, single-frame kernel profile, bench BoW leg + drop-in timing
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_bow2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bow.py tests/test_gpu_dropin.py > $O/tests.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/mb_bow_single.py 200 > $O/mb.txt 2>&1
python3 tools/prof_summary.py $(find $O/p -name "*kernel_stats.csv") > $O/summary.txt
A="--steps 2 --warmup 1 --cpu-sample 1 --latency-frames 0 --no-direct --no-stereo --no-undistort --no-c4 --no-a11"
timeout -k 10 400 python bench.py $A > $O/bench.json 2> $O/bench.err
