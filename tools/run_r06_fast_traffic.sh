#!/bin/bash
# FAST alone (tools/mb_fast.py stage 0, 1,024 C2 frames): FETCH_SIZE / WRITE_SIZE per launch with the
# product's 23,000-B LDS floor per workgroup and without it (libygzfe_f0.so), plus the stage times
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_fast_traffic}
mkdir -p $O
R="rocprofv3 --output-format csv --kernel-include-regex k_fast_"
for lib in libygzfe.so ${LIBS:-libygzfe_f0.so}; do
B="python3 tools/mb_fast.py --child 1024 $PWD/orb-ygz-slam_amd/lib/$lib"
YGZ_MB_STAGES=0 timeout -s KILL 120 $R --pmc FETCH_SIZE -d $O/$lib/fetch -o run -- $B > $O/$lib.fetch.log 2>&1
YGZ_MB_STAGES=0 timeout -s KILL 120 $R --pmc WRITE_SIZE -d $O/$lib/write -o run -- $B > $O/$lib.write.log 2>&1
YGZ_MB_STAGES=0 timeout -k 10 120 python tools/mb_fast.py 1024 $PWD/orb-ygz-slam_amd/lib/$lib > $O/$lib.mb.txt 2>&1
done
