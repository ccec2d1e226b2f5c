#!/bin/bash
# A/B timing of library variants (YGZFE_LIB) on the C2 batch bench; stops at
# the first run that ends other than by a clean exit or a Python error.
O=gpurun_out/${1:-variants}
shift
mkdir -p $O
for v in "$@"; do
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$v timeout -k 10 150 python bench.py --workload c2batch --steps 10 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-c4 --no-undistort --no-bow --no-stereo --no-direct > $O/$v.json 2> $O/$v.err
  rc=$?
  echo "$v rc=$rc" >> $O/rc.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
