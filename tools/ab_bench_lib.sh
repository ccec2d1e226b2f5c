#!/bin/bash
# A/B of library builds on the bench's C5 step (headline legs only): tools/ab_bench_lib.sh OUT lib1.so lib2.so ...
# (extra bench arguments in $BENCH_ARGS, e.g. "--schedule pipe --chunks 4")
out=$1; shift
mkdir -p $out
for lib in "$@" "$@"; do
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 \
    --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin $BENCH_ARGS \
    >> $out/$(basename $lib .so).jsonl 2>> $out/err.log || exit 1
done
