#!/bin/bash
# the default bench line and the serial-schedule rocprof summary of the same command on one box
# (so the roofline's HIP-event launch average and the rocprof average come from the same GPU)
set -e
O=gpurun_out/${1:-r05bp}
mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
bash tools/run_r05_prof_serial.sh ${1:-r05bp}
