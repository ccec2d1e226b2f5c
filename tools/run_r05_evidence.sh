#!/bin/bash
# Round-5 closing evidence on one box: the GPU suite in the driver's order, smoke, the default bench
# line, drop-in timing, rocprof summaries (pipe = the bench's schedule; serial = the roofline's
# kernel-alone durations over the same chunk batches) and the PMC passes
set -e
bash tools/run_r05_final.sh ${1:-r05ev}
bash tools/run_r05_prof_serial.sh ${1:-r05ev}/serial
