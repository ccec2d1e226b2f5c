#!/bin/bash
# Round-6 evidence on one box: the GPU suite, smoke, the default bench line, drop-in call-site
# timing, rocprofv3 kernel summaries of the bench's command (pipe = the bench's schedule; serial =
# the roofline's kernel-alone durations over the same chunk batches) and the PMC passes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06ev}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
bash tools/run_dropin_time.sh ${1:-r06ev}/dropin
A="--steps 5 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py $A > $O/prof_bench.json 2> $O/prof_bench.err
python tools/prof_summary.py $(find $O/prof -name '*kernel_stats.csv') > $O/kernel_summary_pipe.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profs -o run -- python bench.py --schedule serial --chunks 4 $A > $O/prof_serial_bench.json 2> $O/prof_serial_bench.err
python tools/prof_summary.py $(find $O/profs -name '*kernel_stats.csv') > $O/kernel_summary.txt 2>&1 || true
bash tools/run_pmc.sh ${1:-r06ev}
