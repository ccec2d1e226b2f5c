#!/bin/bash
# Round-5 evidence run: the GPU suite in the driver's order, smoke, the default bench line,
# drop-in call-site timing, a rocprofv3 kernel summary of a short bench, PMC passes for the
# traffic figures (tools/run_pmc.sh -> tools/pmc_traffic.py)
set -e
O=gpurun_out/${1:-r05final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
bash tools/run_dropin_time.sh ${1:-r05final}/dropin
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 --latency-frames 0 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-a11 --no-dropin > $O/prof_bench.json 2> $O/prof_bench.err
python tools/prof_summary.py $(find $O/prof -name '*kernel_stats.csv') > $O/kernel_summary.txt 2>&1 || true
bash tools/run_pmc.sh ${1:-r05final}
