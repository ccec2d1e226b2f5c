#!/bin/bash
# Round-4 evidence run: parity suite, smoke, bench line, rocprofv3 kernel summary of a
# short bench, PMC passes (tools/run_pmc.sh) for profiles/r04_traffic.json
set -e
O=gpurun_out/${1:-r04final}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 5 --warmup 2 > $O/prof_bench.json 2> $O/prof_bench.err
python tools/prof_summary.py $(find $O/prof -name '*kernel_stats.csv') > $O/kernel_summary.txt 2>&1 || true
bash tools/run_pmc.sh ${1:-r04final}
# diagnostics: SparseImgAlign solver-wave stamps, octree block timeline (diag builds)
timeout -k 10 200 python tools/mb_align.py --diag --reps 3 > $O/mb_align_diag.txt 2>&1
STAMPK=3 YGZ_DIAG_LIB=$PWD/orb-ygz-slam_amd/lib/libygzfe_diag3.so timeout -k 10 200 python tools/diag_blocks.py 1024 > $O/diag_oct.txt 2>&1
