set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/b.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 150 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/pq/p3 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/pq.log 2>&1
