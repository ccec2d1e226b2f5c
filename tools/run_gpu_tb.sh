set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/b.log 2>&1
