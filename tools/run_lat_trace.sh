set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lat
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d gpurun_out/lat/tr -o run -- python3 bench.py --frames 512 --steps 2 --warmup 1 --cpu-sample 0 --latency-frames 60 --no-direct --no-stereo --no-bow --no-undistort --no-c4 --no-stage-timing > gpurun_out/lat/bench.json 2> gpurun_out/lat/bench.err
