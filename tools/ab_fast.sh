#!/bin/bash
# FAST A/B on the GPU box: strips (default) vs the per-cell kernel (YGZFE_FAST_CELLS=1),
# alternating runs of tools/mb_fast.py (1024 bench frames, ms per 1024 frames).
out=${1:-gpurun_out/ab_fast}
mkdir -p "$out"
for i in 1 2; do
  timeout -k 10 200 python tools/mb_fast.py 1024 libygzfe.so >> "$out/strips.txt" 2>/dev/null || exit 1
  YGZFE_FAST_CELLS=1 timeout -k 10 200 python tools/mb_fast.py 1024 libygzfe.so >> "$out/cells.txt" 2>/dev/null || exit 1
done
