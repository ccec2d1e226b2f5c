#!/bin/bash
# Per-kernel FAST times (rocprofv3 --kernel-trace --stats) of library variants on the
# bench frames: tools/prof_fast_variants.sh OUTDIR lib1.so [lib2.so ...]
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for lib in "$@"; do
  n=$(basename "$lib" .so)
  YGZ_MB_STAGES=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$n" -o run \
    -- python tools/mb_fast.py 1024 "$lib" > "$out/$n.log" 2>&1 || exit 1
done
