#!/bin/bash
# Hamming PMC: MFMA busy, VALU / LDS instructions, waits (one rocprofv3 pass per lib)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_hampmc}
mkdir -p $O
for lib in libygzfe.so libygzfe_h18p1.so; do
  YGZFE_LIB=$PWD/orb-ygz-slam_amd/lib/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA -d $O/${lib%.so} -o pmc --output-format csv -- python3 tools/mb_hamming.py --n 936 --reps 5 > $O/${lib%.so}.txt 2>&1
done
