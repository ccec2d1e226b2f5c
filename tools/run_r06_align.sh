#!/bin/bash
# SparseImgAlign batch kernels A/B: k_sparse_align_reg (one pair per CU) vs k_sparse_align_x2
# (two pairs per CU), results compared record by record; then the align / C5 parity tests
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06_align}
mkdir -p $O
for r in 1 2; do
YGZFE_ALIGN_X2_MIN=1000000 timeout -k 10 180 python tools/mb_align.py --reps 10 --save $O/reg.npy > $O/mb_reg_$r.txt 2>&1
timeout -k 10 180 python tools/mb_align.py --reps 10 --save $O/x2.npy > $O/mb_x2_$r.txt 2>&1
done
python - <<'PY' > $O/cmp.txt 2>&1
import numpy as np, sys
O = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r06_align"
PY
python -c "
import numpy as np
a=np.load('$O/reg.npy'); b=np.load('$O/x2.npy')
na=a[:,7].copy().view(np.int32); nb=b[:,7].copy().view(np.int32)
print('pairs', len(a), 'n_visible equal', int((na==nb).sum()), 'max |dq|,|dt|', float(np.abs(a[:,:7]-b[:,:7]).max()))
" >> $O/cmp.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_align_batch.py tests/test_gpu_c5.py tests/test_gpu_align.py > $O/tests.txt 2>&1
