"""Batch extraction of B bench-shaped C2 frames (resident), repeated: the command
that rocprofv3 PMC passes wrap (tools/run_pmc_cmd.sh TAG tools/mb_extract.py B reps)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import ygzfe  # noqa: E402
import _scenes as S  # noqa: E402
from bench import sweep_index  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
sc = S.PlaneScene(11, W, H)
xi = np.array([0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015], np.float32)
frames = np.stack([sc.render(*ygzfe.trajectory_pose(sweep_index(i), xi), noise_seed=i) for i in range(B)])
b = ygzfe.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, B)
b.upload(frames)
for _ in range(reps):
    b.extract(B)
b.check()
print("ok", B, reps)
