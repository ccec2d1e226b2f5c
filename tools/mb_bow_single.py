"""Single-frame DBoW2 calls through the host C ABI, for a rocprofv3 kernel trace:
python tools/mb_bow_single.py [reps] -- the bench's synthetic k=10 L=6 vocabulary and one
936-descriptor frame (random bits), `reps` transform_each / transform calls, host ms printed."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ygzfe  # noqa: E402
import _vocab as V  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
parent, is_leaf, desc, weight = V.synth_vocab(6, 10, 6)
voc = ygzfe.Vocabulary.from_arrays(10, 6, 0, 0, parent, is_leaf, desc, weight, device=0)
d0 = np.random.default_rng(1).integers(0, 256, (936, 32), dtype=np.uint8)
for name, fn in (("transform_each", voc.transform_each), ("transform", voc.transform)):
    for _ in range(5):
        fn(d0, 4)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn(d0, 4)
        ts.append(time.perf_counter() - t)
    print(f"{name}: median {np.median(ts) * 1e3:.4f} ms over {reps}", flush=True)
