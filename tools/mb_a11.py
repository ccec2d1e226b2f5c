"""Row a11 host-path breakdown: per-call wall time of MatchFrame.set and the two
SearchByProjection forms (the bench's tracking_searches line), for rocprofv3."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ygzfe  # noqa: E402
import _scenes as S  # noqa: E402

p = S.match_pair("C2", 0)
bnd = (0.0, float(p["W"]), 0.0, float(p["H"]))
Q1, qd1, ur, bl1 = S.projection_queries(p, 0, th=7.0, level_mode="mixed")
Q2, qd2, _, bl2 = S.projection_queries(p, 10, th=3.0 * 2.5, level_mode="band")
mf = ygzfe.MatchFrame(0)
t = {"set": [], "best": [], "ratio": []}
for it in range(60):
    t0 = time.perf_counter()
    cur = mf.set(p["k1"], p["d1"], ur, bnd)
    t1 = time.perf_counter()
    ygzfe.search_projection_best(cur, Q1, qd1, bl1, 100, True)
    t2 = time.perf_counter()
    ygzfe.search_projection_ratio(cur, Q2, qd2, bl2, 0.8)
    t3 = time.perf_counter()
    if it >= 10:
        t["set"].append(t1 - t0)
        t["best"].append(t2 - t1)
        t["ratio"].append(t3 - t2)
print({k: round(float(np.median(v)) * 1e3, 4) for k, v in t.items()})
