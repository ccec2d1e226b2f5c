"""Per-scene k_match_resolve timing (run under rocprofv3 --kernel-trace): each scene's
best search 20 times, in scene order; prints scene, queries, passes, re-scans."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ygzfe  # noqa: E402
import _scenes as S  # noqa: E402

for cfg, seed in (("C2", 0), ("C2", 1), ("C4", 2)):
    p = S.match_pair(cfg, seed)
    bnd = (0.0, float(p["W"]), 0.0, float(p["H"]))
    for th, lm in ((7.0, "mixed"), (15.0, "band"), (14.0, "none")):
        Q, qd, ur, bl = S.projection_queries(p, seed, th=th, level_mode=lm)
        cur = ygzfe.MatchFrame(0).set(p["k1"], p["d1"], ur, bnd)
        for _ in range(20):
            ygzfe.search_projection_best(cur, Q, qd, bl, 100, True)
        print(cfg, seed, th, lm, len(Q), cur.resolve_passes(), cur.rescans(), flush=True)
