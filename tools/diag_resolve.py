"""k_match_resolve diagnostics: passes taken / hand-over per pass budget, and the serial
replay's re-scan count, on the test scenes."""
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
        row = []
        for b in ("0", "8", "32", "128", "1024", "4096"):
            os.environ["YGZFE_MATCH_PASSES"] = b
            r, n = ygzfe.search_projection_best(cur, Q, qd, bl, 100, True)
            row.append((b, cur.resolve_passes(), cur.rescans(), n))
        print(cfg, seed, th, lm, len(Q), row, flush=True)
