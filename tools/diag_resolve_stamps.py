"""s_memrealtime stamps inside k_match_resolve (make diag STAMPK=5): entry, after the
prologue, after pass 1, after the pass loop, exit — per scene, µs."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ygzfe  # noqa: E402

ygzfe.LIB_PATH = os.path.join(ROOT, "orb-ygz-slam_amd", "lib", "libygzfe_diag.so")
import _scenes as S  # noqa: E402

L = ygzfe.lib()
buf = np.zeros(8, np.uint64)  # slots: 0 entry, 1 prologue, 3 pass 1, 4 loop, 5 exit, 6/7 pass 2
for cfg, seed in (("C2", 0), ("C2", 1), ("C4", 2)):
    p = S.match_pair(cfg, seed)
    bnd = (0.0, float(p["W"]), 0.0, float(p["H"]))
    for th, lm in ((7.0, "mixed"), (15.0, "band"), (14.0, "none")):
        Q, qd, ur, bl = S.projection_queries(p, seed, th=th, level_mode=lm)
        cur = ygzfe.MatchFrame(0).set(p["k1"], p["d1"], ur, bnd)
        rows = []
        for _ in range(5):
            ygzfe.search_projection_best(cur, Q, qd, bl, 100, True)
            L.ygzfe_diag_match_stamps(buf.ctypes.data_as(C.c_void_p), 8)
            t = buf.astype(np.int64)
            rows.append([(t[1] - t[0]) / 100, (t[3] - t[1]) / 100, (t[4] - t[1]) / 100, (t[5] - t[4]) / 100,
                         (t[6] - t[3]) / 100, (t[7] - t[6]) / 100])
        med = np.median(np.array(rows), 0)
        print(cfg, seed, th, lm, "passes", cur.resolve_passes(),
              "prologue %.2f pass1 %.2f loop %.2f epilogue %.2f | pass2 link %.2f decide %.2f" % tuple(med), flush=True)
