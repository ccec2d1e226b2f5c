"""Phase breakdown of k_sparse_align_reg from the diagnostic build's s_memtime stamps.
Runs one C3 pair through lib/libygzfe_diag.so (make -C orb-ygz-slam_amd diag)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ygzfe  # noqa: E402

ygzfe.LIB_PATH = os.path.join(ROOT, "orb-ygz-slam_amd", "lib", "libygzfe_diag.so")
import numpy as np  # noqa: E402
import _scenes as S  # noqa: E402

sc = S.PlaneScene(0)
ex = ygzfe.ORBextractor(1000, 2.0, 4, 20, 7)
q_ref = S.quat_from_rotvec([0.01, -0.02, 0.005]).astype(np.float32)
t_ref = np.array([0.05, -0.03, 0.02], np.float32)
v, w = S.motion(0)
q_cur, t_cur = S.se3_mul(S.quat_from_rotvec(w), v, q_ref.astype(np.float64), t_ref.astype(np.float64))
fr = ex.ComputePyramid(sc.render(q_ref, t_ref, 1))
fc = ex.ComputePyramid(sc.render(q_cur.astype(np.float32), t_cur.astype(np.float32), 2))
kps, _ = ex.extract(fr)
Pw, ok = sc.map_points(q_ref, t_ref, kps)
xyz = np.array([S.quat_rot(q_ref.astype(np.float64), p) + t_ref for p in Pw], np.float32)
al = ygzfe.SparseImgAlign(3, 1)
buf = (C.c_ulonglong * 4096)()
for rep in range(3):
    ygzfe.lib().ygzfe_diag_stamps(buf, 4096)
    res = al.run(fr, fc, sc.camera(), kps, xyz, ok, ygzfe.SE3.make())
    n = ygzfe.lib().ygzfe_diag_stamps(buf, 4096)
st = sorted([(buf[2 * i], buf[2 * i + 1]) for i in range(n)], key=lambda x: x[1])
names = {9: "start", 1: "L0 (level H in)", 2: "L0b + inverse", 3: "A passed (solver)", 4: "B passed",
         5: "L1", 6: "partials reduced", 7: "chi2 read", 8: "x solved", 10: "exp+mul done",
         11: "w1 residual start", 12: "w1 residual done", 13: "w15 residual done"}
print("n_features", len(kps), "n_visible", res.n_visible, "stamps", n, "total cycles", st[-1][1] - st[0][1])
tot, cnt = {}, {}
for (a, ta), (b, tb) in zip(st, st[1:]):
    k = (a, b)
    tot[k] = tot.get(k, 0) + (tb - ta)
    cnt[k] = cnt.get(k, 0) + 1
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {names.get(k[0], k[0]):20s} -> {names.get(k[1], k[1]):20s}: {v:8d} cycles over {cnt[k]:3d}  ({v / cnt[k]:.0f} each)")
