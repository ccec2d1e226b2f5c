"""Seeded synthetic inputs shared by tests and bench.

Frames: splitmix64 rectangles + noise (ygzfe.synth_texture).  Align pairs:
renders of a textured plane Z = 3 m seen by the EuRoC camera under a known
small motion (ygzfe.render_plane), with map points back-projected onto the
plane.
"""
import numpy as np

import ygzfe

CONFIGS = {
    # name: (W, H, nfeatures, scale, levels, ini, min)  — BASELINE.json configs
    "C1": (640, 480, 500, 1.2, 8, 20, 7),
    "C2": (752, 480, 1000, 2.0, 4, 20, 7),
    "C4": (640, 480, 2000, 1.2, 8, 20, 7),
}

PLANE_Z = 3.0
TEXEL = 0.0065  # metres per texture pixel (~1 image pixel at Z=3 with fx=458)
TEX_W, TEX_H = 2048, 1536


def frame(seed, W, H):
    return ygzfe.synth_texture(seed, W, H)


def quat_from_rotvec(w):
    w = np.asarray(w, np.float64)
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.array([0, 0, 0, 1], np.float64)
    s = np.sin(th / 2) / th
    return np.array([w[0] * s, w[1] * s, w[2] * s, np.cos(th / 2)])


def quat_mul(a, b):
    x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1]
    y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2]
    z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0]
    w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2]
    return np.array([x, y, z, w])


def quat_rot(q, v):
    qv = q[:3]
    uv = 2 * np.cross(qv, v)
    return v + q[3] * uv + np.cross(qv, uv)


def se3_mul(qa, ta, qb, tb):
    return quat_mul(qa, qb), quat_rot(qa, tb) + ta


def se3_inv(q, t):
    qi = np.array([-q[0], -q[1], -q[2], q[3]])
    return qi, -quat_rot(qi, t)


def se3_log_inf(qa, ta, qb, tb):
    """|log(A^-1 B)|_inf (rotation vector + translation, small-motion form)."""
    qi, ti = se3_inv(np.asarray(qa, np.float64), np.asarray(ta, np.float64))
    q, t = se3_mul(qi, ti, np.asarray(qb, np.float64), np.asarray(tb, np.float64))
    if q[3] < 0:
        q = -q
    rv = 2 * q[:3]
    return float(max(np.abs(rv).max(), np.abs(t).max()))


class PlaneScene:
    """Textured plane at Z=PLANE_Z, EuRoC intrinsics, camera poses T_cw."""

    def __init__(self, seed=7, W=752, H=480):
        self.W, self.H = W, H
        self.tex = ygzfe.synth_texture(1000 + seed, TEX_W, TEX_H)
        self.cam = ygzfe.EUROC_CAM

    def render(self, q_cw, t_cw, noise_seed=0, noise_amp=2):
        return ygzfe.render_plane(self.tex, TEXEL, PLANE_Z, self.cam, q_cw, t_cw, self.W, self.H, noise_seed,
                                  noise_amp)

    def map_points(self, q_cw, t_cw, kps):
        """World points on the plane seen at the keypoints (level-0 px) from pose T_cw."""
        uv = np.stack([kps["x"], kps["y"]], 1) if len(kps) else np.zeros((0, 2), np.float32)
        return ygzfe.backproject_plane(self.cam, q_cw, t_cw, uv, PLANE_Z)

    def camera(self):
        return ygzfe.Camera(*self.cam)


def motion(seed, scale=1.0):
    """True relative motion delta = (0.02,-0.01,0.015 m; 0.005,-0.004,0.003 rad) + seeded jitter (§8d)."""
    rng = np.random.default_rng(seed)
    v = np.array([0.02, -0.01, 0.015]) * scale + rng.uniform(-0.003, 0.003, 3)
    w = np.array([0.005, -0.004, 0.003]) * scale + rng.uniform(-0.001, 0.001, 3)
    return v, w
