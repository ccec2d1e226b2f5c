"""The synthetic scene of the offline sequence mode: a textured plane
Z_w = PLANE_Z seen by the EuRoC camera (EuRoC.yaml:8-11), rendered on the device
(ygzfe.render_plane / render_plane_device), with the pose algebra its map points use.

The datasets are not available, so C5Shard (sequence.py) renders its frames from this
scene; the tests (tests/_scenes.py) build their align / match / direct inputs on it too.
"""
import numpy as np

PLANE_Z = 3.0
TEXEL = 0.0065  # metres per texture pixel (~1 image pixel at Z = 3 with fx = 458)
TEX_W, TEX_H = 2048, 1536


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


class PlaneScene:
    """Textured plane at Z = PLANE_Z, EuRoC intrinsics, camera poses T_cw."""

    def __init__(self, seed=7, W=752, H=480):
        from . import synth_texture, EUROC_CAM
        self.W, self.H = W, H
        self.tex = synth_texture(1000 + seed, TEX_W, TEX_H)
        self.cam = EUROC_CAM

    def render(self, q_cw, t_cw, noise_seed=0, noise_amp=2):
        from . import render_plane
        return render_plane(self.tex, TEXEL, PLANE_Z, self.cam, q_cw, t_cw, self.W, self.H, noise_seed, noise_amp)

    def map_points(self, q_cw, t_cw, kps):
        """World points on the plane seen at the keypoints (level-0 px) from pose T_cw."""
        from . import backproject_plane
        uv = np.stack([kps["x"], kps["y"]], 1) if len(kps) else np.zeros((0, 2), np.float32)
        return backproject_plane(self.cam, q_cw, t_cw, uv, PLANE_Z)

    def camera(self):
        from . import Camera
        return Camera(*self.cam)
