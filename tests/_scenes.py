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

# the plane, its texture scale and the pose algebra live in the package (ygzfe.scene:
# the sequence mode renders from them); re-exported for the tests
from ygzfe.scene import PLANE_Z, TEXEL, TEX_W, TEX_H, PlaneScene, quat_mul, quat_rot, se3_inv, se3_mul  # noqa: F401,E402


def frame(seed, W, H):
    return ygzfe.synth_texture(seed, W, H)


def quat_from_rotvec(w):
    w = np.asarray(w, np.float64)
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.array([0, 0, 0, 1], np.float64)
    s = np.sin(th / 2) / th
    return np.array([w[0] * s, w[1] * s, w[2] * s, np.cos(th / 2)])


def se3_log_inf(qa, ta, qb, tb):
    """|log(A^-1 B)|_inf (rotation vector + translation, small-motion form)."""
    qi, ti = se3_inv(np.asarray(qa, np.float64), np.asarray(ta, np.float64))
    q, t = se3_mul(qi, ti, np.asarray(qb, np.float64), np.asarray(tb, np.float64))
    if q[3] < 0:
        q = -q
    rv = 2 * q[:3]
    return float(max(np.abs(rv).max(), np.abs(t).max()))


def world_to_cam(pose, Pw):
    """xyz_ref = T_cw * P_w (the SparseImgAlign map-point snapshot), float32 [n, 3]."""
    q, t = (np.asarray(a, np.float64) for a in pose)
    Pw = np.asarray(Pw, np.float64).reshape(-1, 3)
    return np.array([quat_rot(q, p) + t for p in Pw], np.float32).reshape(-1, 3)


def motion(seed, scale=1.0):
    """True relative motion delta = (0.02,-0.01,0.015 m; 0.005,-0.004,0.003 rad) + seeded jitter (§8d)."""
    rng = np.random.default_rng(seed)
    v = np.array([0.02, -0.01, 0.015]) * scale + rng.uniform(-0.003, 0.003, 3)
    w = np.array([0.005, -0.004, 0.003]) * scale + rng.uniform(-0.001, 0.001, 3)
    return v, w


def project(cam, q_cw, t_cw, Pw):
    """Level-0 pixel of world points under T_cw (pinhole, Frame::World2Pixel)."""
    Pc = np.array([quat_rot(q_cw, p) + t_cw for p in Pw]).reshape(-1, 3)
    fx, fy, cx, cy = cam
    return np.stack([fx * Pc[:, 0] / Pc[:, 2] + cx, fy * Pc[:, 1] / Pc[:, 2] + cy], 1), Pc


def direct_scene(seed, n_kf=4, max_obs=5, W=752, H=480, nlevels=4, scale_factor=2.0, n_points=None, cluster=0):
    """SearchLocalPointsDirect inputs (Tracking.cc:2258-2410) on the textured plane.

    n_kf keyframes around the origin and a current frame moved by motion(seed).
    Map points = plane points under keyframe 0's pixel grid; each point is observed
    by a random ordered subset (0..max_obs) of the keyframes, its keypoint there =
    the point's projection with a random octave.  px_proj = the projection into the
    current frame + U(-1.5, 1.5) px (isInFrustum's prediction).  cluster = k adds k
    neighbours within +-1.2 px after every grid point (consecutive points then share
    cells of SearchLocalPointsDirect's 5-px coverage grid).  Returns a dict of
    images, poses and the CSR item arrays of ygzfe.search_direct_batch."""
    rng = np.random.default_rng(1000 + seed)
    sc = PlaneScene(seed, W, H)
    poses = []
    for k in range(n_kf):
        q = quat_from_rotvec(rng.uniform(-0.01, 0.01, 3))
        t = rng.uniform(-0.04, 0.04, 3)
        poses.append((q, t))
    v, w = motion(seed)
    qc, tc = se3_mul(quat_from_rotvec(w), v, *poses[0])
    imgs = [sc.render(q.astype(np.float32), t.astype(np.float32), seed * 16 + k) for k, (q, t) in enumerate(poses)]
    cur = sc.render(qc.astype(np.float32), tc.astype(np.float32), seed * 16 + 15)
    # map points: a jittered pixel grid of keyframe 0, reaching the image edges (border rejections)
    gx, gy = np.meshgrid(np.arange(6, W - 6, 22), np.arange(6, H - 6, 22))
    uv = np.stack([gx.ravel(), gy.ravel()], 1).astype(np.float64) + rng.uniform(-3, 3, (gx.size, 2))
    if n_points is not None:
        uv = uv[rng.permutation(len(uv))[:n_points]]
    if cluster:
        uv = np.concatenate([uv[:, None, :], uv[:, None, :] + rng.uniform(-1.2, 1.2, (len(uv), cluster, 2))],
                            1).reshape(-1, 2)
    Pw = backproject_plane_np(sc.cam, poses[0], uv)
    n = len(Pw)
    px_cur, _ = project(sc.cam, qc, tc, Pw)
    px_proj = (px_cur + rng.uniform(-1.5, 1.5, px_cur.shape)).astype(np.float32)
    item_ptr = [0]
    ref_index, kps, pt_ref, T_cr = [], [], [], []
    for i in range(n):
        m = int(rng.integers(0, max_obs + 1))
        for k in rng.permutation(n_kf)[:min(m, n_kf)]:
            q, t = poses[k]
            px_k, Pc = project(sc.cam, q, t, Pw[i:i + 1])
            kp = np.zeros(1, ygzfe.KP_DTYPE)
            kp["x"], kp["y"] = px_k[0]
            kp["octave"] = int(rng.integers(0, nlevels))
            kp["size"] = 31.0 * scale_factor ** kp["octave"][0]
            kp["angle"] = -1.0
            qi, ti = se3_inv(q, t)
            qcr, tcr = se3_mul(qc, tc, qi, ti)
            T = np.zeros(1, ygzfe.SE3_DTYPE)
            T["q"] = qcr
            T["t"] = tcr
            ref_index.append(k)
            kps.append(kp)
            pt_ref.append(Pc[0])
            T_cr.append(T)
        item_ptr.append(len(ref_index))
    cat = lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dt)  # noqa: E731
    return {"scene": sc, "kf_images": imgs, "cur_image": cur, "poses": poses, "cur_pose": (qc, tc),
            "item_ptr": np.array(item_ptr, np.int32), "ref_index": np.array(ref_index, np.int32),
            "kps": cat(kps, ygzfe.KP_DTYPE), "pt_ref": np.array(pt_ref, np.float32).reshape(-1, 3),
            "T_cr": cat(T_cr, ygzfe.SE3_DTYPE), "px_proj": px_proj, "Pw": Pw}


def backproject_plane_np(cam, pose, uv):
    """World points on Z_w = PLANE_Z seen at level-0 pixels uv from pose T_cw (float64)."""
    q, t = pose
    qi, ti = se3_inv(q, t)
    fx, fy, cx, cy = cam
    d = np.stack([(uv[:, 0] - cx) / fx, (uv[:, 1] - cy) / fy, np.ones(len(uv))], 1)
    dw = np.array([quat_rot(qi, x) for x in d])
    lam = (PLANE_Z - ti[2]) / dw[:, 2]
    return ti + dw * lam[:, None]


EUROC_BASELINE = 0.110073  # m, EuRoC cam0-cam1 (Examples/Stereo/EuRoC.yaml: Camera.bf / fx)


def stereo_scene(seed, W=752, H=480, baseline=EUROC_BASELINE):
    """A rectified stereo pair of the textured plane: the right camera is the left one
    shifted by `baseline` along its x axis (X_r = X_l - b), so disparity = fx * b / Z."""
    sc = PlaneScene(seed, W, H)
    rng = np.random.default_rng(500 + seed)
    q = quat_from_rotvec(rng.uniform(-0.15, 0.15, 3))  # tilted plane: depth varies over the image
    t = rng.uniform(-0.2, 0.2, 3)
    left = sc.render(q.astype(np.float32), t.astype(np.float32), seed * 2 + 1)
    right = sc.render(q.astype(np.float32), (t - np.array([baseline, 0, 0])).astype(np.float32), seed * 2 + 2)
    fx = sc.cam[0]
    return {"scene": sc, "left": left, "right": right, "pose": (q, t), "mb": float(baseline),
            "mbf": float(np.float32(baseline) * np.float32(fx))}


# ---------------------------------------------------------------- ORBmatcher search inputs
def _oracle_extract(cfg, img):
    import _oracle as O
    W, H, nf, sf, nl, ini, mn = CONFIGS[cfg]
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    return orc.extract(orc.pyramid(img)), orc


def match_pair(cfg="C2", seed=0, motion_scale=1.0):
    """Two rendered frames of the textured plane (frame 1 moved by motion(seed)) with their
    keypoints / descriptors (oracle extraction, identical to the GPU's) and the map points of
    frame 0's keypoints on the plane."""
    W, H = CONFIGS[cfg][:2]
    sc = PlaneScene(seed, W, H)
    q0, t0 = np.array([0, 0, 0, 1.0]), np.zeros(3)
    v, w = motion(seed, motion_scale)
    q1, t1 = quat_from_rotvec(w), v
    f0 = sc.render(q0.astype(np.float32), t0.astype(np.float32), 3 * seed + 1)
    f1 = sc.render(q1.astype(np.float32), t1.astype(np.float32), 3 * seed + 2)
    (k0, d0), orc = _oracle_extract(cfg, f0)
    (k1, d1), _ = _oracle_extract(cfg, f1)
    uv0 = np.stack([k0["x"], k0["y"]], 1).astype(np.float64)
    Pw = backproject_plane_np(sc.cam, (q0, t0), uv0)
    return {"cfg": cfg, "W": W, "H": H, "sc": sc, "poses": ((q0, t0), (q1, t1)), "k0": k0, "d0": d0, "k1": k1,
            "d1": d1, "Pw": Pw, "scale": orc.scale}


def projection_queries(p, seed, th=7.0, level_mode="mixed", blocks_frac=0.8, stereo_frac=0.3, valid_frac=0.9,
                       noise=1.0, flip_bits=8):
    """SearchByProjection(CurrentFrame, LastFrame, ...) queries: frame 0's map points projected into
    frame 1 (+ noise), radius th * mvScaleFactors[octave], a level window per `level_mode`
    (ORBmatcher.cc:1272-1279), the MapPoint descriptor = frame 0's descriptor with a few bits
    flipped, random VALID / BLOCKS / STEREO flags.  Returns (queries, q_desc, u_right of frame 1,
    train_blocked)."""
    import ygzfe
    rng = np.random.default_rng(7000 + seed)
    (q1, t1) = p["poses"][1]
    px, Pc = project(p["sc"].cam, q1, t1, p["Pw"])
    n = len(px)
    Q = np.zeros(n, ygzfe.MATCH_QUERY_DTYPE)
    Q["u"] = px[:, 0] + rng.uniform(-noise, noise, n)
    Q["v"] = px[:, 1] + rng.uniform(-noise, noise, n)
    oct_ = p["k0"]["octave"]
    Q["radius"] = (np.float32(th) * p["scale"][oct_]).astype(np.float32)
    mode = rng.integers(0, 4, n) if level_mode == "mixed" else np.full(n, {"none": 0, "fwd": 1, "bwd": 2, "band": 3}[level_mode])
    Q["min_level"] = np.where(mode == 0, -1, np.where(mode == 1, oct_, np.where(mode == 2, 0, oct_ - 1)))
    Q["max_level"] = np.where(mode == 0, -1, np.where(mode == 1, -1, np.where(mode == 2, oct_, oct_ + 1)))
    Q["angle"] = p["k0"]["angle"]
    fx = p["sc"].cam[0]
    Q["u_right"] = Q["u"] - np.float32(fx * 0.11) / Pc[:, 2].astype(np.float32)
    inside = (Q["u"] >= 0) & (Q["u"] <= p["W"]) & (Q["v"] >= 0) & (Q["v"] <= p["H"])
    flags = np.where(inside & (rng.random(n) < valid_frac), ygzfe.MQ_VALID, 0)
    flags |= np.where(rng.random(n) < blocks_frac, ygzfe.MQ_BLOCKS, 0)
    flags |= np.where(rng.random(n) < stereo_frac, ygzfe.MQ_STEREO, 0)
    Q["flags"] = flags
    qd = p["d0"].copy()
    for i in range(n):  # MapPoint::GetDescriptor() != the keypoint's: a few bits apart
        for b in rng.integers(0, 256, rng.integers(0, flip_bits + 1)):
            qd[i, b // 8] ^= np.uint8(1 << (b % 8))
    n1 = len(p["k1"])
    ur = np.where(rng.random(n1) < 0.5, p["k1"]["x"] - rng.uniform(5, 60, n1), -1.0).astype(np.float32)
    blocked = (rng.random(n1) < 0.1).astype(np.uint8)
    return Q, qd, ur, blocked


def feature_vector(desc, n_nodes, seed):
    """A DBoW2-like FeatureVector: node of each feature from its descriptor bits (node-sorted CSR)."""
    node = (desc[:, 0].astype(np.int64) * 131 + desc[:, 5] + seed) % n_nodes
    order = np.argsort(node, kind="stable")
    nodes, counts = np.unique(node[order], return_counts=True)
    ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    return nodes.astype(np.int32) * 7 + 3, ptr, order.astype(np.int32)
