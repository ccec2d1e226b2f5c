"""GPU direct alignment vs the oracle.

SparseImgAlign::run (SparseImageAlign.cc:20-49): pose within 1e-4 (|log(T_gpu^-1 T_cpu)|_inf).
Align2D (Align.cc:8-105) and FindDirectProjection (ORBmatcher.cc:1573-1602): bit-exact.
"""
import numpy as np
import pytest

import _oracle as O
import _scenes as S

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-4


def align_case(gpu, seed, n_usable_frac=1.0, max_level=3, min_level=1, motion_scale=1.0, method=0, nfeatures=None):
    sc = S.PlaneScene(seed)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    nf = nfeatures or nf
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    # reference camera at a generic pose, current = ref moved by the true motion
    q_ref = S.quat_from_rotvec([0.01, -0.02, 0.005]).astype(np.float32)
    t_ref = np.array([0.05, -0.03, 0.02], np.float32)
    v, w = S.motion(seed, motion_scale)
    q_d = S.quat_from_rotvec(w)
    q_cur, t_cur = S.se3_mul(q_d, v, q_ref.astype(np.float64), t_ref.astype(np.float64))
    f_ref = sc.render(q_ref, t_ref, seed * 2 + 1)
    f_cur = sc.render(q_cur.astype(np.float32), t_cur.astype(np.float32), seed * 2 + 2)
    fr_ref, fr_cur = ex.ComputePyramid(f_ref), ex.ComputePyramid(f_cur)
    kps, _ = ex.extract(fr_ref)
    Pw, ok = sc.map_points(q_ref, t_ref, kps)
    xyz = np.array([S.quat_rot(q_ref.astype(np.float64), p) + t_ref for p in Pw], np.float32)
    rng = np.random.default_rng(seed)
    usable = (ok.astype(bool) & (rng.random(len(kps)) < n_usable_frac)).astype(np.uint8)
    T0 = gpu.SE3.make()
    cam = sc.camera()
    res = gpu.SparseImgAlign(max_level, min_level, method=method).run(fr_ref, fr_cur, cam, kps, xyz, usable, T0)
    ocam = O.Cam(*sc.cam)
    oT0 = O.se3_from((0, 0, 0, 1), (0, 0, 0))
    ores = O.sparse_align(orc.pyramid(f_ref), orc.pyramid(f_cur), orc.inv_scale, ocam, kps, xyz, usable, max_level,
                          min_level, oT0, method=method)
    true_q, true_t = q_d, v
    return res, ores, (true_q, true_t)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_sparse_align_pose_parity(gpu, seed):
    res, ores, (tq, tt) = align_case(gpu, seed)
    gq, gt = res.T_cur_ref.as_arrays()
    oq, ot = np.array(ores.T.q[:]), np.array(ores.T.t[:])
    err = S.se3_log_inf(gq, gt, oq, ot)
    assert err <= POSE_TOL, f"GPU vs CPU pose differ by {err}"
    assert res.n_visible == ores.n_visible and res.n_visible > 100
    # the solver actually recovers the synthetic motion
    assert S.se3_log_inf(gq, gt, tq, tt) < 5e-3


def test_sparse_align_partial_usable(gpu):
    res, ores, _ = align_case(gpu, 5, n_usable_frac=0.3)
    gq, gt = res.T_cur_ref.as_arrays()
    assert S.se3_log_inf(gq, gt, np.array(ores.T.q[:]), np.array(ores.T.t[:])) <= POSE_TOL
    assert res.n_visible == ores.n_visible


def test_sparse_align_no_usable(gpu):
    """No usable map point: GN on an empty system keeps the initial pose."""
    res, ores, _ = align_case(gpu, 6, n_usable_frac=0.0)
    gq, gt = res.T_cur_ref.as_arrays()
    assert res.n_visible == 0 and ores.n_visible == 0
    assert S.se3_log_inf(gq, gt, np.array(ores.T.q[:]), np.array(ores.T.t[:])) <= POSE_TOL


def test_sparse_align_single_level(gpu):
    res, ores, _ = align_case(gpu, 7, max_level=2, min_level=2)
    gq, gt = res.T_cur_ref.as_arrays()
    assert S.se3_log_inf(gq, gt, np.array(ores.T.q[:]), np.array(ores.T.t[:])) <= POSE_TOL


def patches_around(img, pts, rng):
    H, W = img.shape
    pwb = np.zeros((len(pts), 100), np.uint8)
    p = np.zeros((len(pts), 64), np.uint8)
    for i, (x, y) in enumerate(pts):
        x, y = int(x), int(y)
        blk = img[y - 5:y + 5, x - 5:x + 5].astype(np.int32)
        blk = np.clip(blk + rng.integers(-2, 3, blk.shape), 0, 255).astype(np.uint8)
        pwb[i] = blk.reshape(-1)
        p[i] = blk[1:9, 1:9].reshape(-1)
    return pwb, p


def test_align2d_bitexact(gpu):
    W, H = 752, 480
    img = S.frame(9, W, H)
    ex = gpu.ORBextractor(1000, 2.0, 4, 20, 7)
    fr = ex.ComputePyramid(img)
    rng = np.random.default_rng(0)
    pts = np.stack([rng.integers(20, W - 20, 500), rng.integers(20, H - 20, 500)], 1)
    pwb, p = patches_around(img, pts, rng)
    guess = (pts + rng.uniform(-2.5, 2.5, pts.shape)).astype(np.float32)
    # include out-of-bounds guesses (the loop breaks without converging)
    guess[:5] = [[1, 1], [W - 2, 100], [100, H - 1], [-10, 5], [400, 2]]
    conv, px = gpu.align2d_batch(fr, 0, pwb, p, guess)
    for i in range(len(pts)):
        ok, q = O.align2d(img, pwb[i], p[i], guess[i])
        assert ok == conv[i], i
        assert np.array_equal(q, px[i]), (i, q, px[i])
    assert conv.mean() > 0.5


def test_find_direct_projection_bitexact(gpu):
    sc = S.PlaneScene(4)
    W, H, nf, sf, nl, ini, mn = (640, 480, 500, 1.2, 8, 20, 7)
    sc.W, sc.H = W, H
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    q_kf, t_kf = np.array([0, 0, 0, 1], np.float32), np.zeros(3, np.float32)
    v, w = S.motion(1, 2.0)
    q_c = S.quat_from_rotvec(w).astype(np.float32)
    t_c = v.astype(np.float32)
    f_kf, f_c = sc.render(q_kf, t_kf, 1), sc.render(q_c, t_c, 2)
    fr_kf, fr_c = ex.ComputePyramid(f_kf), ex.ComputePyramid(f_c)
    kps, _ = ex.extract(fr_kf)
    Pw, ok = sc.map_points(q_kf, t_kf, kps)
    kps, Pw = kps[ok.astype(bool)], Pw[ok.astype(bool)]
    n = len(kps)
    pt_ref = Pw.astype(np.float32)  # T_kf = identity
    Tcr = np.zeros(n, gpu.SE3_DTYPE)
    Tcr["q"] = q_c
    Tcr["t"] = t_c
    proj = np.array([S.quat_rot(q_c.astype(np.float64), p) + t_c for p in Pw])
    cam = sc.cam
    px0 = np.stack([cam[0] * proj[:, 0] / proj[:, 2] + cam[2], cam[1] * proj[:, 1] / proj[:, 2] + cam[3]], 1)
    px0 = (px0 + np.random.default_rng(0).uniform(-1.5, 1.5, px0.shape)).astype(np.float32)
    px, lvl, okg = gpu.find_direct_projection_batch([fr_kf], fr_c, sc.camera(), np.zeros(n, np.int32), kps, pt_ref,
                                                    Tcr, px0)
    rl, cl = orc.pyramid(f_kf), orc.pyramid(f_c)
    rp = (O.C.c_void_p * 16)(*[l.ctypes.data for l in rl])
    cp = (O.C.c_void_p * 16)(*[l.ctypes.data for l in cl])
    lw = (O.C.c_int * 16)(*[l.shape[1] for l in rl])
    lh = (O.C.c_int * 16)(*[l.shape[0] for l in rl])
    sc_ = (O.C.c_float * 16)(*orc.scale.tolist())
    isc = (O.C.c_float * 16)(*orc.inv_scale.tolist())
    T = O.se3_from(q_c, t_c)
    ocam = O.Cam(*cam)
    n_ok = 0
    for i in range(n):
        q = np.array(px0[i], np.float32)
        sl = O.C.c_int()
        okc = O.lib().ygzo_find_direct_projection(O.C.byref(ocam), rp, lw, lh, cp, lw, lh, nl, sc_, isc,
                                                  O.C.c_float(orc.inv_sigma2[1]), O.C.byref(T), O._p(pt_ref[i]),
                                                  O._p(kps[i:i + 1]), O._p(q), O.C.byref(sl))
        assert bool(okc) == okg[i], i
        assert sl.value == lvl[i], i
        assert np.array_equal(q, px[i]), (i, q, px[i])
        n_ok += okc
    assert n_ok > n // 3


@pytest.mark.parametrize("seed", [0, 1])
def test_search_direct_batch_bitexact(gpu, seed):
    """Batched SearchLocalPointsDirect (Tracking.cc:2258-2410): every point's first
    converged in-border observation, in the listed keyframe order, bit-exact."""
    d = S.direct_scene(seed, n_kf=4, max_obs=5)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    kf_fr = [ex.ComputePyramid(im) for im in d["kf_images"]]
    cur_fr = ex.ComputePyramid(d["cur_image"])
    cam = d["scene"].camera()
    args = (d["item_ptr"], d["ref_index"], d["kps"], d["pt_ref"], d["T_cr"], d["px_proj"])
    px, m = gpu.search_direct_batch(kf_fr, cur_fr, cam, *args)
    opx, om = O.search_direct(orc, [orc.pyramid(im) for im in d["kf_images"]], orc.pyramid(d["cur_image"]),
                              O.Cam(*d["scene"].cam), *args)
    assert np.array_equal(m, om)
    assert np.array_equal(px, opx)
    n = len(m)
    hit = m >= 0
    # coverage: most points with observations match, some fall back to a later keyframe,
    # points without observations never match, and the border rule fires
    has_obs = np.diff(d["item_ptr"]) > 0
    assert not hit[~has_obs].any()
    assert hit[has_obs].mean() > 0.5, hit[has_obs].mean()
    assert (m[hit] > d["item_ptr"][:-1][hit]).any()
    assert ((px[hit] >= 20).all() and (px[hit, 0] < W - 20).all() and (px[hit, 1] < H - 20).all())
    assert n > 500


def test_search_direct_batch_edges(gpu):
    """No points, points without observations, and a keyframe list of length 1."""
    d = S.direct_scene(3, n_kf=1, max_obs=1, n_points=40)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    kf_fr = [ex.ComputePyramid(im) for im in d["kf_images"]]
    cur_fr = ex.ComputePyramid(d["cur_image"])
    cam = d["scene"].camera()
    px, m = gpu.search_direct_batch(kf_fr, cur_fr, cam, np.zeros(1, np.int32), d["ref_index"][:0], d["kps"][:0],
                                    d["pt_ref"][:0], d["T_cr"][:0], d["px_proj"][:0])
    assert len(px) == 0 and len(m) == 0
    ip = np.zeros(6, np.int32)
    px, m = gpu.search_direct_batch(kf_fr, cur_fr, cam, ip, d["ref_index"][:0], d["kps"][:0], d["pt_ref"][:0],
                                    d["T_cr"][:0], d["px_proj"][:5])
    assert (m == -1).all() and (px == 0).all()
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    args = (d["item_ptr"], d["ref_index"], d["kps"], d["pt_ref"], d["T_cr"], d["px_proj"])
    px, m = gpu.search_direct_batch(kf_fr, cur_fr, cam, *args)
    opx, om = O.search_direct(orc, [orc.pyramid(im) for im in d["kf_images"]], orc.pyramid(d["cur_image"]),
                              O.Cam(*d["scene"].cam), *args)
    assert np.array_equal(m, om) and np.array_equal(px, opx)
    with pytest.raises(gpu.YgzfeError):
        bad = d["ref_index"].copy()
        bad[:] = 7
        gpu.search_direct_batch(kf_fr, cur_fr, cam, d["item_ptr"], bad, d["kps"], d["pt_ref"], d["T_cr"],
                                d["px_proj"])


@pytest.mark.parametrize("seed", [0, 2])
def test_search_local_points_direct_grid_bitexact(gpu, seed):
    """Tracking::SearchLocalPointsDirect whole (Tracking.cc:2258-2410): the cache phase with the
    5-px coverage grid replayed in order (clustered projections: >= 10 % of the cache points are
    grid-skipped), mnCacheHitTh, then the local-map phase.  matched_item, px, status (hence the
    mvKeys / mvMatchedFrom order) and the counts bit-exact with the oracle."""
    d = S.direct_scene(seed, n_kf=4, max_obs=5, cluster=2)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    kf_fr = [ex.ComputePyramid(im) for im in d["kf_images"]]
    cur_fr = ex.ComputePyramid(d["cur_image"])
    kl = [orc.pyramid(im) for im in d["kf_images"]]
    cl = orc.pyramid(d["cur_image"])
    cam = d["scene"].camera()
    args = (d["item_ptr"], d["ref_index"], d["kps"], d["pt_ref"], d["T_cr"], d["px_proj"])
    n = len(d["item_ptr"]) - 1
    n_cache = (3 * n) // 5
    seen = set()
    for th in (10 ** 6, 150, 20):
        px, m, st, cs, ran = gpu.search_local_points_direct(kf_fr, cur_fr, cam, n_cache, *args, cache_hit_th=th)
        opx, om, ost, ocs, oran = O.search_local_points_direct(orc, kl, cl, O.Cam(*d["scene"].cam), n_cache, *args,
                                                               cache_hit_th=th)
        assert np.array_equal(st, ost), th
        assert np.array_equal(m, om) and np.array_equal(px, opx), th
        assert (cs, ran) == (ocs, oran), th
        seen.add(ran)
        assert (st[:n_cache] == gpu.DIRECT_GRID_SKIP).mean() >= 0.1
        assert (st[n_cache:] != gpu.DIRECT_GRID_SKIP).all()
    assert seen == {True, False}
    # the local-map-only form is the same replay with no cache points
    px, m = gpu.search_direct_batch(kf_fr, cur_fr, cam, *args)
    opx, om, ost, _, _ = O.search_local_points_direct(orc, kl, cl, O.Cam(*d["scene"].cam), 0, *args)
    assert np.array_equal(m, om) and np.array_equal(px, opx)


def test_search_local_points_direct_dense_chunks(gpu):
    """SearchLocalPointsDirect with > 2,048 cache points (two replay chunks: the grid marks
    of the first reach the second) and 5-point clusters, so that some points' earliest
    possible marker of their cell is itself undecided until the ordered pass over the
    chunk (checked below from the local-only form's matches).  Statuses, matches, pixels
    and counts bit-exact with the oracle's sequential loop (Tracking.cc:2258-2410)."""
    d = S.direct_scene(4, n_kf=3, max_obs=3, cluster=4)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    kf_fr = [ex.ComputePyramid(im) for im in d["kf_images"]]
    cur_fr = ex.ComputePyramid(d["cur_image"])
    kl = [orc.pyramid(im) for im in d["kf_images"]]
    cl = orc.pyramid(d["cur_image"])
    cam = d["scene"].camera()
    args = (d["item_ptr"], d["ref_index"], d["kps"], d["pt_ref"], d["T_cr"], d["px_proj"])
    n = len(d["item_ptr"]) - 1
    n_cache = (3 * n) // 5
    assert n_cache > 2048
    # every point's first in-border match (no grid) -> its matched cell; the first chunk's
    # earliest possible marker per cell and the points that wait on an undecided one
    px_all, m_all = gpu.search_direct_batch(kf_fr, cur_fr, cam, *args)
    gs, gcols = 5, W // 5
    ncell = (H // 5) * gcols

    def cell(p):
        k = int(np.float32(p[1]) / np.float32(gs)) * gcols + int(np.float32(p[0]) / np.float32(gs))
        return k if 0 <= k < ncell else -2

    c = [cell(d["px_proj"][i]) for i in range(2048)]
    first = {}
    for k in range(2048):
        if m_all[k] >= 0:
            mk = cell(px_all[k])
            if mk >= 0:
                first.setdefault(mk, k)
    waits = [k for k in range(2048) if c[k] >= 0 and first.get(c[k], 1 << 30) < k
             and c[first[c[k]]] >= 0 and first.get(c[first[c[k]]], 1 << 30) < first[c[k]]]
    assert len(waits) >= 5, len(waits)
    for th in (10 ** 6, 150):
        px, m, st, cs, ran = gpu.search_local_points_direct(kf_fr, cur_fr, cam, n_cache, *args, cache_hit_th=th)
        opx, om, ost, ocs, oran = O.search_local_points_direct(orc, kl, cl, O.Cam(*d["scene"].cam), n_cache, *args,
                                                               cache_hit_th=th)
        assert np.array_equal(st, ost), th
        assert np.array_equal(m, om) and np.array_equal(px, opx), th
        assert (cs, ran) == (ocs, oran), th
        assert (st[:n_cache] == gpu.DIRECT_GRID_SKIP).mean() >= 0.2
        assert (st[2048:n_cache] == gpu.DIRECT_GRID_SKIP).any()


def test_search_direct_items_own_tcr(gpu):
    """Items of one keyframe whose T_cr differ (the C ABI takes a T_cr per item; the call
    packs one per keyframe only while they agree): bit-exact with the oracle."""
    d = S.direct_scene(1, n_kf=4, max_obs=5)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    kf_fr = [ex.ComputePyramid(im) for im in d["kf_images"]]
    cur_fr = ex.ComputePyramid(d["cur_image"])
    T = d["T_cr"].copy()
    T["t"][::3, 0] += np.float32(2e-3)
    T["t"][1::7, 1] -= np.float32(1e-3)
    args = (d["item_ptr"], d["ref_index"], d["kps"], d["pt_ref"], T, d["px_proj"])
    px, m = gpu.search_direct_batch(kf_fr, cur_fr, cam := d["scene"].camera(), *args)
    opx, om = O.search_direct(orc, [orc.pyramid(im) for im in d["kf_images"]], orc.pyramid(d["cur_image"]),
                              O.Cam(*d["scene"].cam), *args)
    assert np.array_equal(m, om) and np.array_equal(px, opx)
    base, bm = gpu.search_direct_batch(kf_fr, cur_fr, cam, *(args[:4] + (d["T_cr"], args[5])))
    assert not np.array_equal(base, px)  # the per-item poses were used
