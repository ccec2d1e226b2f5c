"""Property tests of the CPU oracle (test infrastructure), independent of the
reference binaries: each restated primitive against its definition.

  FAST-9/16 + cornerScore<16> (OpenCV, ORBextractor.cc:765)   brute force segment test
  resize x2 -> INTER_AREA (ORBextractor.cc:1139)             (a+b+c+d+2)>>2 in numpy
  GaussianBlur 7x7 (ORBextractor.cc:1083)                     constant images, mirror symmetry
  DescriptorDistance (ORBmatcher.cc:1507-1523)                numpy popcount
  DistributeOctTree (ORBextractor.cc:533-723)                 output invariants
  SE3::exp (se3.hpp:407-428)                                  Rodrigues in float64
  Align2D (Align.cc:8-105)                                    recovers a known sub-pixel shift
"""
import ctypes as C

import numpy as np
import pytest

import _oracle as O

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
        (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def brute_best_barrier(patch):
    """Largest b such that 9 contiguous ring pixels are all > v+b or all < v-b (-1: none)."""
    v = int(patch[3, 3])
    d = np.array([int(patch[3 + dy, 3 + dx]) for dx, dy in RING])
    best = -1
    for s in range(16):
        arc = d[(s + np.arange(9)) % 16]
        best = max(best, int(arc.min() - v) - 1, int(v - arc.max()) - 1)
    return best


def test_fast9_score_closed_form_vs_brute_force():
    rng = np.random.default_rng(0)
    lib = O.lib()
    n_corners = 0
    for trial in range(3000):
        patch = rng.integers(0, 256, size=(7, 7), dtype=np.uint8)
        if trial % 2:  # make many of them corners: push an arc up or down
            s = rng.integers(16)
            sign = 1 if rng.integers(2) else -1
            for k in range(int(rng.integers(9, 13))):
                dx, dy = RING[(s + k) % 16]
                patch[3 + dy, 3 + dx] = np.clip(int(patch[3, 3]) + sign * int(rng.integers(10, 120)), 0, 255)
        patch = np.ascontiguousarray(patch)
        b = brute_best_barrier(patch)
        for t in (5, 20):
            is_corner = b >= t
            ptr = C.c_void_p(patch.ctypes.data + 3 * 7 + 3)
            if is_corner:
                n_corners += 1
                assert lib.ygzo_corner_score16(ptr, 7, t) == b
            xs, ys, sc = O.fast9_roi(patch, t)
            # a 7x7 ROI has exactly one testable pixel (3,3); NMS keeps it iff it is a corner
            assert len(xs) == int(is_corner)
    assert n_corners > 500


@pytest.mark.parametrize("seed", [0, 1])
def test_fast9_vector_segment_test_equals_scalar(seed):
    """The oracle's 16-pixel vector segment test (the CPU baseline's FAST) finds
    exactly the scalar test's corners, scores and NMS survivors: ROIs of every
    width (block and tail columns), corner-rich noise and smooth ramps."""
    rng = np.random.default_rng(seed)
    lib = O.lib()
    for trial in range(60):
        h, w = int(rng.integers(7, 60)), int(rng.integers(7, 90))
        img = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
        if trial % 3 == 1:  # piecewise-flat blocks: long runs, ties
            img = (rng.integers(0, 6, size=(h // 4 + 2, w // 4 + 2)) * 50).astype(np.uint8).repeat(4, 0).repeat(4, 1)[:h, :w]
        img = np.ascontiguousarray(img)
        for t in (5, 20, 60):
            lib.ygzo_fast9_force_scalar(1)
            ref = O.fast9_roi(img, t)
            lib.ygzo_fast9_force_scalar(0)
            got = O.fast9_roi(img, t)
            for a, b in zip(ref, got):
                assert np.array_equal(a, b), (trial, t)


def test_resize_exact_half_is_area_average():
    rng = np.random.default_rng(1)
    src = rng.integers(0, 256, size=(60, 94), dtype=np.uint8)
    got = O.resize(src, 47, 30)
    s = src.astype(np.int32)
    want = ((s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2).astype(np.uint8)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("value", [0, 17, 128, 255])
def test_blur_constant_image(value):
    img = np.full((40, 53), value, np.uint8)
    assert np.array_equal(O.blur7(img, 0), img)  # CV4 taps sum to 256


def test_blur_mirror_symmetry():
    """REFLECT_101 borders and a symmetric kernel: blur(flip(x)) == flip(blur(x))."""
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, size=(33, 47), dtype=np.uint8)
    for variant in (0, 1):
        b = O.blur7(img, variant)
        assert np.array_equal(O.blur7(np.ascontiguousarray(img[:, ::-1]), variant), b[:, ::-1])
        assert np.array_equal(O.blur7(np.ascontiguousarray(img[::-1]), variant), b[::-1])


def test_descriptor_distance_and_best2():
    rng = np.random.default_rng(3)
    q = rng.integers(0, 256, size=(50, 32), dtype=np.uint8)
    t = rng.integers(0, 256, size=(70, 32), dtype=np.uint8)
    t[10] = q[5]  # an exact match
    t[11] = q[5]  # ... twice: the first index wins
    dist = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(2)
    for i in range(5):
        assert O.lib().ygzo_descriptor_distance(O._p(q[i]), O._p(t[i])) == dist[i, i]
    bi, bd, sd = O.hamming_best2(q, t)
    assert np.array_equal(bd, dist.min(1))
    assert np.array_equal(bi, dist.argmin(1))  # argmin returns the first minimum
    assert bi[5] == 10 and bd[5] == 0
    srt = np.sort(dist, 1)
    assert np.array_equal(sd, srt[:, 1])


def test_octree_invariants():
    rng = np.random.default_rng(4)
    img = np.full((240, 376), 128, np.int32)
    for _ in range(300):
        x, y = rng.integers(0, 376), rng.integers(0, 240)
        img[y:y + rng.integers(3, 20), x:x + rng.integers(3, 20)] = rng.integers(0, 256)
    img = np.clip(img + rng.integers(-3, 4, img.shape), 0, 255).astype(np.uint8)
    orc = O.OrbOracle(1000, 2.0, 4, 20, 7)
    budget = orc.feat_per_level[1]
    kps, ncand = orc.octree_level(img, 1)
    assert ncand > budget
    assert budget <= len(kps) <= budget + 3  # splitting stops at the first node count >= N
    pts = {(float(k["x"]), float(k["y"])) for k in kps}
    assert len(pts) == len(kps)
    assert np.all(kps["octave"] == 1)


def rodrigues(w):
    th = np.linalg.norm(w)
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-12:
        return np.eye(3) + K
    return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K


def test_se3_exp_matches_rodrigues():
    rng = np.random.default_rng(5)
    for _ in range(50):
        x = (rng.standard_normal(6) * [0.1, 0.1, 0.1, 0.3, 0.3, 0.3]).astype(np.float32)
        T = O.SE3()
        O.lib().ygzo_se3_exp(O._p(x), C.byref(T))
        p = rng.standard_normal(3).astype(np.float32)
        out = np.zeros(3, np.float32)
        O.lib().ygzo_se3_act(C.byref(T), O._p(p), O._p(out))
        w, v = x[3:].astype(np.float64), x[:3].astype(np.float64)
        R = rodrigues(w)
        th = np.linalg.norm(w)
        K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
        V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * K + (th - np.sin(th)) / th ** 3 * K @ K
        want = R @ p + V @ v
        assert np.allclose(out, want, atol=2e-5)


def test_align2d_recovers_subpixel_shift():
    yy, xx = np.mgrid[0:64, 0:64].astype(np.float64)
    img = (128 + 60 * np.sin(xx / 5.0) * np.cos(yy / 7.0) + 30 * np.sin((xx + yy) / 9.0)).astype(np.uint8)
    u0, v0 = 30, 31
    rpb = np.ascontiguousarray(img[v0 - 5:v0 + 5, u0 - 5:u0 + 5])  # 10x10 with border, centre (u0, v0)
    rp = np.ascontiguousarray(rpb[1:9, 1:9])
    ok, px = O.align2d(img, rpb, rp, (u0 + 0.6, v0 - 0.4))
    assert ok
    assert abs(px[0] - u0) < 0.1 and abs(px[1] - v0) < 0.1


def test_search_direct_is_first_in_border_success():
    """ygzo_search_direct (Tracking.cc:2337-2395) == FindDirectProjection per item in
    order, first converged result inside the 20 px border, and recovers the true pixel."""
    import _scenes as S
    d = S.direct_scene(5, n_kf=3, max_obs=3, n_points=120)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    kl = [orc.pyramid(im) for im in d["kf_images"]]
    cl = orc.pyramid(d["cur_image"])
    cam = O.Cam(*d["scene"].cam)
    px, m = O.search_direct(orc, kl, cl, cam, d["item_ptr"], d["ref_index"], d["kps"], d["pt_ref"], d["T_cr"],
                            d["px_proj"])
    cp = (C.c_void_p * 16)(*[l.ctypes.data for l in cl])
    lw = (C.c_int * 16)(*[l.shape[1] for l in cl])
    lh = (C.c_int * 16)(*[l.shape[0] for l in cl])
    sc = (C.c_float * 16)(*orc.scale.tolist())
    isc = (C.c_float * 16)(*orc.inv_scale.tolist())
    for i in range(len(m)):
        want = -1
        for k in range(d["item_ptr"][i], d["item_ptr"][i + 1]):
            rp = (C.c_void_p * 16)(*[l.ctypes.data for l in kl[d["ref_index"][k]]])
            q = np.array(d["px_proj"][i], np.float32)
            sl = C.c_int()
            ok = O.lib().ygzo_find_direct_projection(C.byref(cam), rp, lw, lh, cp, lw, lh, nl, sc, isc,
                                                     C.c_float(orc.inv_sigma2[1]),
                                                     C.byref(O.se3_from(d["T_cr"][k]["q"], d["T_cr"][k]["t"])),
                                                     O._p(d["pt_ref"][k]), O._p(d["kps"][k:k + 1]), O._p(q),
                                                     C.byref(sl))
            if ok and 20 <= q[0] < W - 20 and 20 <= q[1] < H - 20:
                want = k
                assert np.array_equal(q, px[i])
                break
        assert m[i] == want, i
    hit = m >= 0
    assert hit.sum() > 20
    true_px, _ = S.project(d["scene"].cam, *d["cur_pose"], d["Pw"])
    assert np.median(np.abs(px[hit] - true_px[hit])) < 0.5


def _py_transform(parent, is_leaf, desc, weight, f, levelsup, L):
    """TemplatedVocabulary::transform (TemplatedVocabulary.h:1241-1281) in plain Python."""
    children = {}
    for i in range(1, len(parent)):
        children.setdefault(int(parent[i]), []).append(i)
    words = np.cumsum(is_leaf) - 1
    node, level, nid = 0, 0, 0
    while children.get(node):
        level += 1
        ch = children[node]
        d = [int(np.unpackbits(np.bitwise_xor(f, desc[c])).sum()) for c in ch]
        node = ch[int(np.argmin(d))]  # argmin = first minimum
        if level == L - levelsup:
            nid = node
    return (int(words[node]) if is_leaf[node] else 0), float(weight[node]), nid


@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 0), (5, 1), (0, 2), (5, 3)])
def test_bow_oracle_matches_python_restatement(scoring, weighting):
    """oracle/bow.c == a plain-Python DBoW2 transform + BowVector / FeatureVector
    (addWeight / addIfNotExist, normalize L1 / L2, DotProduct's / size())."""
    import _vocab as V
    k, L = 6, 3
    parent, is_leaf, desc, weight = V.synth_vocab(1, k, L)
    voc = O.Vocab(k, L, scoring, weighting, parent, is_leaf, desc, weight)
    rng = np.random.default_rng(2)
    # features near vocabulary leaves (repeats -> shared words), plus random ones
    leaves = np.where(is_leaf)[0]
    f = desc[rng.choice(leaves, 60)] ^ (rng.integers(0, 256, (60, 32), dtype=np.uint8) &
                                        rng.integers(0, 256, (60, 32), dtype=np.uint8) &
                                        rng.integers(0, 256, (60, 32), dtype=np.uint8))
    f = np.concatenate([f, f[:10], rng.integers(0, 256, (10, 32), dtype=np.uint8)])
    w, wt, nid = voc.transform_each(f, 1)
    bow = {}
    fv = {}
    for i, x in enumerate(f):
        ew, ewt, enid = _py_transform(parent, is_leaf, desc, weight, x, 1, L)
        assert (w[i], wt[i], nid[i]) == (ew, ewt, enid), i
        if ewt > 0:
            if weighting in (0, 1):
                bow[ew] = bow.get(ew, 0.0) + ewt
            else:
                bow.setdefault(ew, ewt)
            fv.setdefault(enid, []).append(i)
    keys = sorted(bow)
    vals = [bow[kk] for kk in keys]
    if scoring == 5:
        if weighting in (0, 1):
            vals = [v / float(len(vals)) for v in vals]
    else:
        norm = 0.0
        if scoring == 1:
            for v in vals:
                norm += v * v
            norm = norm ** 0.5
        else:
            for v in vals:
                norm += abs(v)
        if norm > 0:
            vals = [v / norm for v in vals]
    (bw, bv), (fn, ff) = voc.transform(f, 1)
    assert bw.tolist() == keys
    assert bv.tolist() == vals
    assert fn.tolist() == [n for n in sorted(fv) for _ in fv[n]]
    assert ff.tolist() == [i for n in sorted(fv) for i in fv[n]]


def _replay_local_points_direct(first, proj, n_cache, W, H, grid_size, th):
    """Tracking.cc:2258-2410 in Python over per-point first successes (item, px) or None."""
    gr, gc = H // grid_size, W // grid_size
    grid = np.zeros(gr * gc, bool)
    status, cnt = [], 0
    for i in range(n_cache):
        k = int(np.float32(proj[i, 1]) / np.float32(grid_size)) * gc + int(np.float32(proj[i, 0]) / np.float32(grid_size))
        if 0 <= k < len(grid) and grid[k]:
            status.append(2)
            continue
        if first[i] is None:
            status.append(0)
            continue
        status.append(1)
        cnt += 1
        px = first[i][1]
        k = int(px[1] / np.float32(grid_size)) * gc + int(px[0] / np.float32(grid_size))
        grid[k] = True
    ran = not cnt > th
    for i in range(n_cache, len(proj)):
        status.append(3 if not ran else (1 if first[i] is not None else 0))
    return np.array(status), cnt, ran


def test_search_local_points_direct_replays_the_grid():
    """ygzo_search_local_points_direct == the per-point first success (ygzo_search_direct) replayed
    through Tracking.cc:2258-2410's coverage grid and mnCacheHitTh rule, on clustered points."""
    import _scenes as S
    d = S.direct_scene(6, n_kf=2, max_obs=2, n_points=40, cluster=2)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    kl = [orc.pyramid(im) for im in d["kf_images"]]
    cl = orc.pyramid(d["cur_image"])
    cam = O.Cam(*d["scene"].cam)
    args = (d["item_ptr"], d["ref_index"], d["kps"], d["pt_ref"], d["T_cr"], d["px_proj"])
    px1, m1 = O.search_direct(orc, kl, cl, cam, *args)
    first = [(m1[i], px1[i]) if m1[i] >= 0 else None for i in range(len(m1))]
    n = len(m1)
    n_cache = (2 * n) // 3
    for th in (10 ** 6, 3, -1):
        px, m, st, cs, ran = O.search_local_points_direct(orc, kl, cl, cam, n_cache, *args, cache_hit_th=th)
        want, wcnt, wran = _replay_local_points_direct(first, d["px_proj"], n_cache, W, H, 5, th)
        assert np.array_equal(st, want), th
        assert cs == wcnt and ran == wran
        ok = st == 1
        assert np.array_equal(m[ok], m1[ok]) and np.array_equal(px[ok], px1[ok])
        assert (m[~ok] == -1).all() and (px[~ok] == 0).all()
    assert (want[:n_cache] == 2).mean() >= 0.1
    assert ((want[:n_cache] == 1).sum() > 3) and (want[n_cache:] == 3).all()


def test_align_gn_matches_round4_oracle():
    """The GN SparseImgAlign oracle reproduces round 4's restatement bit for bit on a fixed
    scene (tests/golden/align_gn_r04.json, made by tests/golden/make_align_gn_r04.py from
    oracle/align.c at 651410b): round 5's refactor into align_residuals() changed the speed
    of the CPU baseline (2.3x slower, fixed) and must not change its outputs."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_align_gn_r04 as G
    with open(G.FIXTURE) as f:
        want = json.load(f)["outputs"]
    got, _ = G.run(None, G.scene_inputs())
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g["n_visible"] == w["n_visible"] > 100
        assert g["iters"] == w["iters"]
        for k in ("q", "t", "H"):
            assert np.array_equal(np.float32(g[k]), np.float32(w[k])), k
        assert np.float32(g["chi2"]) == np.float32(w["chi2"])
