"""ctypes view of the CPU oracle (oracle/build/libygzoracle.so).

TEST INFRASTRUCTURE ONLY: the parity checker for the HIP product path.  The
functions mirror oracle/ygz_oracle.h; numpy arrays in, numpy arrays out.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "libygzoracle.so")
REF_FAST_PATH = os.path.join(ORACLE_DIR, "_ref", "libfastref.so")

MAXL = 16

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == 28


class Orb(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_double), ("nlevels", C.c_int),
                ("ini_th", C.c_int), ("min_th", C.c_int), ("blur_variant", C.c_int),
                ("scale", C.c_float * MAXL), ("inv_scale", C.c_float * MAXL),
                ("sigma2", C.c_float * MAXL), ("inv_sigma2", C.c_float * MAXL),
                ("feat_per_level", C.c_int * MAXL), ("umax", C.c_int * 16), ("dso_grid", C.c_int)]


class Cam(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float)]


class SE3(C.Structure):
    _fields_ = [("q", C.c_float * 4), ("t", C.c_float * 3)]


class AlignOut(C.Structure):
    _fields_ = [("T", SE3), ("n_visible", C.c_int), ("chi2", C.c_float),
                ("iters", C.c_int * MAXL), ("H", C.c_float * 36)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR], stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def se3_from(q, t):
    s = SE3()
    for i in range(4):
        s.q[i] = float(q[i])
    for i in range(3):
        s.t[i] = float(t[i])
    return s


class OrbOracle:
    """ORBextractor restated (ORBextractor.cc:412-470)."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7,
                 blur_variant=0):
        self.o = Orb()
        lib().ygzo_orb_init(C.byref(self.o), nfeatures, C.c_float(scale_factor), nlevels, ini_th,
                            min_th, blur_variant)
        self.nlevels = nlevels

    @property
    def feat_per_level(self):
        return [self.o.feat_per_level[i] for i in range(self.nlevels)]

    @property
    def scale(self):
        return np.array([self.o.scale[i] for i in range(self.nlevels)], np.float32)

    @property
    def inv_scale(self):
        return np.array([self.o.inv_scale[i] for i in range(self.nlevels)], np.float32)

    @property
    def inv_sigma2(self):
        return np.array([self.o.inv_sigma2[i] for i in range(self.nlevels)], np.float32)

    @property
    def umax(self):
        return [self.o.umax[i] for i in range(16)]

    def level_sizes(self, W, H):
        w = (C.c_int * MAXL)()
        h = (C.c_int * MAXL)()
        lib().ygzo_level_sizes(C.byref(self.o), W, H, w, h)
        return [(w[i], h[i]) for i in range(self.nlevels)]

    def pyramid(self, img):
        img = np.ascontiguousarray(img, np.uint8)
        H, W = img.shape
        sizes = self.level_sizes(W, H)
        levels = [np.zeros((h, w), np.uint8) for (w, h) in sizes]
        ptrs = (C.c_void_p * MAXL)(*[l.ctypes.data for l in levels])
        lib().ygzo_compute_pyramid(C.byref(self.o), _p(img), W, H, W, ptrs)
        return levels

    def _lvl_args(self, levels):
        ptrs = (C.c_void_p * MAXL)(*[l.ctypes.data for l in levels])
        lw = (C.c_int * MAXL)(*[l.shape[1] for l in levels])
        lh = (C.c_int * MAXL)(*[l.shape[0] for l in levels])
        return ptrs, lw, lh

    def extract(self, levels, existing=None, cap=None):
        """ORBSLAM_KEYPOINT extraction on a prebuilt pyramid -> (kps, desc)."""
        existing = np.zeros(0, KP_DTYPE) if existing is None else np.ascontiguousarray(existing, KP_DTYPE)
        cap = cap or (sum(self.feat_per_level) + 8 * self.nlevels + len(existing))
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        ptrs, lw, lh = self._lvl_args(levels)
        n = lib().ygzo_extract_orbslam(C.byref(self.o), ptrs, lw, lh, _p(existing), len(existing),
                                       _p(kps), _p(desc), cap)
        assert n >= 0
        return kps[:n].copy(), desc[:n].copy()

    def extract_dso(self, levels, existing=None, cap=4096):
        existing = np.zeros(0, KP_DTYPE) if existing is None else np.ascontiguousarray(existing, KP_DTYPE).copy()
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        ptrs, lw, lh = self._lvl_args(levels)
        n = lib().ygzo_extract_dso(C.byref(self.o), ptrs, lw, lh, _p(existing), len(existing),
                                   _p(kps), _p(desc), cap)
        assert n >= 0
        return kps[:n].copy(), desc[:n].copy(), existing

    def octree_level(self, lvl, level, cap=8192):
        lvl = np.ascontiguousarray(lvl, np.uint8)
        out = np.zeros(cap, KP_DTYPE)
        nc = C.c_int()
        n = lib().ygzo_octree_level(C.byref(self.o), _p(lvl), lvl.shape[1], lvl.shape[0], level,
                                    _p(out), cap, C.byref(nc))
        return out[:n].copy(), nc.value

    def ic_angle(self, img, x, y):
        lib().ygzo_ic_angle.restype = C.c_float
        return lib().ygzo_ic_angle(_p(img), img.shape[1], img.shape[0], img.shape[1], C.c_float(x),
                                   C.c_float(y), self.o.umax)


def blur7(img, variant=0):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros_like(img)
    lib().ygzo_gaussian_blur7(_p(img), img.shape[1], img.shape[0], img.shape[1], _p(out),
                              img.shape[1], variant)
    return out


def resize(src, dw, dh):
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros((dh, dw), np.uint8)
    lib().ygzo_resize(_p(src), src.shape[1], src.shape[0], src.shape[1], _p(out), dw, dh, dw)
    return out


def fast9_roi(roi, threshold, cap=8192):
    roi = np.ascontiguousarray(roi, np.uint8)
    xs = np.zeros(cap, np.int16)
    ys = np.zeros(cap, np.int16)
    sc = np.zeros(cap, np.uint8)
    n = lib().ygzo_fast9_roi(_p(roi), roi.shape[1], roi.shape[0], roi.shape[1], threshold,
                             _p(xs), _p(ys), _p(sc), cap)
    return xs[:n].copy(), ys[:n].copy(), sc[:n].copy()


def fast10_detect(img, barrier, sse=True, x0=0, y0=0, w=None, h=None, cap=1 << 20):
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    w = W - x0 if w is None else w
    h = H - y0 if h is None else h
    xs = np.zeros(cap, np.int16)
    ys = np.zeros(cap, np.int16)
    fn = lib().ygzo_fast10_detect_sse2 if sse else lib().ygzo_fast10_detect_plain
    ptr = C.c_void_p(img.ctypes.data + y0 * W + x0)
    n = fn(ptr, w, h, W, barrier, _p(xs), _p(ys), cap)
    return xs[:n].copy(), ys[:n].copy()


def fast10_scores(img, xs, ys, threshold, x0=0, y0=0):
    img = np.ascontiguousarray(img, np.uint8)
    W = img.shape[1]
    out = np.zeros(len(xs), np.int32)
    for i, (x, y) in enumerate(zip(xs, ys)):
        ptr = C.c_void_p(img.ctypes.data + (int(y) + y0) * W + int(x) + x0)
        out[i] = lib().ygzo_fast10_score(ptr, W, threshold)
    return out


def fast10_pipeline(img, barrier, x0=0, y0=0, w=None, h=None, scalar=False):
    """detect_sse2 + score + nonmax_3x3 in one pass (ygzo_fast10_detect_score_nms) -> (xs, ys, scores)."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    w = W - x0 if w is None else w
    h = H - y0 if h is None else h
    cap = w * h // 2 + 16
    xs, ys, sc = np.zeros(cap, np.int16), np.zeros(cap, np.int16), np.zeros(cap, np.int32)
    lib().ygzo_fast10_force_scalar(1 if scalar else 0)
    try:
        n = lib().ygzo_fast10_detect_score_nms(C.c_void_p(img.ctypes.data + y0 * W + x0), w, h, W, barrier, _p(xs),
                                              _p(ys), _p(sc), cap)
    finally:
        lib().ygzo_fast10_force_scalar(0)
    return xs[:n].copy(), ys[:n].copy(), sc[:n].copy()


def bench_fast10(img, barrier, x0, y0, w, h, reps=20):
    """The restated FAST-10 pipeline timed in C -> (kept corners, mean seconds)."""
    img = np.ascontiguousarray(img, np.uint8)
    W = img.shape[1]
    s = C.c_double()
    n = lib().ygzo_bench_fast10(C.c_void_p(img.ctypes.data + y0 * W + x0), w, h, W, barrier, reps, C.byref(s))
    return n, s.value


def fast10_nonmax(xs, ys, scores):
    xs = np.ascontiguousarray(xs, np.int16)
    ys = np.ascontiguousarray(ys, np.int16)
    scores = np.ascontiguousarray(scores, np.int32)
    keep = np.zeros(max(1, len(xs)), np.int32)
    n = lib().ygzo_fast10_nonmax(_p(xs), _p(ys), _p(scores), len(xs), _p(keep))
    return keep[:n].copy()


def undistort_map(cam, dist, W, H):
    """initUndistortRectifyMap(K, D, I, K, (W, H), CV_16SC2) -> (map1[H,W,2] i16, map2[H,W] u16)."""
    c = np.ascontiguousarray(cam, np.float32)
    d = np.ascontiguousarray(dist, np.float32).ravel()
    m1 = np.zeros((H, W, 2), np.int16)
    m2 = np.zeros((H, W), np.uint16)
    lib().ygzo_undistort_map(_p(c), _p(d) if len(d) else None, len(d), W, H, _p(m1), _p(m2))
    return m1, m2


def remap_linear(src, map1, map2):
    """remap(src, map1, map2, INTER_LINEAR, BORDER_CONSTANT 0) for CV_8U."""
    src = np.ascontiguousarray(src, np.uint8)
    H, W = src.shape
    DH, DW = map2.shape
    out = np.zeros((DH, DW), np.uint8)
    lib().ygzo_remap_linear(_p(src), W, H, W, _p(np.ascontiguousarray(map1)), _p(np.ascontiguousarray(map2)),
                            DW, DH, _p(out), DW)
    return out


def remap_linear_f32(src, map1, map2):
    """remap(src, map1, map2, INTER_LINEAR, BORDER_CONSTANT 0) for CV_32F (the RGB-D depth image)."""
    src = np.ascontiguousarray(src, np.float32)
    H, W = src.shape
    DH, DW = map2.shape
    out = np.zeros((DH, DW), np.float32)
    lib().ygzo_remap_linear_f32(_p(src), W, H, W, _p(np.ascontiguousarray(map1)), _p(np.ascontiguousarray(map2)),
                                DW, DH, _p(out), DW)
    return out


def hamming_best2(q, t):
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    nq = len(q)
    bi = np.zeros(nq, np.int32)
    bd = np.zeros(nq, np.int32)
    sd = np.zeros(nq, np.int32)
    lib().ygzo_hamming_best2(_p(q), nq, _p(t), len(t), _p(bi), _p(bd), _p(sd))
    return bi, bd, sd


ALIGN_GN, ALIGN_LM = 0, 1  # NLLSSolver's methods (NLSSolver_impl.hpp:8-13)


def sparse_align(ref_levels, cur_levels, inv_scale, cam, kps, xyz_ref, usable, max_level,
                 min_level, T_init, method=ALIGN_GN):
    rp = (C.c_void_p * MAXL)(*[l.ctypes.data for l in ref_levels])
    cp = (C.c_void_p * MAXL)(*[l.ctypes.data for l in cur_levels])
    lw = (C.c_int * MAXL)(*[l.shape[1] for l in ref_levels])
    lh = (C.c_int * MAXL)(*[l.shape[0] for l in ref_levels])
    inv = (C.c_float * MAXL)(*[float(v) for v in inv_scale])
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    xyz = np.ascontiguousarray(xyz_ref, np.float32)
    us = np.ascontiguousarray(usable, np.uint8)
    out = AlignOut()
    lib().ygzo_sparse_align_method(rp, cp, lw, lh, inv, C.byref(cam), _p(kps), _p(xyz), _p(us), len(kps),
                                   max_level, min_level, C.byref(T_init), int(method), C.byref(out))
    return out


def align2d(cur, rpb, rp, px, n_iter=10):
    cur = np.ascontiguousarray(cur, np.uint8)
    px = np.array(px, np.float32)
    ok = lib().ygzo_align2d(_p(cur), cur.shape[1], cur.shape[0], cur.shape[1],
                            _p(np.ascontiguousarray(rpb, np.uint8)),
                            _p(np.ascontiguousarray(rp, np.uint8)), n_iter, _p(px))
    return bool(ok), px


def search_direct(orc, kf_levels, cur_levels, cam, item_ptr, ref_index, kps, pt_ref, T_cr, px_proj, border=20.0):
    """SearchLocalPointsDirect's per-point search (Tracking.cc:2337-2395) -> (px_out, matched)."""
    nl = len(cur_levels)
    flat = [l for lv in kf_levels for l in lv]
    rp = (C.c_void_p * max(1, len(flat)))(*[l.ctypes.data for l in flat])
    cp = (C.c_void_p * MAXL)(*[l.ctypes.data for l in cur_levels])
    lw = (C.c_int * MAXL)(*[l.shape[1] for l in cur_levels])
    lh = (C.c_int * MAXL)(*[l.shape[0] for l in cur_levels])
    sc = (C.c_float * MAXL)(*orc.scale.tolist())
    isc = (C.c_float * MAXL)(*orc.inv_scale.tolist())
    item_ptr = np.ascontiguousarray(item_ptr, np.int32)
    n = len(item_ptr) - 1
    T = (SE3 * max(1, len(T_cr)))(*[se3_from(r["q"], r["t"]) for r in T_cr])
    px_out = np.zeros((max(n, 0), 2), np.float32)
    matched = np.zeros(max(n, 0), np.int32)
    lib().ygzo_search_direct(C.byref(cam), rp, cp, lw, lh, nl, sc, isc, C.c_float(orc.inv_sigma2[1]), n,
                             _p(item_ptr), _p(np.ascontiguousarray(ref_index, np.int32)),
                             _p(np.ascontiguousarray(kps, KP_DTYPE)), _p(np.ascontiguousarray(pt_ref, np.float32)),
                             T, _p(np.ascontiguousarray(px_proj, np.float32)), C.c_float(border), _p(px_out),
                             _p(matched))
    return px_out, matched


def search_local_points_direct(orc, kf_levels, cur_levels, cam, n_cache, item_ptr, ref_index, kps, pt_ref, T_cr,
                               px_proj, border=20.0, grid_size=5, cache_hit_th=150):
    """Tracking::SearchLocalPointsDirect (Tracking.cc:2258-2410) whole ->
    (px_out, matched, status, cache_success, local_ran)."""
    nl = len(cur_levels)
    flat = [l for lv in kf_levels for l in lv]
    rp = (C.c_void_p * max(1, len(flat)))(*[l.ctypes.data for l in flat])
    cp = (C.c_void_p * MAXL)(*[l.ctypes.data for l in cur_levels])
    lw = (C.c_int * MAXL)(*[l.shape[1] for l in cur_levels])
    lh = (C.c_int * MAXL)(*[l.shape[0] for l in cur_levels])
    sc = (C.c_float * MAXL)(*orc.scale.tolist())
    isc = (C.c_float * MAXL)(*orc.inv_scale.tolist())
    item_ptr = np.ascontiguousarray(item_ptr, np.int32)
    n = len(item_ptr) - 1
    T = (SE3 * max(1, len(T_cr)))(*[se3_from(r["q"], r["t"]) for r in T_cr])
    px_out = np.zeros((max(n, 0), 2), np.float32)
    matched = np.zeros(max(n, 0), np.int32)
    status = np.zeros(max(n, 0), np.int32)
    lr = C.c_int()
    cs = lib().ygzo_search_local_points_direct(
        C.byref(cam), rp, cp, lw, lh, nl, sc, isc, C.c_float(orc.inv_sigma2[1]), int(n_cache), n - int(n_cache),
        _p(item_ptr), _p(np.ascontiguousarray(ref_index, np.int32)), _p(np.ascontiguousarray(kps, KP_DTYPE)),
        _p(np.ascontiguousarray(pt_ref, np.float32)), T, _p(np.ascontiguousarray(px_proj, np.float32)),
        C.c_float(border), int(grid_size), int(cache_hit_th), _p(px_out), _p(matched), _p(status), C.byref(lr))
    return px_out, matched, status, cs, bool(lr.value)


def stereo_matches(orc, left_levels, right_levels, kl, dl, kr, dr, mb, mbf):
    """Frame::ComputeStereoMatches (Frame.cc:509-682) -> (uRight, depth, sad)."""
    lp = (C.c_void_p * MAXL)(*[l.ctypes.data for l in left_levels])
    rp = (C.c_void_p * MAXL)(*[l.ctypes.data for l in right_levels])
    lw = (C.c_int * MAXL)(*[l.shape[1] for l in left_levels])
    lh = (C.c_int * MAXL)(*[l.shape[0] for l in left_levels])
    sc = (C.c_float * MAXL)(*orc.scale.tolist())
    isc = (C.c_float * MAXL)(*orc.inv_scale.tolist())
    kl = np.ascontiguousarray(kl, KP_DTYPE)
    kr = np.ascontiguousarray(kr, KP_DTYPE)
    dl = np.ascontiguousarray(dl, np.uint8)
    dr = np.ascontiguousarray(dr, np.uint8)
    ur = np.zeros(max(1, len(kl)), np.float32)
    dep = np.zeros(max(1, len(kl)), np.float32)
    sad = np.zeros(max(1, len(kl)), np.int32)
    lib().ygzo_stereo_matches(lp, rp, lw, lh, len(left_levels), sc, isc, _p(kl), _p(dl), len(kl), _p(kr), _p(dr),
                              len(kr), C.c_float(mb), C.c_float(mbf), _p(ur), _p(dep), _p(sad))
    n = len(kl)
    return ur[:n], dep[:n], sad[:n]


def stereo_from_rgbd(im_depth, kps, mbf):
    im = np.ascontiguousarray(im_depth, np.float32)
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    ur = np.zeros(max(1, len(kps)), np.float32)
    dep = np.zeros(max(1, len(kps)), np.float32)
    lib().ygzo_stereo_from_rgbd(_p(im), im.shape[1], im.shape[0], im.shape[1], _p(kps), len(kps), C.c_float(mbf),
                                _p(ur), _p(dep))
    return ur[:len(kps)], dep[:len(kps)]


class Vocab:
    """DBoW2 TemplatedVocabulary restated (oracle/bow.c)."""

    def __init__(self, k, L, scoring, weighting, parent, is_leaf, desc, weight):
        lib().ygzo_vocab_create.restype = C.c_void_p
        self.keep = [np.ascontiguousarray(parent, np.int32), np.ascontiguousarray(is_leaf, np.uint8),
                     np.ascontiguousarray(desc, np.uint8), np.ascontiguousarray(weight, np.float64)]
        self.h = C.c_void_p(lib().ygzo_vocab_create(k, L, scoring, weighting, len(parent),
                                                    *[_p(a) for a in self.keep]))
        assert self.h.value

    def __del__(self):
        if getattr(self, "h", None) and self.h.value:
            lib().ygzo_vocab_destroy(self.h)

    def transform_each(self, desc, levelsup=4):
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        w, wt, nid = np.zeros(n, np.int32), np.zeros(n, np.float64), np.zeros(n, np.int32)
        for i in range(n):
            a, b, c = C.c_int(), C.c_double(), C.c_int(0)
            lib().ygzo_bow_transform_one(self.h, _p(d[i]), levelsup, C.byref(a), C.byref(b), C.byref(c))
            w[i], wt[i], nid[i] = a.value, b.value, c.value
        return w, wt, nid

    def transform(self, desc, levelsup=4):
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        m = max(n, 1)
        bw, bv = np.zeros(m, np.int32), np.zeros(m, np.float64)
        fn, ff = np.zeros(m, np.int32), np.zeros(m, np.int32)
        nw, nf = C.c_int(), C.c_int()
        lib().ygzo_compute_bow(self.h, _p(d), n, levelsup, _p(bw), _p(bv), C.byref(nw), _p(fn), _p(ff), C.byref(nf))
        return (bw[:nw.value].copy(), bv[:nw.value].copy()), (fn[:nf.value].copy(), ff[:nf.value].copy())


# ---------------------------------------------------------------- ORBmatcher searches (oracle/match.c)
class MFrame(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("u_right", C.c_void_p), ("n", C.c_int),
                ("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float)]


def mframe(kps, desc, u_right=None, bounds=(0.0, 752.0, 0.0, 480.0)):
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    ur = None if u_right is None else np.ascontiguousarray(u_right, np.float32)
    f = MFrame(kps.ctypes.data, desc.ctypes.data, None if ur is None else ur.ctypes.data, len(kps), *bounds)
    f._keep = (kps, desc, ur)
    return f


def search_projection_best(cur, q, q_desc, blocked=None, th_dist=100, check_ori=True):
    q = np.ascontiguousarray(q)
    d = np.ascontiguousarray(q_desc, np.uint8)
    bl = None if blocked is None else np.ascontiguousarray(blocked, np.uint8)
    out = np.zeros(max(cur.n, 1), np.int32)
    nm = lib().ygzo_search_projection_best(C.byref(cur), _p(q), _p(d), len(q), None if bl is None else _p(bl),
                                           th_dist, int(check_ori), _p(out))
    return out[:cur.n], nm


def search_projection_ratio(F, q, q_desc, blocked=None, nnratio=0.6):
    q = np.ascontiguousarray(q)
    d = np.ascontiguousarray(q_desc, np.uint8)
    bl = None if blocked is None else np.ascontiguousarray(blocked, np.uint8)
    out = np.zeros(max(F.n, 1), np.int32)
    nm = lib().ygzo_search_projection_ratio(C.byref(F), _p(q), _p(d), len(q), None if bl is None else _p(bl),
                                            C.c_float(nnratio), _p(out))
    return out[:F.n], nm


def search_for_initialization(F1, F2, prev, window=100, nnratio=0.9, check_ori=True):
    prev = np.ascontiguousarray(prev, np.float32).reshape(-1, 2).copy()
    m12 = np.zeros(max(F1.n, 1), np.int32)
    nm = lib().ygzo_search_for_initialization(C.byref(F1), C.byref(F2), _p(prev), window, C.c_float(nnratio),
                                              int(check_ori), _p(m12))
    return m12[:F1.n], nm, prev


def search_by_bow(kf, F, kf_usable, fv_kf, fv_f, nnratio=0.7, check_ori=False):
    us = np.ascontiguousarray(kf_usable, np.uint8)
    kn, kp, kfe = (np.ascontiguousarray(a, np.int32) for a in fv_kf)
    fn, fp, ffe = (np.ascontiguousarray(a, np.int32) for a in fv_f)
    out = np.zeros(max(F.n, 1), np.int32)
    nm = lib().ygzo_search_by_bow(C.byref(kf), C.byref(F), _p(us), len(kn), _p(kn), _p(kp), _p(kfe), len(fn), _p(fn),
                                  _p(fp), _p(ffe), C.c_float(nnratio), int(check_ori), _p(out))
    return out[:F.n], nm


def features_in_area(F, x, y, r, min_level=-1, max_level=-1):
    out = np.zeros(max(F.n, 1), np.int32)
    n = lib().ygzo_features_in_area(C.byref(F), C.c_float(x), C.c_float(y), C.c_float(r), int(min_level), int(max_level),
                                    _p(out))
    return out[:n]


class RefFast:
    """The reference's own Thirdparty/fast, compiled by oracle/Makefile (oracle/_ref)."""

    def __init__(self):
        self.lib = C.CDLL(REF_FAST_PATH)

    @staticmethod
    def available():
        return os.path.exists(REF_FAST_PATH)

    def pipeline_bench(self, img, barrier, x0, y0, w, h, reps=20):
        """The reference's detect_sse2 + score + nonmax_3x3, timed in C++ -> (kept corners, mean seconds)."""
        img = np.ascontiguousarray(img, np.uint8)
        W = img.shape[1]
        s = C.c_double()
        n = self.lib.ref_fast10_pipeline_bench(C.c_void_p(img.ctypes.data + y0 * W + x0), w, h, W, barrier, reps,
                                               C.byref(s))
        return n, s.value

    def detect(self, img, barrier, sse=True, x0=0, y0=0, w=None, h=None, cap=1 << 20):
        img = np.ascontiguousarray(img, np.uint8)
        H, W = img.shape
        w = W - x0 if w is None else w
        h = H - y0 if h is None else h
        xs = np.zeros(cap, np.int16)
        ys = np.zeros(cap, np.int16)
        ptr = C.c_void_p(img.ctypes.data + y0 * W + x0)
        n = self.lib.ref_fast10_detect(ptr, w, h, W, barrier, int(sse), _p(xs), _p(ys), cap)
        return xs[:n].copy(), ys[:n].copy()

    def scores(self, img, xs, ys, threshold, x0=0, y0=0):
        img = np.ascontiguousarray(img, np.uint8)
        W = img.shape[1]
        xs = np.ascontiguousarray(xs, np.int16)
        ys = np.ascontiguousarray(ys, np.int16)
        out = np.zeros(len(xs), np.int32)
        ptr = C.c_void_p(img.ctypes.data + y0 * W + x0)
        self.lib.ref_fast10_score(ptr, W, _p(xs), _p(ys), len(xs), threshold, _p(out))
        return out

    def nonmax(self, xs, ys, scores):
        xs = np.ascontiguousarray(xs, np.int16)
        ys = np.ascontiguousarray(ys, np.int16)
        scores = np.ascontiguousarray(scores, np.int32)
        keep = np.zeros(max(1, len(xs)), np.int32)
        n = self.lib.ref_fast10_nonmax(_p(xs), _p(ys), _p(scores), len(xs), _p(keep))
        return keep[:n].copy()


# ---------------------------------------------------------------- CPU baseline driver (oracle/bench.c)
class BenchStats(C.Structure):
    _fields_ = [("t_pyr", C.c_double), ("t_extract", C.c_double), ("t_hamming", C.c_double), ("t_align", C.c_double),
                ("frames", C.c_int), ("pairs", C.c_int), ("keypoints", C.c_longlong), ("visible", C.c_longlong)]


def bench_pipeline(frames, cam, plane_z, r3, cz, cfg, threads=1):
    """The per-frame hot path of the restatement over frames[n][H][W] on `threads`
    host threads (contiguous chunks) -> (wall seconds, BenchStats)."""
    frames = np.ascontiguousarray(frames, np.uint8)
    n, H, W = frames.shape
    W_, H_, nf, sf, nl, ini, mn = cfg
    c = (C.c_float * 4)(*[float(v) for v in cam])
    r3 = np.ascontiguousarray(r3, np.float32)
    cz = np.ascontiguousarray(cz, np.float32)
    st = BenchStats()
    L = lib()
    L.ygzo_bench_pipeline.restype = C.c_double
    wall = L.ygzo_bench_pipeline(_p(frames), n, W, H, c, C.c_float(plane_z), _p(r3), _p(cz), nf, C.c_float(sf), nl,
                                 ini, mn, threads, C.byref(st))
    return wall, st


def bench_fast9(img, threshold, reps=20):
    """cv::FAST(img, threshold, nonmax) restated, timed -> (corners, mean seconds)."""
    img = np.ascontiguousarray(img, np.uint8)
    s = C.c_double()
    n = lib().ygzo_bench_fast9(_p(img), img.shape[1], img.shape[0], threshold, reps, C.byref(s))
    return n, s.value
