"""ygzfe — Python view of the MI355X front-end C ABI (include/ygzfe.h).

Mirrors the reference's hot-path interfaces so tests read like the reference:
  ORBextractor      ORBextractor.h:37-192   (ctor, operator(), ComputePyramid, getters)
  Frame             Frame::mvImagePyramid   (device-resident pyramid)
  ORBmatcher        ORBmatcher.h:38-178     (DescriptorDistance, dense / windowed search)
  SparseImgAlign    SparseImageAlign.h:37-60 (run)
  Align2D / FindDirectProjection            Align.h:20-26, ORBmatcher.cc:1573-1602
  Batch             many frames resident in HBM (bench / multi-GPU path)

All compute runs in lib/libygzfe.so on the GPU; there is no CPU fallback: the
module raises if the library or a HIP device is missing.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("YGZFE_LIB") or os.path.join(PKG_ROOT, "lib", "libygzfe.so")  # YGZFE_LIB: A/B builds
SYNTH_PATH = os.path.join(PKG_ROOT, "lib", "libygzsynth.so")
SYNTH_HIP_PATH = os.path.join(PKG_ROOT, "lib", "libygzsynth_hip.so")

MAX_LEVELS = 16
ORBSLAM_KEYPOINT, FAST_KEYPOINT, DSO_KEYPOINT = 0, 1, 2
BLUR_CV4, BLUR_CV3 = 0, 1
OK, EINVAL, EHIP, ECAP, ENOMEM, ESTATE = 0, -1, -2, -3, -4, -5

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


class YgzfeError(RuntimeError):
    pass


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32), ("blur_variant", C.c_int32)]


class Camera(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float)]


class SE3(C.Structure):
    _fields_ = [("q", C.c_float * 4), ("t", C.c_float * 3)]

    @staticmethod
    def make(q=(0, 0, 0, 1), t=(0, 0, 0)):
        s = SE3()
        for i in range(4):
            s.q[i] = float(q[i])
        for i in range(3):
            s.t[i] = float(t[i])
        return s

    def as_arrays(self):
        return np.array(self.q[:], np.float32), np.array(self.t[:], np.float32)


class AlignResult(C.Structure):
    _fields_ = [("T_cur_ref", SE3), ("n_visible", C.c_int32), ("chi2", C.c_float), ("H", C.c_float * 36)]


SE3_DTYPE = np.dtype([("q", "<f4", 4), ("t", "<f4", 3)])
ALIGN_RESULT_DTYPE = np.dtype([("q", "<f4", 4), ("t", "<f4", 3), ("n_visible", "<i4"), ("chi2", "<f4"),
                               ("H", "<f4", 36)])

_lib = None


def lib():
    """Load libygzfe.so; raise loudly when it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise YgzfeError(f"{LIB_PATH} missing: run `make -C orb-ygz-slam_amd` (or __graft_entry__.build())")
        # torch ships its own libamdhip64.so.7; whichever copy loads first
        # serves the whole process, and torch refuses to run on a runtime it
        # was not built with.  Load torch's first so device pointers and
        # streams can be shared with it later in the same process.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        L.ygzfe_last_error.restype = C.c_char_p
        L.ygzfe_batch_stream.restype = C.c_void_p
        _lib = L
    return _lib


def _check(rc, what=""):
    if rc != OK:
        msg = lib().ygzfe_last_error().decode(errors="replace")
        raise YgzfeError(f"{what} failed ({rc}): {msg}")
    return rc


def _p(a):
    return C.c_void_p(a.ctypes.data)


def device_count():
    return lib().ygzfe_device_count()


def slot_bytes(kp_cap):
    """Bytes of one offline-sequence result slot (ygzfe_slot_bytes)."""
    L = lib()
    L.ygzfe_slot_bytes.restype = C.c_size_t
    return int(L.ygzfe_slot_bytes(kp_cap))


def orb_plan(nfeatures, scale_factor, nlevels, ini_th=20, min_th=7, width=752, height=480, blur=BLUR_CV4):
    """Host-only extraction plan (ygzfe_orb_plan): level sizes, budgets, FAST cells, umax."""
    p = OrbParams(nfeatures, scale_factor, nlevels, ini_th, min_th, blur)
    w, h, b, nc = (np.zeros(nlevels, np.int32) for _ in range(4))
    um = np.zeros(16, np.int32)
    _check(lib().ygzfe_orb_plan(C.byref(p), width, height, _p(w), _p(h), _p(b), _p(nc), _p(um)), "orb_plan")
    return {"sizes": list(zip(w.tolist(), h.tolist())), "budget": b.tolist(), "ncells": nc.tolist(),
            "umax": um.tolist()}


class Frame:
    """Device-resident pyramid (Frame::mvImagePyramid)."""

    def __init__(self, extractor, width, height):
        self.ex = extractor
        self.width, self.height = width, height
        self.h = C.c_void_p()
        _check(lib().ygzfe_frame_create(extractor.h, width, height, C.byref(self.h)), "frame_create")

    def __del__(self):
        if getattr(self, "h", None) and self.h.value and _lib is not None:
            _lib.ygzfe_frame_destroy(self.h)
            self.h = None

    def level(self, l):
        w = C.c_int()
        h = C.c_int()
        _check(lib().ygzfe_frame_level(self.h, l, C.byref(w), C.byref(h), None, 0), "frame_level")
        out = np.zeros((h.value, w.value), np.uint8)
        _check(lib().ygzfe_frame_level(self.h, l, None, None, _p(out), w.value), "frame_level")
        return out

    def levels(self):
        return [self.level(l) for l in range(self.ex.nlevels)]

    def set_level(self, l, img):
        img = np.ascontiguousarray(img, np.uint8)
        _check(lib().ygzfe_frame_set_level(self.h, l, _p(img), img.shape[1]), "frame_set_level")


class ORBextractor:
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) (ORBextractor.h:53-57)."""

    def __init__(self, nfeatures=500, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7, device=0,
                 blur=BLUR_CV4):
        self.params = OrbParams(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, blur)
        self.nlevels = nlevels
        self.h = C.c_void_p()
        _check(lib().ygzfe_extractor_create(C.byref(self.params), device, C.byref(self.h)), "extractor_create")

    def __del__(self):
        if getattr(self, "h", None) and self.h.value and _lib is not None:
            _lib.ygzfe_extractor_destroy(self.h)
            self.h = None

    # getters (ORBextractor.h:87-109)
    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return self.params.scale_factor

    def _levels(self):
        arrs = [np.zeros(MAX_LEVELS, np.float32) for _ in range(4)]
        _check(lib().ygzfe_extractor_levels(self.h, None, *[_p(a) for a in arrs]), "levels")
        return [a[:self.nlevels] for a in arrs]

    def GetScaleFactors(self):
        return self._levels()[0]

    def GetInverseScaleFactors(self):
        return self._levels()[1]

    def GetScaleSigmaSquares(self):
        return self._levels()[2]

    def GetInverseScaleSigmaSquares(self):
        return self._levels()[3]

    def FeaturesPerLevel(self):
        out = np.zeros(MAX_LEVELS, np.int32)
        _check(lib().ygzfe_extractor_features_per_level(self.h, _p(out)), "features_per_level")
        return out[:self.nlevels].tolist()

    @property
    def dso_grid(self):
        g = C.c_int32()
        _check(lib().ygzfe_extractor_dso_grid(self.h, C.byref(g), None), "dso_grid")
        return g.value

    @dso_grid.setter
    def dso_grid(self, v):
        g = C.c_int32(v)
        _check(lib().ygzfe_extractor_dso_grid(self.h, None, C.byref(g)), "dso_grid")

    def ComputePyramid(self, image, frame=None):
        """Frame::ComputeImagePyramid -> a device Frame holding mvImagePyramid."""
        image = np.ascontiguousarray(image, np.uint8)
        H, W = image.shape
        frame = frame if frame is not None else Frame(self, W, H)
        _check(lib().ygzfe_compute_pyramid(self.h, frame.h, _p(image), W), "compute_pyramid")
        return frame

    def extract(self, frame, method=ORBSLAM_KEYPOINT, existing=None, cap=None):
        """operator()(Frame*, keypoints, descriptors, method) (ORBextractor.cc:1031-1127).

        Returns (keypoints[KP_DTYPE], descriptors uint8[n,32]); rows of `existing`
        come first (their angles are recomputed in DSO mode, as the reference does)."""
        existing = np.zeros(0, KP_DTYPE) if existing is None else np.ascontiguousarray(existing, KP_DTYPE)
        ne = len(existing)
        cap = cap or (ne + 8192)
        kps = np.zeros(cap, KP_DTYPE)
        kps[:ne] = existing
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int()
        rc = lib().ygzfe_extract(self.h, frame.h, method, _p(kps), ne, cap, _p(desc), C.byref(n))
        if rc == ECAP:
            return self.extract(frame, method, existing, cap=n.value)
        _check(rc, "extract")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def __call__(self, image, mask=None):
        """operator()(image, mask, keypoints, descriptors) (ORBextractor.cc:970-1028)."""
        frame = self.ComputePyramid(image)
        return self.extract(frame, ORBSLAM_KEYPOINT)


def debug_dso_cells(img, g, barrier, device=0):
    """The DSO_KEYPOINT cell kernel's own FAST-10 pass (ygzfe_debug_dso_cells): for each g x g
    cell of the grid, row-major, the cell-relative corners in raster order (int16[n, 2] (x, y)),
    from one pass at `barrier` over the kernel's scan region; border cells are empty."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    ncells = (H // g) * (W // g)
    flags = np.zeros((max(ncells, 1), g, g), np.uint8)
    _check(lib().ygzfe_debug_dso_cells(device, _p(img), W, H, int(g), int(barrier), _p(flags)), "debug_dso_cells")
    out = []
    for k in range(ncells):
        ys, xs = np.nonzero(flags[k])  # raster order (row-major nonzero)
        out.append(np.stack([xs, ys], 1).astype(np.int16))
    return out


def fast10_detect(img, barrier, rois, sse=True, cap=None, device=0):
    """Thirdparty/fast FAST-10 on the GPU (ygzfe_fast10_detect): fast_corner_detect_10_sse2 (sse) or
    fast_corner_detect_10 over each ROI (x0, y0, w, h) of `img` -> list of int16[n, 2] (x, y) corner
    arrays, ROI-relative and in the reference's raster order.  `cap` (corners per ROI) defaults to
    1 << 16 bounded by the largest ROI's pixel count; when a ROI holds more, the call is repeated
    once with the cap the first call's counts report (ygzfe.h: ECAP, counts = corners found)."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    rois = np.ascontiguousarray(rois, np.int32).reshape(-1, 4)
    n = len(rois)
    area = max(1, int((rois[:, 2].clip(0) * rois[:, 3].clip(0)).max())) if n else 1
    retry = cap is None
    cap = min(area, 1 << 16) if cap is None else cap
    while True:
        xy = np.zeros((max(n, 1), cap, 2), np.int16)
        counts = np.zeros(max(n, 1), np.int32)
        rc = lib().ygzfe_fast10_detect(device, _p(img), W, H, W, _p(rois), n, int(barrier), int(bool(sse)), _p(xy),
                                       cap, _p(counts))
        if rc == ECAP and retry:
            retry = False
            cap = int(counts.max())
            continue
        _check(rc, "fast10_detect")
        break
    return [xy[r, :counts[r]].copy() for r in range(n)]


class Undistort:
    """Frame::ComputeImagePyramid's undistortion (Frame.cc:775-790): the CV_16SC2
    initUndistortRectifyMap maps, built on the device once per camera, and the
    INTER_LINEAR remap applied per frame."""

    def __init__(self, cam, dist, width, height, device=0):
        cam = cam if isinstance(cam, Camera) else Camera(*[float(c) for c in cam])
        d = np.ascontiguousarray(dist, np.float32).ravel()
        self.width, self.height, self.device = width, height, device
        self.h = C.c_void_p()
        _check(lib().ygzfe_undistort_create(device, C.byref(cam), _p(d) if len(d) else None, len(d), width, height,
                                            C.byref(self.h)), "undistort_create")

    def __del__(self):
        if getattr(self, "h", None) and self.h.value and _lib is not None:
            _lib.ygzfe_undistort_destroy(self.h)
            self.h = None

    def maps(self):
        """(map1 int16[H, W, 2], map2 uint16[H, W]) -- OpenCV's CV_16SC2 + CV_16UC1 pair."""
        m1 = np.zeros((self.height, self.width, 2), np.int16)
        m2 = np.zeros((self.height, self.width), np.uint16)
        _check(lib().ygzfe_undistort_maps(self.h, _p(m1), _p(m2)), "undistort_maps")
        return m1, m2

    def apply_device(self, d_src, src_pitch, src_stride, d_dst, dst_pitch, dst_stride, n_images, stream=None):
        _check(lib().ygzfe_undistort_apply_device(self.h, C.c_void_p(d_src), C.c_size_t(src_pitch), src_stride,
                                                  C.c_void_p(d_dst), C.c_size_t(dst_pitch), dst_stride, n_images,
                                                  C.c_void_p(stream)), "undistort_apply")

    def apply_f32_device(self, d_src, src_pitch, src_stride, d_dst, dst_pitch, dst_stride, n_images, stream=None):
        """remap of n CV_32F device images (pitch / stride in floats): Frame.cc:799-804."""
        _check(lib().ygzfe_undistort_apply_f32_device(self.h, C.c_void_p(d_src), C.c_size_t(src_pitch), src_stride,
                                                      C.c_void_p(d_dst), C.c_size_t(dst_pitch), dst_stride, n_images,
                                                      C.c_void_p(stream)), "undistort_apply_f32")

    def remap_image(self, image):
        """cv::remap(mImGray / mImRight, ..., INTER_LINEAR) on a host u8 image (Frame.cc:786-797)."""
        image = np.ascontiguousarray(image, np.uint8)
        out = np.zeros_like(image)
        _check(lib().ygzfe_undistort_image(self.h, _p(image), image.shape[1], _p(out), out.shape[1]), "undistort_image")
        return out

    def remap_depth(self, depth):
        """cv::remap(mImDepth, ..., INTER_LINEAR) on a host CV_32F depth image (Frame.cc:799-804)."""
        depth = np.ascontiguousarray(depth, np.float32)
        out = np.zeros_like(depth)
        _check(lib().ygzfe_undistort_depth(self.h, _p(depth), depth.shape[1], _p(out), out.shape[1]), "undistort_depth")
        return out

    def ComputePyramid(self, extractor, image, frame=None):
        """ComputeImagePyramid with mDistCoef != 0: remap(image) -> level 0 -> levels."""
        image = np.ascontiguousarray(image, np.uint8)
        H, W = image.shape
        frame = frame if frame is not None else Frame(extractor, W, H)
        _check(lib().ygzfe_compute_pyramid_undistorted(extractor.h, frame.h, self.h, _p(image), W),
               "compute_pyramid_undistorted")
        return frame


class ORBmatcher:
    """Hamming hot subset of ORBmatcher (ORBmatcher.h:38-178)."""

    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30

    def __init__(self, nnratio=0.6, checkOri=True, device=0):
        self.nnratio, self.checkOri, self.device = nnratio, checkOri, device

    @staticmethod
    def DescriptorDistance(a, b):
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return lib().ygzfe_descriptor_distance(_p(a), _p(b))

    def best2(self, query, train):
        q = np.ascontiguousarray(query, np.uint8).reshape(-1, 32)
        t = np.ascontiguousarray(train, np.uint8).reshape(-1, 32)
        nq = len(q)
        bi = np.zeros(nq, np.int32)
        bd = np.zeros(nq, np.int32)
        sd = np.zeros(nq, np.int32)
        _check(lib().ygzfe_hamming_best2(self.device, _p(q), nq, _p(t), len(t), _p(bi), _p(bd), _p(sd)),
               "hamming_best2")
        return bi, bd, sd

    def window_distances(self, query, train, row_ptr, cand):
        q = np.ascontiguousarray(query, np.uint8).reshape(-1, 32)
        t = np.ascontiguousarray(train, np.uint8).reshape(-1, 32)
        row_ptr = np.ascontiguousarray(row_ptr, np.int32)
        cand = np.ascontiguousarray(cand, np.int32)
        out = np.zeros(max(1, len(cand)), np.int32)
        _check(lib().ygzfe_hamming_csr(self.device, _p(q), len(q), _p(t), len(t), _p(row_ptr), _p(cand), _p(out)),
               "hamming_csr")
        return out[:len(cand)]


MATCH_QUERY_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("radius", "<f4"), ("u_right", "<f4"),
                              ("min_level", "<i4"), ("max_level", "<i4"), ("angle", "<f4"), ("flags", "<i4")])
MQ_VALID, MQ_BLOCKS, MQ_STEREO = 1, 2, 4


class Bounds(C.Structure):
    """Frame::mnMinX / mnMaxX / mnMinY / mnMaxY (Frame.cc:501-507)."""
    _fields_ = [("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float)]


class MatchFrame:
    """The searched Frame's state on the device (mvKeys, mDescriptors, mvuRight, bounds;
    the 64 x 48 grid of AssignFeaturesToGrid is built there)."""

    def __init__(self, device=0):
        self.h = C.c_void_p()
        _check(lib().ygzfe_match_frame_create(device, C.byref(self.h)), "match_frame_create")
        self.n = 0

    def __del__(self):
        if getattr(self, "h", None) and self.h.value and _lib is not None:
            _lib.ygzfe_match_frame_destroy(self.h)
            self.h = None

    def set(self, kps, desc, u_right=None, bounds=(0.0, 752.0, 0.0, 480.0)):
        kps = np.ascontiguousarray(kps, KP_DTYPE)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        ur = None if u_right is None else np.ascontiguousarray(u_right, np.float32)
        b = Bounds(*[float(x) for x in bounds])
        _check(lib().ygzfe_match_frame_set(self.h, _p(kps), _p(desc), len(kps), None if ur is None else _p(ur),
                                           C.byref(b)), "match_frame_set")
        self.n = len(kps)
        return self

    def rescans(self):
        """Queries of the last search whose top-K candidates the sequential skips used up."""
        r = C.c_int()
        _check(lib().ygzfe_match_frame_stats(self.h, C.byref(r)), "match_frame_stats")
        return r.value

    def resolve_passes(self):
        """Parallel-resolve passes of the last search (-1: the serial replay decided)."""
        r = C.c_int()
        _check(lib().ygzfe_match_frame_resolve_stats(self.h, C.byref(r)), "match_frame_resolve_stats")
        return r.value

    def from_batch(self, batch, frame, bounds=(0.0, 752.0, 0.0, 480.0)):
        b = Bounds(*[float(x) for x in bounds])
        _check(lib().ygzfe_match_frame_from_batch(self.h, batch.h, frame, C.byref(b)), "match_frame_from_batch")
        return self


def search_projection_best(cur, queries, q_desc, blocked=None, th_dist=100, check_ori=True):
    """SearchByProjection(CurrentFrame, LastFrame | pKF, ...) (ORBmatcher.cc:1218-1469):
    -> (train_match int32[cur.n]: -1 untouched / -2 NULLed by the rotation check / query, nmatches)."""
    q = np.ascontiguousarray(queries, MATCH_QUERY_DTYPE)
    d = np.ascontiguousarray(q_desc, np.uint8).reshape(-1, 32)
    bl = None if blocked is None else np.ascontiguousarray(blocked, np.uint8)
    out = np.zeros(max(cur.n, 1), np.int32)
    nm = C.c_int()
    _check(lib().ygzfe_search_projection_best(cur.h, _p(q), _p(d), len(q), None if bl is None else _p(bl), th_dist,
                                              int(check_ori), _p(out), C.byref(nm)), "search_projection_best")
    return out[:cur.n], nm.value


def search_projection_ratio(F, queries, q_desc, blocked=None, nnratio=0.6):
    """SearchByProjection(F, vpMapPoints, th, checkLevel) (ORBmatcher.cc:43-126) -> (train_match, nmatches)."""
    q = np.ascontiguousarray(queries, MATCH_QUERY_DTYPE)
    d = np.ascontiguousarray(q_desc, np.uint8).reshape(-1, 32)
    bl = None if blocked is None else np.ascontiguousarray(blocked, np.uint8)
    out = np.zeros(max(F.n, 1), np.int32)
    nm = C.c_int()
    _check(lib().ygzfe_search_projection_ratio(F.h, _p(q), _p(d), len(q), None if bl is None else _p(bl),
                                               C.c_float(nnratio), _p(out), C.byref(nm)), "search_projection_ratio")
    return out[:F.n], nm.value


def search_for_initialization(F1, F2, prev_matched, window_size=100, nnratio=0.9, check_ori=True):
    """SearchForInitialization (ORBmatcher.cc:375-478) -> (vnMatches12, nmatches, vbPrevMatched updated)."""
    prev = np.ascontiguousarray(prev_matched, np.float32).reshape(-1, 2).copy()
    m12 = np.zeros(max(F1.n, 1), np.int32)
    nm = C.c_int()
    _check(lib().ygzfe_search_for_initialization(F1.h, F2.h, _p(prev), window_size, C.c_float(nnratio),
                                                 int(check_ori), _p(m12), C.byref(nm)), "search_for_initialization")
    return m12[:F1.n], nm.value, prev


def search_by_bow(kf, F, kf_usable, fv_kf, fv_f, nnratio=0.7, check_ori=False):
    """SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.cc:155-263).  fv_* = (nodes, ptr, feats)
    node-sorted CSR FeatureVectors -> (f_match int32[F.n]: KF index or -1, nmatches)."""
    us = np.ascontiguousarray(kf_usable, np.uint8)
    kn, kp, kfe = (np.ascontiguousarray(a, np.int32) for a in fv_kf)
    fn, fp, ffe = (np.ascontiguousarray(a, np.int32) for a in fv_f)
    out = np.zeros(max(F.n, 1), np.int32)
    nm = C.c_int()
    _check(lib().ygzfe_search_by_bow(kf.h, F.h, _p(us), len(kn), _p(kn), _p(kp), _p(kfe), len(fn), _p(fn), _p(fp),
                                     _p(ffe), C.c_float(nnratio), int(check_ori), _p(out), C.byref(nm)),
           "search_by_bow")
    return out[:F.n], nm.value


class SparseImgAlign:
    """SparseImgAlign(n_levels, min_level, n_iter=10, method=GaussNewton) (SparseImageAlign.h:37-60)."""
    GaussNewton, LevenbergMarquardt = 0, 1  # NLLSSolver's methods (NLSSolver.h:40-43)

    def __init__(self, max_level, min_level, n_iter=10, method=0):
        self.max_level, self.min_level, self.method = max_level, min_level, int(method)

    def run(self, ref_frame, cur_frame, cam, kps, xyz_ref, usable, T_init):
        kps = np.ascontiguousarray(kps, KP_DTYPE)
        xyz = np.ascontiguousarray(xyz_ref, np.float32).reshape(-1, 3)
        us = np.ascontiguousarray(usable, np.uint8)
        res = AlignResult()
        _check(lib().ygzfe_sparse_align_method(ref_frame.h, cur_frame.h, C.byref(cam), _p(kps), _p(xyz), _p(us),
                                               len(kps), self.max_level, self.min_level, C.byref(T_init),
                                               self.method, C.byref(res)),
               "sparse_align")
        return res


def align2d_batch(cur_frame, level, patches_with_border, patches, px, n_iter=10):
    pwb = np.ascontiguousarray(patches_with_border, np.uint8).reshape(-1, 100)
    p = np.ascontiguousarray(patches, np.uint8).reshape(-1, 64)
    px = np.ascontiguousarray(px, np.float32).reshape(-1, 2).copy()
    conv = np.zeros(len(px), np.uint8)
    _check(lib().ygzfe_align2d_batch(cur_frame.h, level, len(px), _p(pwb), _p(p), n_iter, _p(px), _p(conv)),
           "align2d_batch")
    return conv.astype(bool), px


def find_direct_projection_batch(ref_frames, cur_frame, cam, ref_index, kp_ref, pt_ref, T_cr, px):
    refs = (C.c_void_p * len(ref_frames))(*[f.h.value for f in ref_frames])
    ref_index = np.ascontiguousarray(ref_index, np.int32)
    kp_ref = np.ascontiguousarray(kp_ref, KP_DTYPE)
    pt_ref = np.ascontiguousarray(pt_ref, np.float32).reshape(-1, 3)
    T_cr = np.ascontiguousarray(T_cr, SE3_DTYPE)
    px = np.ascontiguousarray(px, np.float32).reshape(-1, 2).copy()
    n = len(px)
    lvl = np.zeros(n, np.int32)
    ok = np.zeros(n, np.uint8)
    _check(lib().ygzfe_find_direct_projection_batch(refs, cur_frame.h, C.byref(cam), n, _p(ref_index), _p(kp_ref),
                                                    _p(pt_ref), _p(T_cr), _p(px), _p(lvl), _p(ok)),
           "find_direct_projection_batch")
    return px, lvl, ok.astype(bool)


def stereo_matches(left_frame, right_frame, kl, dl, kr, dr, mb, mbf):
    """Frame::ComputeStereoMatches (Frame.cc:509-682) -> (mvuRight, mvDepth), float32[nl], -1 = none."""
    kl = np.ascontiguousarray(kl, KP_DTYPE)
    kr = np.ascontiguousarray(kr, KP_DTYPE)
    dl = np.ascontiguousarray(dl, np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(dr, np.uint8).reshape(-1, 32)
    ur = np.zeros(len(kl), np.float32)
    dep = np.zeros(len(kl), np.float32)
    _check(lib().ygzfe_stereo_matches(left_frame.h, right_frame.h, _p(kl), _p(dl), len(kl), _p(kr), _p(dr), len(kr),
                                      C.c_float(mb), C.c_float(mbf), _p(ur), _p(dep)), "stereo_matches")
    return ur, dep


def stereo_from_rgbd(im_depth, kps, mbf, device=0):
    """Frame::ComputeStereoFromRGBD (Frame.cc:684-700) -> (mvuRight, mvDepth)."""
    im = np.ascontiguousarray(im_depth, np.float32)
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    ur = np.zeros(len(kps), np.float32)
    dep = np.zeros(len(kps), np.float32)
    _check(lib().ygzfe_stereo_from_rgbd(device, _p(im), im.shape[1], im.shape[0], im.shape[1], _p(kps), len(kps),
                                        C.c_float(mbf), _p(ur), _p(dep)), "stereo_from_rgbd")
    return ur, dep


class Vocabulary:
    """ORBVocabulary = TemplatedVocabulary<FORB::TDescriptor, FORB> (Thirdparty/DBoW2) in HBM."""

    def __init__(self, handle, device):
        self.h, self.device = handle, device
        v = [C.c_int() for _ in range(6)]
        _check(lib().ygzfe_vocab_info(self.h, *[C.byref(x) for x in v]), "vocab_info")
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words = [x.value for x in v]

    @classmethod
    def from_arrays(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight, device=0):
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        weight = np.ascontiguousarray(weight, np.float64)
        h = C.c_void_p()
        _check(lib().ygzfe_vocab_create(device, k, L, scoring, weighting, len(parent), _p(parent), _p(is_leaf),
                                        _p(desc), _p(weight), C.byref(h)), "vocab_create")
        return cls(h, device)

    @classmethod
    def load_text(cls, path, device=0):
        """loadFromTextFile (TemplatedVocabulary.h:1362)."""
        h = C.c_void_p()
        _check(lib().ygzfe_vocab_load_text(device, str(path).encode(), C.byref(h)), "vocab_load_text")
        return cls(h, device)

    @classmethod
    def load_binary(cls, path, device=0):
        """loadFromBinaryFile (TemplatedVocabulary.h:1478)."""
        h = C.c_void_p()
        _check(lib().ygzfe_vocab_load_binary(device, str(path).encode(), C.byref(h)), "vocab_load_binary")
        return cls(h, device)

    def __del__(self):
        if getattr(self, "h", None) and self.h.value and _lib is not None:
            _lib.ygzfe_vocab_destroy(self.h)
            self.h = None

    def transform_each(self, desc, levelsup=4):
        """transform(feature, word, weight, &nid, levelsup) per descriptor -> (word, weight, nid)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        w = np.zeros(n, np.int32)
        wt = np.zeros(n, np.float64)
        nid = np.zeros(n, np.int32)
        _check(lib().ygzfe_bow_transform(self.h, _p(d), n, levelsup, _p(w), _p(wt), _p(nid)), "bow_transform")
        return w, wt, nid

    def transform(self, desc, levelsup=4):
        """Frame::ComputeBoW -> (BowVector {word: value}, FeatureVector {node: [features]}), as
        (words int32[], values float64[]) and (nodes int32[], features int32[]) in map order."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        m = max(n, 1)
        bw, bv = np.zeros(m, np.int32), np.zeros(m, np.float64)
        fn, ff = np.zeros(m, np.int32), np.zeros(m, np.int32)
        nw, nf = C.c_int(), C.c_int()
        _check(lib().ygzfe_compute_bow(self.h, _p(d), n, levelsup, _p(bw), _p(bv), C.byref(nw), _p(fn), _p(ff),
                                       C.byref(nf)), "compute_bow")
        return (bw[:nw.value].copy(), bv[:nw.value].copy()), (fn[:nf.value].copy(), ff[:nf.value].copy())


def search_direct_batch(ref_frames, cur_frame, cam, item_ptr, ref_index, kp_ref, pt_ref, T_cr, px_proj, border=20.0):
    """Tracking::SearchLocalPointsDirect's per-point search (Tracking.cc:2337-2395), batched:
    point i tries items [item_ptr[i], item_ptr[i+1]) (its keyframes in SelectNearestKeyframe
    order) with FindDirectProjection from px_proj[i] and keeps the first converged pixel inside
    the border.  Returns (px_out float32[n,2], matched_item int32[n], -1 = no match)."""
    refs = (C.c_void_p * max(1, len(ref_frames)))(*[f.h.value for f in ref_frames])
    item_ptr = np.ascontiguousarray(item_ptr, np.int32)
    n = len(item_ptr) - 1
    ref_index = np.ascontiguousarray(ref_index, np.int32)
    kp_ref = np.ascontiguousarray(kp_ref, KP_DTYPE)
    pt_ref = np.ascontiguousarray(pt_ref, np.float32).reshape(-1, 3)
    T_cr = np.ascontiguousarray(T_cr, SE3_DTYPE)
    px_proj = np.ascontiguousarray(px_proj, np.float32).reshape(-1, 2)
    px_out = np.zeros((max(n, 0), 2), np.float32)
    matched = np.zeros(max(n, 0), np.int32)
    _check(lib().ygzfe_search_direct_batch(refs, len(ref_frames), cur_frame.h, C.byref(cam), n, _p(item_ptr),
                                           _p(ref_index), _p(kp_ref), _p(pt_ref), _p(T_cr), _p(px_proj),
                                           C.c_float(border), _p(px_out), _p(matched)),
           "search_direct_batch")
    return px_out, matched


DIRECT_FAILED, DIRECT_MATCHED, DIRECT_GRID_SKIP, DIRECT_NOT_RUN = 0, 1, 2, 3


def search_local_points_direct(ref_frames, cur_frame, cam, n_cache, item_ptr, ref_index, kp_ref, pt_ref, T_cr,
                               px_proj, border=20.0, grid_size=5, cache_hit_th=150):
    """Tracking::SearchLocalPointsDirect (Tracking.cc:2258-2410) whole: points [0, n_cache) are the
    cache (5-px coverage grid, replayed in order), the rest the local-map points (searched only
    when the cache gave <= cache_hit_th successes).  Returns (px_out float32[n,2], matched_item
    int32[n], status int32[n] (DIRECT_*), cache_success, local_ran)."""
    refs = (C.c_void_p * max(1, len(ref_frames)))(*[f.h.value for f in ref_frames])
    item_ptr = np.ascontiguousarray(item_ptr, np.int32)
    n = len(item_ptr) - 1
    ref_index = np.ascontiguousarray(ref_index, np.int32)
    kp_ref = np.ascontiguousarray(kp_ref, KP_DTYPE)
    pt_ref = np.ascontiguousarray(pt_ref, np.float32).reshape(-1, 3)
    T_cr = np.ascontiguousarray(T_cr, SE3_DTYPE)
    px_proj = np.ascontiguousarray(px_proj, np.float32).reshape(-1, 2)
    px_out = np.zeros((max(n, 0), 2), np.float32)
    matched = np.zeros(max(n, 0), np.int32)
    status = np.zeros(max(n, 0), np.int32)
    cs, lr = C.c_int(), C.c_int()
    _check(lib().ygzfe_search_local_points_direct(refs, len(ref_frames), cur_frame.h, C.byref(cam), int(n_cache),
                                                  n - int(n_cache), _p(item_ptr), _p(ref_index), _p(kp_ref),
                                                  _p(pt_ref), _p(T_cr), _p(px_proj), C.c_float(border), int(grid_size),
                                                  int(cache_hit_th), _p(px_out), _p(matched), _p(status),
                                                  C.byref(cs), C.byref(lr)),
           "search_local_points_direct")
    return px_out, matched, status, cs.value, bool(lr.value)


class Batch:
    """Frames resident in HBM, one launch per stage (the bench / multi-GPU path)."""

    def __init__(self, params_or_extractor_args, device, width, height, max_frames):
        p = params_or_extractor_args
        if not isinstance(p, OrbParams):
            p = OrbParams(*p)
        self.params = p
        self.device, self.width, self.height, self.max_frames = device, width, height, max_frames
        self.h = C.c_void_p()
        _check(lib().ygzfe_batch_create(C.byref(p), device, width, height, max_frames, C.byref(self.h)),
               "batch_create")
        pitch = C.c_size_t()
        cap = C.c_int()
        nl = C.c_int()
        _check(lib().ygzfe_batch_info(self.h, C.byref(pitch), C.byref(cap), C.byref(nl)), "batch_info")
        self.frame_pitch, self.kp_cap, self.nlevels = pitch.value, cap.value, nl.value

    def __del__(self):
        if getattr(self, "h", None) and self.h.value and _lib is not None:
            _lib.ygzfe_batch_destroy(self.h)
            self.h = None

    @property
    def stream(self):
        return lib().ygzfe_batch_stream(self.h)

    def frames_ptr(self):
        """Device pointer of the pyramid slots (frame i level 0 at + i * frame_pitch)."""
        p = C.c_void_p()
        _check(lib().ygzfe_batch_frames(self.h, C.byref(p)), "batch_frames")
        return p.value

    def upload(self, frames):
        frames = np.ascontiguousarray(frames, np.uint8)
        _check(lib().ygzfe_batch_upload(self.h, _p(frames), len(frames)), "batch_upload")

    def upload_undistorted(self, und, frames):
        frames = np.ascontiguousarray(frames, np.uint8)
        _check(lib().ygzfe_batch_upload_undistorted(self.h, und.h, _p(frames), len(frames)), "upload_undistorted")

    def undistort_device(self, und, d_raw, raw_pitch, n_frames, stream=None):
        _check(lib().ygzfe_batch_undistort_device(self.h, und.h, C.c_void_p(d_raw), C.c_size_t(raw_pitch), n_frames,
                                                  C.c_void_p(stream)), "batch_undistort")

    def bind(self, pyramids=0, kps=0, desc=0, counts=0):
        _check(lib().ygzfe_batch_bind_buffers(self.h, C.c_void_p(pyramids or None), C.c_void_p(kps or None),
                                              C.c_void_p(desc or None), C.c_void_p(counts or None)), "bind")

    def extract(self, n_frames, stream=None):
        _check(lib().ygzfe_batch_extract(self.h, n_frames, C.c_void_p(stream)), "batch_extract")

    def extract_split(self, n_frames, kp_stream, desc_stream):
        _check(lib().ygzfe_batch_extract_split(self.h, n_frames, C.c_void_p(kp_stream), C.c_void_p(desc_stream)),
               "batch_extract_split")

    def check(self):
        _check(lib().ygzfe_batch_check(self.h), "batch_check")

    def result(self, i):
        kps = np.zeros(self.kp_cap, KP_DTYPE)
        desc = np.zeros((self.kp_cap, 32), np.uint8)
        n = C.c_int()
        _check(lib().ygzfe_batch_result(self.h, i, _p(kps), self.kp_cap, _p(desc), C.byref(n)), "batch_result")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def level_size(self, level):
        w, h, st = C.c_int(), C.c_int(), C.c_int()
        _check(lib().ygzfe_batch_level(self.h, 0, level, None, C.byref(w), C.byref(h), C.byref(st)), "batch_level")
        return w.value, h.value

    def stats(self, n_frames):
        """Per-level totals over frames [0, n) of the last extract: (FAST candidates, octree keypoints)."""
        cand = np.zeros(self.nlevels, np.int64)
        sel = np.zeros(self.nlevels, np.int64)
        _check(lib().ygzfe_batch_stats(self.h, n_frames, _p(cand), _p(sel)), "batch_stats")
        return cand, sel

    def read_level(self, i, level, blurred=False):
        """Host copy of pyramid level `level` of frame i (or its 7x7 blurred copy)."""
        w, h = self.level_size(level)
        out = np.zeros((h, w), np.uint8)
        _check(lib().ygzfe_batch_read_level(self.h, i, level, int(bool(blurred)), _p(out), w), "batch_read_level")
        return out

    def match(self, n_pairs, d_qframe, d_tframe, d_bi, d_bd, d_sd, stream=None):
        _check(lib().ygzfe_batch_match(self.h, n_pairs, C.c_void_p(d_qframe), C.c_void_p(d_tframe), C.c_void_p(d_bi),
                                       C.c_void_p(d_bd), C.c_void_p(d_sd), C.c_void_p(stream)), "batch_match")

    def sparse_align(self, n_pairs, d_ref_idx, d_cur_idx, d_xyz, d_usable, cam, max_level, min_level, d_T_init,
                     d_out, stream=None):
        _check(lib().ygzfe_batch_sparse_align(self.h, n_pairs, C.c_void_p(d_ref_idx), C.c_void_p(d_cur_idx),
                                              C.c_void_p(d_xyz), C.c_void_p(d_usable), C.byref(cam), max_level,
                                              min_level, C.c_void_p(d_T_init), C.c_void_p(d_out),
                                              C.c_void_p(stream)), "batch_sparse_align")

    def stereo(self, n_pairs, d_left_idx, d_right_idx, mb, mbf, d_u_right, d_depth, stream=None):
        _check(lib().ygzfe_batch_stereo(self.h, n_pairs, C.c_void_p(d_left_idx), C.c_void_p(d_right_idx),
                                        C.c_float(mb), C.c_float(mbf), C.c_void_p(d_u_right), C.c_void_p(d_depth),
                                        C.c_void_p(stream)), "batch_stereo")

    def stereo_rgbd(self, n_frames, d_depth_images, depth_pitch, stride, mbf, d_u_right, d_depth, stream=None):
        _check(lib().ygzfe_batch_stereo_rgbd(self.h, n_frames, C.c_void_p(d_depth_images), C.c_size_t(depth_pitch),
                                             stride, C.c_float(mbf), C.c_void_p(d_u_right), C.c_void_p(d_depth),
                                             C.c_void_p(stream)), "batch_stereo_rgbd")

    def compute_bow(self, vocab, n_frames, levelsup, d_bow_words, d_bow_values, d_n_words, d_fv_nodes, d_fv_feats,
                    d_n_fv, stream=None):
        _check(lib().ygzfe_batch_compute_bow(self.h, vocab.h, n_frames, levelsup, C.c_void_p(d_bow_words),
                                             C.c_void_p(d_bow_values), C.c_void_p(d_n_words),
                                             C.c_void_p(d_fv_nodes), C.c_void_p(d_fv_feats), C.c_void_p(d_n_fv),
                                             C.c_void_p(stream)), "batch_compute_bow")

    def pack_slots(self, frame_begin, n_frames, d_align, global_first, d_slots, slot_pitch, stream=None):
        """Device-side packing of the offline sequence mode's per-frame result slots
        (ygzfe_batch_pack_slots; layout in include/ygzfe.h and ygzfe.dist)."""
        _check(lib().ygzfe_batch_pack_slots(self.h, frame_begin, n_frames, C.c_void_p(d_align or None), global_first,
                                            C.c_void_p(d_slots), C.c_size_t(slot_pitch), C.c_void_p(stream)),
               "batch_pack_slots")

    def timing(self, enable=True):
        ms = (C.c_float * 16)()
        names = (C.c_char_p * 16)()
        n = lib().ygzfe_batch_timing(self.h, int(enable), ms, names, 16)
        return {names[i].decode(): ms[i] for i in range(n)}


# ---------------------------------------------------------------- synthetic inputs (tests / bench)
_synth = None


def synth():
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise YgzfeError(f"{SYNTH_PATH} missing: run `make -C orb-ygz-slam_amd`")
        _synth = C.CDLL(SYNTH_PATH)
        _synth.ygzs_backproject_plane.restype = C.c_int
    return _synth


def synth_texture(seed, W, H):
    out = np.zeros((H, W), np.uint8)
    synth().ygzs_texture(C.c_uint64(seed), W, H, _p(out))
    return out


EUROC_CAM = (458.654, 457.296, 367.215, 248.375)


def trajectory_pose(k, xi):
    q = np.zeros(4, np.float32)
    t = np.zeros(3, np.float32)
    xi = np.ascontiguousarray(xi, np.float32)
    synth().ygzs_trajectory_pose(k, _p(xi), _p(q), _p(t))
    return q, t


def render_plane(tex, texel, plane_z, cam, q_cw, t_cw, W, H, noise_seed=0, noise_amp=2):
    tex = np.ascontiguousarray(tex, np.uint8)
    out = np.zeros((H, W), np.uint8)
    camv = np.array(cam, np.float32)
    synth().ygzs_render_plane(_p(tex), tex.shape[1], tex.shape[0], C.c_double(texel), C.c_double(plane_z),
                              _p(camv), _p(np.ascontiguousarray(q_cw, np.float32)),
                              _p(np.ascontiguousarray(t_cw, np.float32)), W, H, C.c_uint64(noise_seed), noise_amp,
                              _p(out))
    return out


def backproject_plane(cam, q_cw, t_cw, uv, plane_z):
    camv = np.array(cam, np.float32)
    q = np.ascontiguousarray(q_cw, np.float32)
    t = np.ascontiguousarray(t_cw, np.float32)
    uv = np.asarray(uv, np.float32).reshape(-1, 2)
    out = np.zeros((len(uv), 3), np.float32)
    ok = np.zeros(len(uv), np.uint8)
    P = np.zeros(3, np.float32)
    for i, (u, v) in enumerate(uv):
        ok[i] = synth().ygzs_backproject_plane(_p(camv), _p(q), _p(t), C.c_float(u), C.c_float(v),
                                               C.c_double(plane_z), _p(P))
        out[i] = P
    return out, ok


_synth_hip = None


def _synth_hip_lib():
    global _synth_hip
    if _synth_hip is None:
        lib()  # torch's HIP runtime first (see lib())
        if not os.path.exists(SYNTH_HIP_PATH):
            raise YgzfeError(f"{SYNTH_HIP_PATH} missing: run `make -C orb-ygz-slam_amd`")
        _synth_hip = C.CDLL(SYNTH_HIP_PATH)
    return _synth_hip


def render_plane_device(d_tex, tex_w, tex_h, texel, plane_z, cam, d_q, d_t, d_seeds, n_frames, W, H, d_out, pitch,
                        noise_amp=2, stream=None):
    """The synthetic plane sequence rendered on the device (synth/plane_points.hip):
    frame i (pose d_q[i], d_t[i], noise seed d_seeds[i]) -> d_out + i * pitch."""
    c = (C.c_float * 4)(*[float(v) for v in cam])
    rc = _synth_hip_lib().ygzs_render_plane_device(C.c_void_p(d_tex), tex_w, tex_h, C.c_double(texel),
                                                   C.c_double(plane_z), c, C.c_void_p(d_q), C.c_void_p(d_t),
                                                   C.c_void_p(d_seeds), n_frames, W, H, noise_amp, C.c_void_p(d_out),
                                                   C.c_size_t(pitch), C.c_void_p(stream))
    if rc != 0:
        raise YgzfeError("render_plane_device launch failed")


def plane_points_device(d_kps, cap, n_frames, cam, d_r3, d_cz, plane_z, d_xyz, stream=None):
    """Synthetic map points for bench.py: back-project every keypoint of frame i
    onto the plane Z_w = plane_z (one fused HIP pass; synth/plane_points.hip)."""
    c = (C.c_float * 4)(*[float(v) for v in cam])
    rc = _synth_hip_lib().ygzs_plane_points(C.c_void_p(d_kps), KP_DTYPE.itemsize // 4, cap, n_frames, c, C.c_void_p(d_r3),
                                      C.c_void_p(d_cz), C.c_float(plane_z), C.c_void_p(d_xyz), C.c_void_p(stream))
    if rc != 0:
        raise YgzfeError("plane_points launch failed")
