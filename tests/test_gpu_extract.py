"""GPU ORB extraction vs the CPU oracle: bit-exact keypoints and descriptors.

Reference path: ORBextractor::operator()(Frame*, ..., ORBSLAM_KEYPOINT)
(ORBextractor.cc:1031-1127) and (..., DSO_KEYPOINT) (ORBextractor.cc:1275-1386).
"""
import os

import numpy as np
import pytest

import _oracle as O
import _scenes as S

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load_test1_png():
    from PIL import Image
    return np.array(Image.open(os.path.join(GOLDEN, "test1.png")))


def assert_kps_equal(a, b, what=""):
    assert len(a) == len(b), f"{what}: {len(a)} vs {len(b)} keypoints"
    for f in a.dtype.names:
        if not np.array_equal(a[f], b[f]):
            bad = np.nonzero(a[f] != b[f])[0]
            raise AssertionError(f"{what}: field {f} differs at rows {bad[:10]}: {a[f][bad[:5]]} vs {b[f][bad[:5]]}")


def make(gpu, cfg, blur=0):
    W, H, nf, sf, nl, ini, mn = S.CONFIGS[cfg]
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn, blur=blur)
    orc = O.OrbOracle(nf, sf, nl, ini, mn, blur_variant=blur)
    return W, H, ex, orc


@pytest.mark.parametrize("cfg", ["C1", "C2", "C4"])
def test_pyramid_bitexact(gpu, cfg):
    W, H, ex, orc = make(gpu, cfg)
    for seed in (0, 5):
        img = S.frame(seed, W, H)
        fr = ex.ComputePyramid(img)
        ref = orc.pyramid(img)
        for l, (g, r) in enumerate(zip(fr.levels(), ref)):
            assert g.shape == r.shape
            assert np.array_equal(g, r), f"{cfg} level {l}: {np.count_nonzero(g != r)} px differ"


@pytest.mark.parametrize("cfg", ["C1", "C2", "C4"])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_extract_orbslam_bitexact(gpu, cfg, seed):
    W, H, ex, orc = make(gpu, cfg)
    img = S.frame(seed, W, H)
    fr = ex.ComputePyramid(img)
    kg, dg = ex.extract(fr)
    kr, dr = orc.extract(orc.pyramid(img))
    assert len(kr) > 100
    assert_kps_equal(kg, kr, f"{cfg}/{seed}")
    assert np.array_equal(dg, dr), f"{np.count_nonzero((dg != dr).any(1))} descriptor rows differ"


def test_extract_test1_png(gpu):
    img = load_test1_png()
    H, W = img.shape
    ex = gpu.ORBextractor(1000, 2.0, 4, 20, 7)
    orc = O.OrbOracle(1000, 2.0, 4, 20, 7)
    kg, dg = ex(img)
    kr, dr = orc.extract(orc.pyramid(img))
    assert_kps_equal(kg, kr, "test1.png")
    assert np.array_equal(dg, dr)


def test_extract_blur_cv3(gpu):
    W, H, ex, orc = make(gpu, "C2", blur=1)
    img = S.frame(11, W, H)
    kg, dg = ex.extract(ex.ComputePyramid(img))
    kr, dr = orc.extract(orc.pyramid(img))
    assert_kps_equal(kg, kr)
    assert np.array_equal(dg, dr)


def test_extract_with_existing(gpu):
    """Frame with direct-tracked keypoints: their descriptor rows come first (ORBextractor.cc:1088-1099)."""
    W, H, ex, orc = make(gpu, "C1")
    img = S.frame(3, W, H)
    lv = orc.pyramid(img)
    base, _ = orc.extract(lv)
    rng = np.random.default_rng(0)
    existing = base[rng.choice(len(base), 40, replace=False)].copy()
    existing["x"] += rng.uniform(-1.5, 1.5, 40).astype(np.float32)
    existing["angle"] = rng.uniform(0, 360, 40).astype(np.float32)
    kg, dg = ex.extract(ex.ComputePyramid(img), existing=existing)
    kr, dr = orc.extract(lv, existing=existing)
    assert_kps_equal(kg, kr)
    assert np.array_equal(dg, dr)
    assert_kps_equal(kg[:40], existing)


def test_extract_dso_bitexact_and_state(gpu):
    """DSO_KEYPOINT: grid state mnGridSize carries across frames (ORBextractor.cc:1295,1380)."""
    W, H, ex, orc = make(gpu, "C2")
    for seed in (4, 5, 6):
        img = S.frame(seed, W, H)
        lv = orc.pyramid(img)
        base, _ = orc.extract(lv)
        existing = base[:60].copy()
        kg, dg = ex.extract(ex.ComputePyramid(img), method=gpu.DSO_KEYPOINT, existing=existing)
        kr, dr, ex_r = orc.extract_dso(lv, existing=existing)
        assert_kps_equal(kg, kr, f"dso seed {seed}")
        assert np.array_equal(dg, dr)
        assert ex.dso_grid == orc.o.dso_grid


def test_batch_matches_single(gpu):
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    frames = np.stack([S.frame(s, W, H) for s in range(6)])
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, 8)
    b.upload(frames)
    b.extract(len(frames))
    b.check()
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    for i in range(len(frames)):
        kg, dg = b.result(i)
        kr, dr = orc.extract(orc.pyramid(frames[i]))
        assert_kps_equal(kg, kr, f"batch frame {i}")
        assert np.array_equal(dg, dr)


@pytest.mark.parametrize("cfg,size", [("C4", (640, 480)), ("C1", (641, 479))])
def test_batch_linear_pyramid_chain(gpu, cfg, size):
    """A batch of >= 64 frames forms its INTER_LINEAR levels in one launch (a workgroup
    per frame, k_pyramid_linear_chain): every level of every frame equals the oracle's
    cv::resize chain (ORBextractor.cc:1129-1150), odd sizes included; keypoints of a
    few frames too."""
    W, H = size
    _, _, nf, sf, nl, ini, mn = S.CONFIGS[cfg]
    F = 64
    base = [S.frame(s, W, H) for s in range(4)]
    frames = np.stack([np.roll(base[i % 4], 3 * i, axis=1) for i in range(F)])
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, F)
    b.upload(frames)
    b.extract(F)
    b.check()
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    for i in (0, 1, 37, F - 1):
        lv = orc.pyramid(frames[i])
        for l in range(nl):
            got = b.read_level(i, l)
            assert np.array_equal(got, lv[l]), f"frame {i} level {l}"
    for i in (0, F - 1):
        kg, dg = b.result(i)
        kr, dr = orc.extract(orc.pyramid(frames[i]))
        assert_kps_equal(kg, kr, f"{cfg} batch frame {i}")
        assert np.array_equal(dg, dr)


def test_featureless_frame(gpu):
    """Edge case: a flat image has no FAST corners -> empty result, no hang."""
    W, H, ex, orc = make(gpu, "C2")
    img = np.full((H, W), 77, np.uint8)
    kg, dg = ex.extract(ex.ComputePyramid(img))
    kr, dr = orc.extract(orc.pyramid(img))
    assert len(kg) == len(kr) == 0


@pytest.mark.parametrize("size,cfg,blur", [((752, 480), "C2", 0), ((640, 480), "C1", 0), ((641, 479), "C1", 1),
                                           ((97, 61), "C1", 0), ((30, 20), "C2", 1)])
def test_batch_blur_every_pixel(gpu, size, cfg, blur):
    """GaussianBlur(7x7, sigma 2, REFLECT_101) of every level, border columns
    and rows included (ORBextractor.cc:1079-1084), vs the oracle's blur7."""
    W, H = size
    _, _, nf, sf, nl, ini, mn = S.CONFIGS[cfg]
    # levels must stay >= 1 px: cap nlevels for the tiny image
    while nl > 1 and round(min(W, H) / sf ** (nl - 1)) < 2:
        nl -= 1
    frames = np.stack([S.frame(s, W, H) for s in (11, 12)])
    b = gpu.Batch((nf, sf, nl, ini, mn, blur), 0, W, H, 2)
    b.upload(frames)
    b.extract(len(frames))
    for i in range(len(frames)):
        for l in range(b.nlevels):
            lv = b.read_level(i, l)
            got = b.read_level(i, l, blurred=True)
            want = O.blur7(lv, blur)
            if not np.array_equal(got, want):
                bad = np.argwhere(got != want)
                raise AssertionError(f"frame {i} level {l} {lv.shape}: {len(bad)} px differ, first {bad[:5].tolist()}")


@pytest.mark.parametrize("W,H,nl", [(752, 480, 4), (1280, 720, 4), (776, 488, 4), (752, 480, 3), (752, 480, 2)])
def test_batch_fused_area_pyramid(gpu, W, H, nl):
    """An all-area pyramid (scale 2.0: every level an exact x2 INTER_AREA) is formed in the
    batch path by the level-0 blur strips (k_blur7's fused mode, K = nl - 1 levels), the
    separate pyramid pass skipped: every level and every blurred level of every frame equal
    the oracle's (ORBextractor.cc:1129-1150, 1079-1084), widths whose last strip is short
    (776: 8 columns) and heights whose last strip is (720, 488) included; keypoints and
    descriptors too."""
    frames = np.stack([S.frame(s, W, H) for s in (21, 22, 23)])
    b = gpu.Batch((1000, 2.0, nl, 20, 7, 0), 0, W, H, 4)
    b.upload(frames)
    b.extract(len(frames))
    b.check()
    orc = O.OrbOracle(1000, 2.0, nl, 20, 7)
    for i in range(len(frames)):
        lv = orc.pyramid(frames[i])
        for l in range(nl):
            got = b.read_level(i, l)
            assert np.array_equal(got, lv[l]), f"frame {i} level {l}: {np.count_nonzero(got != lv[l])} px differ"
            bl = b.read_level(i, l, blurred=True)
            assert np.array_equal(bl, O.blur7(lv[l], 0)), f"frame {i} blurred level {l}"
        kg, dg = b.result(i)
        kr, dr = orc.extract(lv)
        assert_kps_equal(kg, kr, f"frame {i}")
        assert np.array_equal(dg, dr)


@pytest.mark.parametrize("cfg", ["C2", "C4"])
@pytest.mark.parametrize("kind", ["uniform", "checker"])
def test_dense_noise_frames_capacity(gpu, cfg, kind):
    """Worst-case FAST density: uniform noise (most pixels are corners at minTh 7 / iniTh 20) and
    a 1-px checkerboard with noise.  The per-cell candidate slots and the per-level key limit
    must hold whatever the image; extraction stays bit-exact with the oracle."""
    W, H, ex, orc = make(gpu, cfg)
    rng = np.random.default_rng(99)
    if kind == "uniform":
        img = rng.integers(0, 256, (H, W), dtype=np.uint8)
    else:
        yy, xx = np.mgrid[0:H, 0:W]
        img = np.where((xx + yy) % 2 == 0, 200, 40).astype(np.int32) + rng.integers(-12, 13, (H, W))
        img = np.clip(img, 0, 255).astype(np.uint8)
    k, d = ex.extract(ex.ComputePyramid(img))
    rk, rd = orc.extract(orc.pyramid(img))
    assert_kps_equal(k, rk, f"{cfg} {kind}")
    assert np.array_equal(d, rd)
    assert len(k) >= 0.5 * CONFIG_NF[cfg]


CONFIG_NF = {c: S.CONFIGS[c][2] for c in S.CONFIGS}
