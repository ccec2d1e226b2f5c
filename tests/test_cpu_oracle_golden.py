"""The CPU oracle's FAST-10 (ORBextractor DSO path, Thirdparty/fast) against the
reference's own outputs: tests/golden/fast10_ref.npz, produced by
tests/golden/make_golden.py from the reference sources compiled in oracle/_ref.

This pins oracle/fast10.c (restating fast_10.cpp, faster_corner_10_sse.cpp,
fast_10_score.cpp, nonmax_3x3.cpp) before it is trusted as the GPU checker.
"""
import os

import numpy as np
import pytest

import _oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FIX = np.load(os.path.join(GOLDEN, "fast10_ref.npz"))  # allow_pickle=False (default)


def image(name):
    if name == "test1":
        from PIL import Image
        return np.array(Image.open(os.path.join(GOLDEN, "test1.png")))
    return FIX[f"{name}/img"]


IMAGES = ("test1", "synth_a", "synth_b")
THRESHOLDS = (5, 7, 20, 75)


def test_known_answer_167():
    """Thirdparty/fast/test/test.cpp:300,332 -- 167 corners at threshold 75 on test1.png."""
    img = image("test1")
    H, W = img.shape
    assert len(FIX["test1/t75/s1/xy"]) == 167
    for sse in (False, True):
        xs, ys = O.fast10_detect(img, 75, sse=sse, x0=3, y0=3, w=W - 6, h=H - 6)
        assert len(xs) == 167


@pytest.mark.parametrize("name", IMAGES)
@pytest.mark.parametrize("th", THRESHOLDS)
def test_fast10_detect_score_nonmax(name, th):
    img = image(name)
    H, W = img.shape
    for sse in (0, 1):
        xs, ys = O.fast10_detect(img, th, sse=bool(sse), x0=3, y0=3, w=W - 6, h=H - 6)
        want = FIX[f"{name}/t{th}/s{sse}/xy"]
        got = np.stack([xs, ys], 1).astype(np.int16)
        assert np.array_equal(got, want), f"{name} th={th} sse={sse}: {len(got)} vs {len(want)}"
    xs, ys = FIX[f"{name}/t{th}/s1/xy"].T
    sc = O.fast10_scores(img, xs, ys, th, x0=3, y0=3)
    assert np.array_equal(sc, FIX[f"{name}/t{th}/score"])
    keep = O.fast10_nonmax(xs, ys, sc)
    assert np.array_equal(keep, FIX[f"{name}/t{th}/keep"])


@pytest.mark.parametrize("g", (18, 19, 22, 30))
@pytest.mark.parametrize("th", (20, 5))
def test_dso_cells(g, th):
    """DSO cells (ORBextractor.cc:1317-1345): < 22 px wide -> plain tree over the whole cell."""
    img = image("test1")
    cells = FIX[f"dso/g{g}/cells"]
    xy, offs = FIX[f"dso/g{g}/t{th}/xy"], FIX[f"dso/g{g}/t{th}/offs"]
    for i, (x, y) in enumerate(cells):
        xs, ys = O.fast10_detect(img, th, sse=True, x0=int(x), y0=int(y), w=g, h=g)
        want = xy[offs[i]:offs[i + 1]]
        assert np.array_equal(np.stack([xs, ys], 1).astype(np.int16), want), f"cell {i} at {(x, y)}"


@pytest.mark.skipif(not O.RefFast.available(), reason="oracle/_ref not built (reference checkout absent)")
def test_live_reference_random_frames():
    """Where the reference's fast lib is built (this container), cross-check fresh inputs too."""
    ref = O.RefFast()
    rng = np.random.default_rng(7)
    for trial in range(3):
        img = rng.integers(0, 256, size=(64, 80), dtype=np.uint8)
        img = ((img.astype(np.int32) + np.roll(img, 1, 0)) // 2).astype(np.uint8)
        for th in (5, 20):
            a = ref.detect(img, th, sse=True, x0=3, y0=3, w=74, h=58)
            b = O.fast10_detect(img, th, sse=True, x0=3, y0=3, w=74, h=58)
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
            sa = ref.scores(img, a[0], a[1], th, x0=3, y0=3)
            assert np.array_equal(sa, O.fast10_scores(img, a[0], a[1], th, x0=3, y0=3))


@pytest.mark.parametrize("name", IMAGES)
@pytest.mark.parametrize("th", THRESHOLDS)
def test_fast10_vector_pipeline(name, th):
    """The 16-pixel vector FAST-10 (detect + score + dense-map 3x3 NMS, the CPU baseline's
    path) == the scalar restatement == the reference library's survivors and scores."""
    img = image(name)
    H, W = img.shape
    xy, sc, keep = FIX[f"{name}/t{th}/s1/xy"], FIX[f"{name}/t{th}/score"], FIX[f"{name}/t{th}/keep"]
    for scalar in (False, True):
        xs, ys, s = O.fast10_pipeline(img, th, x0=3, y0=3, w=W - 6, h=H - 6, scalar=scalar)
        assert np.array_equal(np.stack([xs, ys], 1).astype(np.int16), xy[keep]), (name, th, scalar)
        assert np.array_equal(s, sc[keep]), (name, th, scalar)
    O.lib().ygzo_fast10_force_scalar(1)
    try:
        xs1, ys1 = O.fast10_detect(img, th, sse=True, x0=3, y0=3, w=W - 6, h=H - 6)
    finally:
        O.lib().ygzo_fast10_force_scalar(0)
    assert np.array_equal(np.stack([xs1, ys1], 1).astype(np.int16), xy)
