"""Row a9 on the GPU against the reference's own outputs: tests/golden/fast10_ref.npz, written by
tests/golden/make_golden.py from Thirdparty/fast compiled here (oracle/_ref), read directly (no
oracle in between).

* test1.png (Thirdparty/fast/test/data, the reference's known-answer image: 167 corners at
  threshold 75, test.cpp:300,332) and two seeded frames, thresholds {5, 7, 20, 75}, on the
  in-bounds interior (3, 3, W-6, H-6): fast_corner_detect_10 (plain) and
  fast_corner_detect_10_sse2, corner lists in order;
* the DSO cell path (ORBextractor.cc:1317-1345): fast_corner_detect_10_sse2 on g x g cells,
  g in {18, 19, 22, 30} (g < 22 -> the plain scan over the whole cell,
  faster_corner_10_sse.cpp:192-194), thresholds 20 and 5.

The GPU runs the same segment test as k_dso_cells (csrc/dso.hip fast10_corner) through the C ABI
(ygzfe_fast10_detect), and k_dso_cells itself through its debug pass (ygzfe_debug_dso_cells)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIX = np.load(os.path.join(GOLDEN, "fast10_ref.npz"))  # allow_pickle=False (default)


def _image(name):
    if name == "test1":
        from PIL import Image
        return np.array(Image.open(os.path.join(GOLDEN, "test1.png")))
    return FIX[f"{name}/img"]


@pytest.mark.parametrize("name", ["test1", "synth_a", "synth_b"])
@pytest.mark.parametrize("th", [5, 7, 20, 75])
@pytest.mark.parametrize("sse", [0, 1])
def test_fast10_detect_matches_reference(gpu, name, th, sse):
    img = _image(name)
    H, W = img.shape
    (xy,) = gpu.fast10_detect(img, th, [(3, 3, W - 6, H - 6)], sse=bool(sse))
    want = FIX[f"{name}/t{th}/s{sse}/xy"]
    assert xy.shape == want.shape, f"{name} t{th} s{sse}: {len(xy)} corners vs the reference's {len(want)}"
    assert np.array_equal(xy, want)


def test_fast10_known_answer_167(gpu):
    img = _image("test1")
    H, W = img.shape
    (xy,) = gpu.fast10_detect(img, 75, [(3, 3, W - 6, H - 6)], sse=True)
    assert len(xy) == 167  # Thirdparty/fast/test/test.cpp:300,332


@pytest.mark.parametrize("g", [18, 19, 22, 30])
@pytest.mark.parametrize("th", [20, 5])
def test_fast10_dso_cells_match_reference(gpu, g, th):
    img = _image("test1")
    cells = FIX[f"dso/g{g}/cells"].astype(np.int32)
    rois = np.concatenate([cells, np.full((len(cells), 2), g, np.int32)], 1)
    got = gpu.fast10_detect(img, th, rois, sse=True)
    xy, offs = FIX[f"dso/g{g}/t{th}/xy"], FIX[f"dso/g{g}/t{th}/offs"]
    for k in range(len(cells)):
        want = xy[offs[k]:offs[k + 1]]
        assert np.array_equal(got[k], want), f"g {g} th {th} cell {tuple(cells[k])}: {got[k].tolist()} vs " \
                                             f"{want.tolist()}"


@pytest.mark.parametrize("g", [18, 19, 22, 30])
@pytest.mark.parametrize("th", [20, 5])
def test_dso_cell_kernel_matches_reference(gpu, g, th):
    """k_dso_cells itself (its debug pass: the cell kernel's LDS tile, scan region and segment
    test, ORBextractor.cc:1317-1345) against the reference's fast_corner_detect_10_sse2 corner
    lists of the same cells."""
    img = _image("test1")
    H, W = img.shape
    got = gpu.debug_dso_cells(img, g, th)
    cols = W // g
    cells = FIX[f"dso/g{g}/cells"].astype(np.int32)
    xy, offs = FIX[f"dso/g{g}/t{th}/xy"], FIX[f"dso/g{g}/t{th}/offs"]
    n_corners = 0
    for k, (x0, y0) in enumerate(cells):
        assert x0 % g == 0 and y0 % g == 0
        want = xy[offs[k]:offs[k + 1]]
        mine = got[(y0 // g) * cols + x0 // g]
        assert np.array_equal(mine, want), f"g {g} th {th} cell ({x0}, {y0}): {mine.tolist()} vs {want.tolist()}"
        n_corners += len(want)
    assert n_corners > 0


def test_fast10_rejects_out_of_bounds_roi(gpu):
    img = _image("synth_b")
    H, W = img.shape
    with pytest.raises(gpu.YgzfeError):
        gpu.fast10_detect(img, 20, [(0, 0, W, H)], sse=False)  # the plain scan's ring would leave the image
