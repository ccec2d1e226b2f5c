"""Handle lifetimes across the C ABI: an extractor destroyed before its frames (the order a
garbage collector may pick for a reference cycle) is released by the last frame's destroy,
and the frames stay usable until then (include/ygzfe.h, ygzfe_extractor_destroy)."""
import gc

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_extractor_destroyed_before_frames(gpu):
    import _scenes as S
    ex = gpu.ORBextractor(1000, 2.0, 4, 20, 7)
    img = S.frame(0, 752, 480)
    frames = [ex.ComputePyramid(img) for _ in range(3)]
    ref_kps, ref_desc = ex.extract(frames[0])
    lib = gpu.lib()
    h = ex.h
    ex.h = None  # the Python wrapper no longer owns it
    lib.ygzfe_extractor_destroy(h)  # deferred: three frames borrow it
    # the frames still work (their extractor's stream, plans and mutex are alive)
    lvl = frames[1].level(1)
    assert lvl.shape == (240, 376)
    for f in frames:  # the last destroy releases the extractor
        lib.ygzfe_frame_destroy(f.h)
        f.h = None
    del frames
    gc.collect()
    # a fresh extractor afterwards extracts the same keypoints
    ex2 = gpu.ORBextractor(1000, 2.0, 4, 20, 7)
    k2, d2 = ex2.extract(ex2.ComputePyramid(img))
    assert np.array_equal(k2, ref_kps) and np.array_equal(d2, ref_desc)
