"""Two extractors used from two host threads at once, as Frame's stereo constructor does
(Frame.cc:728-731: `thread threadLeft(&Frame::ExtractORB, this, 0, imLeft); thread
threadRight(&Frame::ExtractORB, this, 1, imRight);`).  Each thread owns one handle (its
own streams, pinned staging, workspace and captured graph); the calls interleave on
the device.  Every result must equal the oracle's, frame by frame."""
import threading

import numpy as np
import pytest

import _oracle as O
import _scenes as S

pytestmark = pytest.mark.gpu


def test_two_extractors_two_threads(gpu):
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    left = [S.frame(100 + i, W, H) for i in range(6)]
    right = [np.roll(S.frame(200 + i, W, H), 5, axis=1) for i in range(6)]
    want = {side: [orc.extract(orc.pyramid(im)) for im in ims] for side, ims in (("L", left), ("R", right))}
    got = {"L": [None] * 6, "R": [None] * 6}
    errors = []

    def run(side, ims):
        try:
            ex = gpu.ORBextractor(nf, sf, nl, ini, mn, device=0)
            for rep in range(4):  # repeated: graph replays interleave with the other thread's
                for i, im in enumerate(ims):
                    k, d = ex.extract(ex.ComputePyramid(im))
                    if rep == 3:
                        got[side][i] = (k.copy(), d.copy())
        except Exception as e:  # surfaced in the main thread
            errors.append((side, repr(e)))

    th = [threading.Thread(target=run, args=("L", left)), threading.Thread(target=run, args=("R", right))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    assert all(not t.is_alive() for t in th), "extraction thread did not finish"
    for side in ("L", "R"):
        for i in range(6):
            kg, dg = got[side][i]
            kr, dr = want[side][i]
            assert len(kg) == len(kr), (side, i)
            for fld in kg.dtype.names:
                assert np.array_equal(kg[fld], kr[fld]), (side, i, fld)
            assert np.array_equal(dg, dr), (side, i)
