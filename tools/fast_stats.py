"""FAST cell statistics of the C5 workload (how often do cells retry at
minThFAST, how many pixels survive the 4-point screen per pass, how many corners per pass).
CPU only: the C5 frames rendered on the host (the same scene, poses and noise as
ygzfe.sequence.C5Shard), the cell ROIs of ComputeKeyPointsOctTree (ORBextractor.cc:725-781),
the oracle's cv::FAST restatement per ROI (tests/_oracle.py fast9_roi) and the compass screen
restated in numpy.  Usage: python tools/fast_stats.py [n_frames]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ygzfe  # noqa: E402
import _oracle as O  # noqa: E402
from ygzfe import scene  # noqa: E402
from ygzfe.sequence import C2, C5_FRAMES, SCENE_SEED, XI, sweep_index  # noqa: E402


def cells(w, h):
    """ComputeKeyPointsOctTree's cell ROIs (iniX, iniY, maxX, maxY) of a w x h level."""
    minb, maxx, maxy = 16, w - 16, h - 16  # EDGE_THRESHOLD 19: 19 - 3, cols - 19 + 3
    width, height = maxx - minb, maxy - minb
    ncols, nrows = width // 30, height // 30
    if ncols == 0 or nrows == 0:
        return []
    wc, hc = int(np.ceil(width / ncols)), int(np.ceil(height / nrows))
    out = []
    for i in range(nrows):
        iy = minb + i * hc
        my = iy + hc + 6
        if iy >= maxy - 3:
            continue
        my = min(my, maxy)
        for j in range(ncols):
            ix = minb + j * wc
            mx = ix + wc + 6
            if ix >= maxx - 6:
                continue
            mx = min(mx, maxx)
            out.append((ix, iy, mx, my))
    return out


def screen(roi, th):
    """Pixels of the ROI interior [3, -3) passing the 4-point compass test at th."""
    r = roi.astype(np.int16)
    v = r[3:-3, 3:-3]
    T, B, L, R = r[:-6, 3:-3], r[6:, 3:-3], r[3:-3, :-6], r[3:-3, 6:]
    bv = np.minimum(np.maximum(T, B), np.maximum(L, R))
    dv = np.maximum(np.minimum(T, B), np.minimum(L, R))
    return int(((bv - v > th) | (v - dv > th)).sum())


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    W, H, nf, sf, nl, ini, mn = C2
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    sc = scene.PlaneScene(SCENE_SEED, W, H)
    frames = np.linspace(0, C5_FRAMES - 1, n).astype(int)
    tot = {}
    for g in frames:
        q, t = ygzfe.trajectory_pose(sweep_index(int(g)), XI)
        img = sc.render(q, t, int(g))
        lv = orc.pyramid(img)
        for l, im in enumerate(lv):
            st = tot.setdefault(l, dict(cells=0, retry=0, px=0, surv1=0, surv2=0, corn1=0, corn2=0, empty=0))
            for ix, iy, mx, my in cells(im.shape[1], im.shape[0]):
                roi = im[iy:my, ix:mx]
                st["cells"] += 1
                st["px"] += max(roi.shape[0] - 6, 0) * max(roi.shape[1] - 6, 0)
                st["surv1"] += screen(roi, ini)
                c1 = len(O.fast9_roi(roi, ini)[0])
                st["corn1"] += c1
                if c1 == 0:
                    st["retry"] += 1
                    st["surv2"] += screen(roi, mn)
                    c2 = len(O.fast9_roi(roi, mn)[0])
                    st["corn2"] += c2
                    st["empty"] += c2 == 0
    print(f"C5 frames sampled: {n} (C2: {W}x{H}, FAST {ini}/{mn}); per frame:")
    print("level  cells  retried  interior_px  screen_surv_ini  corners_ini  screen_surv_min  corners_min  empty")
    for l, st in tot.items():
        print(f"{l:5d} {st['cells'] / n:6.1f} {st['retry'] / n:8.1f} {st['px'] / n:12.0f} {st['surv1'] / n:16.0f} "
              f"{st['corn1'] / n:12.0f} {st['surv2'] / n:16.0f} {st['corn2'] / n:12.1f} {st['empty'] / n:6.1f}")


if __name__ == "__main__":
    main()
