"""oracle/match.c (the ORBmatcher searches' CPU restatement) against a second, independent
pure-Python restatement of the same reference loops, on small random frames.  The reference
itself cannot be built here (OpenCV / Eigen absent), so two restatements written
apart from each other must agree before the C one is trusted as the GPU checker."""
import math

import numpy as np
import pytest

import _oracle as O

COLS, ROWS, TH_HIGH, TH_LOW, HISTO = 64, 48, 100, 50, 30
f32 = np.float32


def roundf(v):
    """C roundf: half away from zero (exact in double for a float argument)."""
    v = float(v)
    return int(math.copysign(math.floor(abs(v) + 0.5), v))


def popc(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


class PyFrame:
    """Frame::AssignFeaturesToGrid / PosInGrid / GetFeaturesInArea (Frame.cc:314-330, 424-493)."""

    def __init__(self, kps, desc, u_right, bounds):
        self.kps, self.desc, self.ur = kps, desc, u_right
        self.minx, self.maxx, self.miny, self.maxy = (f32(b) for b in bounds)
        self.iw = f32(COLS) / f32(self.maxx - self.minx)
        self.ih = f32(ROWS) / f32(self.maxy - self.miny)
        self.grid = [[[] for _ in range(ROWS)] for _ in range(COLS)]
        for i, k in enumerate(kps):
            px = roundf(f32(f32(k["x"]) - self.minx) * self.iw)
            py = roundf(f32(f32(k["y"]) - self.miny) * self.ih)
            if 0 <= px < COLS and 0 <= py < ROWS:
                self.grid[px][py].append(i)

    def in_area(self, x, y, r, minL=-1, maxL=-1):
        x, y, r = f32(x), f32(y), f32(r)
        out = []
        c0 = max(0, int(math.floor(f32(f32(x - self.minx) - r) * self.iw)))
        if c0 >= COLS:
            return out
        c1 = min(COLS - 1, int(math.ceil(f32(f32(x - self.minx) + r) * self.iw)))
        if c1 < 0:
            return out
        r0 = max(0, int(math.floor(f32(f32(y - self.miny) - r) * self.ih)))
        if r0 >= ROWS:
            return out
        r1 = min(ROWS - 1, int(math.ceil(f32(f32(y - self.miny) + r) * self.ih)))
        if r1 < 0:
            return out
        chk = minL > 0 or maxL >= 0
        for ix in range(c0, c1 + 1):
            for iy in range(r0, r1 + 1):
                for j in self.grid[ix][iy]:
                    k = self.kps[j]
                    if chk and (k["octave"] < minL or (maxL >= 0 and k["octave"] > maxL)):
                        continue
                    if abs(f32(k["x"]) - x) < r and abs(f32(k["y"]) - y) < r:
                        out.append(j)
        return out


def three_maxima(h):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(h):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if m2 < f32(0.1) * f32(m1):
        i2 = i3 = -1
    elif m3 < f32(0.1) * f32(m1):
        i3 = -1
    return i1, i2, i3


def rot_bin(a, b):
    rot = f32(f32(a) - f32(b))
    if rot < 0:
        rot = f32(rot + f32(360))
    v = float(f32(rot * (f32(1) / f32(HISTO))))
    b = roundf(v)
    return 0 if b == HISTO else b


def py_best(F, Q, qd, blocked, th, ori):
    blocked = np.array(blocked, bool)
    out = np.full(len(F.kps), -1)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    for i, q in enumerate(Q):
        if not q["flags"] & 1:
            continue
        cand = F.in_area(q["u"], q["v"], q["radius"], q["min_level"], q["max_level"])
        best, bi = 256, -1
        for j in cand:
            if blocked[j]:
                continue
            if q["flags"] & 4 and F.ur is not None and F.ur[j] > 0 and abs(f32(q["u_right"]) - F.ur[j]) > q["radius"]:
                continue
            d = popc(qd[i], F.desc[j])
            if d < best:
                best, bi = d, j
        if cand and best <= th:
            out[bi] = i
            blocked[bi] = bool(q["flags"] & 2)
            nm += 1
            if ori:
                hist[rot_bin(q["angle"], F.kps[bi]["angle"])].append(bi)
    if ori:
        keep = three_maxima([len(h) for h in hist])
        for b in range(HISTO):
            if b not in keep:
                for j in hist[b]:
                    out[j] = -2
                    nm -= 1
    return out, nm


def py_init(F1, F2, prev, window, ratio, ori):
    m12 = np.full(len(F1.kps), -1)
    mdist = np.full(len(F2.kps), 2 ** 31 - 1)
    m21 = np.full(len(F2.kps), -1)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    for i1, k1 in enumerate(F1.kps):
        if k1["octave"] > 0:
            continue
        cand = F2.in_area(prev[i1, 0], prev[i1, 1], window, 0, 0)
        best = best2 = 2 ** 31 - 1
        bi = -1
        for j in cand:
            d = popc(F1.desc[i1], F2.desc[j])
            if mdist[j] <= d:
                continue
            if d < best:
                best2, best, bi = best, d, j
            elif d < best2:
                best2 = d
        if best <= TH_LOW and best < f32(best2) * f32(ratio):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                nm -= 1
            m12[i1], m21[bi], mdist[bi] = bi, i1, best
            nm += 1
            if ori:
                hist[rot_bin(k1["angle"], F2.kps[bi]["angle"])].append(i1)
    if ori:
        keep = three_maxima([len(h) for h in hist])
        for b in range(HISTO):
            if b not in keep:
                for i1 in hist[b]:
                    if m12[i1] >= 0:
                        m12[i1] = -1
                        nm -= 1
    return m12, nm


def random_frame(rng, n, W=160, H=120):
    kps = np.zeros(n, O.KP_DTYPE)
    kps["x"] = rng.uniform(-3, W + 3, n)
    kps["y"] = rng.uniform(-3, H + 3, n)
    kps["octave"] = rng.integers(0, 3, n)
    kps["angle"] = rng.uniform(0, 360, n)
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    desc[:, :20] &= 0x0F  # correlated descriptors: distances spread around the thresholds
    return kps, desc


@pytest.mark.parametrize("seed", range(4))
def test_features_in_area(seed):
    rng = np.random.default_rng(seed)
    kps, desc = random_frame(rng, 300)
    b = (0.0, 160.0, 0.0, 120.0)
    F = PyFrame(kps, desc, None, b)
    Fo = O.mframe(kps, desc, None, b)
    for _ in range(200):
        x, y, r = rng.uniform(-10, 170), rng.uniform(-10, 130), rng.uniform(0.5, 30)
        lo, hi = rng.integers(-1, 3), rng.integers(-1, 3)
        assert list(O.features_in_area(Fo, x, y, r, lo, hi)) == F.in_area(x, y, r, lo, hi)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("ori", [True, False])
def test_projection_best_and_init(seed, ori):
    rng = np.random.default_rng(100 + seed)
    b = (0.0, 160.0, 0.0, 120.0)
    k1, d1 = random_frame(rng, 250)
    k0, d0 = random_frame(rng, 200)
    d0[:120] = d1[:120] ^ (rng.random((120, 32)) < 0.05).astype(np.uint8)  # true matches with a few flipped bits
    ur = np.where(rng.random(250) < 0.5, k1["x"] - 10, -1).astype(np.float32)
    F = PyFrame(k1, d1, ur, b)
    import ygzfe
    Q = np.zeros(200, ygzfe.MATCH_QUERY_DTYPE)
    Q["u"] = np.where(np.arange(200) < 120, k1["x"][:200] + rng.uniform(-2, 2, 200), rng.uniform(0, 160, 200))
    Q["v"] = np.where(np.arange(200) < 120, k1["y"][:200] + rng.uniform(-2, 2, 200), rng.uniform(0, 120, 200))
    Q["radius"] = rng.choice([4.0, 8.0, 20.0], 200)
    Q["min_level"] = rng.integers(-1, 2, 200)
    Q["max_level"] = rng.integers(-1, 3, 200)
    Q["angle"] = rng.uniform(0, 360, 200)
    Q["u_right"] = Q["u"] - 10
    Q["flags"] = rng.integers(0, 8, 200) | 1
    bl = (rng.random(250) < 0.1).astype(np.uint8)
    for th in (50, 100):
        want = py_best(F, Q, d0, bl, th, ori)
        got = O.search_projection_best(O.mframe(k1, d1, ur, b), Q, d0, bl, th, ori)
        assert got[1] == want[1] and np.array_equal(got[0], want[0])
    F0 = PyFrame(k0, d0, None, b)
    prev = np.stack([k0["x"], k0["y"]], 1).astype(np.float32)
    for window in (10, 40):
        want = py_init(F0, PyFrame(k1, d1, None, b), prev, window, 0.9, ori)
        got = O.search_for_initialization(O.mframe(k0, d0, None, b), O.mframe(k1, d1, None, b), prev, window, 0.9,
                                          ori)
        assert got[1] == want[1] and np.array_equal(got[0], want[0])


def test_three_maxima_ten_percent_rule():
    import ctypes as C
    L = O.lib()
    for h in ([5, 0, 0, 100, 9, 11], [0] * 30, [3, 3, 3, 3], [1, 50, 4, 6, 7], [10, 1, 10, 2]):
        h = list(h) + [0] * (30 - len(h))
        a, b, c = C.c_int(-1), C.c_int(-1), C.c_int(-1)
        arr = (C.c_int * 30)(*h)
        L.ygzo_compute_three_maxima(arr, 30, C.byref(a), C.byref(b), C.byref(c))
        assert (a.value, b.value, c.value) == three_maxima(h)
