"""Prototype of the path-code octree (design check, CPU only): DistributeOctTree
(ORBextractor.cc:533-723) restated over keys sorted by their quadrant path, checked
against oracle/orb.c's list simulation on random and clustered candidate sets.

Claim being checked: after P main-loop passes the list is, section by section
(creation depth e = P, P-1, ..., 0), the nodes created at depth e (all of depth P's
fresh nodes; singletons only below P), each section in the order fo_e that the
push_front passes leave (fo_0 = root ascending; fo_e = reverse(fo_{e-1}) of the
parents, then quadrant descending).  With the root field and the odd depths'
quadrants complemented in the code, fo_e is the ascending code order for odd e and
its reverse for even e.  Each final round divides, in (count desc, list position
asc) order, the front nodes created by the previous round (or section P)."""
import ctypes as C
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _oracle as O  # noqa: E402

D = 14  # path depth carried in the code


def f32(v):
    return float(np.float32(v))


def ceil_half(d):
    return int(math.ceil(f32(f32(d) / 2)))


def codes(xs, ys, hX, nIni, H0):
    out = []
    for x, y in zip(xs, ys):
        idx = int(f32(f32(x) / hX))
        idx = min(idx, nIni - 1)
        x0, x1, y0, y1 = int(f32(hX * idx)), int(f32(hX * (idx + 1))), 0, H0
        c = (nIni - 1 - idx) << (2 * D)  # root descending in the flipped order
        for d in range(1, D + 1):
            mx, my = x0 + ceil_half(x1 - x0), y0 + ceil_half(y1 - y0)
            q = (x >= mx) + 2 * (y >= my)
            if q & 1: x0 = mx
            else: x1 = mx
            if q & 2: y0 = my
            else: y1 = my
            t = q ^ 3 if d & 1 else q  # flipped at odd depths
            c |= t << (2 * (D - d))
        out.append(c)
    return out


def prefix(c, d):
    return c >> (2 * (D - d))


def quad_at(c, d):  # real quadrant of the node at depth d (unflip)
    t = (c >> (2 * (D - d))) & 3
    return t ^ 3 if d & 1 else t


def octree_paths(xs, ys, resp, minX, maxX, minY, maxY, N):
    n = len(xs)
    if n == 0:
        return []
    nIni = max(1, int(np.round(np.float32(maxX - minX) / np.float32(maxY - minY))))  # roundf: half away
    r = f32(f32(maxX - minX) / f32(maxY - minY))
    nIni = max(1, int(math.floor(r + 0.5)))
    hX = f32(f32(maxX - minX) / nIni)
    H0 = maxY - minY
    cd = codes(xs, ys, hX, nIni, H0)
    order = sorted(range(n), key=lambda i: (cd[i], i))
    sc = [cd[i] for i in order]

    def lcp(a, b):  # deepest d with equal prefix (-1: roots differ)
        if prefix(a, 0) != prefix(b, 0):
            return -1
        d = 0
        while d < D and prefix(a, d + 1) == prefix(b, d + 1):
            d += 1
        return d

    L = [-1] + [lcp(sc[j - 1], sc[j]) for j in range(1, n)] + [-1]  # L[j]: between j-1 and j
    m = [max(L[j], L[j + 1]) for j in range(n)]
    size = lambda d: sum(1 for j in range(n) if L[j] < d)
    single = lambda d: sum(1 for j in range(n) if m[j] < d)
    P, final = 0, False
    prev = size(0)
    while True:
        P += 1
        assert P <= D, "keys not separated within D levels"
        s = size(P)
        nexp = s - single(P)
        if s >= N or s == prev:
            break
        if s + 3 * nexp > N:
            final = True
            break
        prev = s
    # main-loop list: node = (start, len, depth) over the sorted keys
    secs = {}
    j = 0
    while j < n:
        if m[j] + 1 <= P:
            e, ln = m[j] + 1, 1
        else:
            e, ln = P, 1
            while j + ln < n and L[j + ln] >= P:
                ln += 1
        secs.setdefault(e, []).append((j, ln, e))
        j += ln
    lst = []
    for e in range(P, -1, -1):
        nodes = secs.get(e, [])
        lst += nodes if e % 2 == 1 else nodes[::-1]
    if final:
        seq = 0
        fresh = [nd for nd in secs.get(P, []) if nd[1] > 1]  # array order
        # creation order = reverse fo_P
        fo = fresh if P % 2 == 1 else fresh[::-1]
        cands = [(nd[1], len(fo) - 1 - k, nd) for k, nd in enumerate(fo)]  # (count, seq)
        seq = len(fo)
        done = False
        while not done:
            prevSize = len(lst)
            cands.sort(key=lambda t: (t[0], t[1]))
            newc = []
            for cnt, sq, nd in reversed(cands):
                st, ln, dep = nd
                # children at dep+1: runs by prefix(dep+1); quadrant order ascending
                ch = []
                k = st
                while k < st + ln:
                    e2 = 1
                    while k + e2 < st + ln and L[k + e2] >= dep + 1:
                        e2 += 1
                    ch.append((k, e2, dep + 1))
                    k += e2
                ch.sort(key=lambda c: quad_at(sc[c[0]], dep + 1))
                i = lst.index(nd)
                del lst[i]
                for c in ch:
                    lst.insert(0, c)
                    if c[1] > 1:
                        newc.append((c[1], seq, c))
                    seq += 1
                if len(lst) >= N:
                    break
            if len(lst) >= N or len(lst) == prevSize:
                done = True
            cands = newc
    out = []
    for st, ln, dep in lst:
        best = max(range(st, st + ln), key=lambda k: (resp[order[k]], -order[k]))
        out.append(order[best])
    return out


def oracle_octree(xs, ys, resp, minX, maxX, minY, maxY, N):
    n = len(xs)
    kp = np.zeros(max(n, 1), O.KP_DTYPE)
    kp["x"][:n] = xs
    kp["y"][:n] = ys
    kp["response"][:n] = resp
    kp["class_id"][:n] = np.arange(n)
    out = np.zeros(max(4 * N + 64, n + 1), O.KP_DTYPE)
    lib = O.lib()
    lib.ygzo_distribute_octree.restype = C.c_int
    k = lib.ygzo_distribute_octree(kp.ctypes.data_as(C.c_void_p), n, minX, maxX, minY, maxY, N,
                                   out.ctypes.data_as(C.c_void_p), len(out))
    return [int(v) for v in out["class_id"][:k]]


def case(rng, W, H, n, N, clustered):
    minX, maxX, minY, maxY = 16, W - 16, 16, H - 16
    w, h = maxX - minX, maxY - minY
    if clustered:
        cx, cy = rng.integers(0, w, 6), rng.integers(0, h, 6)
        pts = set()
        while len(pts) < n:
            k = rng.integers(0, 6)
            s = rng.choice([2, 6, 30])
            x = int(np.clip(cx[k] + rng.normal(0, s), 0, w - 1))
            y = int(np.clip(cy[k] + rng.normal(0, s), 0, h - 1))
            pts.add((x, y))
        pts = list(pts)
    else:
        flat = rng.choice(w * h, n, replace=False)
        pts = [(int(v % w), int(v // w)) for v in flat]
    rng.shuffle(pts)
    xs = [p[0] for p in pts]
    ys = [p[1] for p in pts]
    resp = [int(v) for v in rng.integers(20, 40, n)]
    return xs, ys, resp, minX, maxX, minY, maxY, N


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    bad = 0
    for t in range(int(sys.argv[1]) if len(sys.argv) > 1 else 200):
        W, H = [(752, 480), (376, 240), (188, 120), (640, 480), (1241, 376), (94, 60)][t % 6]
        n = int(rng.integers(1, 1500))
        N = int(rng.integers(1, 600))
        args = case(rng, W, H, n, N, t % 3 == 0)
        a = octree_paths(*args)
        b = oracle_octree(*args)
        if a != b:
            bad += 1
            print("MISMATCH", t, W, H, n, N, len(a), len(b))
    print("bad", bad)


def octree_arrays(xs, ys, resp, minX, maxX, minY, maxY, N, Dn=None):
    """The kernel's formulation: flat arrays, list = node records (start, len, depth) in
    list order; final rounds divide the front nodes by (count desc, position asc)."""
    n = len(xs)
    if n == 0:
        return []
    r = f32(f32(maxX - minX) / f32(maxY - minY))
    nIni = max(1, int(math.floor(r + 0.5)))
    hX = f32(f32(maxX - minX) / nIni)
    H0 = maxY - minY
    cd = codes(xs, ys, hX, nIni, H0)
    order = sorted(range(n), key=lambda i: cd[i])
    sc = [cd[i] for i in order]
    assert len(set(sc)) == n
    L = [-1] * (n + 1)
    for j in range(1, n):
        x = sc[j - 1] ^ sc[j]
        if x >> (2 * D):
            L[j] = -1
        else:
            L[j] = (2 * D - x.bit_length()) // 2
    hL = np.bincount([v + 1 for v in L[:n]], minlength=D + 2)
    hm = np.bincount([max(L[j], L[j + 1]) + 1 for j in range(n)], minlength=D + 2)
    cL, cm = np.cumsum(hL), np.cumsum(hm)
    P, final, prev = 0, False, int(cL[0])
    while True:
        P += 1
        s = int(cL[P])
        nexp = s - int(cm[P])
        if s >= N or s == prev:
            break
        if s + 3 * nexp > N:
            final = True
            break
        prev = s
    heads = [j for j in range(n) if L[j] < P]
    sec = {j: min(max(L[j], L[j + 1]) + 1, P) for j in heads}
    cnt = np.bincount([sec[j] for j in heads], minlength=P + 1)
    base = {e: int(sum(cnt[e + 1:P + 1])) for e in range(P + 1)}
    rank = {}
    run = [0] * (P + 1)
    for j in heads:
        rank[j] = run[sec[j]]
        run[sec[j]] += 1
    nxt = heads[1:] + [n]
    lst = [None] * len(heads)
    for j, jn in zip(heads, nxt):
        e = sec[j]
        pos = base[e] + (rank[j] if e % 2 == 1 else cnt[e] - 1 - rank[j])
        lst[pos] = (j, jn - j, e)
    front = int(cnt[P])
    if final:
        while True:
            prevSize = len(lst)
            cand = [p for p in range(front) if lst[p][1] > 1]
            cand.sort(key=lambda p: (-lst[p][1], p))
            def children(nd):
                st, ln, dep = nd
                b = [st] + [k for k in range(st + 1, st + ln) if L[k] == dep]
                ch = [(b[i], (b[i + 1] if i + 1 < len(b) else st + ln) - b[i], dep + 1) for i in range(len(b))]
                return ch if (dep + 1) % 2 == 1 else ch[::-1]   # list-front order (quadrant descending)
            ech = [len(children(lst[p])) for p in cand]
            cum = np.cumsum([e - 1 for e in ech])
            cut = next((i for i in range(len(cand)) if prevSize + cum[i] >= N), len(cand) - 1)
            proc = cand[:cut + 1]
            newfront = []
            for p in reversed(proc):
                newfront += children(lst[p])
            ps = set(proc)
            lst = newfront + [lst[p] for p in range(len(lst)) if p not in ps]
            front = len(newfront)
            if len(lst) >= N or len(lst) == prevSize:
                break
    out = []
    for st, ln, dep in lst:
        best = max(range(st, st + ln), key=lambda k: (resp[order[k]], -order[k]))
        out.append(order[best])
    return out


def check_arrays(ntests):
    rng = np.random.default_rng(7)
    bad = 0
    for t in range(ntests):
        W, H = [(752, 480), (376, 240), (188, 120), (640, 480), (1241, 376), (94, 60)][t % 6]
        n = int(rng.integers(1, 1500))
        N = int(rng.integers(1, 600))
        args = case(rng, W, H, n, N, t % 3 == 0)
        if octree_arrays(*args) != oracle_octree(*args):
            bad += 1
            print("MISMATCH(arrays)", t, W, H, n, N)
    print("arrays bad", bad)
