"""The tracking-path ORBmatcher searches on the GPU (csrc/match.hip) against the oracle's
literal restatement of the reference loops (oracle/match.c), bit-exact on every output:

  SearchByProjection(CurrentFrame, LastFrame, th, bMono, checkLevel)   ORBmatcher.cc:1218-1350
  SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)   ORBmatcher.cc:1352-1469
  SearchByProjection(F, vpMapPoints, th, checkLevel)                  ORBmatcher.cc:43-126
  SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, ws)     ORBmatcher.cc:375-478
  SearchByBoW(pKF, F, vpMapPointMatches)                              ORBmatcher.cc:155-263

C2 (EuRoC 752x480, 1000 features) and C4 (TUM 640x480, 2000 features) frame pairs, rotation
check on and off, plus dense windows where the sequential skips exhaust the GPU's per-query
top-K list (the re-scan path).

Every test runs twice: with the parallel resolve (k_match_resolve, the default) and with
the serial replay alone (YGZFE_MATCH_PASSES=0); test_resolve_long_chains drives the resolve
through long dependency chains."""
import os

import numpy as np
import pytest

import _oracle as O
import _scenes as S

pytestmark = pytest.mark.gpu

PAIRS = {}


@pytest.fixture(autouse=True, params=["resolve", "serial"])
def decide(request):
    old = os.environ.get("YGZFE_MATCH_PASSES")
    if request.param == "serial":
        os.environ["YGZFE_MATCH_PASSES"] = "0"
    else:
        os.environ.pop("YGZFE_MATCH_PASSES", None)
    yield request.param
    if old is None:
        os.environ.pop("YGZFE_MATCH_PASSES", None)
    else:
        os.environ["YGZFE_MATCH_PASSES"] = old


def pair(cfg, seed):
    if (cfg, seed) not in PAIRS:
        PAIRS[(cfg, seed)] = S.match_pair(cfg, seed)
    return PAIRS[(cfg, seed)]


def bounds(p):
    return (0.0, float(p["W"]), 0.0, float(p["H"]))


def gpu_frame(gpu, kps, desc, ur, p):
    return gpu.MatchFrame(0).set(kps, desc, ur, bounds(p))


@pytest.mark.parametrize("cfg,seed", [("C2", 0), ("C2", 1), ("C4", 2)])
@pytest.mark.parametrize("check_ori", [True, False])
def test_search_by_projection_last_frame(gpu, cfg, seed, check_ori, decide):
    p = pair(cfg, seed)
    for th, lm in ((7.0, "mixed"), (15.0, "band"), (14.0, "none")):
        Q, qd, ur, bl = S.projection_queries(p, seed, th=th, level_mode=lm)
        cur = gpu_frame(gpu, p["k1"], p["d1"], ur, p)
        got, gn = gpu.search_projection_best(cur, Q, qd, bl, 100, check_ori)
        want, wn = O.search_projection_best(O.mframe(p["k1"], p["d1"], ur, bounds(p)), Q, qd, bl, 100, check_ori)
        assert gn == wn and np.array_equal(got, want), (th, lm, gn, wn, np.flatnonzero(got != want)[:10])
        assert wn > 50  # the scene really matches
        assert (cur.resolve_passes() >= 1) == (decide == "resolve")  # the path under test decided


@pytest.mark.parametrize("check_ori", [True, False])
def test_search_by_projection_keyframe_relocalisation(gpu, check_ori):
    """The sAlreadyFound / ORBdist form: any assigned keypoint blocks (every query BLOCKS)."""
    p = pair("C2", 0)
    Q, qd, ur, bl = S.projection_queries(p, 3, th=10.0, level_mode="band", stereo_frac=0.0)
    Q["flags"] |= 2
    cur = gpu_frame(gpu, p["k1"], p["d1"], None, p)
    for orbdist in (50, 64, 100):
        got, gn = gpu.search_projection_best(cur, Q, qd, bl, orbdist, check_ori)
        want, wn = O.search_projection_best(O.mframe(p["k1"], p["d1"], None, bounds(p)), Q, qd, bl, orbdist,
                                            check_ori)
        assert gn == wn and np.array_equal(got, want)


@pytest.mark.parametrize("cfg,seed", [("C2", 1), ("C4", 2)])
def test_search_by_projection_local_map_ratio(gpu, cfg, seed, decide):
    p = pair(cfg, seed)
    for nnratio, lm in ((0.8, "band"), (0.6, "mixed"), (1.0, "none")):
        Q, qd, ur, bl = S.projection_queries(p, seed + 10, th=3.0 * 2.5, level_mode=lm)
        F = gpu_frame(gpu, p["k1"], p["d1"], ur, p)
        got, gn = gpu.search_projection_ratio(F, Q, qd, bl, nnratio)
        want, wn = O.search_projection_ratio(O.mframe(p["k1"], p["d1"], ur, bounds(p)), Q, qd, bl, nnratio)
        assert gn == wn and np.array_equal(got, want), (nnratio, lm)
        assert wn > 30
        assert (F.resolve_passes() >= 1) == (decide == "resolve")


@pytest.mark.parametrize("cfg,seed", [("C2", 0), ("C4", 2)])
@pytest.mark.parametrize("check_ori", [True, False])
@pytest.mark.parametrize("window", [100, 30])
def test_search_for_initialization(gpu, cfg, seed, check_ori, window):
    """Tracking.cc:825-826: ORBmatcher(0.9, true).SearchForInitialization(..., 100)."""
    p = pair(cfg, seed)
    rng = np.random.default_rng(seed)
    prev = np.stack([p["k0"]["x"], p["k0"]["y"]], 1).astype(np.float32) + rng.uniform(-2, 2, (len(p["k0"]), 2))
    prev = prev.astype(np.float32)
    F1 = gpu_frame(gpu, p["k0"], p["d0"], None, p)
    F2 = gpu_frame(gpu, p["k1"], p["d1"], None, p)
    got, gn, gprev = gpu.search_for_initialization(F1, F2, prev, window, 0.9, check_ori)
    want, wn, wprev = O.search_for_initialization(O.mframe(p["k0"], p["d0"], None, bounds(p)),
                                                  O.mframe(p["k1"], p["d1"], None, bounds(p)), prev, window, 0.9,
                                                  check_ori)
    assert gn == wn and np.array_equal(got, want)
    assert np.array_equal(gprev, wprev)
    assert wn > 20


@pytest.mark.parametrize("check_ori", [True, False])
@pytest.mark.parametrize("n_nodes", [40, 400])
def test_search_by_bow(gpu, check_ori, n_nodes, decide):
    """Tracking.cc:1018-1020 ORBmatcher(0.7, false) and :1847 (0.75, true)."""
    p = pair("C2", 1)
    rng = np.random.default_rng(n_nodes)
    usable = (rng.random(len(p["k0"])) < 0.85).astype(np.uint8)
    fv0 = S.feature_vector(p["d0"], n_nodes, 0)
    fv1 = S.feature_vector(p["d1"], n_nodes, 0)
    # drop some nodes on each side so the lower_bound walk skips
    keep0 = rng.random(len(fv0[0])) < 0.9
    fv0 = sub_fv(fv0, keep0)
    KF = gpu_frame(gpu, p["k0"], p["d0"], None, p)
    F = gpu_frame(gpu, p["k1"], p["d1"], None, p)
    for nnratio in (0.7, 0.75, 0.95):
        got, gn = gpu.search_by_bow(KF, F, usable, fv0, fv1, nnratio, check_ori)
        want, wn = O.search_by_bow(O.mframe(p["k0"], p["d0"], None, bounds(p)),
                                   O.mframe(p["k1"], p["d1"], None, bounds(p)), usable, fv0, fv1, nnratio, check_ori)
        assert gn == wn and np.array_equal(got, want), nnratio
        assert wn > 10
        assert (F.resolve_passes() >= 1) == (decide == "resolve")


@pytest.mark.parametrize("mode", ["init", "bow"])
def test_query_frame_upload_in_flight(gpu, mode, decide):
    """SearchForInitialization / SearchByBoW read the query frame's descriptors on the device
    from the train frame's stream.  The query frame is set (async upload on its own stream)
    with that stream held for 20 ms (YGZFE_DEBUG_SET_HOLD_US) and the search starts at once:
    it must wait for the upload (ev_ready) and still equal the oracle."""
    p = pair("C2", 0)
    F2 = gpu_frame(gpu, p["k1"], p["d1"], None, p)
    os.environ["YGZFE_DEBUG_SET_HOLD_US"] = "20000"
    try:
        F1 = gpu_frame(gpu, p["k0"], p["d0"], None, p)  # fresh device buffers, upload held
    finally:
        os.environ.pop("YGZFE_DEBUG_SET_HOLD_US", None)
    if mode == "init":
        rng = np.random.default_rng(3)
        prev = (np.stack([p["k0"]["x"], p["k0"]["y"]], 1) + rng.uniform(-2, 2, (len(p["k0"]), 2))).astype(np.float32)
        got, gn, _ = gpu.search_for_initialization(F1, F2, prev, 100, 0.9, True)
        want, wn, _ = O.search_for_initialization(O.mframe(p["k0"], p["d0"], None, bounds(p)),
                                                  O.mframe(p["k1"], p["d1"], None, bounds(p)), prev, 100, 0.9, True)
    else:
        usable = np.ones(len(p["k0"]), np.uint8)
        fv0 = S.feature_vector(p["d0"], 40, 0)
        fv1 = S.feature_vector(p["d1"], 40, 0)
        got, gn = gpu.search_by_bow(F1, F2, usable, fv0, fv1, 0.75, True)
        want, wn = O.search_by_bow(O.mframe(p["k0"], p["d0"], None, bounds(p)),
                                   O.mframe(p["k1"], p["d1"], None, bounds(p)), usable, fv0, fv1, 0.75, True)
    assert gn == wn and np.array_equal(got, want)
    assert wn > 10


def sub_fv(fv, keep):
    nodes, ptr, feats = fv
    nn, pp, ff = [], [0], []
    for k in np.flatnonzero(keep):
        nn.append(nodes[k])
        ff.extend(feats[ptr[k]:ptr[k + 1]])
        pp.append(len(ff))
    return np.array(nn, np.int32), np.array(pp, np.int32), np.array(ff, np.int32)


def test_dense_windows_exhaust_topk(gpu):
    """Wide windows and every query blocking: later queries find their K best candidates taken
    and the GPU re-scans them; INIT with a huge window re-assigns keypoints (vMatchedDistance)."""
    p = pair("C2", 0)
    Q, qd, ur, bl = S.projection_queries(p, 9, th=40.0, level_mode="none", blocks_frac=1.0, stereo_frac=0.0,
                                         valid_frac=1.0, flip_bits=40)
    cur = gpu_frame(gpu, p["k1"], p["d1"], None, p)
    for check_ori in (True, False):
        got, gn = gpu.search_projection_best(cur, Q, qd, None, 100, check_ori)
        want, wn = O.search_projection_best(O.mframe(p["k1"], p["d1"], None, bounds(p)), Q, qd, None, 100, check_ori)
        assert gn == wn and np.array_equal(got, want)
        assert cur.rescans() > 0  # the re-scan path really ran
    got, gn = gpu.search_projection_ratio(cur, Q, qd, None, 0.9)
    want, wn = O.search_projection_ratio(O.mframe(p["k1"], p["d1"], None, bounds(p)), Q, qd, None, 0.9)
    assert gn == wn and np.array_equal(got, want)
    prev = np.full((len(p["k0"]), 2), (376.0, 240.0), np.float32)  # every window the whole image
    F1 = gpu_frame(gpu, p["k0"], p["d0"], None, p)
    got, gn, _ = gpu.search_for_initialization(F1, cur, prev, 500, 0.95, True)
    want, wn, _ = O.search_for_initialization(O.mframe(p["k0"], p["d0"], None, bounds(p)),
                                              O.mframe(p["k1"], p["d1"], None, bounds(p)), prev, 500, 0.95, True)
    assert gn == wn and np.array_equal(got, want)
    assert cur.rescans() > 0


def test_empty_inputs(gpu):
    p = pair("C2", 0)
    cur = gpu_frame(gpu, p["k1"], p["d1"], None, p)
    empty = np.zeros(0, gpu.MATCH_QUERY_DTYPE)
    got, gn = gpu.search_projection_best(cur, empty, np.zeros((0, 32), np.uint8), None, 100, True)
    assert gn == 0 and (got == -1).all()
    none = gpu.MatchFrame(0).set(np.zeros(0, gpu.KP_DTYPE), np.zeros((0, 32), np.uint8), None, bounds(p))
    Q, qd, _, _ = S.projection_queries(p, 1)
    got, gn = gpu.search_projection_best(none, Q, qd, None, 100, True)
    assert gn == 0 and len(got) == 0


def test_resolve_long_chains(gpu, decide):
    """Every query blocking and windows of 40 px: each query's best candidates are taken by
    the ones before it, so decisions feed each other in long chains (many resolve passes,
    re-scans in most passes); the result equals the oracle's and the serial replay's."""
    p = pair("C2", 0)
    Q, qd, ur, bl = S.projection_queries(p, 9, th=40.0, level_mode="none", blocks_frac=1.0, stereo_frac=0.0,
                                         valid_frac=1.0, flip_bits=40)
    cur = gpu_frame(gpu, p["k1"], p["d1"], None, p)
    got, gn = gpu.search_projection_best(cur, Q, qd, None, 100, True)
    want, wn = O.search_projection_best(O.mframe(p["k1"], p["d1"], None, bounds(p)), Q, qd, None, 100, True)
    assert gn == wn and np.array_equal(got, want)
    if decide == "resolve":
        assert cur.resolve_passes() > 8, cur.resolve_passes()
    else:
        assert cur.resolve_passes() == -1
