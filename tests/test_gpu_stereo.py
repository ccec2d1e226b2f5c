"""GPU stereo vs the oracle.

Frame::ComputeStereoMatches (Frame.cc:509-682): row-band Hamming, 11x11 SAD
sliding window + parabola, median outlier cut — mvuRight / mvDepth bit-exact.
Frame::ComputeStereoFromRGBD (Frame.cc:684-700): bit-exact.
"""
import numpy as np
import pytest

import _oracle as O
import _scenes as S

pytestmark = pytest.mark.gpu


def _extract_pair(gpu, cfg, d):
    W, H, nf, sf, nl, ini, mn = cfg
    ex_l = gpu.ORBextractor(nf, sf, nl, ini, mn)
    ex_r = gpu.ORBextractor(nf, sf, nl, ini, mn)  # the stereo Frame's two extractors
    fl, fr = ex_l.ComputePyramid(d["left"]), ex_r.ComputePyramid(d["right"])
    kl, dl = ex_l.extract(fl)
    kr, dr = ex_r.extract(fr)
    return ex_l, ex_r, fl, fr, kl, dl, kr, dr


@pytest.mark.parametrize("cfg,seed", [("C2", 0), ("C2", 1), ("C1", 2), ("C4", 3)])
def test_stereo_matches_bitexact(gpu, cfg, seed):
    W, H, nf, sf, nl, ini, mn = S.CONFIGS[cfg]
    d = S.stereo_scene(seed, W, H)
    ex_l, ex_r, fl, fr, kl, dl, kr, dr = _extract_pair(gpu, S.CONFIGS[cfg], d)
    ur, dep = gpu.stereo_matches(fl, fr, kl, dl, kr, dr, d["mb"], d["mbf"])
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    our, odep, osad = O.stereo_matches(orc, orc.pyramid(d["left"]), orc.pyramid(d["right"]), kl, dl, kr, dr, d["mb"],
                                       d["mbf"])
    assert np.array_equal(ur, our)
    assert np.array_equal(dep, odep)
    ok = dep > 0
    assert ok.mean() > 0.3, ok.mean()
    # the recovered depth is the plane's depth at the keypoint (sanity of the restatement)
    sc = d["scene"]
    Pw, _ = sc.map_points(d["pose"][0].astype(np.float32), d["pose"][1].astype(np.float32), kl[ok])
    Pc = np.array([S.quat_rot(d["pose"][0], p) + d["pose"][1] for p in Pw])
    rel = np.abs(dep[ok] - Pc[:, 2]) / Pc[:, 2]
    assert np.median(rel) < 0.05, np.median(rel)
    assert (osad[ok] >= 0).all() and (osad[~ok] == -1).all()


def test_stereo_edges(gpu):
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    d = S.stereo_scene(4, W, H)
    ex_l, ex_r, fl, fr, kl, dl, kr, dr = _extract_pair(gpu, S.CONFIGS["C2"], d)
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    ll, rl = orc.pyramid(d["left"]), orc.pyramid(d["right"])
    # no left keypoints, no right keypoints, one left keypoint
    ur, dep = gpu.stereo_matches(fl, fr, kl[:0], dl[:0], kr, dr, d["mb"], d["mbf"])
    assert len(ur) == 0
    ur, dep = gpu.stereo_matches(fl, fr, kl, dl, kr[:0], dr[:0], d["mb"], d["mbf"])
    assert (ur == -1).all() and (dep == -1).all()
    for sl in (slice(0, 1), slice(0, 7), slice(3, 300)):
        ur, dep = gpu.stereo_matches(fl, fr, kl[sl], dl[sl], kr, dr, d["mb"], d["mbf"])
        our, odep, _ = O.stereo_matches(orc, ll, rl, kl[sl], dl[sl], kr, dr, d["mb"], d["mbf"])
        assert np.array_equal(ur, our) and np.array_equal(dep, odep)
    # identical images: disparities ~0 (clamped to 0.01 px, Frame.cc:661-664), all SADs 0, so the
    # median cut (SAD >= 2.1 x 0) drops every match, as in the reference
    ur, dep = gpu.stereo_matches(fl, fl, kl, dl, kl, dl, d["mb"], d["mbf"])
    our, odep, _ = O.stereo_matches(orc, ll, ll, kl, dl, kl, dl, d["mb"], d["mbf"])
    assert np.array_equal(ur, our) and np.array_equal(dep, odep)
    with pytest.raises(gpu.YgzfeError):
        gpu.stereo_matches(fl, fr, kl, dl, kr, dr, 0.0, d["mbf"])


def test_batch_stereo_matches_single(gpu):
    import torch
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    scenes = [S.stereo_scene(10 + i, W, H) for i in range(3)]
    frames = np.stack([im for d in scenes for im in (d["left"], d["right"])])
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, len(frames))
    b.upload(frames)
    b.extract(len(frames))
    b.check()
    cap = b.kp_cap
    dev = torch.device("cuda", 0)
    li = torch.tensor([0, 2, 4], dtype=torch.int32, device=dev)
    ri = torch.tensor([1, 3, 5], dtype=torch.int32, device=dev)
    ur = torch.zeros((3, cap), dtype=torch.float32, device=dev)
    dep = torch.zeros((3, cap), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    b.stereo(3, li.data_ptr(), ri.data_ptr(), scenes[0]["mb"], scenes[0]["mbf"], ur.data_ptr(), dep.data_ptr())
    b.check()
    ur, dep = ur.cpu().numpy(), dep.cpu().numpy()
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    for p, d in enumerate(scenes):
        kl, dl = b.result(2 * p)
        kr, dr = b.result(2 * p + 1)
        fl, fr = ex.ComputePyramid(d["left"]), ex.ComputePyramid(d["right"])
        sur, sdep = gpu.stereo_matches(fl, fr, kl, dl, kr, dr, d["mb"], d["mbf"])
        n = len(kl)
        assert np.array_equal(ur[p, :n], sur) and np.array_equal(dep[p, :n], sdep)
        assert (dep[p, :n] > 0).mean() > 0.3


def test_stereo_from_rgbd_bitexact(gpu):
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C4"]
    rng = np.random.default_rng(7)
    img = S.frame(7, W, H)
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    kps, _ = ex.extract(ex.ComputePyramid(img))
    depth = rng.uniform(0.5, 4.0, (H, W)).astype(np.float32)
    depth[rng.random((H, W)) < 0.2] = 0.0  # holes
    mbf = 40.0  # TUM1.yaml Camera.bf
    ur, dep = gpu.stereo_from_rgbd(depth, kps, mbf)
    our, odep = O.stereo_from_rgbd(depth, kps, mbf)
    assert np.array_equal(ur, our) and np.array_equal(dep, odep)
    assert (dep > 0).mean() > 0.6
