"""Batched SparseImgAlign (ygzfe_batch_sparse_align, the bench path) vs the oracle, pair by pair.

SparseImgAlign::run (SparseImageAlign.cc:20-49) of frame k-1 -> k for every pair of a resident
batch; pose within 1e-4 (|log(T_gpu^-1 T_cpu)|_inf) and the same visible-feature count.  Up to 960
reference features per pair run in k_sparse_align_reg's register / LDS form (one feature per thread
of waves 1..15); more take its generic path (sparse_align_generic: global scratch, Eigen's pivoted
LDLT), exercised here with 2000-feature extractions.  Fast motion makes features leave the image
during the iterations, which exercises the out-of-bounds H correction.
"""
import numpy as np
import pytest

import _oracle as O
import _scenes as S

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-4
XI = np.array([0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015], np.float32)


def run_batch_align(gpu, F, stride, max_level, min_level, usable_frac=1.0, seed=11, nfeatures=None):
    import torch
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    nf = nfeatures or nf
    sc = S.PlaneScene(seed, W, H)
    poses = [gpu.trajectory_pose(k * stride, XI) for k in range(F)]
    frames = np.stack([sc.render(q, t, noise_seed=k) for k, (q, t) in enumerate(poses)])
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, F)
    b.upload(frames)
    b.extract(F)
    b.check()
    cap = b.kp_cap
    P = F - 1
    kps = [b.result(i)[0] for i in range(F)]
    xyz = np.zeros((P, cap, 3), np.float32)
    usable = np.zeros((P, cap), np.uint8)
    rng = np.random.default_rng(seed)
    for p in range(P):
        q, t = poses[p]
        Pw, ok = sc.map_points(q, t, kps[p])
        n = len(kps[p])
        xyz[p, :n] = [S.quat_rot(q.astype(np.float64), w) + t for w in Pw]
        usable[p, :n] = ok.astype(bool) & (rng.random(n) < usable_frac)
    d_xyz = torch.from_numpy(xyz).cuda()
    d_us = torch.from_numpy(usable).cuda()
    ref_idx = torch.arange(0, P, dtype=torch.int32, device="cuda")
    cur_idx = torch.arange(1, F, dtype=torch.int32, device="cuda")
    T0 = torch.zeros((P, 7), dtype=torch.float32, device="cuda")
    T0[:, 3] = 1.0
    out = torch.zeros((P, 45), dtype=torch.float32, device="cuda")
    b.sparse_align(P, ref_idx.data_ptr(), cur_idx.data_ptr(), d_xyz.data_ptr(), d_us.data_ptr(), sc.camera(),
                   max_level, min_level, T0.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    res = out.cpu().numpy()
    nvis = out[:, 7].contiguous().view(torch.int32).cpu().numpy()
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    ocam = O.Cam(*sc.cam)
    oT0 = O.se3_from((0, 0, 0, 1), (0, 0, 0))
    pyrs = [orc.pyramid(f) for f in frames]
    errs = []
    for p in range(P):
        n = len(kps[p])
        o = O.sparse_align(pyrs[p], pyrs[p + 1], orc.inv_scale, ocam, kps[p], xyz[p, :n], usable[p, :n], max_level,
                           min_level, oT0)
        err = S.se3_log_inf(res[p, 0:4], res[p, 4:7], np.array(o.T.q[:]), np.array(o.T.t[:]))
        errs.append(err)
        assert err <= POSE_TOL, f"pair {p}: GPU vs CPU pose differ by {err}"
        assert nvis[p] == o.n_visible, f"pair {p}: n_visible {nvis[p]} vs {o.n_visible}"
    return np.array(errs), nvis


def test_batch_align_levels_3_1(gpu):
    errs, nvis = run_batch_align(gpu, F=6, stride=1, max_level=3, min_level=1)
    assert (nvis > 100).all()


def test_batch_align_fast_motion(gpu):
    """4x the per-frame motion: features cross the level borders between iterations."""
    run_batch_align(gpu, F=5, stride=4, max_level=3, min_level=1)


def test_batch_align_partial_usable(gpu):
    run_batch_align(gpu, F=4, stride=2, max_level=3, min_level=1, usable_frac=0.4, seed=3)


def test_batch_align_level0_register_kernel(gpu):
    """Level 0 (752x480) exceeds the LDS image budget: the register-resident kernel runs."""
    run_batch_align(gpu, F=3, stride=1, max_level=2, min_level=0)


def test_batch_align_generic_path_over_960_features(gpu):
    """ORBextractor(2000, 2.0, 4) on 752x480: ~1900 reference features per pair (> 960), so every
    pair runs sparse_align_generic; levels 3..1 and 2..0."""
    errs, nvis = run_batch_align(gpu, F=4, stride=1, max_level=3, min_level=1, nfeatures=2000, seed=5)
    assert (nvis > 960).all()
    run_batch_align(gpu, F=3, stride=2, max_level=2, min_level=0, nfeatures=2000, seed=6, usable_frac=0.8)
