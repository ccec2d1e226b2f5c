"""Offline sequence mode on the device: the bench's device-side
frame renderer against the host renderer, and ygzfe_batch_pack_slots against the
numpy slot packing of ygzfe.dist (the layout the RCCL gather moves to rank 0)."""
import numpy as np
import pytest
import torch

import _scenes as S
from ygzfe import dist as D

pytestmark = pytest.mark.gpu


def _poses(n, xi=(0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015)):
    import ygzfe
    xi = np.array(xi, np.float32)
    return [ygzfe.trajectory_pose(g, xi) for g in range(n)]


def test_render_plane_device_matches_host(gpu):
    ygzfe = gpu
    sc = S.PlaneScene(11)
    poses = _poses(3)
    dev = torch.device("cuda", 0)
    tex = torch.from_numpy(sc.tex).to(dev)
    q = torch.from_numpy(np.stack([p[0] for p in poses])).to(dev)
    t = torch.from_numpy(np.stack([p[1] for p in poses])).to(dev)
    seeds = torch.arange(3, dtype=torch.int64, device=dev)
    pitch = 752 * 480 + 64
    out = torch.zeros(3 * pitch, dtype=torch.uint8, device=dev)
    ygzfe.render_plane_device(tex.data_ptr(), S.TEX_W, S.TEX_H, S.TEXEL, S.PLANE_Z, sc.cam, q.data_ptr(),
                              t.data_ptr(), seeds.data_ptr(), 3, 752, 480, out.data_ptr(), pitch, noise_amp=0)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for i, (qq, tt) in enumerate(poses):
        want = sc.render(qq, tt, noise_seed=0, noise_amp=0)
        assert np.array_equal(got[i * pitch:i * pitch + 752 * 480].reshape(480, 752), want), f"frame {i}"
    # with noise: every frame distinct, noise bounded by +-2 around the clean render
    ygzfe.render_plane_device(tex.data_ptr(), S.TEX_W, S.TEX_H, S.TEXEL, S.PLANE_Z, sc.cam, q.data_ptr(),
                              t.data_ptr(), seeds.data_ptr(), 3, 752, 480, out.data_ptr(), pitch, noise_amp=2)
    noisy = out.cpu().numpy()
    for i, (qq, tt) in enumerate(poses):
        clean = sc.render(qq, tt, noise_seed=0, noise_amp=0).astype(np.int32)
        d = noisy[i * pitch:i * pitch + 752 * 480].reshape(480, 752).astype(np.int32) - clean
        assert np.abs(d).max() <= 2 and (d != 0).mean() > 0.5


def test_pack_slots_matches_numpy(gpu):
    ygzfe = gpu
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    sc = S.PlaneScene(11)
    F = 6
    poses = _poses(F)
    frames = np.stack([sc.render(q, t, noise_seed=g) for g, (q, t) in enumerate(poses)])
    b = ygzfe.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, F)
    b.upload(frames)
    b.extract(F)
    b.check()
    cap = b.kp_cap
    dev = torch.device("cuda", 0)
    P = F - 1
    res = [b.result(i) for i in range(F)]
    xyz = np.zeros((P, cap, 3), np.float32)
    us = np.zeros((P, cap), np.uint8)
    for p in range(P):
        k = res[p][0]
        Pw, ok = sc.map_points(*poses[p], k)
        xyz[p, :len(k)] = S.world_to_cam(poses[p], Pw)
        us[p, :len(k)] = ok
    ref_idx = torch.arange(0, P, dtype=torch.int32, device=dev)
    cur_idx = ref_idx + 1
    T0 = torch.zeros((P, 7), dtype=torch.float32, device=dev)
    T0[:, 3] = 1
    out = torch.zeros((P, 45), dtype=torch.float32, device=dev)
    xyz_d = torch.from_numpy(xyz).to(dev)
    us_d = torch.from_numpy(us).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    b.sparse_align(P, ref_idx.data_ptr(), cur_idx.data_ptr(), xyz_d.data_ptr(), us_d.data_ptr(), sc.camera(), 3, 1,
                   T0.data_ptr(), out.data_ptr(), st)
    S_b = ygzfe.slot_bytes(cap)
    assert S_b == D.slot_bytes(cap)
    for fb, n, g0 in ((0, F, 100), (1, F - 1, 7)):  # whole batch; a halo-shard (frame 0 = halo)
        slots = torch.full((n, S_b), 0xAB, dtype=torch.uint8, device=dev)
        b.pack_slots(fb, n, out.data_ptr(), g0, slots.data_ptr(), S_b, st)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        align = np.zeros(F, D.ALIGN_DTYPE)
        for f in range(1, F):
            r = o[f - 1]
            align[f] = (tuple(r[0:4]), tuple(r[4:7]), int(r[7:8].view(np.int32)[0]), float(r[8]))
        kps = np.zeros((F, cap), ygzfe.KP_DTYPE)
        desc = np.zeros((F, cap, 32), np.uint8)
        counts = np.array([len(k) for k, _ in res], np.int32)
        for i, (k, d) in enumerate(res):
            kps[i, :len(k)] = k
            desc[i, :len(k)] = d
        want = D.pack_slots(counts[fb:], kps[fb:], desc[fb:], align[fb:], global_first=g0,
                            has_align=np.arange(fb, F) >= 1)
        got = slots.cpu().numpy()
        assert np.array_equal(got, want)
        s1 = D.unpack_slot(got[1], cap, ygzfe.KP_DTYPE)
        assert s1["has_align"] and s1["n_visible"] > 100 and s1["frame"] == g0 + 1
