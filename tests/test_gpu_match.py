"""GPU Hamming matching vs the oracle (ORBmatcher.cc:1507-1523 + search loops): bit-exact."""
import numpy as np
import pytest

import _oracle as O
import _scenes as S

pytestmark = pytest.mark.gpu


def rand_desc(rng, n):
    return rng.integers(0, 256, (n, 32), dtype=np.uint8)


@pytest.mark.parametrize("nq,nt", [(1, 1), (100, 37), (1000, 1000), (300, 2500), (2000, 2000)])
def test_best2_random(gpu, nq, nt):
    rng = np.random.default_rng(nq * 7 + nt)
    q, t = rand_desc(rng, nq), rand_desc(rng, nt)
    # plant exact duplicates and ties so the first-index rule is exercised
    t[nt // 2] = q[0]
    if nt > 3:
        t[nt - 1] = q[0]
    m = gpu.ORBmatcher()
    bi, bd, sd = m.best2(q, t)
    ri, rd, rs = O.hamming_best2(q, t)
    assert np.array_equal(bi, ri) and np.array_equal(bd, rd) and np.array_equal(sd, rs)
    assert bd[0] == 0 and bi[0] == nt // 2


def test_best2_empty_train(gpu):
    rng = np.random.default_rng(1)
    q = rand_desc(rng, 5)
    bi, bd, sd = gpu.ORBmatcher().best2(q, np.zeros((0, 32), np.uint8))
    assert (bi == -1).all() and (bd == 257).all() and (sd == 257).all()


def test_descriptor_distance(gpu):
    rng = np.random.default_rng(2)
    a, b = rand_desc(rng, 50), rand_desc(rng, 50)
    for i in range(50):
        assert gpu.ORBmatcher.DescriptorDistance(a[i], b[i]) == O.lib().ygzo_descriptor_distance(O._p(a[i]), O._p(b[i]))


def test_window_csr(gpu):
    rng = np.random.default_rng(3)
    q, t = rand_desc(rng, 200), rand_desc(rng, 300)
    counts = rng.integers(0, 40, 200)
    row_ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    cand = rng.integers(0, 300, row_ptr[-1]).astype(np.int32)
    d = gpu.ORBmatcher().window_distances(q, t, row_ptr, cand)
    for i in range(200):
        for k in range(row_ptr[i], row_ptr[i + 1]):
            assert d[k] == O.lib().ygzo_descriptor_distance(O._p(q[i]), O._p(t[cand[k]]))


def test_best2_on_extracted_frames(gpu):
    """C2: descriptors of frame k vs frame k+1 of a rendered sequence (dense 1000x1000-class search)."""
    sc = S.PlaneScene(3)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    q0, t0 = np.array([0, 0, 0, 1], np.float32), np.zeros(3, np.float32)
    v, w = S.motion(0)
    q1 = S.quat_from_rotvec(w).astype(np.float32)
    f0 = sc.render(q0, t0, 1)
    f1 = sc.render(q1, v.astype(np.float32), 2)
    k0, d0 = ex(f0)
    k1, d1 = ex(f1)
    bi, bd, sd = gpu.ORBmatcher().best2(d1, d0)
    ri, rd, rs = O.hamming_best2(d1, d0)
    assert np.array_equal(bi, ri) and np.array_equal(bd, rd) and np.array_equal(sd, rs)
    # sanity: most keypoints find a close match in the previous frame
    assert np.mean(bd < 50) > 0.5


@pytest.mark.parametrize("nt", [31, 32, 33, 64, 95])
def test_best2_tile_edges_and_ties(gpu, nt):
    """Train sizes around the 32-row MFMA tile; many equal distances (first index wins)."""
    rng = np.random.default_rng(nt)
    base = rand_desc(rng, 4)
    t = base[rng.integers(0, 4, nt)]          # heavy duplication -> ties everywhere
    q = np.concatenate([base, rand_desc(rng, 61)])
    bi, bd, sd = gpu.ORBmatcher().best2(q, t)
    ri, rd, rs = O.hamming_best2(q, t)
    assert np.array_equal(bi, ri) and np.array_equal(bd, rd) and np.array_equal(sd, rs)


@pytest.mark.parametrize("nt", [8191, 8192, 8193, 9000])
def test_best2_fused_key_boundary(gpu, nt):
    """hamming.hip's FP4 form keeps the key in the accumulators for train sets of <= 8,192
    rows (tile index < 256) and builds it per element above that: both sides of the switch,
    with duplicates of a query planted at the first and last rows and across tile 255."""
    rng = np.random.default_rng(nt)
    q, t = rand_desc(rng, 70), rand_desc(rng, nt)
    for r in (0, 8160, 8191 % nt, nt - 1):
        t[r] = q[1]
    t[8190 % nt] = q[2]
    t[nt - 2] = q[2]
    bi, bd, sd = gpu.ORBmatcher().best2(q, t)
    ri, rd, rs = O.hamming_best2(q, t)
    assert np.array_equal(bi, ri) and np.array_equal(bd, rd) and np.array_equal(sd, rs)
    assert bi[1] == 0 and bd[1] == 0 and sd[1] == 0


def test_best2_extreme_distances(gpu):
    """All-zero vs all-one descriptors: distances 0 and 256 (the key's full range)."""
    z, o = np.zeros((1, 32), np.uint8), np.full((1, 32), 255, np.uint8)
    q = np.concatenate([z, o, z, o])
    t = np.concatenate([o, o, z, o, z])
    bi, bd, sd = gpu.ORBmatcher().best2(q, t)
    ri, rd, rs = O.hamming_best2(q, t)
    assert np.array_equal(bi, ri) and np.array_equal(bd, rd) and np.array_equal(sd, rs)
    assert bd[0] == 0 and bi[0] == 2 and sd[0] == 0
    t1 = np.concatenate([o])
    bi, bd, sd = gpu.ORBmatcher().best2(z, t1)
    assert bi[0] == 0 and bd[0] == 256 and sd[0] == 257


def test_batch_match_pairs(gpu):
    """ygzfe_batch_match (the bench path): frame k vs frame k-1 of a batch, every pair."""
    import torch
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    F = 5
    frames = np.stack([S.frame(20 + s, W, H) for s in range(F)])
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, F)
    b.upload(frames)
    b.extract(F)
    b.check()
    P = F - 1
    cap = b.kp_cap
    qf = torch.arange(1, F, dtype=torch.int32, device="cuda")
    tf = torch.arange(0, P, dtype=torch.int32, device="cuda")
    bi = torch.full((P, cap), -7, dtype=torch.int32, device="cuda")
    bd, sd = torch.empty_like(bi), torch.empty_like(bi)
    b.match(P, qf.data_ptr(), tf.data_ptr(), bi.data_ptr(), bd.data_ptr(), sd.data_ptr())
    torch.cuda.synchronize()
    res = [b.result(i) for i in range(F)]
    for p in range(P):
        dq, dt = res[p + 1][1], res[p][1]
        ri, rd, rs = O.hamming_best2(dq, dt)
        n = len(dq)
        assert np.array_equal(bi[p, :n].cpu().numpy(), ri)
        assert np.array_equal(bd[p, :n].cpu().numpy(), rd)
        assert np.array_equal(sd[p, :n].cpu().numpy(), rs)
