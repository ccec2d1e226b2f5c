"""The bench's extraction schedule (ygzfe_batch_extract_split: keypoint rows on one stream, blur +
orientation/rBRIEF on a second) gives exactly the keypoints and descriptors of the single-stream
ygzfe_batch_extract (itself pinned to the oracle in test_gpu_batch / test_gpu_extract), frame by frame,
and the same per-frame counts in bound device buffers; the dense Hamming that follows it in the bench
step matches a numpy brute force on those descriptors."""
import numpy as np
import pytest

import _scenes as S

pytestmark = pytest.mark.gpu
XI = np.array([0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015], np.float32)


def _frames(gpu, F, stride, seed=11):
    W, H = S.CONFIGS["C2"][:2]
    sc = S.PlaneScene(seed, W, H)
    poses = [gpu.trajectory_pose(k * stride, XI) for k in range(F)]
    return np.stack([sc.render(q, t, noise_seed=k) for k, (q, t) in enumerate(poses)])


@pytest.mark.parametrize("F,stride", [(5, 1), (9, 7)])
def test_extract_split_equals_extract(gpu, F, stride):
    import torch
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    frames = _frames(gpu, F, stride)
    a = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, F)
    a.upload(frames)
    a.extract(F)
    a.check()
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, F)
    counts = torch.zeros(F, dtype=torch.int32, device="cuda")
    b.bind(counts=counts.data_ptr())
    b.upload(frames)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    b.extract_split(F, s1.cuda_stream, s2.cuda_stream)
    torch.cuda.synchronize()
    b.check()
    c = counts.cpu().numpy()
    for i in range(F):
        ka, da = a.result(i)
        kb, db = b.result(i)
        assert len(ka) == len(kb) == c[i], (i, len(ka), len(kb), c[i])
        assert (ka == kb).all(), f"frame {i}: keypoints differ"
        assert (da == db).all(), f"frame {i}: descriptors differ"


def test_bench_step_hamming_on_split_descriptors(gpu):
    import torch
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    F = 4
    frames = _frames(gpu, F, 3, seed=5)
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, F)
    cap = b.kp_cap
    desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(F, dtype=torch.int32, device="cuda")
    b.bind(desc=desc.data_ptr(), counts=counts.data_ptr())
    b.upload(frames)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    b.extract_split(F, s1.cuda_stream, s2.cuda_stream)
    P = F - 1
    qf = torch.arange(1, F, dtype=torch.int32, device="cuda")
    tf = torch.arange(0, P, dtype=torch.int32, device="cuda")
    bi, bd, sd = (torch.full((P, cap), -7, dtype=torch.int32, device="cuda") for _ in range(3))
    s2.wait_stream(s1)
    b.match(P, qf.data_ptr(), tf.data_ptr(), bi.data_ptr(), bd.data_ptr(), sd.data_ptr(), s2.cuda_stream)
    torch.cuda.synchronize()
    d, c = desc.cpu().numpy(), counts.cpu().numpy()
    pc = np.unpackbits(np.arange(256, dtype=np.uint8)[:, None], axis=1).sum(1)
    for p in range(P):
        q, t = d[p + 1, :c[p + 1]], d[p, :c[p]]
        D = pc[q[:, None, :] ^ t[None, :, :]].sum(2)
        o = np.sort(D, axis=1)
        nq = len(q)
        assert (bd[p, :nq].cpu().numpy() == o[:, 0]).all()
        assert (sd[p, :nq].cpu().numpy() == o[:, 1]).all()
        assert (bi[p, :nq].cpu().numpy() == np.argmin(D, axis=1)).all()  # first index on ties
