"""GPU undistortion vs the CPU oracle, bit-exact (§8(f) rank 1).

Reference path: Frame::ComputeImagePyramid (Frame.cc:775-790) --
initUndistortRectifyMap(K, D, I, K, size, CV_16SC2) once per camera and
remap(INTER_LINEAR, BORDER_CONSTANT 0) per frame, then the ORB pyramid."""
import numpy as np
import pytest

import _cameras as CAM
import _oracle as O
import _scenes as S
from test_gpu_extract import assert_kps_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(CAM.ALL))
def test_maps_bitexact(gpu, name):
    cam, dist, (W, H) = CAM.ALL[name]
    g1, g2 = gpu.Undistort(cam, dist, W, H).maps()
    r1, r2 = O.undistort_map(cam, dist, W, H)
    assert np.array_equal(g1, r1), f"map1: {np.count_nonzero((g1 != r1).any(-1))} px differ"
    assert np.array_equal(g2, r2), f"map2: {np.count_nonzero(g2 != r2)} px differ"


@pytest.mark.parametrize("name", sorted(CAM.ALL))
def test_remap_batch_bitexact(gpu, name):
    import torch
    cam, dist, (W, H) = CAM.ALL[name]
    und = gpu.Undistort(cam, dist, W, H)
    m1, m2 = O.undistort_map(cam, dist, W, H)
    n = 11  # two frame groups of the kernel, the second partial
    rng = np.random.default_rng(7)
    frames = np.stack([S.frame(s, W, H) for s in range(n - 1)] + [rng.integers(0, 256, (H, W), dtype=np.uint8)])
    src = torch.from_numpy(frames).cuda()
    pitch = W * H + 64  # padded destination pitch
    dst = torch.full((n, pitch), 7, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    und.apply_device(src.data_ptr(), W * H, W, dst.data_ptr(), pitch, W, n, st.cuda_stream)
    torch.cuda.synchronize()
    out = dst.cpu().numpy()
    for i in range(n):
        ref = O.remap_linear(frames[i], m1, m2)
        got = out[i, :W * H].reshape(H, W)
        assert np.array_equal(got, ref), f"frame {i}: {np.count_nonzero(got != ref)} px differ"
        assert (out[i, W * H:] == 7).all(), "wrote past the image"


def test_remap_strided_unaligned(gpu):
    import torch
    cam, dist, (W, H) = CAM.EUROC
    und = gpu.Undistort(cam, dist, W, H)
    m1, m2 = O.undistort_map(cam, dist, W, H)
    img = S.frame(3, W, H)
    src = torch.zeros((H, W + 5), dtype=torch.uint8, device="cuda")
    src[:, :W] = torch.from_numpy(img).cuda()
    dst = torch.zeros(H * (W + 3) + 1, dtype=torch.uint8, device="cuda")
    # destination offset by one byte and row stride W + 3: the scalar path
    und.apply_device(src.data_ptr(), 0, W + 5, dst.data_ptr() + 1, 0, W + 3, 1)
    got = dst[1:].cpu().numpy().reshape(H, W + 3)[:, :W]
    assert np.array_equal(got, O.remap_linear(img, m1, m2))


@pytest.mark.parametrize("name", ["euroc", "tum1"])
def test_undistorted_extraction_bitexact(gpu, name):
    cam, dist, (W, H) = CAM.ALL[name]
    cfg = {"euroc": "C2", "tum1": "C1"}[name]
    _, _, nf, sf, nl, ini, mn = S.CONFIGS[cfg]
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    und = gpu.Undistort(cam, dist, W, H)
    m1, m2 = O.undistort_map(cam, dist, W, H)
    img = S.frame(4, W, H)
    fr = und.ComputePyramid(ex, img)
    ref_levels = orc.pyramid(O.remap_linear(img, m1, m2))
    for l, (g, r) in enumerate(zip(fr.levels(), ref_levels)):
        assert np.array_equal(g, r), f"level {l}: {np.count_nonzero(g != r)} px differ"
    kg, dg = ex.extract(fr)
    kr, dr = orc.extract(ref_levels)
    assert len(kr) > 100
    assert_kps_equal(kg, kr, name)
    assert np.array_equal(dg, dr)


def test_batch_upload_undistorted_matches_single(gpu):
    cam, dist, (W, H) = CAM.EUROC
    _, _, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    und = gpu.Undistort(cam, dist, W, H)
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, 4)
    frames = np.stack([S.frame(s, W, H) for s in range(3)])
    b.upload_undistorted(und, frames)
    b.extract(3)
    b.check()
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    m1, m2 = O.undistort_map(cam, dist, W, H)
    for i in range(3):
        kg, dg = b.result(i)
        kr, dr = orc.extract(orc.pyramid(O.remap_linear(frames[i], m1, m2)))
        assert_kps_equal(kg, kr, f"frame {i}")
        assert np.array_equal(dg, dr)


def test_batch_undistort_device_then_extract(gpu):
    import torch
    cam, dist, (W, H) = CAM.EUROC
    _, _, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    und = gpu.Undistort(cam, dist, W, H)
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, 9)
    frames = np.stack([S.frame(10 + s, W, H) for s in range(9)])
    raw = torch.from_numpy(frames).cuda()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    b.undistort_device(und, raw.data_ptr(), W * H, 9, s.cuda_stream)
    b.extract(9, s.cuda_stream)
    torch.cuda.synchronize()
    b.check()
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    m1, m2 = O.undistort_map(cam, dist, W, H)
    for i in (0, 8):
        kg, dg = b.result(i)
        kr, dr = orc.extract(orc.pyramid(O.remap_linear(frames[i], m1, m2)))
        assert_kps_equal(kg, kr, f"frame {i}")
        assert np.array_equal(dg, dr)


def test_size_mismatch_fails_loudly(gpu):
    cam, dist, _ = CAM.EUROC
    und = gpu.Undistort(cam, dist, 640, 480)
    ex = gpu.ORBextractor(1000, 2.0, 4, 20, 7)
    with pytest.raises(gpu.YgzfeError):
        und.ComputePyramid(ex, S.frame(0, 752, 480))
    b = gpu.Batch((1000, 2.0, 4, 20, 7, 0), 0, 752, 480, 2)
    with pytest.raises(gpu.YgzfeError):
        b.upload_undistorted(und, np.zeros((1, 480, 752), np.uint8))
    with pytest.raises(gpu.YgzfeError):
        gpu.Undistort(cam, np.zeros(13, np.float32), 64, 64)
