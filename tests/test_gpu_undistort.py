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


def _depth_image(seed, W, H):
    """TUM-like CV_32F depth (Tracking.cc GrabImageRGBD: uint16 / 5000 -> metres): a tilted
    plane with steps, holes (0 = no depth) and a few large values."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    d = (0.8 + 0.002 * xx + 0.003 * yy + 0.25 * ((xx // 97 + yy // 71) % 3)).astype(np.float32)
    raw = np.round(d * 5000).astype(np.uint16)
    raw[rng.random((H, W)) < 0.05] = 0
    raw[rng.random((H, W)) < 0.001] = 65535
    return (raw.astype(np.float32) * np.float32(1.0 / 5000)).astype(np.float32)


@pytest.mark.parametrize("name", sorted(CAM.ALL))
def test_remap_depth_f32_bitexact(gpu, name):
    """Frame.cc:799-804 (RGB-D): remap(mImDepth, map1, map2, INTER_LINEAR) on CV_32F, host in / out
    and batched on the device, bit-exact against the oracle's float remapBilinear."""
    import torch
    cam, dist, (W, H) = CAM.ALL[name]
    und = gpu.Undistort(cam, dist, W, H)
    m1, m2 = O.undistort_map(cam, dist, W, H)
    depths = [_depth_image(s, W, H) for s in range(3)]
    for d in depths[:1]:
        got = und.remap_depth(d)
        ref = O.remap_linear_f32(d, m1, m2)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), \
            f"{np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))} px differ"
        # the "wild" model maps most of the frame outside the source (BORDER_CONSTANT 0)
        assert (ref > 0).mean() > (0.2 if name == "wild" else 0.5)
    src = torch.from_numpy(np.stack(depths)).cuda()
    pitch = W * H + 16
    dst = torch.full((3, pitch), -1.0, dtype=torch.float32, device="cuda")
    und.apply_f32_device(src.data_ptr(), W * H, W, dst.data_ptr(), pitch, W, 3)
    out = dst.cpu().numpy()
    for i, d in enumerate(depths):
        ref = O.remap_linear_f32(d, m1, m2)
        assert np.array_equal(out[i, :W * H].reshape(H, W).view(np.uint32), ref.view(np.uint32)), f"image {i}"
        assert (out[i, W * H:] == -1.0).all(), "wrote past the image"


def test_remap_image_host_bitexact(gpu):
    """The u8 host-in / host-out remap the drop-in Frame::ComputeImagePyramid uses (Frame.cc:786-797)."""
    for name in ("tum1", "odd"):
        cam, dist, (W, H) = CAM.ALL[name]
        und = gpu.Undistort(cam, dist, W, H)
        m1, m2 = O.undistort_map(cam, dist, W, H)
        img = S.frame(4, W, H)
        assert np.array_equal(und.remap_image(img), O.remap_linear(img, m1, m2)), name


def test_rgbd_depth_undistorted_then_stereo(gpu):
    """The C4 (TUM1, distorted) RGB-D path: depth undistorted (Frame.cc:799-804) then
    ComputeStereoFromRGBD (:684-700) at the undistorted keypoints, both against the oracle."""
    cam, dist, (W, H) = CAM.TUM1
    und = gpu.Undistort(cam, dist, W, H)
    m1, m2 = O.undistort_map(cam, dist, W, H)
    _, _, nf, sf, nl, ini, mn = S.CONFIGS["C4"]
    img = und.remap_image(S.frame(9, W, H))
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn, device=0)
    kps, _ = ex.extract(ex.ComputePyramid(img))
    depth = _depth_image(9, W, H)
    dg = und.remap_depth(depth)
    ur, dp = gpu.stereo_from_rgbd(dg, kps, 40.0)
    dref = O.remap_linear_f32(depth, m1, m2)
    rur, rdp = O.stereo_from_rgbd(dref, kps, 40.0)
    assert np.array_equal(dp, rdp) and np.array_equal(ur, rur)
    assert (dp > 0).mean() > 0.5
