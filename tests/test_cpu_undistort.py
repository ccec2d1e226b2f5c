"""CPU checks of the undistortion restatement (oracle/undistort.c), the
§8(f) rank-1 row: Frame::ComputeImagePyramid's initUndistortRectifyMap +
remap(INTER_LINEAR) (Frame.cc:775-790).

OpenCV is not in the image, so the restatement is pinned by properties of the
algorithm rather than by OpenCV outputs (parity unpinned against OpenCV
itself): zero distortion is the identity map and remap a byte copy; the
fixed-point map rounds the closed-form distortion model to 1/32 px; integer
shifts of the image move the remap output exactly."""
import numpy as np
import pytest

import _cameras as CAM
import _oracle as O


def _model(cam, dist, W, H):
    """Closed-form distorted source position of every output pixel (float64)."""
    fx, fy, cx, cy = (float(np.float32(c)) for c in cam)
    k = np.zeros(12)
    d = np.asarray(dist, np.float32).astype(np.float64)
    k[:len(d)] = d
    k1, k2, p1, p2, k3, k4, k5, k6 = k[:8]
    v, u = np.mgrid[0:H, 0:W].astype(np.float64)
    x, y = (u - cx) / fx, (v - cy) / fy
    r2 = x * x + y * y
    kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
    xd = x * kr + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * kr + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return fx * xd + cx, fy * yd + cy


def _decode(m1, m2):
    return m1[..., 0] + (m2 & 31) / 32.0, m1[..., 1] + (m2 >> 5) / 32.0


def test_zero_distortion_identity():
    cam, _, (W, H) = CAM.EUROC
    m1, m2 = O.undistort_map(cam, (), W, H)
    ys, xs = np.mgrid[0:H, 0:W]
    assert np.array_equal(m1[..., 0], xs) and np.array_equal(m1[..., 1], ys)
    assert not m2.any()
    img = np.random.default_rng(3).integers(0, 256, (H, W), dtype=np.uint8)
    assert np.array_equal(O.remap_linear(img, m1, m2), img)


@pytest.mark.parametrize("name", sorted(CAM.ALL))
def test_map_is_model_rounded_to_1_32(name):
    cam, dist, (W, H) = CAM.ALL[name]
    m1, m2 = O.undistort_map(cam, dist, W, H)
    assert m2.max() < 1024
    u, v = _model(cam, dist, W, H)
    gu, gv = _decode(m1, m2)
    # cvRound(u * 32) / 32: half a 1/32 step, plus the incremental row walk's ulps
    assert np.abs(gu - u).max() <= 1 / 64 + 1e-9
    assert np.abs(gv - v).max() <= 1 / 64 + 1e-9


def test_principal_point_is_fixed():
    cam, dist, (W, H) = CAM.EUROC
    cam = (cam[0], cam[1], 300.0, 200.0)  # integer principal point: x = y = 0 there
    m1, m2 = O.undistort_map(cam, dist, W, H)
    assert tuple(m1[200, 300]) == (300, 200) and m2[200, 300] == 0


def test_remap_integer_shift_is_exact():
    H, W = 60, 80
    img = np.random.default_rng(1).integers(0, 256, (H, W), dtype=np.uint8)
    ys, xs = np.mgrid[0:H, 0:W]
    m1 = np.stack([xs + 3, ys - 2], -1).astype(np.int16)
    out = O.remap_linear(img, m1, np.zeros((H, W), np.uint16))
    ref = np.zeros_like(img)
    ref[2:, :W - 3] = img[:H - 2, 3:]
    assert np.array_equal(out, ref)  # BORDER_CONSTANT 0 outside


def test_remap_half_pixel_rounds_like_fixed_point():
    H, W = 8, 8
    img = np.zeros((H, W), np.uint8)
    img[:, 1::2] = 255
    ys, xs = np.mgrid[0:H, 0:W]
    m1 = np.stack([xs, ys], -1).astype(np.int16)
    m2 = np.full((H, W), 16, np.uint16)  # tx = 16/32, ty = 0
    out = O.remap_linear(img, m1, m2)
    # (a * 2^14 + b * 2^14 + 2^14) >> 15 = (a + b + 1) >> 1 inside; the last column blends with the 0 border
    exp = np.full((H, W), 128, np.uint8)
    exp[:, W - 1] = (255 * 16384 + 16384) >> 15
    assert np.array_equal(out, exp)


def test_remap_fully_outside_is_zero():
    H, W = 10, 12
    img = np.full((H, W), 200, np.uint8)
    m1 = np.full((H, W, 2), -5, np.int16)
    assert not O.remap_linear(img, m1, np.zeros((H, W), np.uint16)).any()
    m1[..., 0] = -1  # straddles the left edge: only the sx + 1 = 0 tap is inside
    m1[..., 1] = 3
    out = O.remap_linear(img, m1, np.full((H, W), 16, np.uint16))
    assert (out == 100).all()


def _remap_f32_numpy(src, m1, m2):
    """A second, vectorised restatement of remapBilinear<float> (BORDER_CONSTANT 0): the
    float weights c_y * c_x, summed S00 w0 + S01 w1 + S10 w2 + S11 w3 in float32."""
    H, W = src.shape
    sx, sy = m1[..., 0].astype(np.int64), m1[..., 1].astype(np.int64)
    tx, ty = (m2 & 31).astype(np.float32), (m2 >> 5).astype(np.float32)
    f32 = np.float32
    cx1, cy1 = tx * f32(1 / 32), ty * f32(1 / 32)
    cx0, cy0 = f32(1) - cx1, f32(1) - cy1
    w = [cy0 * cx0, cy0 * cx1, cy1 * cx0, cy1 * cx1]

    def tap(x, y):
        ok = (x >= 0) & (x < W) & (y >= 0) & (y < H)
        return np.where(ok, src[np.clip(y, 0, H - 1), np.clip(x, 0, W - 1)], f32(0)).astype(np.float32)

    v = [tap(sx, sy), tap(sx + 1, sy), tap(sx, sy + 1), tap(sx + 1, sy + 1)]
    out = ((v[0] * w[0] + v[1] * w[1]).astype(np.float32) + v[2] * w[2]).astype(np.float32) + v[3] * w[3]
    outside = (sx >= W) | (sx + 1 < 0) | (sy >= H) | (sy + 1 < 0)
    return np.where(outside, f32(0), out.astype(np.float32)).astype(np.float32)


@pytest.mark.parametrize("name", ["tum1", "odd", "wild"])
def test_remap_f32_matches_numpy_restatement(name):
    """Frame.cc:799-804 (the RGB-D depth remap): the C restatement equals an independent
    vectorised one bit for bit, including the BORDER_CONSTANT edge taps."""
    cam, dist, (W, H) = CAM.ALL[name]
    m1, m2 = O.undistort_map(cam, dist, W, H)
    rng = np.random.default_rng(3)
    src = (rng.random((H, W)) * 4.0).astype(np.float32)
    src[rng.random((H, W)) < 0.05] = 0.0
    got = O.remap_linear_f32(src, m1, m2)
    want = _remap_f32_numpy(src, m1, m2)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_remap_f32_zero_distortion_is_copy():
    cam, _, (W, H) = CAM.TUM1
    m1, m2 = O.undistort_map(cam, (), W, H)
    src = np.random.default_rng(5).random((H, W)).astype(np.float32)
    assert np.array_equal(O.remap_linear_f32(src, m1, m2), src)
