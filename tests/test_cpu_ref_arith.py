"""The oracle's floating-point restatements against the reference's own arithmetic.

* rBRIEF's angle (ORBextractor.cc:108-109): `float a = (float)cos(angle)` under
  `using namespace std` is std::cos(float), i.e. the C library's cosf / sinf.
  oracle/orb.c ygzo_sincosf restates glibc's algorithm; it is compared here bit
  for bit with this image's libm (glibc 2.35) over EVERY float in [0, 2pi) --
  the range angle * pi/180 takes for fastAtan2 angles -- and on a stride
  sample of all finite floats.
* The reference is built `g++ -O3 -march=native -std=c++11` (CMakeLists.txt:14,21).
  C++ keeps GCC's -ffp-contract=fast, so on an FMA machine GET_VALUE
  (ORBextractor.cc:114-116) and the Shi-Tomasi discriminant (:1186) are fused
  multiply-adds.  tests/probe/ref_arith_probe.cpp holds those expression shapes;
  it is compiled here with the reference's flags and compared with the
  oracle's explicit fma form on many angles / patches.
"""
import ctypes as C
import os
import shutil
import subprocess
import threading

import numpy as np
import pytest

import _oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))


def _bits(f):
    return int(np.float32(f).view(np.uint32))


def _sweep(ranges, threads=8):
    L = O.lib()
    L.ygzo_sincosf_sweep.restype = C.c_int64
    L.ygzo_sincosf_sweep.argtypes = [C.c_uint32, C.c_uint32]
    out = [0] * len(ranges)
    sem = threading.Semaphore(threads)

    def run(i, lo, hi):
        with sem:  # ctypes drops the GIL: the ranges run in parallel
            out[i] = L.ygzo_sincosf_sweep(lo, hi)

    ths = [threading.Thread(target=run, args=(i, lo, hi)) for i, (lo, hi) in enumerate(ranges)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return out


def test_sincosf_every_float_in_0_2pi():
    """All 1,086,918,619 floats in [0, 2pi): restated sinf/cosf == libm sinf/cosf."""
    hi = _bits(np.float32(2 * np.pi))  # first float >= 2pi (6.2831855 > 2pi): exclusive bound
    assert float(np.float32(2 * np.pi)) > 2 * np.pi
    n = 64
    edges = np.linspace(0, hi, n + 1).astype(np.int64)
    bad = _sweep([(int(edges[i]), int(edges[i + 1])) for i in range(n)])
    assert sum(bad) == 0, f"{sum(bad)} mismatches"


def test_sincosf_sampled_all_finite():
    """Stride sample over every finite float of both signs (incl. the |y| >= 120 reduction)."""
    ranges = []
    for sign in (0, 0x80000000):
        for start in range(0, 0x7F800000, 0x7F800000 // 256):
            lo = sign + start
            ranges.append((lo, lo + 4000))
    assert sum(_sweep(ranges)) == 0


def _cpu_has_fma():
    try:
        return " fma " in open("/proc/cpuinfo").read().replace("\n", " ")
    except OSError:
        return False


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ absent: cannot compile the probe with the reference's flags")
    if not _cpu_has_fma():
        pytest.skip("host CPU has no FMA: -march=native would not contract here")
    so = str(tmp_path_factory.mktemp("probe") / "ref_arith_probe.so")
    subprocess.check_call([gxx, "-Wall", "-O3", "-march=native", "-Wno-reorder", "-std=c++11", "-fPIC", "-shared",
                           os.path.join(HERE, "probe", "ref_arith_probe.cpp"), "-o", so])
    lib = C.CDLL(so)
    lib.probe_shi_tomasi.restype = C.c_float
    return lib


def _angles(n, seed=5):
    """fastAtan2 outputs of random IC moments plus uniform angles in [0, 360)."""
    rng = np.random.default_rng(seed)
    L = O.lib()
    L.ygzo_fast_atan2.restype = C.c_float
    m = rng.integers(-60000, 60000, size=(n // 2, 2))
    a = [L.ygzo_fast_atan2(C.c_float(float(y)), C.c_float(float(x))) for y, x in m]
    u = rng.uniform(0, 360, size=n - len(a)).astype(np.float32)
    return np.concatenate([np.array(a, np.float32), u, np.float32([0, 90, 180, 270, 359.99997, 45, 135])])


def test_rbrief_offsets_match_reference_build(probe):
    """GET_VALUE's 512 rotated offsets: oracle (glibc sincosf + explicit fma) == the
    reference's expression compiled with its own flags, on 20,000 angles."""
    L = O.lib()
    L.ygzo_bit_pattern.restype = C.POINTER(C.c_int)
    pat = np.ctypeslib.as_array(L.ygzo_bit_pattern(), shape=(1024,)).astype(np.int32).copy()
    dy0, dx0, dy1, dx1 = (np.zeros(512, np.int32) for _ in range(4))
    differ_from_double_cos = 0
    for ang in _angles(20000):
        probe.probe_offsets(O._p(pat), C.c_float(float(ang)), O._p(dy0), O._p(dx0))
        L.ygzo_orb_sample_offsets(C.c_float(float(ang)), O._p(dy1), O._p(dx1))
        assert np.array_equal(dy0, dy1) and np.array_equal(dx0, dx1), f"angle {ang!r}"
        r = np.float32(ang) * np.float32(np.pi / 180.0)
        differ_from_double_cos += np.float32(np.cos(np.float64(r))) != np.float32(np.cos(r))
    # the substitution this replaced, (float)cos((double)x), really is a different function
    assert differ_from_double_cos > 0


def test_sincos_probe_equals_oracle(probe):
    """std::cos(float)/std::sin(float) as compiled by the reference's flags == ygzo_sincosf."""
    y = np.random.default_rng(3).uniform(-7, 7, 200000).astype(np.float32)
    s0, c0 = np.zeros_like(y), np.zeros_like(y)
    probe.probe_sincos(O._p(y), len(y), O._p(s0), O._p(c0))
    s1, c1 = C.c_float(), C.c_float()
    for i in range(0, len(y), 97):
        O.lib().ygzo_sincosf(C.c_float(float(y[i])), C.byref(s1), C.byref(c1))
        assert np.float32(s1.value).view(np.uint32) == s0[i].view(np.uint32)
        assert np.float32(c1.value).view(np.uint32) == c0[i].view(np.uint32)


def test_shi_tomasi_matches_reference_build(probe):
    """ShiTomasiScore (ORBextractor.cc:1152-1187): oracle == reference expression + flags."""
    rng = np.random.default_rng(11)
    L = O.lib()
    L.ygzo_shi_tomasi.restype = C.c_float
    for trial in range(6):
        img = rng.integers(0, 256, size=(40, 48), dtype=np.uint8)
        if trial % 2:
            img = ((img.astype(np.int32) + np.roll(img, 1, 1) + np.roll(img, 1, 0)) // 3).astype(np.uint8)
        H, W = img.shape
        for v in range(H):
            for u in range(W):
                a = probe.probe_shi_tomasi(O._p(img), W, H, W, u, v)
                b = L.ygzo_shi_tomasi(O._p(img), W, H, W, u, v)
                assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32) or (np.isnan(a) and np.isnan(b)), \
                    (trial, u, v, a, b)
