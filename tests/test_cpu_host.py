"""Host-side logic and the C-ABI library, without a GPU.

* the extraction plan (level sizes, budgets, FAST cell grid, umax) computed by
  the product library (ygzfe_orb_plan) and by the oracle, against the tables of
  SURVEY.md §8a derived from ORBextractor.cc:416-467, 728-781, 1131-1132;
* lib/libygzfe.so loads and exports every function include/ygzfe.h declares;
* the product library does not link or contain the oracle.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import _oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "orb-ygz-slam_amd")
HEADER = os.path.join(ROOT, "include", "ygzfe.h")

SIZES = {
    "C1": [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161), (179, 134)],
    "C2": [(752, 480), (376, 240), (188, 120), (94, 60)],
}
BUDGETS = {
    "C1": [109, 90, 75, 63, 52, 44, 36, 31],
    "C2": [533, 267, 133, 67],
    "C4": [434, 362, 302, 251, 209, 175, 145, 122],
}
PARAMS = {"C1": (500, 1.2, 8, 640, 480), "C2": (1000, 2.0, 4, 752, 480), "C4": (2000, 1.2, 8, 640, 480)}


@pytest.fixture(scope="module")
def ygzfe():
    lib = os.path.join(PKG, "lib", "libygzfe.so")
    if not os.path.exists(lib):  # hipcc cross-compiles for gfx950 without a GPU
        subprocess.check_call(["make", "-s", "-C", PKG])
    import ygzfe as m
    return m


@pytest.mark.parametrize("cfg", ["C1", "C2", "C4"])
def test_plan_tables(ygzfe, cfg):
    nf, sf, nl, W, H = PARAMS[cfg]
    plan = ygzfe.orb_plan(nf, sf, nl, 20, 7, W, H)
    assert plan["budget"] == BUDGETS[cfg]
    assert sum(plan["budget"]) == nf
    want = SIZES["C1" if cfg == "C4" else cfg]
    assert plan["sizes"] == want
    orc = O.OrbOracle(nf, sf, nl, 20, 7)
    assert orc.level_sizes(W, H) == want
    assert orc.feat_per_level == BUDGETS[cfg]
    assert plan["umax"] == orc.umax


def test_cell_grid_c2(ygzfe):
    """C2 level 0 has 14x24 cells; level 3 (94x60) has none (nRows = int(28/30) = 0)."""
    plan = ygzfe.orb_plan(1000, 2.0, 4, 20, 7, 752, 480)
    assert plan["ncells"][0] == 14 * 24
    assert plan["ncells"][3] == 0


def test_umax_table(ygzfe):
    """ORBextractor.cc:453-467 for HALF_PATCH_SIZE = 15 (a symmetric quarter circle)."""
    um = ygzfe.orb_plan(500, 1.2, 8)["umax"]
    assert um == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]


def test_invalid_params_fail_loudly(ygzfe):
    with pytest.raises(ygzfe.YgzfeError):
        ygzfe.orb_plan(1000, 1.0, 4)  # scale factor must be > 1
    with pytest.raises(ygzfe.YgzfeError):
        ygzfe.orb_plan(1000, 2.0, 17)  # > YGZFE_MAX_LEVELS


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ygzfe_[a-z0-9_]+)\s*\(", src)))


def test_abi_exports_every_declared_symbol(ygzfe):
    names = declared_functions()
    assert len(names) > 30
    lib = C.CDLL(ygzfe.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"declared in include/ygzfe.h but not exported: {missing}"


def test_product_library_does_not_contain_the_oracle(ygzfe):
    out = subprocess.run(["nm", "-D", "--defined-only", ygzfe.LIB_PATH], capture_output=True, text=True).stdout
    assert "ygzo_" not in out
    needed = subprocess.run(["readelf", "-d", ygzfe.LIB_PATH], capture_output=True, text=True).stdout
    assert "ygzoracle" not in needed and "fastref" not in needed


def test_kp_layout_matches_cv_keypoint(ygzfe):
    """ygzfe_kp is cv::KeyPoint's 28-byte layout."""
    assert ygzfe.KP_DTYPE.itemsize == 28
    assert list(ygzfe.KP_DTYPE.names) == ["x", "y", "size", "angle", "response", "octave", "class_id"]
    assert C.sizeof(ygzfe.SE3) == 28


def test_compat_adapter_builds_and_fails_loudly_without_gpu(ygzfe):
    """compat/ygz_compat.hpp (the drop-in C++ classes) compiles into a Tracking.cc-shaped
    caller; with no HIP device the product path reports an error instead of falling back."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "compat")])
    exe = os.path.join(ROOT, "compat", "build", "tracking_demo")
    if ygzfe.device_count() > 0:
        pytest.skip("a GPU is visible: tests/test_gpu_compat.py runs the demo")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "no HIP device" in r.stdout


def _e4m3_encode(v):
    """extract.hip upload_pattern's OCP E4M3 encoding of an integer |v| <= 16."""
    a = abs(v)
    if a == 0:
        return 0
    e = 0
    while (2 << e) <= a:
        e += 1
    return (0x80 if v < 0 else 0) | ((e + 7) << 3) | (((a << 3) >> e) & 7)


def _e4m3_decode(b):
    if b & 0x7F == 0:
        return 0.0
    s = -1.0 if b & 0x80 else 1.0
    return s * (1 + (b & 7) / 8) * 2.0 ** (((b >> 3) & 15) - 7)


def test_pattern_fp8_exact():
    """k_orient_desc reads the rBRIEF pattern as FP8 (E4M3) point pairs and converts them with
    v_cvt_pk_f32_fp8: every coordinate of the ORB pattern (ORBextractor.cc:152-410,
    include/ygzfe_pattern.inc) must be an integer that E4M3 holds exactly."""
    txt = open(os.path.join(ROOT, "include", "ygzfe_pattern.inc")).read()
    body = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    vals = [int(x) for x in re.findall(r"-?\d+", body)]
    assert len(vals) == 1024
    assert max(abs(v) for v in vals) <= 16
    for v in set(vals):
        assert _e4m3_decode(_e4m3_encode(v)) == float(v), v
