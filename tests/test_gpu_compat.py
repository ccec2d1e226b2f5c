"""The drop-in C++ adapter (compat/ygz_compat.hpp) driven by a Tracking.cc-shaped
caller (compat/tracking_demo.cpp): extractor ctor + getters, ComputePyramid +
operator()(Frame), ORBmatcher best/second + DescriptorDistance, SparseImgAlign
(3,1).run on a known translation, Align2D on a known sub-pixel offset."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tracking_demo(gpu):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "compat")])
    r = subprocess.run([os.path.join(ROOT, "compat", "build", "tracking_demo")], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")
