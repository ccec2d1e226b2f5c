"""The reference's own call sites, verbatim, against the drop-in headers
(compat/dropin/: ORBextractor.h, SparseImageAlign.h, Align.h, ORBmatcherGPU.h +
ORBmatcher_gpu.inc) and test stubs of Frame / MapPoint / KeyFrame / ORBmatcher,
built -std=c++11 like the reference (tests/dropin/dropin_calls.cpp): every
result is compared with the CPU oracle inside the program."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_call_sites_compile_and_match_the_oracle(gpu):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "compat"), "dropin"])
    r = subprocess.run([os.path.join(ROOT, "compat", "build", "dropin_calls")], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")
    for line in ("mpAlign->run(&mLastFrame, &mCurrentFrame, TCR)", "DSO_KEYPOINT", "ORBSLAM_KEYPOINT",
                 "SearchForInitialization", "SearchByBoW", "ygz::Align2D", "SearchLocalPointsDirect() [3 keyframes, mnCacheHitTh 150]",
                 "SearchLocalPointsDirect() [3 keyframes, mnCacheHitTh 1073741824]",
                 "SearchLocalPointsDirect() [130 keyframes, mnCacheHitTh 150]",
                 "the pyramid pool grew past its soft capacity", "matcher.FindDirectProjection",
                 "Frame::ComputeStereoMatches()", "Frame::ComputeBoW()", "remap(mImDepth) CV_32F"):
        assert line in r.stdout
