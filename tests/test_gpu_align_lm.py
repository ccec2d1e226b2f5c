"""SparseImgAlign constructed with LevenbergMarquardt (SparseImageAlign.h:37-41 -> NLLSSolver::optimize,
NLSSolver_impl.hpp:8-13) on the GPU vs the oracle's restatement of optimizeLevenbergMarquardt
(NLSSolver_impl.hpp:95-212; oracle/align.c ygzo_sparse_align_method): pose within 1e-4, the same
visible count (n_meas_ of the last computeResiduals) and chi2_, and getFisherInformation's H_ as the
last trial left it (damped).  Both the register kernel (<= 960 features) and the generic path
(ORBextractor(2000): ~1,900 features) are covered, with small and large motions (failed trials,
mu growth) and partially usable map points."""
import numpy as np
import pytest

import _scenes as S
from test_gpu_align import POSE_TOL, align_case

pytestmark = pytest.mark.gpu
LM = 1


def _check(res, ores, what):
    gq, gt = res.T_cur_ref.as_arrays()
    err = S.se3_log_inf(gq, gt, np.array(ores.T.q[:]), np.array(ores.T.t[:]))
    assert err <= POSE_TOL, f"{what}: LM pose differs from the oracle by {err}"
    assert res.n_visible == ores.n_visible, f"{what}: n_visible {res.n_visible} vs {ores.n_visible}"
    assert abs(res.chi2 - ores.chi2) <= 1e-3 * max(1.0, abs(ores.chi2)), f"{what}: chi2 {res.chi2} vs {ores.chi2}"
    H, oH = np.array(res.H[:]), np.array(ores.H[:])
    assert np.allclose(H, oH, rtol=2e-3, atol=1e-2 * np.abs(oH).max()), f"{what}: damped H differs"
    return err


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
@pytest.mark.parametrize("motion_scale", [1.0, 3.0])
def test_sparse_align_lm_pose_parity(gpu, seed, motion_scale):
    res, ores, _ = align_case(gpu, seed, motion_scale=motion_scale, method=LM)
    _check(res, ores, f"seed {seed} x{motion_scale}")
    assert res.n_visible > 100


def test_sparse_align_lm_partial_usable(gpu):
    res, ores, _ = align_case(gpu, 5, n_usable_frac=0.3, method=LM)
    _check(res, ores, "30% usable")


def test_sparse_align_lm_generic_path(gpu):
    """> 960 usable features: sparse_align_generic runs the same LM rounds."""
    res, ores, _ = align_case(gpu, 6, method=LM, nfeatures=2000)
    assert ores.n_visible > 960
    _check(res, ores, "generic")


def test_sparse_align_gn_unchanged_by_method_arg(gpu):
    """method=GaussNewton through the method entry point equals the default path."""
    res, ores, _ = align_case(gpu, 1, method=0)
    _check_gn = S.se3_log_inf(*res.T_cur_ref.as_arrays(), np.array(ores.T.q[:]), np.array(ores.T.t[:]))
    assert _check_gn <= POSE_TOL and res.n_visible == ores.n_visible
