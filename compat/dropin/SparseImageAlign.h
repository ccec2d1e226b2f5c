// SparseImageAlign.h — drop-in replacement of the reference's
// include/SparseImageAlign.h (SparseImageAlign.h:19-118) over the gfx950
// SparseImgAlign kernel (include/ygzfe.h ygzfe_sparse_align).
//
//   mpAlign = new ygz::SparseImgAlign(nLevels - 1, 1);          Tracking.cc:284
//   size_t ret = mpAlign->run(&mLastFrame, &mCurrentFrame, TCR);  Tracking.cc:2171
// compile unchanged.  run() reads what SparseImageAlign.cc reads:
//   ref_frame->mvKeys / N / mvpMapPoints / mvbOutlier / mTcw / mvImagePyramid,
//   cur_frame->mTcw / mvImagePyramid, Frame::fx / fy / cx / cy;
// the initial estimate is T_cur_from_ref = cur->mTcw * ref->mTcw.inverse()
// (SparseImageAlign.cc:36: TCR is output only), xyz_ref = ref->mTcw *
// MapPoint::GetWorldPos() for the usable features (:67-86), both evaluated with
// the caller's own Sophus / Eigen types.  Levels max_level..min_level, 10
// Gauss-Newton iterations each (iterations[], :38-43; n_iter is ignored as
// there), return n_meas_ / 16.  getFisherInformation() = H_ / (float)(5e-4 *
// 255 * 255) (:51-55).
//
// Method: NLLSSolver::optimize dispatches on method_ (NLSSolver_impl.hpp:8-13) to
// optimizeGaussNewton (:18-91, what Tracking.cc:284 constructs) or
// optimizeLevenbergMarquardt (:95-212); both run on the GPU
// (ygzfe_sparse_align_method).
#ifndef YGZ_SPARSE_IMAGE_ALIGN_
#define YGZ_SPARSE_IMAGE_ALIGN_

#include <cstdio>
#include <type_traits>
#include <vector>

#include "Common.h"
#include "ygzfe_dropin.h"

namespace ygz {

class SparseImgAlign {
public:
    enum Method { GaussNewton, LevenbergMarquardt };  // NLLSSolver's methods (NLSSolver.h:40-43)

    SparseImgAlign(int n_levels, int min_level, int n_iter = 10, Method method = GaussNewton, bool display = false,
                   bool verbose = false)
        : max_level_(n_levels), min_level_(min_level), method_(method) {
        (void)n_iter;  // iterations[] overrides it per level (SparseImageAlign.cc:38-43)
        (void)display;
        (void)verbose;
        for (int i = 0; i < 36; i++) H_[i] = 0.f;
    }

    template <class FrameT, class SE3T>
    size_t run(FrameT *ref_frame, FrameT *cur_frame, SE3T &TCR) {
        if (ref_frame->mvKeys.empty()) return 0;  // SparseImageAlign.cc:24-27
        const SE3T T_cur_from_ref = cur_frame->mTcw * ref_frame->mTcw.inverse();
        const int n = ref_frame->N;
        std::vector<float> xyz(3 * (size_t)(n > 0 ? n : 0), 0.f);
        std::vector<uint8_t> usable((size_t)(n > 0 ? n : 0), 0);
        for (int i = 0; i < n; i++) {
            auto *mp = ref_frame->mvpMapPoints[i];
            if (mp == nullptr || mp->isBad() || ref_frame->mvbOutlier[i] == true) continue;
            const Vector3f p = ref_frame->mTcw * mp->GetWorldPos();  // SparseImageAlign.cc:86
            xyz[3 * (size_t)i + 0] = p[0];
            xyz[3 * (size_t)i + 1] = p[1];
            xyz[3 * (size_t)i + 2] = p[2];
            usable[i] = 1;
        }
        dropin::PyramidPool &pool = dropin::PyramidPool::instance();
        ygzfe_frame *ref = pool.find_or_upload(ref_frame->mvImagePyramid);
        ygzfe_frame *cur = pool.find_or_upload(cur_frame->mvImagePyramid);
        if (!ref || !cur) return 0;
        ygzfe_camera cam;
        cam.fx = FrameT::fx;
        cam.fy = FrameT::fy;
        cam.cx = FrameT::cx;
        cam.cy = FrameT::cy;
        const auto q = T_cur_from_ref.unit_quaternion();
        const auto t = T_cur_from_ref.translation();
        ygzfe_se3 T0;
        T0.q[0] = q.x();
        T0.q[1] = q.y();
        T0.q[2] = q.z();
        T0.q[3] = q.w();
        T0.t[0] = t[0];
        T0.t[1] = t[1];
        T0.t[2] = t[2];
        ygzfe_align_result r;
        const int method = method_ == LevenbergMarquardt ? YGZFE_ALIGN_LEVENBERG_MARQUARDT : YGZFE_ALIGN_GAUSS_NEWTON;
        if (ygzfe_sparse_align_method(ref, cur, &cam, dropin::as_kp(ref_frame->mvKeys.data()), xyz.data(),
                                      usable.data(), n, max_level_, min_level_, &T0, method, &r) != YGZFE_OK) {
            dropin::log_once("SparseImgAlign::run", dropin::last_error());
            return 0;
        }
        typedef typename std::decay<decltype(T_cur_from_ref.unit_quaternion())>::type Quat;
        typedef typename std::decay<decltype(T_cur_from_ref.translation())>::type Vec;
        Vec tr;
        tr[0] = r.T_cur_ref.t[0];
        tr[1] = r.T_cur_ref.t[1];
        tr[2] = r.T_cur_ref.t[2];
        TCR = SE3T(Quat(r.T_cur_ref.q[3], r.T_cur_ref.q[0], r.T_cur_ref.q[1], r.T_cur_ref.q[2]), tr);
        for (int i = 0; i < 36; i++) H_[i] = r.H[i];
        return (size_t)(r.n_visible > 0 ? r.n_visible : 0);
    }

    // SparseImageAlign.cc:51-55
    Eigen::Matrix<float, 6, 6> getFisherInformation() {
        const float sigma_i_sq = 5e-4 * 255 * 255;
        Eigen::Matrix<float, 6, 6> I;
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 6; c++) I(r, c) = H_[6 * r + c] / sigma_i_sq;
        return I;
    }

protected:
    int max_level_, min_level_;
    Method method_;
    float H_[36];
};

}  // namespace ygz

#endif
