// ORBextractor.h — drop-in replacement of the reference's include/ORBextractor.h
// (ORBextractor.h:37-192) over the gfx950 extractor (include/ygzfe.h).
//
// Same class, namespace, enum and public members, so Frame.cc / Tracking.cc
// compile unchanged:
//   ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)       Tracking.cc:255-261
//   operator()(InputArray image, InputArray mask, keypoints, descriptors)    ORBextractor.h:71-75
//   operator()(Frame*, keypoints, descriptors, KeyPointMethod, leftEye)      Frame.cc:337/340/346
//   ComputePyramid(cv::Mat) + the public mvImagePyramid                      Frame.cc:807-813, 515, 604
//   GetLevels / GetScaleFactor / GetScaleFactors / ... (getters)             Frame.cc:119-125
// The reference's src/ORBextractor.cc is not compiled with this header (its
// functions live in libygzfe.so); Frame is a template parameter of the Frame
// overload so this header needs only the reference's Common.h (OpenCV types).
//
// Semantics kept from ORBextractor.cc:1031-1127: the left eye extracts on the
// Frame's pyramid (frame->mvImagePyramid) and computes descriptors for the
// frame's existing keypoints (rows 0..N-1, angles recomputed in DSO mode) before
// the new ones, appended to `keypoints`; the right eye computes the pyramid of
// frame->mImRight and ignores existing keypoints; an empty result releases the
// descriptor matrix.  FAST_KEYPOINT (flagged buggy at ORBextractor.cc:1191,
// never called) returns no keypoints.
#ifndef YGZ_ORBEXTRACTOR_H_
#define YGZ_ORBEXTRACTOR_H_

#include "Common.h"
#include "ygzfe_dropin.h"

namespace ygz {

class Frame;

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    typedef enum { ORBSLAM_KEYPOINT, FAST_KEYPOINT, DSO_KEYPOINT } KeyPointMethod;

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
        : nfeatures(nfeatures), scaleFactor(scaleFactor), nlevels(nlevels), iniThFAST(iniThFAST),
          minThFAST(minThFAST) {
        ygzfe_orb_params p;
        p.nfeatures = nfeatures;
        p.scale_factor = scaleFactor;
        p.nlevels = nlevels;
        p.ini_th_fast = iniThFAST;
        p.min_th_fast = minThFAST;
        p.blur_variant = YGZFE_BLUR_CV4;
        if (ygzfe_extractor_create(&p, dropin::device(), &ex_) != YGZFE_OK) ex_ = nullptr;
        std::vector<float> s(YGZFE_MAX_LEVELS), is(YGZFE_MAX_LEVELS), s2(YGZFE_MAX_LEVELS), is2(YGZFE_MAX_LEVELS);
        if (ex_ && ygzfe_extractor_levels(ex_, nullptr, s.data(), is.data(), s2.data(), is2.data()) == YGZFE_OK) {
            mvScaleFactor.assign(s.begin(), s.begin() + nlevels);
            mvInvScaleFactor.assign(is.begin(), is.begin() + nlevels);
            mvLevelSigma2.assign(s2.begin(), s2.begin() + nlevels);
            mvInvLevelSigma2.assign(is2.begin(), is2.begin() + nlevels);
        }
        mvImagePyramid.resize(nlevels);
        if (ex_) dropin::PyramidPool::instance().set_extractor(ex_, nlevels);
    }

    ~ORBextractor() {
        if (ex_) {
            dropin::PyramidPool::instance().forget_extractor(ex_);
            ygzfe_extractor_destroy(ex_);
        }
    }

    ORBextractor(const ORBextractor &) = delete;
    ORBextractor &operator=(const ORBextractor &) = delete;

    // ORBextractor.cc:970-1028
    void operator()(cv::InputArray _image, cv::InputArray _mask, std::vector<cv::KeyPoint> &_keypoints,
                    cv::OutputArray _descriptors) {
        (void)_mask;
        if (_image.empty()) return;
        cv::Mat image = _image.getMat();
        ComputePyramid(image);
        _keypoints.clear();
        extract(last_, _keypoints, 0, YGZFE_ORBSLAM_KEYPOINT, _descriptors);
    }

    // ORBextractor.cc:1031-1127
    template <class FrameT>
    void operator()(FrameT *frame, std::vector<cv::KeyPoint> &_keypoints, cv::OutputArray _descriptors,
                    KeyPointMethod method, bool leftEye = true) {
        ygzfe_frame *f = nullptr;
        if (leftEye == false) {
            ComputePyramid(frame->mImRight);
            f = last_;
        } else {
            mvImagePyramid = frame->mvImagePyramid;
            f = dropin::PyramidPool::instance().find_or_upload(frame->mvImagePyramid);
        }
        if (method == FAST_KEYPOINT) {  // never called by the reference (ORBextractor.cc:1191)
            _descriptors.release();
            return;
        }
        const int n_exist = leftEye ? frame->N : 0;
        extract(f, _keypoints, n_exist, method == DSO_KEYPOINT ? YGZFE_DSO_KEYPOINT : YGZFE_ORBSLAM_KEYPOINT,
                _descriptors, leftEye ? &frame->mvKeys : nullptr);
    }

    int inline GetLevels() { return nlevels; }
    float inline GetScaleFactor() { return (float)scaleFactor; }
    std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
    std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
    std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

    std::vector<cv::Mat> mvImagePyramid;

    // ORBextractor.cc:1129-1150: the pyramid on the GPU; mvImagePyramid gets host
    // copies of the levels in fresh buffers that nothing writes afterwards (the
    // reference resizes into its own, ORBextractor.cc:1135-1146; a Frame shares them,
    // FrameGPU.h).  Level 0 is the image (:1135), copied here while the GPU builds the
    // levels above it, which come back in one DMA.
    void ComputePyramid(cv::Mat image) {
        last_ = nullptr;
        mvImagePyramid.assign(nlevels, cv::Mat());
        if (image.empty() || !ex_) return;
        dropin::PyramidPool &pool = dropin::PyramidPool::instance();
        ygzfe_frame *f = pool.compute(ex_, nlevels, image.data, image.cols, image.rows, image.step[0]);
        if (!f) return;
        std::vector<uint8_t *> dst(nlevels);
        std::vector<int> ds(nlevels);
        for (int l = 0; l < nlevels; l++) {
            int w = 0, h = 0;
            if (ygzfe_frame_level(f, l, &w, &h, nullptr, 0) != YGZFE_OK) return;  // sizes only, no device work
            mvImagePyramid[l].create(h, w, CV_8U);
            dst[l] = mvImagePyramid[l].data;
            ds[l] = (int)mvImagePyramid[l].step[0];
        }
        for (int y = 0; y < image.rows; y++)
            std::memcpy(dst[0] + (size_t)y * ds[0], image.data + (size_t)y * image.step[0], (size_t)image.cols);
        if (nlevels > 1 && ygzfe_frame_levels(f, 1, nlevels - 1, &dst[1], &ds[1]) != YGZFE_OK) {
            mvImagePyramid.assign(nlevels, cv::Mat());
            return;
        }
        pool.bind(f, mvImagePyramid[0]);
        last_ = f;
    }

    ygzfe_extractor *handle() const { return ex_; }

protected:
    // extraction on device pyramid f; rows 0..n_exist-1 describe (*exist)[0..n_exist),
    // new keypoints are appended to `keypoints`
    void extract(ygzfe_frame *f, std::vector<cv::KeyPoint> &keypoints, int n_exist, int method,
                 cv::OutputArray descriptors, std::vector<cv::KeyPoint> *exist = nullptr) {
        if (!f || !ex_) {
            descriptors.release();
            return;
        }
        if (!exist) n_exist = 0;
        std::vector<cv::KeyPoint> rows(exist ? exist->begin() : keypoints.begin(),
                                       exist ? exist->begin() + n_exist : keypoints.begin());
        int cap = n_exist + 4096, n = 0;
        std::vector<uint8_t> desc;
        int rc = YGZFE_ECAP;
        for (int tries = 0; tries < 3 && rc == YGZFE_ECAP; tries++) {
            rows.resize(cap);
            desc.resize((size_t)cap * 32);
            rc = ygzfe_extract(ex_, f, method, dropin::as_kp(rows.data()), n_exist, cap, desc.data(), &n);
            if (rc == YGZFE_ECAP) cap = n;
        }
        if (rc != YGZFE_OK) {  // the reference never throws: no new keypoints
            descriptors.release();
            return;
        }
        if (exist)  // DSO mode recomputes the existing keypoints' angles (ORBextractor.cc:1383-1385)
            for (int i = 0; i < n_exist; i++) (*exist)[i].angle = rows[i].angle;
        keypoints.insert(keypoints.end(), rows.begin() + n_exist, rows.begin() + n);
        if (n == 0) {
            descriptors.release();
            return;
        }
        descriptors.create(n, 32, CV_8U);
        cv::Mat d = descriptors.getMat();
        for (int i = 0; i < n; i++) std::memcpy(d.data + (size_t)i * d.step[0], &desc[(size_t)32 * i], 32);
    }

    int nfeatures = 0;
    double scaleFactor = 0;
    int nlevels = 0;
    int iniThFAST = 0;
    int minThFAST = 0;
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
    ygzfe_extractor *ex_ = nullptr;
    ygzfe_frame *last_ = nullptr;  // the device pyramid of the last ComputePyramid (pool-owned)
};

}  // namespace ygz

#endif
