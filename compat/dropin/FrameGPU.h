// FrameGPU.h — the §8f rows at Frame.cc's own call sites: Frame::ComputeImagePyramid's
// undistortion (Frame.cc:773-805), ComputeStereoMatches (:509-682),
// ComputeStereoFromRGBD (:684-700) and ComputeBoW (:495-500) on the GPU, through
// include/ygzfe.h.  Frame_gpu.inc holds the four member-function bodies that call
// these templates; Frame.h and every caller stay unchanged.  C++11, Frame read
// through the reference's member names (mImGray, mImRight, mImDepth, mK, mDistCoef,
// mbNeedUndistort, mSensor, mvKeys, mDescriptors, mvuRight, mvDepth, mb, mbf,
// mBowVec, mFeatVec, mpORBvocabulary, mpORBextractorLeft / Right, mvImagePyramid).
//
// Vocabulary: TemplatedVocabulary keeps its tree protected, so the device copy is
// loaded from the file System.cc loads (one added line after loadFromTextFile /
// loadFromBinaryFile: gpu::BindVocabulary(mpVocabulary, strVocFile), INTEGRATION.md
// §1).  A Frame whose vocabulary was never bound gets no BoW (logged once): there is
// no CPU fallback.
#ifndef YGZFE_FRAME_GPU_H_
#define YGZFE_FRAME_GPU_H_

#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "ygzfe_dropin.h"

namespace ygz {
namespace gpu {

// ------------------------------------------------------------------ undistortion maps
// initUndistortRectifyMap(K, D, I, K, size, CV_16SC2) once per (K, D, size): the
// reference caches map1 / map2 in static Frame members (Frame.h:268, Frame.cc:776-783)
class UndistortCache {
public:
    static UndistortCache &instance() {
        static UndistortCache *c = new UndistortCache();  // lives as long as the process
        return *c;
    }
    ygzfe_undistort *get(const float K[4], const float *dist, int ndist, int W, int H) {
        std::lock_guard<std::mutex> lk(mu_);
        for (Entry &e : entries_)
            if (e.W == W && e.H == H && e.ndist == ndist && std::memcmp(e.K, K, sizeof(e.K)) == 0 &&
                std::memcmp(e.dist, dist, sizeof(float) * ndist) == 0)
                return e.u;
        Entry e;
        std::memcpy(e.K, K, sizeof(e.K));
        for (int i = 0; i < ndist && i < 12; i++) e.dist[i] = dist[i];
        e.ndist = ndist;
        e.W = W;
        e.H = H;
        ygzfe_camera cam;
        cam.fx = K[0];
        cam.fy = K[1];
        cam.cx = K[2];
        cam.cy = K[3];
        if (ygzfe_undistort_create(dropin::device(), &cam, dist, ndist, W, H, &e.u) != YGZFE_OK) {
            dropin::log_once("initUndistortRectifyMap", dropin::last_error());
            return nullptr;
        }
        entries_.push_back(e);
        return e.u;
    }

private:
    struct Entry {
        float K[4] = {0, 0, 0, 0}, dist[12] = {0};
        int ndist = 0, W = 0, H = 0;
        ygzfe_undistort *u = nullptr;
    };
    std::mutex mu_;
    std::vector<Entry> entries_;
};

template <class FrameT>
inline ygzfe_undistort *undistort_of(const FrameT &F, int W, int H) {
    // Converter::toCvMat(mK): fx = K(0,0), fy = K(1,1), cx = K(0,2), cy = K(1,2) (Tracking.cc:165-169);
    // mDistCoef: 4, 5 or 8 CV_32F coefficients (Tracking.cc:171-204)
    const float K[4] = {F.mK(0, 0), F.mK(1, 1), F.mK(0, 2), F.mK(1, 2)};
    const int nd = F.mDistCoef.rows * F.mDistCoef.cols;
    float d[12] = {0};
    for (int i = 0; i < nd && i < 12; i++) d[i] = F.mDistCoef.template ptr<float>(0)[i];
    return UndistortCache::instance().get(K, d, nd < 12 ? nd : 12, W, H);
}

// Frame.cc:773-805
template <class FrameT>
inline void ComputeImagePyramid(FrameT &F) {
    if (FrameT::mbNeedUndistort) {
        const int W = F.mImGray.cols, H = F.mImGray.rows;
        ygzfe_undistort *u = W > 0 && H > 0 ? undistort_of(F, W, H) : nullptr;
        if (u) {
            // cv::remap(mImGray, img_undistorted, map1, map2, INTER_LINEAR), Frame.cc:786-789
            cv::Mat g(H, W, CV_8U);
            if (ygzfe_undistort_image(u, F.mImGray.data, (int)F.mImGray.step[0], g.data, (int)g.step[0]) == YGZFE_OK)
                F.mImGray = g;
            else
                dropin::log_once("remap(mImGray)", dropin::last_error());
            if (F.mSensor == FrameT::Stereo && !F.mImRight.empty()) {  // :791-797
                cv::Mat r(H, W, CV_8U);
                if (ygzfe_undistort_image(u, F.mImRight.data, (int)F.mImRight.step[0], r.data, (int)r.step[0]) ==
                    YGZFE_OK)
                    F.mImRight = r;
                else
                    dropin::log_once("remap(mImRight)", dropin::last_error());
            }
            if (F.mSensor == FrameT::RGBD && !F.mImDepth.empty()) {  // :799-804
                cv::Mat d(H, W, CV_32F);
                if (ygzfe_undistort_depth(u, F.mImDepth.template ptr<float>(0), (int)(F.mImDepth.step[0] / 4),
                                          d.template ptr<float>(0), (int)(d.step[0] / 4)) == YGZFE_OK)
                    F.mImDepth = d;
                else
                    dropin::log_once("remap(mImDepth)", dropin::last_error());
            }
        }
    }
    // Frame.cc:807-813.  The reference clones the extractor's levels because its
    // extractor resizes into them again for the next image; the drop-in extractor
    // hands out fresh buffers per ComputePyramid that nothing writes afterwards, so the
    // Frame shares them: the same pixels without a copy, and the device pyramid is
    // found by their level-0 pointer
    F.mpORBextractorLeft->ComputePyramid(F.mImGray);
    F.mvImagePyramid = F.mpORBextractorLeft->mvImagePyramid;
}

// Frame.cc:186-188, the copy constructor's pyramid copy (Tracking's
// mLastFrame = Frame(mCurrentFrame), Tracking.cc:718): the same deep copy, and the
// copy's level 0 indexed to the device pyramid of the original (no compare, no upload
// when the next SparseImgAlign::run reads mLastFrame)
template <class MatVec>
inline void CopyImagePyramid(MatVec &dst, const MatVec &src) {
    for (const auto &mat : src) dst.push_back(mat.clone());
    dropin::PyramidPool::instance().alias(dst, src);
}

// Frame.cc:509-682: row-band Hamming search + SAD sub-pixel refinement + median cut,
// over the two extractors' pyramids (:515, 604, 618)
template <class FrameT>
inline void ComputeStereoMatches(FrameT &F) {
    F.mvuRight = std::vector<float>(F.N, -1.0f);
    F.mvDepth = std::vector<float>(F.N, -1.0f);
    if (F.N <= 0 || F.mvKeysRight.empty()) return;
    dropin::PyramidPool &pool = dropin::PyramidPool::instance();
    ygzfe_frame *left = pool.find_or_upload(F.mpORBextractorLeft->mvImagePyramid);
    ygzfe_frame *right = pool.find_or_upload(F.mpORBextractorRight->mvImagePyramid);
    if (!left || !right) {
        dropin::log_once("ComputeStereoMatches", "no device pyramid");
        return;
    }
    const int nr = (int)F.mvKeysRight.size();
    const std::vector<uint8_t> dl = dropin::desc_rows(F.mDescriptors, F.N);
    const std::vector<uint8_t> dr = dropin::desc_rows(F.mDescriptorsRight, nr);
    if (ygzfe_stereo_matches(left, right, dropin::as_kp(F.mvKeys.data()), dl.data(), F.N,
                             dropin::as_kp(F.mvKeysRight.data()), dr.data(), nr, F.mb, F.mbf, F.mvuRight.data(),
                             F.mvDepth.data()) != YGZFE_OK) {
        dropin::log_once("ComputeStereoMatches", dropin::last_error());
        F.mvuRight.assign(F.N, -1.0f);
        F.mvDepth.assign(F.N, -1.0f);
    }
}

// Frame.cc:684-700
template <class FrameT, class MatT>
inline void ComputeStereoFromRGBD(FrameT &F, const MatT &imDepth) {
    F.mvuRight = std::vector<float>(F.N, -1);
    F.mvDepth = std::vector<float>(F.N, -1);
    if (F.N <= 0 || imDepth.empty()) return;
    if (ygzfe_stereo_from_rgbd(dropin::device(), imDepth.template ptr<float>(0), imDepth.cols, imDepth.rows,
                               (int)(imDepth.step[0] / 4), dropin::as_kp(F.mvKeys.data()), F.N, F.mbf,
                               F.mvuRight.data(), F.mvDepth.data()) != YGZFE_OK) {
        dropin::log_once("ComputeStereoFromRGBD", dropin::last_error());
        F.mvuRight.assign(F.N, -1.0f);
        F.mvDepth.assign(F.N, -1.0f);
    }
}

// ------------------------------------------------------------------ vocabulary
class VocabRegistry {
public:
    static VocabRegistry &instance() {
        static VocabRegistry *r = new VocabRegistry();
        return *r;
    }
    void bind(const void *voc, ygzfe_vocab *v) {
        std::lock_guard<std::mutex> lk(mu_);
        map_[voc] = v;
    }
    ygzfe_vocab *find(const void *voc) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = map_.find(voc);
        return it == map_.end() ? nullptr : it->second;
    }

private:
    std::mutex mu_;
    std::map<const void *, ygzfe_vocab *> map_;
};

// System.cc, after mpVocabulary->loadFromTextFile(strVocFile) (or loadFromBinaryFile):
// the same file into HBM, bound to that ORBVocabulary
inline bool BindVocabulary(const void *voc, const char *path, bool binary = false) {
    ygzfe_vocab *v = nullptr;
    const int rc = binary ? ygzfe_vocab_load_binary(dropin::device(), path, &v)
                          : ygzfe_vocab_load_text(dropin::device(), path, &v);
    if (rc != YGZFE_OK) {
        dropin::log_once("BindVocabulary", dropin::last_error());
        return false;
    }
    VocabRegistry::instance().bind(voc, v);
    return true;
}
inline void BindVocabulary(const void *voc, ygzfe_vocab *v) { VocabRegistry::instance().bind(voc, v); }

// Frame.cc:495-500: mpORBvocabulary->transform(toDescriptorVector(mDescriptors), mBowVec, mFeatVec, 4)
template <class FrameT>
inline void ComputeBoW(FrameT &F) {
    if (!F.mBowVec.empty()) return;
    ygzfe_vocab *v = VocabRegistry::instance().find(F.mpORBvocabulary);
    if (!v) {
        dropin::log_once("ComputeBoW", "vocabulary not bound on the GPU (call gpu::BindVocabulary after loading it)");
        return;
    }
    const int n = F.mDescriptors.empty() ? 0 : F.mDescriptors.rows;
    F.mFeatVec.clear();
    if (n == 0) return;
    const std::vector<uint8_t> d = dropin::desc_rows(F.mDescriptors, n);
    std::vector<int32_t> words(n), fn(n), ff(n);
    std::vector<double> values(n);
    int nw = 0, nfv = 0;
    if (ygzfe_compute_bow(v, d.data(), n, 4, words.data(), values.data(), &nw, fn.data(), ff.data(), &nfv) !=
        YGZFE_OK) {
        dropin::log_once("ComputeBoW", dropin::last_error());
        return;
    }
    for (int i = 0; i < nw; i++) F.mBowVec[(unsigned)words[i]] = values[i];
    for (int i = 0; i < nfv; i++) F.mFeatVec[(unsigned)fn[i]].push_back((unsigned)ff[i]);
}

}  // namespace gpu
}  // namespace ygz

#endif
