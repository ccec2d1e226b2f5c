// ygz_compat.hpp — drop-in C++ classes with the reference's hot-path signatures,
// implemented over the ygzfe C ABI (include/ygzfe.h).  Header-only; link
// orb-ygz-slam_amd/lib/libygzfe.so.
//
//   ygz::ORBextractor    ORBextractor.h:45-192  (ctor :53-57, operator() :71-85,
//                        ComputePyramid :112, getters :87-109)
//   ygz::ORBmatcher      ORBmatcher.h:38-178    (DescriptorDistance :94, the Hamming
//                        inner loops of the Search* functions)
//   ygz::SparseImgAlign  SparseImageAlign.h:37-60 (ctor, run :45, getFisherInformation)
//   ygz::Align2D         Align.h:20-26
//
// Without OpenCV the adapters use std::vector<KeyPoint> (KeyPoint has
// cv::KeyPoint's exact 28-byte layout) and row-major N x 32 descriptor
// buffers.  Define YGZ_COMPAT_OPENCV before including to get the cv::Mat /
// cv::KeyPoint overloads the reference's Tracking.cc / Frame.cc call.
// Errors follow the reference's conventions: empty results, run() == 0,
// Align2D() == false; ygz::compat::last_error() carries the message.
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "ygzfe.h"

#ifdef YGZ_COMPAT_OPENCV
#include <opencv2/core/core.hpp>
#endif

namespace ygz {

#ifdef YGZ_COMPAT_OPENCV
using KeyPoint = cv::KeyPoint;
#else
// cv::KeyPoint field order: pt.x, pt.y, size, angle, response, octave, class_id
struct KeyPoint {
    struct Point2f { float x, y; } pt{0.f, 0.f};
    float size = 0.f, angle = -1.f, response = 0.f;
    int octave = 0, class_id = -1;
};
#endif
static_assert(sizeof(KeyPoint) == sizeof(ygzfe_kp), "KeyPoint must have cv::KeyPoint's 28-byte layout");

enum KeyPointMethod { ORBSLAM_KEYPOINT = YGZFE_ORBSLAM_KEYPOINT, FAST_KEYPOINT = YGZFE_FAST_KEYPOINT,
                      DSO_KEYPOINT = YGZFE_DSO_KEYPOINT };

namespace compat {
inline std::string last_error() { return ygzfe_last_error(); }
inline void check(int rc, const char *what) {
    if (rc != YGZFE_OK) throw std::runtime_error(std::string(what) + ": " + ygzfe_last_error());
}
inline ygzfe_kp *as_kp(KeyPoint *p) { return reinterpret_cast<ygzfe_kp *>(p); }
inline const ygzfe_kp *as_kp(const KeyPoint *p) { return reinterpret_cast<const ygzfe_kp *>(p); }
}  // namespace compat

// A frame's device-resident pyramid (Frame::mvImagePyramid, Frame.cc:807-813).
class FramePyramid {
public:
    FramePyramid() = default;
    FramePyramid(const FramePyramid &) = delete;
    FramePyramid &operator=(const FramePyramid &) = delete;
    ~FramePyramid() { ygzfe_frame_destroy(f_); }
    ygzfe_frame *handle() const { return f_; }
    int width() const { return w_; }
    int height() const { return h_; }
    // host copy of one level (the reference reads mvImagePyramid[l] on the host)
    std::vector<uint8_t> level(int l, int *w = nullptr, int *h = nullptr) const {
        int lw = 0, lh = 0;
        compat::check(ygzfe_frame_level(f_, l, &lw, &lh, nullptr, 0), "frame_level");
        std::vector<uint8_t> out((size_t)lw * lh);
        compat::check(ygzfe_frame_level(f_, l, nullptr, nullptr, out.data(), lw), "frame_level");
        if (w) *w = lw;
        if (h) *h = lh;
        return out;
    }

private:
    friend class ORBextractor;
    ygzfe_frame *f_ = nullptr;
    int w_ = 0, h_ = 0;
};

class ORBextractor {
public:
    // ORBextractor.h:53-57 (+ the GPU ordinal)
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0) {
        ygzfe_orb_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, YGZFE_BLUR_CV4};
        compat::check(ygzfe_extractor_create(&p, device, &ex_), "ORBextractor");
        nlevels_ = nlevels;
        scale_factor_ = scaleFactor;
    }
    ORBextractor(const ORBextractor &) = delete;
    ORBextractor &operator=(const ORBextractor &) = delete;
    ~ORBextractor() { ygzfe_extractor_destroy(ex_); }

    // ComputePyramid(cv::Mat image) (ORBextractor.h:112, ORBextractor.cc:1129-1150)
    void ComputePyramid(FramePyramid &f, const uint8_t *image, int width, int height, int stride) {
        if (!f.f_ || f.w_ != width || f.h_ != height) {
            ygzfe_frame_destroy(f.f_);
            f.f_ = nullptr;
            compat::check(ygzfe_frame_create(ex_, width, height, &f.f_), "frame_create");
            f.w_ = width;
            f.h_ = height;
        }
        compat::check(ygzfe_compute_pyramid(ex_, f.f_, image, stride), "ComputePyramid");
    }

    // operator()(Frame*, keypoints, descriptors, method, leftEye) (ORBextractor.h:79-85):
    // `keypoints` holds the frame's existing keypoints on entry (their descriptor
    // rows come first) and all keypoints on return; descriptors = n x 32 bytes.
    void operator()(FramePyramid &f, std::vector<KeyPoint> &keypoints, std::vector<uint8_t> &descriptors,
                    KeyPointMethod method, bool leftEye = true) {
        (void)leftEye;  // both eyes use the same extractor state in the reference's Frame path
        const int n_existing = (int)keypoints.size();
        const int cap = n_existing + capacity_hint(f);
        keypoints.resize(cap);
        descriptors.resize((size_t)cap * 32);
        int n = 0;
        const int rc = ygzfe_extract(ex_, f.f_, (int)method, compat::as_kp(keypoints.data()), n_existing, cap,
                                     descriptors.data(), &n);
        if (rc != YGZFE_OK) {  // the reference never throws: empty result
            keypoints.clear();
            descriptors.clear();
            return;
        }
        keypoints.resize(n);
        descriptors.resize((size_t)n * 32);
    }

    // operator()(InputArray image, InputArray mask, keypoints, descriptors) (ORBextractor.h:71-75)
    void operator()(const uint8_t *image, int width, int height, int stride, std::vector<KeyPoint> &keypoints,
                    std::vector<uint8_t> &descriptors) {
        keypoints.clear();
        descriptors.clear();
        if (!image || width <= 0 || height <= 0) return;  // ORBextractor.cc:972-973
        ComputePyramid(scratch_, image, width, height, stride);
        (*this)(scratch_, keypoints, descriptors, ORBSLAM_KEYPOINT);
    }

#ifdef YGZ_COMPAT_OPENCV
    void operator()(cv::InputArray image, cv::InputArray /*mask*/, std::vector<cv::KeyPoint> &keypoints,
                    cv::OutputArray descriptors) {
        cv::Mat img = image.getMat();
        std::vector<uint8_t> d;
        (*this)(img.data, img.cols, img.rows, (int)img.step, keypoints, d);
        if (keypoints.empty()) { descriptors.release(); return; }
        descriptors.create((int)keypoints.size(), 32, CV_8U);
        std::memcpy(descriptors.getMat().data, d.data(), d.size());
    }
#endif

    // getters (ORBextractor.h:87-109)
    int inline GetLevels() const { return nlevels_; }
    float inline GetScaleFactor() const { return scale_factor_; }
    std::vector<float> inline GetScaleFactors() const { return levels(0); }
    std::vector<float> inline GetInverseScaleFactors() const { return levels(1); }
    std::vector<float> inline GetScaleSigmaSquares() const { return levels(2); }
    std::vector<float> inline GetInverseScaleSigmaSquares() const { return levels(3); }
    std::vector<int> GetFeaturesPerLevel() const {
        std::vector<int> v(nlevels_);
        compat::check(ygzfe_extractor_features_per_level(ex_, v.data()), "features_per_level");
        return v;
    }
    ygzfe_extractor *handle() const { return ex_; }

private:
    std::vector<float> levels(int which) const {
        std::vector<float> a(nlevels_), b(nlevels_), c(nlevels_), d(nlevels_);
        compat::check(ygzfe_extractor_levels(ex_, nullptr, a.data(), b.data(), c.data(), d.data()), "levels");
        return which == 0 ? a : which == 1 ? b : which == 2 ? c : d;
    }
    int capacity_hint(const FramePyramid &f) const {
        // octree output per level <= budget + 3 (+ DSO grid: 3 per 7x7 cell at most)
        int s = 0;
        for (int v : GetFeaturesPerLevel()) s += v + 8;
        return s + 3 * (f.w_ / 7 + 1) * (f.h_ / 7 + 1);
    }
    ygzfe_extractor *ex_ = nullptr;
    int nlevels_ = 0;
    float scale_factor_ = 1.f;
    FramePyramid scratch_;
};

class ORBmatcher {
public:
    static const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;  // ORBmatcher.cc:36-38
    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true, int device = 0)
        : mfNNratio(nnratio), mbCheckOrientation(checkOri), device_(device) {}

    // ORBmatcher::DescriptorDistance (ORBmatcher.cc:1507-1523)
    static int DescriptorDistance(const uint8_t *a, const uint8_t *b) { return ygzfe_descriptor_distance(a, b); }
#ifdef YGZ_COMPAT_OPENCV
    static int DescriptorDistance(const cv::Mat &a, const cv::Mat &b) { return ygzfe_descriptor_distance(a.data, b.data); }
#endif

    // Dense best / second best (the inner loop of SearchByProjection & co.):
    // per query: best train index (first minimum), best and second distances.
    void SearchBest2(const uint8_t *query, int nq, const uint8_t *train, int nt, std::vector<int> &best_idx,
                     std::vector<int> &best_dist, std::vector<int> &second_dist) const {
        best_idx.assign(nq, -1);
        best_dist.assign(nq, 256);
        second_dist.assign(nq, 256);
        if (nq == 0 || nt == 0) return;
        compat::check(ygzfe_hamming_best2(device_, query, nq, train, nt, best_idx.data(), best_dist.data(),
                                          second_dist.data()),
                      "hamming_best2");
    }
    // Windowed candidates (Frame::GetFeaturesInArea lists as CSR): the distance of every
    // (query, candidate) pair, for replaying the reference's sequential assignment rules.
    std::vector<int> SearchWindowed(const uint8_t *query, int nq, const uint8_t *train, int nt,
                                    const std::vector<int> &row_ptr, const std::vector<int> &cand) const {
        std::vector<int> dist(cand.size(), 256);
        if (!cand.empty())
            compat::check(ygzfe_hamming_csr(device_, query, nq, train, nt, row_ptr.data(), cand.data(), dist.data()),
                          "hamming_csr");
        return dist;
    }

    float mfNNratio;
    bool mbCheckOrientation;

private:
    int device_;
};

// Sophus::SE3f as unit quaternion (x, y, z, w) + translation
struct SE3 {
    std::array<float, 4> q{{0.f, 0.f, 0.f, 1.f}};
    std::array<float, 3> t{{0.f, 0.f, 0.f}};
};

class SparseImgAlign {
public:
    // SparseImgAlign(int n_levels, int min_level, int n_iter = 10, Method = GaussNewton, ...) (SparseImageAlign.h:37-43)
    // n_iter is accepted and ignored, as in the reference: run() overrides it per level
    // with iterations[] = {10, ...} (SparseImageAlign.cc:38-43).
    SparseImgAlign(int n_levels, int min_level, int n_iter = 10) : max_level_(n_levels), min_level_(min_level) {
        (void)n_iter;
    }
    // size_t run(Frame* ref, Frame* cur, SE3f& TCR) (SparseImageAlign.cc:20-49): the ref
    // frame's keypoints, xyz_ref = T_ref * P_w per keypoint, usable = has a good MapPoint.
    // TCR: in = initial guess, out = estimate.  Returns the visible-feature count.
    size_t run(const FramePyramid &ref, const FramePyramid &cur, const ygzfe_camera &cam,
               const std::vector<KeyPoint> &kps, const float *xyz_ref, const uint8_t *usable, SE3 &TCR) {
        ygzfe_se3 T0;
        std::memcpy(T0.q, TCR.q.data(), sizeof(T0.q));
        std::memcpy(T0.t, TCR.t.data(), sizeof(T0.t));
        ygzfe_align_result r;
        if (ygzfe_sparse_align(ref.handle(), cur.handle(), &cam, compat::as_kp(kps.data()), xyz_ref, usable,
                               (int)kps.size(), max_level_, min_level_, &T0, &r) != YGZFE_OK)
            return 0;
        std::memcpy(TCR.q.data(), r.T_cur_ref.q, sizeof(r.T_cur_ref.q));
        std::memcpy(TCR.t.data(), r.T_cur_ref.t, sizeof(r.T_cur_ref.t));
        std::memcpy(H_, r.H, sizeof(H_));
        return (size_t)(r.n_visible > 0 ? r.n_visible : 0);
    }
    // getFisherInformation() (SparseImageAlign.cc:51-55): H_ / sigma_i_sq with
    // float sigma_i_sq = 5e-4 * 255 * 255 (double product, 32.5125, rounded to float)
    std::array<float, 36> getFisherInformation() const {
        const float s2 = (float)(5e-4 * 255 * 255);
        std::array<float, 36> I;
        for (int i = 0; i < 36; i++) I[i] = H_[i] / s2;
        return I;
    }
    // H_ of the last linearisation (NLLSSolver::H_), row-major 6x6
    const float *hessian() const { return H_; }

private:
    int max_level_, min_level_;
    float H_[36] = {0};
};

// bool Align2D(const cv::Mat& cur_img, uint8_t* ref_patch_with_border, uint8_t* ref_patch,
//              int n_iter, Vector2f& cur_px_estimate, bool no_simd = false) (Align.h:20-26),
// with the current image given as a FramePyramid level.
inline bool Align2D(const FramePyramid &cur, int level, const uint8_t *ref_patch_with_border,
                    const uint8_t *ref_patch, int n_iter, float cur_px_estimate[2], bool no_simd = false) {
    (void)no_simd;
    uint8_t ok = 0;
    if (ygzfe_align2d_batch(cur.handle(), level, 1, ref_patch_with_border, ref_patch, n_iter, cur_px_estimate,
                            &ok) != YGZFE_OK)
        return false;
    return ok != 0;
}

// Tracking::SearchLocalPointsDirect (Tracking.cc:2258-2410) with its per-point
// FindDirectProjection loop batched on the GPU.  The caller keeps the reference's
// control flow (isBad / isInFrustum / cache set / UpdateLocalMap) and, per
// surviving map point, lists its SelectNearestKeyframe observations
// (Tracking.cc:2412-2432) in order:
//
//   ygz::DirectSearch ds;
//   for (MapPoint *mp : candidates) {            // after isInFrustum(mp, 0.5)
//       ds.add_point(mp->mTrackProjX, mp->mTrackProjY);
//       for (auto &o : SelectNearestKeyframe(mp->GetObservations(), 5))
//           ds.add_observation(slot_of(o.first), o.first->mvKeys[o.second],
//                              o.first->GetPose() * mp->GetWorldPos(), mCurrentFrame.mTcw * o.first->GetPose().inverse());
//   }
//   ds.run(keyframe_pyramids, current_pyramid, cam);   // one GPU pass over all (point, keyframe) items
//   // ds.matched(i) / ds.px(i): the reference's px_ave for point i (or no match)
//
// For the cache pass (Tracking.cc:2268-2325) cache_pass() replays the 5x5-px
// occupancy grid in cache order: a point whose predicted cell is already
// taken is kept untried, a matched point marks the cell of its pixel, an
// unmatched point leaves the cache.
class DirectSearch {
public:
    enum CacheOutcome { kMatched = 0, kKeptUntried = 1, kErased = 2 };

    void clear() { item_ptr_.assign(1, 0); proj_.clear(); ref_.clear(); kps_.clear(); pt_.clear(); T_.clear(); }
    int add_point(float proj_x, float proj_y) {
        if (item_ptr_.empty()) item_ptr_.push_back(0);
        proj_.push_back(proj_x);
        proj_.push_back(proj_y);
        item_ptr_.push_back(item_ptr_.back());
        return (int)proj_.size() / 2 - 1;
    }
    void add_observation(int kf_slot, const KeyPoint &kp, const float pt_ref[3], const SE3 &T_cr) {
        ref_.push_back(kf_slot);
        kps_.push_back(kp);
        pt_.insert(pt_.end(), pt_ref, pt_ref + 3);
        ygzfe_se3 t;
        std::memcpy(t.q, T_cr.q.data(), sizeof(t.q));
        std::memcpy(t.t, T_cr.t.data(), sizeof(t.t));
        T_.push_back(t);
        item_ptr_.back() += 1;
    }
    int n_points() const { return (int)proj_.size() / 2; }
    // FindDirectProjection over every item + first in-border success per point
    void run(const std::vector<const FramePyramid *> &keyframes, const FramePyramid &cur, const ygzfe_camera &cam,
             float border = 20.f) {
        const int n = n_points();
        px_.assign(2 * (size_t)n, 0.f);
        matched_.assign(n, -1);
        if (n == 0) return;
        std::vector<const ygzfe_frame *> h(keyframes.size());
        for (size_t i = 0; i < keyframes.size(); i++) h[i] = keyframes[i]->handle();
        compat::check(ygzfe_search_direct_batch(h.data(), (int)h.size(), cur.handle(), &cam, n, item_ptr_.data(),
                                                ref_.data(), compat::as_kp(kps_.data()), pt_.data(), T_.data(),
                                                proj_.data(), border, px_.data(), matched_.data()),
                      "search_direct_batch");
    }
    bool matched(int i) const { return matched_[i] >= 0; }
    int matched_observation(int i) const { return matched_[i] < 0 ? -1 : matched_[i] - item_ptr_[i]; }
    const float *px(int i) const { return &px_[2 * (size_t)i]; }
    // Tracking.cc:2262-2325: grid_size 5 over level 0 (rows / 5 x cols / 5 cells)
    std::vector<CacheOutcome> cache_pass(int cols, int rows, int grid_size = 5) const {
        const int gr = rows / grid_size, gc = cols / grid_size;
        std::vector<bool> grid((size_t)gr * gc, false);
        std::vector<CacheOutcome> out(n_points());
        for (int i = 0; i < n_points(); i++) {
            const int k = (int)(proj_[2 * i + 1] / grid_size) * gc + (int)(proj_[2 * i] / grid_size);
            if (grid[k]) { out[i] = kKeptUntried; continue; }
            if (matched_[i] < 0) { out[i] = kErased; continue; }
            grid[(size_t)((int)(px_[2 * i + 1] / grid_size) * gc + (int)(px_[2 * i] / grid_size))] = true;
            out[i] = kMatched;
        }
        return out;
    }

private:
    std::vector<int32_t> item_ptr_{0}, ref_, matched_;
    std::vector<float> proj_, pt_, px_;
    std::vector<KeyPoint> kps_;
    std::vector<ygzfe_se3> T_;
};

// Frame::ComputeStereoMatches (Frame.cc:509-682): fills mvuRight / mvDepth (-1 = none)
// from the two extractors' pyramids, keypoints and descriptors.
inline void ComputeStereoMatches(const FramePyramid &left, const FramePyramid &right,
                                 const std::vector<KeyPoint> &keys, const std::vector<uint8_t> &desc,
                                 const std::vector<KeyPoint> &keys_right, const std::vector<uint8_t> &desc_right,
                                 float mb, float mbf, std::vector<float> &uRight, std::vector<float> &depth) {
    uRight.assign(keys.size(), -1.f);
    depth.assign(keys.size(), -1.f);
    if (keys.empty()) return;
    compat::check(ygzfe_stereo_matches(left.handle(), right.handle(), compat::as_kp(keys.data()), desc.data(),
                                       (int)keys.size(), compat::as_kp(keys_right.data()), desc_right.data(),
                                       (int)keys_right.size(), mb, mbf, uRight.data(), depth.data()),
                  "stereo_matches");
}

// ORBVocabulary (TemplatedVocabulary<FORB::TDescriptor, FORB>) resident on the GPU, with the
// loaders System.cc:187-189 calls and the transform Frame::ComputeBoW (Frame.cc:495-500) calls.
// BowVector / FeatureVector come back as their std::map contents in map order.
class ORBVocabulary {
public:
    explicit ORBVocabulary(int device = 0) : device_(device) {}
    ~ORBVocabulary() { ygzfe_vocab_destroy(v_); }
    ORBVocabulary(const ORBVocabulary &) = delete;
    ORBVocabulary &operator=(const ORBVocabulary &) = delete;
    bool loadFromTextFile(const std::string &path) { return reload(ygzfe_vocab_load_text(device_, path.c_str(), &n_)); }
    bool loadFromBinaryFile(const std::string &path) {
        return reload(ygzfe_vocab_load_binary(device_, path.c_str(), &n_));
    }
    bool empty() const {
        int words = 0;
        return !v_ || ygzfe_vocab_info(v_, nullptr, nullptr, nullptr, nullptr, nullptr, &words) != YGZFE_OK ||
               words == 0;
    }
    // transform(features, BowVector&, FeatureVector&, levelsup); desc = n x 32 bytes
    void transform(const uint8_t *desc, int n, std::vector<std::pair<int, double>> &bow,
                   std::vector<std::pair<int, std::vector<unsigned>>> &feat, int levelsup) const {
        bow.clear();
        feat.clear();
        if (!v_ || n <= 0) return;
        std::vector<int32_t> w(n), fn(n), ff(n);
        std::vector<double> val(n);
        int nw = 0, nf = 0;
        compat::check(ygzfe_compute_bow(v_, desc, n, levelsup, w.data(), val.data(), &nw, fn.data(), ff.data(), &nf),
                      "compute_bow");
        for (int i = 0; i < nw; i++) bow.emplace_back(w[i], val[i]);
        for (int i = 0; i < nf; i++) {
            if (feat.empty() || feat.back().first != fn[i]) feat.emplace_back(fn[i], std::vector<unsigned>());
            feat.back().second.push_back((unsigned)ff[i]);
        }
    }
    const ygzfe_vocab *handle() const { return v_; }

private:
    bool reload(int rc) {
        if (rc != YGZFE_OK) return false;
        ygzfe_vocab_destroy(v_);
        v_ = n_;
        n_ = nullptr;
        return true;
    }
    int device_;
    ygzfe_vocab *v_ = nullptr, *n_ = nullptr;
};

}  // namespace ygz
