// ORBmatcherGPU.h — the tracking-path ORBmatcher searches on the GPU, read
// through the reference's own Frame / KeyFrame / MapPoint members.
//
// ORBmatcher.h is kept unchanged (LocalMapping / LoopClosing use its other
// searches); ORBmatcher.cc includes ORBmatcher_gpu.inc in place of the bodies
// of the five tracking searches, which forward here:
//   SearchByProjection(Frame &F, const vector<MapPoint*> &, th, checkLevel)   ORBmatcher.cc:43-126
//   SearchByBoW(KeyFrame *pKF, Frame &F, vector<MapPoint*> &)                ORBmatcher.cc:155-263
//   SearchForInitialization(Frame &F1, Frame &F2, vbPrevMatched, vnMatches12) ORBmatcher.cc:375-478
//   SearchByProjection(Frame &Cur, const Frame &Last, th, bMono, checkLevel)  ORBmatcher.cc:1218-1350
//   SearchByProjection(Frame &Cur, KeyFrame *pKF, sAlreadyFound, th, ORBdist) ORBmatcher.cc:1352-1469
// so Tracking.cc's calls (Tracking.cc:826, 1020, 1171, 1674, 1866, 1933)
// compile and run unchanged.  The projections, windows and flags are formed
// here on the host with the caller's Eigen / Sophus types, exactly as the
// reference forms them; the window search, Hamming distances, the sequential
// rules and the rotation check run on the GPU (include/ygzfe.h
// ygzfe_search_*); the MapPoint assignments are applied back to the Frame.
#ifndef YGZFE_ORBMATCHER_GPU_H_
#define YGZFE_ORBMATCHER_GPU_H_

#include <cmath>
#include <set>
#include <vector>

#include "Common.h"
#include "ygzfe_dropin.h"

namespace ygz {
namespace gpu {

constexpr int kTH_HIGH = 100, kTH_LOW = 50;  // ORBmatcher.cc:36-37

// a per-thread device view of one Frame / KeyFrame (mvKeys, mDescriptors, mvuRight).
// Tracking searches one CurrentFrame several times (motion model, then the local
// map, ...): a view whose rows, descriptors, mvuRight and bounds are byte-equal to
// the last upload is reused without a new upload or grid build.
class MatchView {
public:
    explicit MatchView(int slot) {
        if (ygzfe_match_frame_create(dropin::device(), &h_) != YGZFE_OK) h_ = nullptr;
        (void)slot;
    }
    ~MatchView() { ygzfe_match_frame_destroy(h_); }
    template <class KeyVec, class DescMat>
    bool set(const KeyVec &keys, const DescMat &desc, int n, const float *u_right, const ygzfe_bounds &b) {
        if (!h_) {
            dropin::log_once("ORBmatcher search", "no device match frame (ygzfe_match_frame_create failed)");
            return false;
        }
        const std::vector<uint8_t> d = dropin::desc_rows(desc, n);
        const ygzfe_kp *k = dropin::as_kp(keys.data());
        const size_t kb = sizeof(ygzfe_kp) * (size_t)n;
        if (valid_ && n == n_ && (u_right != nullptr) == has_ur_ && std::memcmp(&b, &b_, sizeof(b)) == 0 &&
            std::memcmp(k, kps_.data(), kb) == 0 && d == desc_ &&
            (!u_right || std::memcmp(u_right, ur_.data(), 4 * (size_t)n) == 0))
            return true;
        valid_ = false;
        if (ygzfe_match_frame_set(h_, k, d.data(), n, u_right, &b) != YGZFE_OK) {
            dropin::log_once("ORBmatcher search", ygzfe_last_error());
            return false;
        }
        n_ = n;
        b_ = b;
        has_ur_ = u_right != nullptr;
        kps_.assign(k, k + n);
        desc_ = d;
        ur_.assign(u_right ? u_right : nullptr, u_right ? u_right + n : nullptr);
        valid_ = true;
        return true;
    }
    ygzfe_match_frame *get() const { return h_; }

private:
    ygzfe_match_frame *h_ = nullptr;
    bool valid_ = false, has_ur_ = false;
    int n_ = 0;
    ygzfe_bounds b_{};
    std::vector<ygzfe_kp> kps_;
    std::vector<uint8_t> desc_;
    std::vector<float> ur_;
};

inline MatchView &view(int slot) {
    static thread_local MatchView *v[2] = {nullptr, nullptr};  // kept for the thread's lifetime
    if (!v[slot]) v[slot] = new MatchView(slot);
    return *v[slot];
}

template <class FrameT>
inline ygzfe_bounds bounds_of() {
    ygzfe_bounds b;
    b.min_x = FrameT::mnMinX;
    b.max_x = FrameT::mnMaxX;
    b.min_y = FrameT::mnMinY;
    b.max_y = FrameT::mnMaxY;
    return b;
}

template <class FrameT>
inline bool set_frame(MatchView &v, const FrameT &F, bool with_uright) {
    const int n = F.N;
    return v.set(F.mvKeys, F.mDescriptors, n,
                 with_uright && (int)F.mvuRight.size() >= n && n > 0 ? F.mvuRight.data() : nullptr,
                 bounds_of<FrameT>());
}

template <class Mat>
inline void append_desc(std::vector<uint8_t> &out, const Mat &d) {
    const size_t o = out.size();
    out.resize(o + 32);
    std::memcpy(&out[o], d.data, 32);
}

inline int failed(const char *where) {
    dropin::log_once(where, ygzfe_last_error());
    return 0;
}

// ORBmatcher::RadiusByViewingCos (ORBmatcher.cc:128-133)
inline float radius_by_viewing_cos(const float &viewCos) { return viewCos > 0.998 ? 2.5f : 4.0f; }

// SearchByProjection(F, vpMapPoints, th, checkLevel) (ORBmatcher.cc:43-126)
template <class FrameT, class MapPointT>
int SearchByProjection(FrameT &F, const std::vector<MapPointT *> &vpMapPoints, const float th, bool checkLevel,
                       float nnratio) {
    const bool bFactor = th != 1.0;
    std::vector<ygzfe_match_query> q(vpMapPoints.size());
    std::vector<uint8_t> qd;
    qd.reserve(32 * vpMapPoints.size());
    for (size_t iMP = 0; iMP < vpMapPoints.size(); iMP++) {
        MapPointT *pMP = vpMapPoints[iMP];
        ygzfe_match_query &Q = q[iMP];
        std::memset(&Q, 0, sizeof(Q));
        Q.min_level = Q.max_level = -1;
        if (!pMP->mbTrackInView || pMP->isBad()) {
            qd.resize(qd.size() + 32, 0);
            continue;
        }
        const int &nPredictedLevel = pMP->mnTrackScaleLevel;
        float r = radius_by_viewing_cos(pMP->mTrackViewCos);
        if (bFactor) r *= th;
        Q.u = pMP->mTrackProjX;
        Q.v = pMP->mTrackProjY;
        Q.radius = r * F.mvScaleFactors[nPredictedLevel];
        if (checkLevel) {
            Q.min_level = nPredictedLevel - 1;
            Q.max_level = nPredictedLevel;
        }
        Q.u_right = pMP->mTrackProjXR;
        Q.flags = YGZFE_MQ_VALID | YGZFE_MQ_STEREO | (pMP->Observations() > 0 ? YGZFE_MQ_BLOCKS : 0);
        append_desc(qd, pMP->GetDescriptor());
    }
    std::vector<uint8_t> blocked((size_t)F.N, 0);
    for (int i = 0; i < F.N; i++) blocked[i] = F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0;
    MatchView &v = view(0);
    if (!set_frame(v, F, true)) return 0;
    std::vector<int32_t> out((size_t)F.N + 1);
    int nmatches = 0;
    if (ygzfe_search_projection_ratio(v.get(), q.data(), qd.data(), (int)q.size(), blocked.data(), nnratio, out.data(),
                                      &nmatches) != YGZFE_OK)
        return failed("SearchByProjection(F, vpMapPoints)");
    for (int i = 0; i < F.N; i++)
        if (out[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[out[i]];
    return nmatches;
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono, checkLevel) (ORBmatcher.cc:1218-1350)
template <class FrameT>
int SearchByProjection(FrameT &CurrentFrame, const FrameT &LastFrame, const float th, const bool bMono,
                       bool checkLevel, bool checkOri) {
    // the reference's own Eigen types and expressions (ORBmatcher.cc:1228-1239)
    const Matrix3f Rcw = CurrentFrame.mTcw.rotationMatrix();
    const Vector3f tcw = CurrentFrame.mTcw.translation();
    const Vector3f twc = -1 * Rcw.transpose() * tcw;
    const Matrix3f Rlw = LastFrame.mTcw.rotationMatrix();
    const Vector3f tlw = LastFrame.mTcw.translation();
    const Vector3f tlc = Rlw * twc + tlw;
    const bool bForward = tlc[2] > CurrentFrame.mb && !bMono;
    const bool bBackward = -tlc[2] > CurrentFrame.mb && !bMono;
    std::vector<ygzfe_match_query> q;
    std::vector<uint8_t> qd;
    std::vector<int> src;  // LastFrame index of each query
    for (int i = 0; i < LastFrame.N; i++) {
        auto *pMP = LastFrame.mvpMapPoints[i];
        if (!pMP || LastFrame.mvbOutlier[i]) continue;
        const Vector3f x3Dw = pMP->GetWorldPos();
        const Vector3f x3Dc = Rcw * x3Dw + tcw;
        const float xc = x3Dc[0];
        const float yc = x3Dc[1];
        const float invzc = 1.0 / x3Dc[2];
        if (invzc < 0) continue;
        const float u = CurrentFrame.fx * xc * invzc + CurrentFrame.cx;
        const float v = CurrentFrame.fy * yc * invzc + CurrentFrame.cy;
        if (u < CurrentFrame.mnMinX || u > CurrentFrame.mnMaxX) continue;
        if (v < CurrentFrame.mnMinY || v > CurrentFrame.mnMaxY) continue;
        const int nLastOctave = LastFrame.mvKeys[i].octave;
        const float radius = th * CurrentFrame.mvScaleFactors[nLastOctave];
        ygzfe_match_query Q;
        Q.u = u;
        Q.v = v;
        Q.radius = radius;
        Q.u_right = u - CurrentFrame.mbf * invzc;
        if (checkLevel == false) {
            Q.min_level = -1;
            Q.max_level = -1;
        } else if (bForward) {
            Q.min_level = nLastOctave;
            Q.max_level = -1;
        } else if (bBackward) {
            Q.min_level = 0;
            Q.max_level = nLastOctave;
        } else {
            Q.min_level = nLastOctave - 1;
            Q.max_level = nLastOctave + 1;
        }
        Q.angle = LastFrame.mvKeys[i].angle;
        Q.flags = YGZFE_MQ_VALID | YGZFE_MQ_STEREO | (pMP->Observations() > 0 ? YGZFE_MQ_BLOCKS : 0);
        q.push_back(Q);
        append_desc(qd, pMP->GetDescriptor());
        src.push_back(i);
    }
    std::vector<uint8_t> blocked((size_t)CurrentFrame.N, 0);
    for (int i = 0; i < CurrentFrame.N; i++)
        blocked[i] = CurrentFrame.mvpMapPoints[i] && CurrentFrame.mvpMapPoints[i]->Observations() > 0;
    MatchView &mv = view(0);
    if (!set_frame(mv, CurrentFrame, true)) return 0;
    std::vector<int32_t> out((size_t)CurrentFrame.N + 1);
    int nmatches = 0;
    if (ygzfe_search_projection_best(mv.get(), q.data(), qd.data(), (int)q.size(), blocked.data(), kTH_HIGH,
                                     checkOri ? 1 : 0, out.data(), &nmatches) != YGZFE_OK)
        return failed("SearchByProjection(CurrentFrame, LastFrame)");
    for (int i2 = 0; i2 < CurrentFrame.N; i2++) {
        if (out[i2] >= 0) CurrentFrame.mvpMapPoints[i2] = LastFrame.mvpMapPoints[src[out[i2]]];
        else if (out[i2] == -2) CurrentFrame.mvpMapPoints[i2] = nullptr;
    }
    return nmatches;
}

// SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (ORBmatcher.cc:1352-1469)
template <class FrameT, class KeyFrameT, class MapPointT>
int SearchByProjection(FrameT &CurrentFrame, KeyFrameT *pKF, const std::set<MapPointT *> &sAlreadyFound,
                       const float th, const int ORBdist, bool checkOri) {
    const Matrix3f Rcw = CurrentFrame.mTcw.rotationMatrix();  // ORBmatcher.cc:1356-1358
    const Vector3f tcw = CurrentFrame.mTcw.translation();
    const Vector3f Ow = -1 * Rcw.transpose() * tcw;
    const std::vector<MapPointT *> vpMPs = pKF->GetMapPointMatches();
    std::vector<ygzfe_match_query> q;
    std::vector<uint8_t> qd;
    std::vector<size_t> src;
    for (size_t i = 0, iend = vpMPs.size(); i < iend; i++) {
        MapPointT *pMP = vpMPs[i];
        if (!pMP || pMP->isBad() || sAlreadyFound.count(pMP)) continue;
        const Vector3f x3Dw = pMP->GetWorldPos();
        const Vector3f x3Dc = Rcw * x3Dw + tcw;
        const float xc = x3Dc[0];
        const float yc = x3Dc[1];
        const float invzc = 1.0 / x3Dc[2];
        const float u = CurrentFrame.fx * xc * invzc + CurrentFrame.cx;
        const float v = CurrentFrame.fy * yc * invzc + CurrentFrame.cy;
        if (u < CurrentFrame.mnMinX || u > CurrentFrame.mnMaxX) continue;
        if (v < CurrentFrame.mnMinY || v > CurrentFrame.mnMaxY) continue;
        const Vector3f PO = x3Dw - Ow;
        const float dist3D = PO.norm();
        const float maxDistance = pMP->GetMaxDistanceInvariance();
        const float minDistance = pMP->GetMinDistanceInvariance();
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int nPredictedLevel = pMP->PredictScale(dist3D, &CurrentFrame);
        ygzfe_match_query Q;
        Q.u = u;
        Q.v = v;
        Q.radius = th * CurrentFrame.mvScaleFactors[nPredictedLevel];
        Q.u_right = 0.f;
        Q.min_level = nPredictedLevel - 1;
        Q.max_level = nPredictedLevel + 1;
        Q.angle = pKF->mvKeys[i].angle;
        Q.flags = YGZFE_MQ_VALID | YGZFE_MQ_BLOCKS;  // any assigned MapPoint makes the keypoint skipped (:1418-1419)
        q.push_back(Q);
        append_desc(qd, pMP->GetDescriptor());
        src.push_back(i);
    }
    std::vector<uint8_t> blocked((size_t)CurrentFrame.N, 0);
    for (int i = 0; i < CurrentFrame.N; i++) blocked[i] = CurrentFrame.mvpMapPoints[i] != nullptr;
    MatchView &mv = view(0);
    if (!set_frame(mv, CurrentFrame, false)) return 0;
    std::vector<int32_t> out((size_t)CurrentFrame.N + 1);
    int nmatches = 0;
    if (ygzfe_search_projection_best(mv.get(), q.data(), qd.data(), (int)q.size(), blocked.data(), ORBdist,
                                     checkOri ? 1 : 0, out.data(), &nmatches) != YGZFE_OK)
        return failed("SearchByProjection(CurrentFrame, pKF, sAlreadyFound)");
    for (int i2 = 0; i2 < CurrentFrame.N; i2++) {
        if (out[i2] >= 0) CurrentFrame.mvpMapPoints[i2] = vpMPs[src[out[i2]]];
        else if (out[i2] == -2) CurrentFrame.mvpMapPoints[i2] = nullptr;
    }
    return nmatches;
}

// SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (ORBmatcher.cc:375-478)
template <class FrameT, class Point2fT>
int SearchForInitialization(FrameT &F1, FrameT &F2, std::vector<Point2fT> &vbPrevMatched,
                            std::vector<int> &vnMatches12, int windowSize, float nnratio, bool checkOri) {
    const int n1 = (int)F1.mvKeys.size(), n2 = (int)F2.mvKeys.size();
    vnMatches12 = std::vector<int>(n1, -1);
    MatchView &a = view(0), &b = view(1);
    if (!a.set(F1.mvKeys, F1.mDescriptors, n1, nullptr, bounds_of<FrameT>()) ||
        !b.set(F2.mvKeys, F2.mDescriptors, n2, nullptr, bounds_of<FrameT>()))
        return 0;
    std::vector<float> prev(2 * (size_t)n1 + 2);
    for (int i = 0; i < n1; i++) {
        prev[2 * i] = vbPrevMatched[i].x;
        prev[2 * i + 1] = vbPrevMatched[i].y;
    }
    int nmatches = 0;
    if (ygzfe_search_for_initialization(a.get(), b.get(), prev.data(), windowSize, nnratio, checkOri ? 1 : 0,
                                        vnMatches12.data(), &nmatches) != YGZFE_OK) {
        vnMatches12.assign(n1, -1);
        return failed("SearchForInitialization");
    }
    for (int i = 0; i < n1; i++)
        if (vnMatches12[i] >= 0) vbPrevMatched[i] = F2.mvKeys[vnMatches12[i]].pt;
    return nmatches;
}

// SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.cc:155-263)
template <class KeyFrameT, class FrameT, class MapPointT>
int SearchByBoW(KeyFrameT *pKF, FrameT &F, std::vector<MapPointT *> &vpMapPointMatches, float nnratio,
                bool checkOri) {
    const std::vector<MapPointT *> vpMapPointsKF = pKF->GetMapPointMatches();
    vpMapPointMatches = std::vector<MapPointT *>(F.N, static_cast<MapPointT *>(NULL));
    const int nkf = (int)pKF->mvKeys.size();
    std::vector<uint8_t> usable((size_t)nkf + 1, 0);
    for (int i = 0; i < nkf && i < (int)vpMapPointsKF.size(); i++)
        usable[i] = vpMapPointsKF[i] && !vpMapPointsKF[i]->isBad();
    // FeatureVectors (std::map<NodeId, std::vector<unsigned>>) as node-sorted CSR
    auto csr = [](const decltype(F.mFeatVec) &fv, std::vector<int32_t> &nodes, std::vector<int32_t> &ptr,
                  std::vector<int32_t> &feats) {
        ptr.push_back(0);
        for (auto it = fv.begin(); it != fv.end(); ++it) {
            nodes.push_back((int32_t)it->first);
            for (size_t k = 0; k < it->second.size(); k++) feats.push_back((int32_t)it->second[k]);
            ptr.push_back((int32_t)feats.size());
        }
    };
    std::vector<int32_t> kn, kp, kfe, fn, fp, ffe;
    csr(pKF->mFeatVec, kn, kp, kfe);
    csr(F.mFeatVec, fn, fp, ffe);
    MatchView &a = view(0), &b = view(1);
    if (!a.set(pKF->mvKeys, pKF->mDescriptors, nkf, nullptr, bounds_of<FrameT>()) ||
        !b.set(F.mvKeys, F.mDescriptors, F.N, nullptr, bounds_of<FrameT>()))
        return 0;
    std::vector<int32_t> out((size_t)F.N + 1);
    int nmatches = 0;
    if (ygzfe_search_by_bow(a.get(), b.get(), usable.data(), (int)kn.size(), kn.data(), kp.data(), kfe.data(),
                            (int)fn.size(), fn.data(), fp.data(), ffe.data(), nnratio, checkOri ? 1 : 0, out.data(),
                            &nmatches) != YGZFE_OK)
        return failed("SearchByBoW");
    for (int i = 0; i < F.N; i++)
        if (out[i] >= 0) vpMapPointMatches[i] = vpMapPointsKF[out[i]];
    return nmatches;
}

}  // namespace gpu
}  // namespace ygz

#endif
