// Test stub of the reference's MapPoint (MapPoint.h): only the members the
// tracking-path call sites read.  Written for the test.
#pragma once
#include "Common.h"
#include "Frame.h"

namespace ygz {
class KeyFrame;
class MapPoint {
public:
    Vector3f mWorldPos;
    Vector3f mNormalVector{0.f, 0.f, 1.f};
    cv::Mat mDescriptor;
    int nObs = 1;
    bool mbBad = false;
    bool mbTrackInView = false;
    int mnTrackScaleLevel = 0;
    float mTrackViewCos = 1.f, mTrackProjX = 0.f, mTrackProjY = 0.f, mTrackProjXR = 0.f;
    float mfMaxDistance = 1e9f, mfMinDistance = 0.f;
    int mnPredictedLevel = 0;
    std::map<KeyFrame *, size_t> mObservations;
    Vector3f GetWorldPos() { return mWorldPos; }
    Vector3f GetNormal() { return mNormalVector; }
    bool isBad() { return mbBad; }
    int Observations() { return nObs; }
    std::map<KeyFrame *, size_t> GetObservations() { return mObservations; }
    cv::Mat GetDescriptor() { return mDescriptor.clone(); }
    float GetMaxDistanceInvariance() { return 1.2f * mfMaxDistance; }
    float GetMinDistanceInvariance() { return 0.8f * mfMinDistance; }
    int PredictScale(const float &, Frame *) { return mnPredictedLevel; }
};

// Frame::isInFrustum (Frame.cc:363-422), written for the test over the stub's pose
inline bool Frame::isInFrustum(MapPoint *pMP, float viewingCosLimit) {
    pMP->mbTrackInView = false;
    const Vector3f P = pMP->GetWorldPos();
    const Vector3f Pc = mTcw * P;
    if (Pc[2] < 0.0f) return false;
    const float invz = 1.0f / Pc[2];
    const float u = fx * Pc[0] * invz + cx;
    const float v = fy * Pc[1] * invz + cy;
    if (u < mnMinX || u > mnMaxX) return false;
    if (v < mnMinY || v > mnMaxY) return false;
    const Vector3f Ow = mTcw.inverse().translation();
    const Vector3f PO = P - Ow;
    const float dist = PO.norm();
    if (dist < pMP->GetMinDistanceInvariance() || dist > pMP->GetMaxDistanceInvariance()) return false;
    const Vector3f Pn = pMP->GetNormal();
    const float viewCos = (PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2]) / dist;
    if (viewCos < viewingCosLimit) return false;
    pMP->mbTrackInView = true;
    pMP->mTrackProjX = u;
    pMP->mTrackProjXR = u - mbf * invz;
    pMP->mTrackProjY = v;
    pMP->mnTrackScaleLevel = pMP->PredictScale(dist, this);
    pMP->mTrackViewCos = viewCos;
    return true;
}
}  // namespace ygz
