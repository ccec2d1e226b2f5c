// Test stub of the reference's MapPoint (MapPoint.h): only the members the
// tracking-path call sites read.  Written for the test.
#pragma once
#include "Common.h"

namespace ygz {
class Frame;
class MapPoint {
public:
    Vector3f mWorldPos;
    cv::Mat mDescriptor;
    int nObs = 1;
    bool mbBad = false;
    bool mbTrackInView = false;
    int mnTrackScaleLevel = 0;
    float mTrackViewCos = 1.f, mTrackProjX = 0.f, mTrackProjY = 0.f, mTrackProjXR = 0.f;
    float mfMaxDistance = 1e9f, mfMinDistance = 0.f;
    int mnPredictedLevel = 0;
    Vector3f GetWorldPos() { return mWorldPos; }
    bool isBad() { return mbBad; }
    int Observations() { return nObs; }
    cv::Mat GetDescriptor() { return mDescriptor.clone(); }
    float GetMaxDistanceInvariance() { return 1.2f * mfMaxDistance; }
    float GetMinDistanceInvariance() { return 0.8f * mfMinDistance; }
    int PredictScale(const float &, Frame *) { return mnPredictedLevel; }
};
}  // namespace ygz
