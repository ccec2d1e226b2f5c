// Test stub of the reference's KeyFrame: the members SearchByBoW / the
// relocalisation search / the direct local-map search read.  Written for the test.
#pragma once
#include "Common.h"

namespace ygz {
class MapPoint;
class KeyFrame {
public:
    std::vector<cv::KeyPoint> mvKeys;
    cv::Mat mDescriptors;
    DBoW2::FeatureVector mFeatVec;
    std::vector<MapPoint *> mvpMapPoints;
    std::vector<cv::Mat> mvImagePyramid;  // shared with the Frame it was made from (KeyFrame.cc:257-260)
    std::vector<float> mvScaleFactors;
    SE3f mTcw;
    long unsigned int mnId = 0;
    bool mbBad = false;
    std::vector<MapPoint *> GetMapPointMatches() { return mvpMapPoints; }
    SE3f GetPose() { return mTcw; }
    bool isBad() { return mbBad; }
};
}  // namespace ygz
