// Test stub of the reference's KeyFrame: the members SearchByBoW / the
// relocalisation search read.  Written for the test.
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
    std::vector<MapPoint *> GetMapPointMatches() { return mvpMapPoints; }
};
}  // namespace ygz
