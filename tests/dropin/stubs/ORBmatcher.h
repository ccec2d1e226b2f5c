// Test stub of the reference's ORBmatcher.h: the constructor, the members and
// the declarations of the five tracking-path searches and FindDirectProjection with the reference's
// signatures (ORBmatcher.h:38-142).  Written for the test.
#pragma once
#include "Common.h"
#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"

namespace ygz {
class ORBmatcher {
public:
    ORBmatcher(float nnratio = 0.6, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}
    int SearchByProjection(Frame &F, const std::vector<MapPoint *> &vpMapPoints, const float th = 3,
                           bool checkLevel = true);
    int SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, const float th, const bool bMono,
                           bool checkLevel = true);
    int SearchByProjection(Frame &CurrentFrame, KeyFrame *pKF, const std::set<MapPoint *> &sAlreadyFound,
                           const float th, const int ORBdist);
    int SearchByBoW(KeyFrame *pKF, Frame &F, std::vector<MapPoint *> &vpMapPointMatches);
    int SearchForInitialization(Frame &F1, Frame &F2, std::vector<cv::Point2f> &vbPrevMatched,
                                std::vector<int> &vnMatches12, int windowSize = 10);
    bool FindDirectProjection(KeyFrame *ref, Frame *curr, MapPoint *mp, Vector2f &px_curr, int &search_level);
    static const int TH_LOW;
    static const int TH_HIGH;
    static const int HISTO_LENGTH;

private:
    float mfNNratio;
    bool mbCheckOrientation;
};
}  // namespace ygz
