// Test stub of the reference's Frame (Frame.h): the members the hot-path call
// sites read, and the two member functions whose bodies hold the call sites
// verbatim (Frame::ExtractORB Frame.cc:332-348, Frame::ComputeImagePyramid
// Frame.cc:807-813).  Written for the test; the drop-in ORBextractor.h comes
// first on the include path, as it would in the reference build.
#pragma once
#include "Common.h"
#include "ORBextractor.h"

namespace ygz {
class MapPoint;

#define FRAME_GRID_ROWS 48
#define FRAME_GRID_COLS 64

class Frame {
public:
    Frame() {}
    Frame(const cv::Mat &imGray, ORBextractor *extractor) : mpORBextractorLeft(extractor), mImGray(imGray.clone()) {
        mnId = nNextId++;
        mnScaleLevels = mpORBextractorLeft->GetLevels();
        mvScaleFactors = mpORBextractorLeft->GetScaleFactors();
        mvInvScaleFactors = mpORBextractorLeft->GetInverseScaleFactors();
        mvLevelSigma2 = mpORBextractorLeft->GetScaleSigmaSquares();
        mvInvLevelSigma2 = mpORBextractorLeft->GetInverseScaleSigmaSquares();
        mnMinX = 0.0f;
        mnMaxX = imGray.cols;
        mnMinY = 0.0f;
        mnMaxY = imGray.rows;
        ComputeImagePyramid();
    }

    void ExtractORB(int flag, const cv::Mat &im);
    void ComputeImagePyramid();
    void ExtractFeatures() {  // the parts of Frame.cc:717-771 the searches depend on
        ExtractORB(0, mImGray);
        N = mvKeys.size();
        mvuRight = std::vector<float>(N, -1);
        mvDepth = std::vector<float>(N, -1);
        mvpMapPoints.resize(N, nullptr);
        mvbOutlier.resize(N, false);
        mbFeatureExtracted = true;
    }
    void SetPose(const SE3f &Tcw) { mTcw = Tcw; }
    bool isInFrustum(MapPoint *pMP, float viewingCosLimit);  // defined in the MapPoint.h stub

    static float fx, fy, cx, cy, invfx, invfy;
    static float mnMinX, mnMaxX, mnMinY, mnMaxY;
    float mbf = 0.f, mb = 0.f;
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysRight;
    std::vector<float> mvuRight, mvDepth;
    cv::Mat mDescriptors, mDescriptorsRight;
    std::vector<MapPoint *> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    std::vector<int> mvMatchedFrom;
    DBoW2::FeatureVector mFeatVec;
    SE3f mTcw;
    std::vector<cv::Mat> mvImagePyramid;
    int mnScaleLevels = 0;
    std::vector<float> mvScaleFactors, mvInvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
    ORBextractor *mpORBextractorLeft = nullptr, *mpORBextractorRight = nullptr;
    cv::Mat mImGray, mImRight;
    bool mbFeatureExtracted = false;
    long unsigned int mnId = 0;
    static long unsigned int nNextId;
};

// Frame.cc:332-348, the call lines verbatim
inline void Frame::ExtractORB(int flag, const cv::Mat &im) {
    (void)im;
        if (flag == 0) {
            if (N > 0 && mbFeatureExtracted == false)
            {
                (*mpORBextractorLeft)(this, mvKeys, mDescriptors, ORBextractor::DSO_KEYPOINT);
            } else {
                (*mpORBextractorLeft)( this,mvKeys,mDescriptors,ORBextractor::ORBSLAM_KEYPOINT );
            }
        } else {
            (*mpORBextractorRight)(this, mvKeysRight, mDescriptorsRight, ORBextractor::ORBSLAM_KEYPOINT, false);
        }
}

// Frame.cc:807-813 verbatim (the undistortion before it is out of this test)
inline void Frame::ComputeImagePyramid() {
        mpORBextractorLeft->ComputePyramid(mImGray);

        mvImagePyramid.resize(mpORBextractorLeft->GetLevels());
        for (int l = 0; l < mpORBextractorLeft->GetLevels(); l++) {
            mvImagePyramid[l] = mpORBextractorLeft->mvImagePyramid[l].clone();
        }
}
}  // namespace ygz
