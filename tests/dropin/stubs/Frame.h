// Test stub of the reference's Frame (Frame.h): the members the hot-path call
// sites read, Frame::ExtractORB with its call sites verbatim (Frame.cc:332-348),
// and ComputeImagePyramid / ComputeStereoMatches / ComputeStereoFromRGBD /
// ComputeBoW with the drop-in bodies (compat/dropin/Frame_gpu.inc), as Frame.cc
// would include them.  Written for the test; the drop-in ORBextractor.h comes
// first on the include path, as it would in the reference build.
#pragma once
#include "Common.h"
#include "FrameGPU.h"
#include "ORBextractor.h"

namespace ygz {
class MapPoint;

#define FRAME_GRID_ROWS 48
#define FRAME_GRID_COLS 64

class Frame {
public:
    typedef enum { Monocular = 0, Stereo, RGBD } SensorType;  // Frame.h:38-41
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

    // the stereo / RGB-D constructors' parts that reach the §8f rows (Frame.cc:181-236):
    // members set, then ComputeImagePyramid (undistortion of every image included)
    Frame(const cv::Mat &imLeft, const cv::Mat &imRight, const cv::Mat &imDepth, SensorType sensor,
          ORBextractor *extractorLeft, ORBextractor *extractorRight, ORBVocabulary *voc, const Eigen::Matrix3f &K,
          const cv::Mat &distCoef, float bf)
        : mbf(bf), mpORBvocabulary(voc), mK(K), mDistCoef(distCoef.clone()), mSensor(sensor),
          mImDepth(imDepth.clone()), mpORBextractorLeft(extractorLeft), mpORBextractorRight(extractorRight),
          mImGray(imLeft.clone()), mImRight(imRight.clone()) {
        mnId = nNextId++;
        mb = mbf / K(0, 0);
        mnScaleLevels = mpORBextractorLeft->GetLevels();
        mvScaleFactors = mpORBextractorLeft->GetScaleFactors();
        mvInvScaleFactors = mpORBextractorLeft->GetInverseScaleFactors();
        ComputeImagePyramid();
    }

    // Frame.cc:156-189 for the members this stub has (deep copies of the images and
    // descriptors, mbFeatureExtracted false), the pyramid copy of :186-188 through the
    // drop-in (gpu::CopyImagePyramid: the one-line edit INTEGRATION.md §1 lists)
    Frame(const Frame &frame)
        : mbf(frame.mbf), mb(frame.mb), N(frame.N), mvKeys(frame.mvKeys), mvKeysRight(frame.mvKeysRight),
          mvuRight(frame.mvuRight), mvDepth(frame.mvDepth), mDescriptors(frame.mDescriptors.clone()),
          mDescriptorsRight(frame.mDescriptorsRight.clone()), mvpMapPoints(frame.mvpMapPoints),
          mvbOutlier(frame.mvbOutlier), mvMatchedFrom(frame.mvMatchedFrom), mFeatVec(frame.mFeatVec),
          mBowVec(frame.mBowVec), mpORBvocabulary(frame.mpORBvocabulary), mK(frame.mK),
          mDistCoef(frame.mDistCoef.clone()), mSensor(frame.mSensor), mImDepth(frame.mImDepth.clone()),
          mTcw(frame.mTcw), mnScaleLevels(frame.mnScaleLevels), mvScaleFactors(frame.mvScaleFactors),
          mvInvScaleFactors(frame.mvInvScaleFactors), mvLevelSigma2(frame.mvLevelSigma2),
          mvInvLevelSigma2(frame.mvInvLevelSigma2), mpORBextractorLeft(frame.mpORBextractorLeft),
          mpORBextractorRight(frame.mpORBextractorRight), mImGray(frame.mImGray.clone()),
          mImRight(frame.mImRight.clone()), mbFeatureExtracted(false), mnId(frame.mnId) {
        gpu::CopyImagePyramid(mvImagePyramid, frame.mvImagePyramid);
    }
    Frame &operator=(const Frame &) = default;  // the reference's implicit member-wise assignment

    void ExtractORB(int flag, const cv::Mat &im);
    void ComputeImagePyramid();
    void ComputeStereoMatches();
    void ComputeStereoFromRGBD(const cv::Mat &imDepth);
    void ComputeBoW();
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
    DBoW2::BowVector mBowVec;
    ORBVocabulary *mpORBvocabulary = nullptr;
    Eigen::Matrix3f mK;
    cv::Mat mDistCoef;
    static bool mbNeedUndistort;
    SensorType mSensor = Monocular;
    cv::Mat mImDepth;
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

// Frame.cc:495-500, 509-700, 773-813: the drop-in bodies
#include "Frame_gpu.inc"
}  // namespace ygz
