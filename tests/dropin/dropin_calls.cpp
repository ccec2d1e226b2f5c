// dropin_calls.cpp — the reference's hot-path call sites, verbatim, compiled
// against the drop-in headers (compat/dropin/) and the test stubs of Frame /
// MapPoint / KeyFrame / ORBmatcher (tests/dropin/stubs/), built -std=c++11 like
// the reference, then run on the GPU and checked against the CPU oracle
// (oracle/ygz_oracle.h; TEST INFRASTRUCTURE):
//
//   Tracking.cc:255   mpORBextractorLeft = new ORBextractor(nFeatures, fScaleFactor, nLevels, ...)
//   Tracking.cc:284   mpAlign = new ygz::SparseImgAlign(nLevels - 1, 1);
//   Frame.cc:807-813  ComputeImagePyramid (stub Frame.h)
//   Frame.cc:337/340  (*mpORBextractorLeft)(this, mvKeys, mDescriptors, ORBextractor::...)   (stub Frame.h)
//   Tracking.cc:2170-2171  SE3f TCR; size_t ret = mpAlign->run(&mLastFrame, &mCurrentFrame, TCR);
//   Tracking.cc:825-826    matcher.SearchForInitialization(mInitialFrame, mCurrentFrame, ...)
//   Tracking.cc:1156,1171  matcher.SearchByProjection(mCurrentFrame, mLastFrame, th, mSensor == System::MONOCULAR)
//   Tracking.cc:1662,1674  matcher.SearchByProjection(mCurrentFrame, mvpLocalMapPoints, th, false)
//   Tracking.cc:1018-1020  matcher.SearchByBoW(mpReferenceKF, mCurrentFrame, vpMapPointMatches)
//   ORBmatcher.cc:1598-1599 ygz::Align2D(curr->mvImagePyramid[search_level], _patch_with_border, ...)
//   Tracking.cc:2201        SearchLocalPointsDirect();   (body: compat/dropin/Tracking_direct_gpu.inc)
//   Tracking.cc:2294        matcher.FindDirectProjection(o.first, &mCurrentFrame, mp, px_curr, level)
//
// Prints one line per check; exit 0 and "OK" when every check passes.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "Align.h"
#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"
#include "ORBmatcher.h"
#include "ORBmatcherGPU.h"
#include "SparseImageAlign.h"
#include "TrackingDirectGPU.h"
#include "ygz_oracle.h"

namespace ygz {
#include "ORBmatcher_gpu.inc"

const int ORBmatcher::TH_HIGH = 100;
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;
float Frame::fx, Frame::fy, Frame::cx, Frame::cy, Frame::invfx, Frame::invfy;
float Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY;
long unsigned int Frame::nNextId = 0;
bool Frame::mbNeedUndistort = false;

struct System {
    enum eSensor { MONOCULAR = 0, STEREO = 1, RGBD = 2 };
};

// the Tracking members the call sites use, with those call sites verbatim
struct Tracking {
    ORBextractor *mpORBextractorLeft = nullptr;
    SparseImgAlign *mpAlign = nullptr;
    Frame mCurrentFrame, mLastFrame, mInitialFrame;
    std::vector<cv::Point2f> mvbPrevMatched;
    std::vector<int> mvIniMatches;
    std::vector<MapPoint *> mvpLocalMapPoints;
    KeyFrame *mpReferenceKF = nullptr;
    int mSensor = System::MONOCULAR;
    // SearchLocalPointsDirect state (Tracking.h:245-248, 282)
    set<MapPoint *> mvpDirectMapPointsCache;
    int mnCacheHitTh = 150;
    KeyFrame *mpLastKeyFrame = nullptr;
    std::vector<MapPoint *> mvpNextLocalMapPoints;  // what the UpdateLocalMap stub installs
    int nUpdateLocalMap = 0;
    void UpdateLocalMap() {
        mvpLocalMapPoints = mvpNextLocalMapPoints;
        nUpdateLocalMap++;
    }
    void SearchLocalPointsDirect();
    void TrackLocalMapDirect() {  // Tracking.cc:2191-2201, the call line verbatim
        SearchLocalPointsDirect();
    }
    // Tracking.cc:2412-2432 verbatim
    vector<std::pair<KeyFrame *, size_t> >
    SelectNearestKeyframe(const std::map<KeyFrame *, size_t> &observations, int n) {
        vector<std::pair<KeyFrame *, size_t> > s;
        for (auto &o: observations) {
            if (!o.first->isBad() && o.first != mpLastKeyFrame)
                s.push_back(make_pair(o.first, o.second));
        }
        sort(s.begin(), s.end(),
             [](const pair<KeyFrame *, size_t> &p1, const pair<KeyFrame *, size_t> &p2) {
                 return p1.first->mnId > p2.first->mnId;
             });

        if ((int) s.size() < n)
            return s;
        else
            return vector<std::pair<KeyFrame *, size_t> >(s.begin(), s.begin() + n);
    }

    Tracking(int nFeatures, float fScaleFactor, int nLevels, int fIniThFAST, int fMinThFAST) {
        mpORBextractorLeft = new ORBextractor(nFeatures, fScaleFactor, nLevels, fIniThFAST, fMinThFAST);
        mpAlign = new ygz::SparseImgAlign(nLevels - 1, 1);
    }
    ~Tracking() {
        delete mpAlign;
        delete mpORBextractorLeft;
    }
    size_t SparseAlign(SE3f &out) {
        SE3f TCR;
        size_t ret = mpAlign->run(&mLastFrame, &mCurrentFrame, TCR);
        out = TCR;
        return ret;
    }
    int Initialization() {
        ORBmatcher matcher(0.9, true);
        int nmatches = matcher.SearchForInitialization(mInitialFrame, mCurrentFrame, mvbPrevMatched, mvIniMatches,
                                                       100);
        return nmatches;
    }
    int MotionModel(int th) {
        ORBmatcher matcher(0.9, true);
        int nmatches = matcher.SearchByProjection(mCurrentFrame, mLastFrame, th, mSensor == System::MONOCULAR);
        return nmatches;
    }
    int LocalPoints(float th) {
        ORBmatcher matcher(0.8);
        int cnt = matcher.SearchByProjection(mCurrentFrame, mvpLocalMapPoints, th, false );
        return cnt;
    }
    int ReferenceKF(std::vector<MapPoint *> &vpMapPointMatches) {
        ORBmatcher matcher(0.7, false);
        int nmatches = matcher.SearchByBoW(mpReferenceKF, mCurrentFrame, vpMapPointMatches);
        return nmatches;
    }
};
#include "Tracking_direct_gpu.inc"
}  // namespace ygz

using namespace ygz;

static int fails = 0;
#define CHECK(cond, ...)                       \
    do {                                       \
        std::printf(__VA_ARGS__);              \
        std::printf(" %s\n", (cond) ? "ok" : "FAILED"); \
        if (!(cond)) fails++;                  \
    } while (0)

static cv::Mat synth(int W, int H, unsigned seed, int dx, int dy) {
    cv::Mat img(H, W, CV_8U);
    std::memset(img.data, 128, (size_t)W * H);
    unsigned s = seed;
    auto rnd = [&](int n) { s = s * 1664525u + 1013904223u; return (int)((s >> 8) % (unsigned)n); };
    for (int r = 0; r < 900; r++) {
        const int x0 = rnd(W + 40) - 20, y0 = rnd(H + 40) - 20, w = 4 + rnd(40), h = 4 + rnd(40), v = rnd(256);
        for (int y = y0; y < y0 + h; y++)
            for (int x = x0; x < x0 + w; x++) {
                const int xx = x + dx, yy = y + dy;
                if (xx >= 0 && yy >= 0 && xx < W && yy < H) img.data[(size_t)yy * W + xx] = (uint8_t)v;
            }
    }
    for (int i = 0; i < W * H; i++) {  // +-1 noise so no two frames are identical
        const int v = img.data[i] + (int)(((uint32_t)(i + seed) * 2654435761u) >> 30) - 1;
        img.data[i] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
    return img;
}

// median wall time (ms) of `reps` calls of fn(): the drop-in path as a Tracking thread sees
// it (bench.py's dropin leg reads the TIMING lines)
template <class Fn>
static double median_ms(int reps, Fn fn) {
    std::vector<double> t;
    for (int i = 0; i < reps; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        fn();
        t.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}
static bool g_timing = false;

static ygzo_mframe mframe(const Frame &F, bool uright) {
    ygzo_mframe f;
    f.kps = reinterpret_cast<const ygzo_kp *>(F.mvKeys.data());
    f.desc = F.mDescriptors.data;
    f.u_right = uright ? F.mvuRight.data() : nullptr;
    f.n = F.N;
    f.min_x = Frame::mnMinX;
    f.max_x = Frame::mnMaxX;
    f.min_y = Frame::mnMinY;
    f.max_y = Frame::mnMaxY;
    return f;
}

// Frame.cc:495-500, 509-700, 773-813 through the drop-in bodies (compat/dropin/Frame_gpu.inc),
// each against the oracle: the TUM1 (C4) RGB-D frame undistorted (gray + CV_32F depth), its
// depths; a rectified EuRoC stereo pair's ComputeStereoMatches; ComputeBoW on a vocabulary
// bound with gpu::BindVocabulary.
static void frame_rows() {
    // TUM1.yaml:8-17 (C4): K, k1 k2 p1 p2 k3 -> Frame::mbNeedUndistort (Tracking.cc:171-204)
    const int W = 640, H = 480, nl = 8;
    Eigen::Matrix3f K;
    K(0, 0) = 517.306408f;
    K(1, 1) = 516.469215f;
    K(0, 2) = 318.643040f;
    K(1, 2) = 255.313989f;
    K(2, 2) = 1.f;
    cv::Mat D(5, 1, CV_32F);
    const float dist[5] = {0.262383f, -0.953104f, -0.005358f, 0.002628f, 1.163314f};
    std::memcpy(D.data, dist, sizeof(dist));
    const float cam4[4] = {K(0, 0), K(1, 1), K(0, 2), K(1, 2)};
    std::vector<int16_t> m1((size_t)2 * W * H);
    std::vector<uint16_t> m2((size_t)W * H);
    ygzo_undistort_map(cam4, dist, 5, W, H, m1.data(), m2.data());
    const cv::Mat gray = synth(W, H, 11u, 0, 0);
    cv::Mat depth(H, W, CV_32F);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {  // TUM-like: uint16 / 5000, holes
            const unsigned h = (((unsigned)x * 73856093u) ^ ((unsigned)y * 19349663u)) % 97u;
            const int raw = h < 5 ? 0 : (int)(5000.f * (0.8f + 0.002f * x + 0.003f * y + 0.25f * ((x / 97 + y / 71) % 3)));
            depth.ptr<float>(y)[x] = (float)raw * (1.0f / 5000);
        }
    ORBextractor ex4(2000, 1.2f, nl, 20, 7);  // TUM1.yaml (C4)
    const bool saved = Frame::mbNeedUndistort;
    Frame::mbNeedUndistort = true;
    Frame F(gray, cv::Mat(), depth, Frame::RGBD, &ex4, nullptr, nullptr, K, D, 40.0f);
    {
        std::vector<uint8_t> ug((size_t)W * H);
        ygzo_remap_linear(gray.data, W, H, W, m1.data(), m2.data(), W, H, ug.data(), W);
        std::vector<float> ud((size_t)W * H);
        ygzo_remap_linear_f32(depth.ptr<float>(0), W, H, W, m1.data(), m2.data(), W, H, ud.data(), W);
        const bool g_ok = F.mImGray.cols == W && std::memcmp(F.mImGray.data, ug.data(), ug.size()) == 0;
        const bool d_ok = F.mImDepth.cols == W && std::memcmp(F.mImDepth.data, ud.data(), ud.size() * 4) == 0;
        ygzo_orb o4;
        ygzo_orb_init(&o4, 2000, 1.2f, nl, 20, 7, 0);
        int lw[YGZO_MAX_LEVELS], lh[YGZO_MAX_LEVELS];
        ygzo_level_sizes(&o4, W, H, lw, lh);
        std::vector<std::vector<uint8_t>> lv(nl);
        uint8_t *lp[YGZO_MAX_LEVELS];
        for (int l = 0; l < nl; l++) {
            lv[l].resize((size_t)lw[l] * lh[l]);
            lp[l] = lv[l].data();
        }
        ygzo_compute_pyramid(&o4, ug.data(), W, H, W, lp);
        bool p_ok = (int)F.mvImagePyramid.size() == nl;
        for (int l = 0; l < nl && p_ok; l++)
            p_ok = std::memcmp(F.mvImagePyramid[l].data, lp[l], lv[l].size()) == 0;
        CHECK(g_ok && d_ok && p_ok, "Frame::ComputeImagePyramid (RGB-D, TUM1 distortion): remap(mImGray) %s, "
              "remap(mImDepth) CV_32F %s, pyramid %s == oracle", g_ok ? "ok" : "differs", d_ok ? "ok" : "differs",
              p_ok ? "ok" : "differs");
        if (g_timing) {
            const double gm = median_ms(20, [&] {
                Frame Fx(gray, cv::Mat(), depth, Frame::RGBD, &ex4, nullptr, nullptr, K, D, 40.0f);
            });
            const double cm = median_ms(5, [&] {
                ygzo_remap_linear(gray.data, W, H, W, m1.data(), m2.data(), W, H, ug.data(), W);
                ygzo_remap_linear_f32(depth.ptr<float>(0), W, H, W, m1.data(), m2.data(), W, H, ud.data(), W);
                ygzo_compute_pyramid(&o4, ug.data(), W, H, W, lp);
            });
            std::printf("TIMING frame_undistort_pyramid_rgbd dropin_ms %.4f oracle_ms %.4f\n", gm, cm);
        }
        // ExtractFeatures, RGB-D branch (Frame.cc:737-750): ExtractORB(0), then ComputeStereoFromRGBD(mImDepth)
        F.ExtractORB(0, F.mImGray);
        F.N = (int)F.mvKeys.size();
        F.ComputeStereoFromRGBD(F.mImDepth);
        std::vector<float> our(F.N), odp(F.N);
        ygzo_stereo_from_rgbd(ud.data(), W, H, W, reinterpret_cast<const ygzo_kp *>(F.mvKeys.data()), F.N, 40.0f,
                              our.data(), odp.data());
        int with_depth = 0;
        for (int i = 0; i < F.N; i++) with_depth += F.mvDepth[i] > 0;
        const bool s_ok = F.N > 500 && (int)F.mvDepth.size() == F.N &&
                          std::memcmp(F.mvDepth.data(), odp.data(), 4 * (size_t)F.N) == 0 &&
                          std::memcmp(F.mvuRight.data(), our.data(), 4 * (size_t)F.N) == 0;
        CHECK(s_ok && with_depth > F.N / 2, "Frame::ComputeStereoFromRGBD(mImDepth) on the undistorted depth: %d "
              "keypoints, %d depths == oracle", F.N, with_depth);
    }
    Frame::mbNeedUndistort = saved;

    // ---------------- ComputeStereoMatches: a rectified EuRoC pair (right = left moved 6 px)
    {
        const int Ws = 752, Hs = 480, ns = 4;
        Eigen::Matrix3f Ks;
        Ks(0, 0) = 458.654f;
        Ks(1, 1) = 457.296f;
        Ks(0, 2) = 367.215f;
        Ks(1, 2) = 248.375f;
        Ks(2, 2) = 1.f;
        const cv::Mat L = synth(Ws, Hs, 21u, 0, 0), R = synth(Ws, Hs, 21u, -6, 0);
        ORBextractor exl(1000, 2.0f, ns, 20, 7), exr(1000, 2.0f, ns, 20, 7);
        const float bf = 0.11f * Ks(0, 0);  // EuRoC.yaml Camera.bf
        Frame S(L, R, cv::Mat(), Frame::Stereo, &exl, &exr, nullptr, Ks, cv::Mat(), bf);
        S.ExtractORB(0, S.mImGray);
        S.ExtractORB(1, S.mImRight);
        S.N = (int)S.mvKeys.size();
        S.ComputeStereoMatches();
        ygzo_orb os;
        ygzo_orb_init(&os, 1000, 2.0f, ns, 20, 7, 0);
        int lw[YGZO_MAX_LEVELS], lh[YGZO_MAX_LEVELS];
        ygzo_level_sizes(&os, Ws, Hs, lw, lh);
        std::vector<std::vector<uint8_t>> ll(ns), rl(ns);
        uint8_t *lp[YGZO_MAX_LEVELS], *rp[YGZO_MAX_LEVELS];
        for (int l = 0; l < ns; l++) {
            ll[l].resize((size_t)lw[l] * lh[l]);
            rl[l].resize((size_t)lw[l] * lh[l]);
            lp[l] = ll[l].data();
            rp[l] = rl[l].data();
        }
        ygzo_compute_pyramid(&os, L.data, Ws, Hs, Ws, lp);
        ygzo_compute_pyramid(&os, R.data, Ws, Hs, Ws, rp);
        const int nr = (int)S.mvKeysRight.size();
        std::vector<float> our(S.N), odp(S.N);
        ygzo_stereo_matches(lp, rp, lw, lh, ns, os.scale, os.inv_scale,
                            reinterpret_cast<const ygzo_kp *>(S.mvKeys.data()), S.mDescriptors.data, S.N,
                            reinterpret_cast<const ygzo_kp *>(S.mvKeysRight.data()), S.mDescriptorsRight.data, nr,
                            S.mb, S.mbf, our.data(), odp.data(), nullptr);
        int with_depth = 0;
        for (int i = 0; i < S.N; i++) with_depth += S.mvDepth[i] > 0;
        const bool ok = S.N > 300 && nr > 300 && std::memcmp(S.mvDepth.data(), odp.data(), 4 * (size_t)S.N) == 0 &&
                        std::memcmp(S.mvuRight.data(), our.data(), 4 * (size_t)S.N) == 0;
        CHECK(ok && with_depth > S.N / 4, "Frame::ComputeStereoMatches(): %d left / %d right keypoints, %d depths "
              "== oracle", S.N, nr, with_depth);
        if (g_timing) {
            const double gm = median_ms(20, [&] { S.ComputeStereoMatches(); });
            const double cm = median_ms(5, [&] {
                ygzo_stereo_matches(lp, rp, lw, lh, ns, os.scale, os.inv_scale,
                                    reinterpret_cast<const ygzo_kp *>(S.mvKeys.data()), S.mDescriptors.data, S.N,
                                    reinterpret_cast<const ygzo_kp *>(S.mvKeysRight.data()), S.mDescriptorsRight.data,
                                    nr, S.mb, S.mbf, our.data(), odp.data(), nullptr);
            });
            std::printf("TIMING compute_stereo_matches dropin_ms %.4f oracle_ms %.4f\n", gm, cm);
        }

        // ---------------- ComputeBoW: vocabularies bound to the Frame's ORBVocabulary: k = 10, L = 3,
        // and ORBvoc.txt's shape k = 10, L = 6 (1,111,111 nodes; the timed one)
        for (const int Lv : {3, 6}) {
        const int k = 10;
        std::vector<int32_t> parent(1, -1);
        std::vector<uint8_t> leaf(1, 0);
        int lvl_begin = 0, lvl_end = 1;
        for (int d = 1; d <= Lv; d++) {
            for (int p = lvl_begin; p < lvl_end; p++)
                for (int c = 0; c < k; c++) {
                    parent.push_back(p);
                    leaf.push_back(d == Lv);
                }
            lvl_begin = lvl_end;
            lvl_end = (int)parent.size();
        }
        const int nn = (int)parent.size();
        std::vector<uint8_t> vdesc((size_t)nn * 32);
        std::vector<double> wgt(nn);
        unsigned sd = 12345u;
        for (int i = 0; i < nn; i++) {
            // a child is its parent's descriptor with a few bits flipped: a real-looking tree
            for (int b = 0; b < 32; b++) vdesc[(size_t)32 * i + b] = i ? vdesc[(size_t)32 * parent[i] + b] : 0;
            if (i == 0) continue;
            for (int f = 0; f < 24; f++) {
                sd = sd * 1664525u + 1013904223u;
                vdesc[(size_t)32 * i + ((sd >> 8) & 31)] ^= (uint8_t)(1u << ((sd >> 16) & 7));
            }
            for (int b = 0; b < 32 && parent[i] == 0; b++) {  // level-1 centres: random
                sd = sd * 1664525u + 1013904223u;
                vdesc[(size_t)32 * i + b] = (uint8_t)(sd >> 24);
            }
            wgt[i] = 0.5 + (double)((sd >> 4) % 1000) / 400.0;
        }
        ygzfe_vocab *gv = nullptr;
        const int rc = ygzfe_vocab_create(dropin::device(), k, Lv, 0, 0, nn, parent.data(), leaf.data(), vdesc.data(),
                                          wgt.data(), &gv);
        ygzo_vocab *ov = ygzo_vocab_create(k, Lv, 0, 0, nn, parent.data(), leaf.data(), vdesc.data(), wgt.data());
        static int voc_token[2];  // stand for the System's ORBVocabulary objects
        gpu::BindVocabulary(&voc_token[Lv == 6], gv);
        S.mpORBvocabulary = reinterpret_cast<ORBVocabulary *>(&voc_token[Lv == 6]);
        S.mBowVec.clear();
        S.ComputeBoW();
        std::vector<int32_t> ow(S.N), ofn(S.N), off(S.N);
        std::vector<double> oval(S.N);
        int onw = 0, onf = 0;
        ygzo_compute_bow(ov, S.mDescriptors.data, S.N, 4, ow.data(), oval.data(), &onw, ofn.data(), off.data(), &onf);
        bool b_ok = rc == YGZFE_OK && (int)S.mBowVec.size() == onw && onw > 20;
        int i = 0;
        for (auto &e : S.mBowVec) {
            b_ok = b_ok && i < onw && (int)e.first == ow[i] && e.second == oval[i];
            i++;
        }
        int j = 0;
        for (auto &e : S.mFeatVec)
            for (unsigned f : e.second) {
                b_ok = b_ok && j < onf && (int)e.first == ofn[j] && (int)f == off[j];
                j++;
            }
        b_ok = b_ok && j == onf;
        CHECK(b_ok, "Frame::ComputeBoW(): BowVector %d words, FeatureVector %d entries == oracle (bound vocabulary, "
              "k %d, L %d, %d nodes)", (int)S.mBowVec.size(), j, k, Lv, nn);
        if (g_timing && Lv == 6) {
            const double gm = median_ms(20, [&] {
                S.mBowVec.clear();
                S.ComputeBoW();
            });
            const double cm = median_ms(5, [&] {
                ygzo_compute_bow(ov, S.mDescriptors.data, S.N, 4, ow.data(), oval.data(), &onw, ofn.data(),
                                 off.data(), &onf);
            });
            std::printf("TIMING compute_bow dropin_ms %.4f oracle_ms %.4f\n", gm, cm);
        }
        ygzo_vocab_destroy(ov);
        }
    }
}

int main(int argc, char **argv) {
    g_timing = argc > 1 && std::strcmp(argv[1], "--time") == 0;
    const int W = 752, H = 480, nl = 4;
    Frame::fx = 458.654f;
    Frame::fy = 457.296f;
    Frame::cx = 367.215f;
    Frame::cy = 248.375f;
    Frame::invfx = 1.f / Frame::fx;
    Frame::invfy = 1.f / Frame::fy;
    const float Z = 3.0f;
    Tracking T(1000, 2.0f, nl, 20, 7);  // EuRoC.yaml:32-45

    // ---------------------------------------------------------------- pyramid + ORB extraction
    const cv::Mat im0 = synth(W, H, 7u, 0, 0), im1 = synth(W, H, 7u, 2, -1);
    T.mLastFrame = Frame(im0, T.mpORBextractorLeft);
    T.mCurrentFrame = Frame(im1, T.mpORBextractorLeft);
    T.mLastFrame.ExtractFeatures();
    T.mCurrentFrame.ExtractFeatures();
    ygzo_orb o;
    ygzo_orb_init(&o, 1000, 2.0f, nl, 20, 7, 0);
    int lw[YGZO_MAX_LEVELS], lh[YGZO_MAX_LEVELS];
    ygzo_level_sizes(&o, W, H, lw, lh);
    std::vector<std::vector<uint8_t>> lv(nl);
    uint8_t *lp[YGZO_MAX_LEVELS];
    for (int l = 0; l < nl; l++) {
        lv[l].resize((size_t)lw[l] * lh[l]);
        lp[l] = lv[l].data();
    }
    for (int fi = 0; fi < 2; fi++) {
        const Frame &F = fi ? T.mCurrentFrame : T.mLastFrame;
        ygzo_compute_pyramid(&o, (fi ? im1 : im0).data, W, H, W, lp);
        bool pyr_ok = (int)F.mvImagePyramid.size() == nl;
        for (int l = 0; l < nl && pyr_ok; l++)
            pyr_ok = F.mvImagePyramid[l].cols == lw[l] && F.mvImagePyramid[l].rows == lh[l] &&
                     std::memcmp(F.mvImagePyramid[l].data, lp[l], lv[l].size()) == 0;
        CHECK(pyr_ok, "Frame::ComputeImagePyramid -> ORBextractor::ComputePyramid (frame %d): levels == oracle", fi);
        std::vector<ygzo_kp> ok_(4096);
        std::vector<uint8_t> od(4096 * 32);
        const int n = ygzo_extract_orbslam(&o, lp, lw, lh, nullptr, 0, ok_.data(), od.data(), 4096);
        const bool same = n == F.N && n > 300 && std::memcmp(ok_.data(), F.mvKeys.data(), sizeof(ygzo_kp) * n) == 0 &&
                          std::memcmp(od.data(), F.mDescriptors.data, (size_t)32 * n) == 0;
        CHECK(same, "(*mpORBextractorLeft)(this, mvKeys, mDescriptors, ORBSLAM_KEYPOINT) (frame %d): %d keypoints "
                    "+ descriptors == oracle", fi, F.N);
    }

    // The pyramid pool's lookups are exact.  A Frame's pyramid is found by its
    // level-0 pointer (the pool holds that buffer, so the address cannot be handed to another
    // image).  A host pyramid in a fresh buffer whose level 0 differs from a pooled one only in
    // pixels the content index does not sample gets its own device pyramid; an identical deep
    // copy is matched by one full compare.
    {
        dropin::PyramidPool &pool = dropin::PyramidPool::instance();
        Frame A(im1, T.mpORBextractorLeft);
        std::vector<cv::Mat> B, Cc;
        for (const cv::Mat &m : A.mvImagePyramid) {
            B.push_back(m.clone());  // plain deep copies: not aliased to A's device pyramid
            Cc.push_back(m.clone());
        }
        std::vector<uint8_t> sampled((size_t)W * H, 0);  // the fingerprint's 512 spread samples
        {
            const size_t n = (size_t)W * H, step = n / 512 + 1;
            size_t i = 7 % n;
            for (int k = 0; k < 512; k++, i = (i + step * 2 + 1) % n) sampled[i] = 1;
        }
        int x = 8;
        while (sampled[(size_t)W + x]) x++;  // row 1 is none of the 8 whole sampled rows
        B[0].data[(size_t)W + x] ^= 0x40;
        ygzfe_frame *fa = pool.find_or_upload(A.mvImagePyramid);
        ygzfe_frame *fb = pool.find_or_upload(B);
        ygzfe_frame *fc = pool.find_or_upload(Cc);
        std::vector<uint8_t> back((size_t)W * H);
        const bool read = fb && ygzfe_frame_level(fb, 0, nullptr, nullptr, back.data(), W) == YGZFE_OK;
        const bool b_ok = read && fb != fa && std::memcmp(back.data(), B[0].data, back.size()) == 0;
        CHECK(fa && b_ok && fc == fa && pool.held() <= 3 * pool.size(),
              "pyramid pool: an unsampled one-pixel change gets its own device pyramid (%s), an identical copy is "
              "matched (%s), %d held host buffers for %d entries", b_ok ? "yes" : "NO", fc == fa ? "yes" : "NO",
              pool.held(), pool.size());
        // A held level-0 buffer rewritten in place (cv::Mat::create / copyTo of the same size
        // reuse it): the pointer is indexed, its fingerprint no longer agrees, so the new pixels
        // are uploaded instead of the old device pyramid being returned.
        for (int xx = 0; xx < W; xx++) A.mvImagePyramid[0].data[xx] ^= 0x5a;  // row 0: a sampled row
        ygzfe_frame *fr = pool.find_or_upload(A.mvImagePyramid);
        const bool rread = fr && ygzfe_frame_level(fr, 0, nullptr, nullptr, back.data(), W) == YGZFE_OK;
        const bool r_ok = rread && std::memcmp(back.data(), A.mvImagePyramid[0].data, back.size()) == 0;
        ygzfe_frame *fr2 = pool.find_or_upload(A.mvImagePyramid);
        CHECK(r_ok && fr2 == fr, "pyramid pool: a held buffer rewritten in place gets the new pixels (%s), then hits "
              "by pointer again (%s)", r_ok ? "yes" : "NO", fr2 == fr ? "yes" : "NO");
    }

    // DSO path: a frame with direct-tracked keypoints and no features yet (Frame.cc:335-337)
    {
        ORBextractor dso_ex(1000, 2.0f, nl, 20, 7);
        Frame Fd(im1, &dso_ex);
        for (int i = 0; i < 60; i++)
            Fd.mvKeys.push_back(cv::KeyPoint(T.mCurrentFrame.mvKeys[i].pt, 7, -1, 0, 0));
        Fd.N = (int)Fd.mvKeys.size();
        std::vector<ygzo_kp> ex(Fd.N);
        std::memcpy(ex.data(), Fd.mvKeys.data(), sizeof(ygzo_kp) * Fd.N);
        Fd.ExtractORB(0, Fd.mImGray);
        ygzo_orb od_;
        ygzo_orb_init(&od_, 1000, 2.0f, nl, 20, 7, 0);
        ygzo_compute_pyramid(&od_, im1.data, W, H, W, lp);
        std::vector<ygzo_kp> ok_(8192);
        std::vector<uint8_t> odesc(8192 * 32);
        const int n = ygzo_extract_dso(&od_, lp, lw, lh, ex.data(), 60, ok_.data(), odesc.data(), 8192);
        const bool same = n == (int)Fd.mvKeys.size() &&
                          std::memcmp(ok_.data(), Fd.mvKeys.data(), sizeof(ygzo_kp) * n) == 0 &&
                          std::memcmp(odesc.data(), Fd.mDescriptors.data, (size_t)32 * n) == 0;
        CHECK(same, "(*mpORBextractorLeft)(this, mvKeys, mDescriptors, DSO_KEYPOINT): %d rows (60 existing) == oracle",
              (int)Fd.mvKeys.size());
    }

    // ---------------------------------------------------------------- SparseImgAlign::run
    // map points of the last frame on the plane Z = 3 m in front of it (identity pose)
    std::vector<MapPoint> mps(T.mLastFrame.N);
    for (int i = 0; i < T.mLastFrame.N; i++) {
        const cv::KeyPoint &kp = T.mLastFrame.mvKeys[i];
        mps[i].mWorldPos = Vector3f((kp.pt.x - Frame::cx) / Frame::fx * Z, (kp.pt.y - Frame::cy) / Frame::fy * Z, Z);
        mps[i].mDescriptor = T.mLastFrame.mDescriptors.row(i).clone();
        mps[i].nObs = 1 + (i % 3 == 0);
        if (i % 17 == 0) mps[i].mbBad = true;
        T.mLastFrame.mvpMapPoints[i] = i % 11 == 5 ? nullptr : &mps[i];
        T.mLastFrame.mvbOutlier[i] = i % 13 == 7;
    }
    SE3f TCR;
    const size_t ret = T.SparseAlign(TCR);
    {
        std::vector<float> xyz(3 * (size_t)T.mLastFrame.N);
        std::vector<uint8_t> us(T.mLastFrame.N);
        for (int i = 0; i < T.mLastFrame.N; i++) {
            MapPoint *mp = T.mLastFrame.mvpMapPoints[i];
            us[i] = mp && !mp->isBad() && !T.mLastFrame.mvbOutlier[i];
            const Vector3f p = T.mLastFrame.mTcw * mps[i].mWorldPos;
            for (int k = 0; k < 3; k++) xyz[3 * i + k] = p[k];
        }
        uint8_t *rp[YGZO_MAX_LEVELS], *cp[YGZO_MAX_LEVELS];
        for (int l = 0; l < nl; l++) {
            rp[l] = T.mLastFrame.mvImagePyramid[l].data;
            cp[l] = T.mCurrentFrame.mvImagePyramid[l].data;
        }
        ygzo_cam cam{Frame::fx, Frame::fy, Frame::cx, Frame::cy};
        ygzo_se3 T0{{0, 0, 0, 1}, {0, 0, 0}};
        ygzo_align_out ao;
        ygzo_sparse_align(rp, cp, lw, lh, o.inv_scale, &cam, reinterpret_cast<const ygzo_kp *>(T.mLastFrame.mvKeys.data()),
                          xyz.data(), us.data(), T.mLastFrame.N, nl - 1, 1, &T0, &ao);
        float err = 0.f;
        const float gq[4] = {TCR.unit_quaternion().x(), TCR.unit_quaternion().y(), TCR.unit_quaternion().z(),
                             TCR.unit_quaternion().w()};
        for (int k = 0; k < 4; k++) err = std::fmax(err, std::fabs(gq[k] - ao.T.q[k]));
        for (int k = 0; k < 3; k++) err = std::fmax(err, std::fabs(TCR.translation()[k] - ao.T.t[k]));
        const float tx = 2.0f * Z / Frame::fx, ty = -1.0f * Z / Frame::fy;  // image shift (2, -1) px at depth Z
        CHECK(ret == (size_t)ao.n_visible && err <= 1e-4f && ret > 100,
              "mpAlign->run(&mLastFrame, &mCurrentFrame, TCR): visible %zu (oracle %d), |dT| %.2e, t (%.4f %.4f) "
              "expected ~(%.4f %.4f)", ret, ao.n_visible, err, TCR.translation()[0], TCR.translation()[1], tx, ty);
        {  // NLSSolver_impl.hpp:8-13: SparseImgAlign(.., LevenbergMarquardt) -> optimizeLevenbergMarquardt
            ygz::SparseImgAlign lm(nl - 1, 1, 10, ygz::SparseImgAlign::LevenbergMarquardt);
            SE3f Tlm;
            const size_t vlm = lm.run(&T.mLastFrame, &T.mCurrentFrame, Tlm);
            ygzo_align_out lo;
            ygzo_sparse_align_method(rp, cp, lw, lh, o.inv_scale, &cam,
                                     reinterpret_cast<const ygzo_kp *>(T.mLastFrame.mvKeys.data()), xyz.data(),
                                     us.data(), T.mLastFrame.N, nl - 1, 1, &T0, YGZO_ALIGN_LM, &lo);
            float el = 0.f;
            const float lq[4] = {Tlm.unit_quaternion().x(), Tlm.unit_quaternion().y(), Tlm.unit_quaternion().z(),
                                 Tlm.unit_quaternion().w()};
            for (int k = 0; k < 4; k++) el = std::fmax(el, std::fabs(lq[k] - lo.T.q[k]));
            for (int k = 0; k < 3; k++) el = std::fmax(el, std::fabs(Tlm.translation()[k] - lo.T.t[k]));
            CHECK(vlm == (size_t)lo.n_visible && el <= 1e-4f && vlm > 100,
                  "SparseImgAlign(.., LevenbergMarquardt).run(): visible %zu (oracle %d), |dT| %.2e", vlm,
                  lo.n_visible, el);
        }
        const auto I = T.mpAlign->getFisherInformation();
        CHECK(std::fabs(I(0, 0) - ao.H[0] / (float)(5e-4 * 255 * 255)) <= 1e-3f * std::fabs(I(0, 0)) + 1e-3f,
              "getFisherInformation() = H / 32.5125: %.4g", I(0, 0));
        if (g_timing) {
            SE3f Tx;
            const double ga = median_ms(30, [&] { T.SparseAlign(Tx); });
            const double ca = median_ms(10, [&] {
                ygzo_sparse_align(rp, cp, lw, lh, o.inv_scale, &cam,
                                  reinterpret_cast<const ygzo_kp *>(T.mLastFrame.mvKeys.data()), xyz.data(), us.data(),
                                  T.mLastFrame.N, nl - 1, 1, &T0, &ao);
            });
            std::printf("TIMING sparse_align dropin_ms %.4f oracle_ms %.4f\n", ga, ca);
            // Frame(im, extractor) + ExtractFeatures: the pyramid and the ORB extraction as Frame.cc:327-348
            // runs them (cv::Mat image on the host, mvKeys / mDescriptors back on the host)
            // steady state: the drop-in's pyramid pool holds 96 device frames, each created
            // (and its extraction graph captured) on first use; Tracking streams past that
            auto one = [&] {
                Frame Fx(im1, T.mpORBextractorLeft);
                Fx.ExtractFeatures();
            };
            for (int i = 0; i < dropin::PyramidPool::soft_capacity() + 4; i++) one();
            const double ge = median_ms(30, one);
            const double gp = median_ms(30, [&] { T.mpORBextractorLeft->ComputePyramid(im1); });
            const double gf = median_ms(30, [&] { Frame Fx(im1, T.mpORBextractorLeft); });
            std::printf("TIMING extract_parts pyramid_ms %.4f frame_ctor_ms %.4f\n", gp, gf);
            std::vector<ygzo_kp> ok_(4096);
            std::vector<uint8_t> od(4096 * 32);
            const double ce = median_ms(10, [&] {
                ygzo_compute_pyramid(&o, im1.data, W, H, W, lp);
                ygzo_extract_orbslam(&o, lp, lw, lh, nullptr, 0, ok_.data(), od.data(), 4096);
            });
            std::printf("TIMING extract dropin_ms %.4f oracle_ms %.4f\n", ge, ce);
        }
    }

    // ---------------------------------------------------------------- SearchByProjection(F, LastF)
    T.mCurrentFrame.SetPose(TCR * T.mLastFrame.mTcw);
    for (int i = 0; i < T.mCurrentFrame.N; i++) T.mCurrentFrame.mvpMapPoints[i] = nullptr;
    {
        // expected: the oracle over the same windows (ORBmatcher.cc:1241-1280 formed here)
        Frame &C = T.mCurrentFrame;
        const Frame &L = T.mLastFrame;
        const Matrix3f Rcw = C.mTcw.rotationMatrix();
        const Vector3f tcw = C.mTcw.translation();
        std::vector<ygzo_mquery> q;
        std::vector<uint8_t> qd;
        std::vector<int> src;
        // the reference's per-point projection and window set-up (ORBmatcher.cc:1241-1280),
        // timed with the oracle's search below as the reference runs them, in one loop
        auto build_last = [&] {
            q.clear();
            qd.clear();
            src.clear();
            for (int i = 0; i < L.N; i++) {
                MapPoint *pMP = L.mvpMapPoints[i];
                if (!pMP || L.mvbOutlier[i]) continue;
                const Vector3f x3Dc = Rcw * pMP->GetWorldPos() + tcw;
                const float invzc = 1.0 / x3Dc[2];
                if (invzc < 0) continue;
                const float u = C.fx * x3Dc[0] * invzc + C.cx, v = C.fy * x3Dc[1] * invzc + C.cy;
                if (u < C.mnMinX || u > C.mnMaxX || v < C.mnMinY || v > C.mnMaxY) continue;
                const int oc = L.mvKeys[i].octave;
                ygzo_mquery Q{u, v, 15 * C.mvScaleFactors[oc], u - C.mbf * invzc, oc - 1, oc + 1, L.mvKeys[i].angle,
                              YGZO_MQ_VALID | YGZO_MQ_STEREO | (pMP->Observations() > 0 ? YGZO_MQ_BLOCKS : 0)};
                q.push_back(Q);
                qd.insert(qd.end(), pMP->mDescriptor.data, pMP->mDescriptor.data + 32);
                src.push_back(i);
            }
        };
        build_last();
        std::vector<int32_t> want(C.N);
        std::vector<uint8_t> blocked(C.N, 0);
        const ygzo_mframe mf = mframe(C, true);
        const int wn = ygzo_search_projection_best(&mf, q.data(), qd.data(), (int)q.size(), blocked.data(), 100, 1,
                                                   want.data());
        const int nmatches = T.MotionModel(15);
        int same = nmatches == wn && nmatches > 100;
        for (int i2 = 0; i2 < C.N && same; i2++) {
            MapPoint *exp = want[i2] >= 0 ? L.mvpMapPoints[src[want[i2]]] : nullptr;
            same = C.mvpMapPoints[i2] == exp;
        }
        CHECK(same, "matcher.SearchByProjection(mCurrentFrame, mLastFrame, th, MONOCULAR): %d matches (oracle %d)",
              nmatches, wn);
        if (g_timing) {
            const double g = median_ms(50, [&] {
                for (int i = 0; i < C.N; i++) C.mvpMapPoints[i] = nullptr;
                T.MotionModel(15);
            });
            const double c = median_ms(50, [&] {
                build_last();
                ygzo_search_projection_best(&mf, q.data(), qd.data(), (int)q.size(), blocked.data(), 100, 1,
                                            want.data());
            });
            std::printf("TIMING search_by_projection_last_frame dropin_ms %.4f oracle_ms %.4f queries %zu\n", g, c,
                        q.size());
        }

        // ---------------- a whole fallback frame in Tracking's call order: Frame(im) (Tracking.cc:390)
        // -> TrackWithMotionModel: ExtractFeatures, ORB mode (:1154), the pose from the last frame
        // (:1160), the map points cleared (:1162), SearchByProjection(mCurrentFrame, mLastFrame, 15,
        // MONOCULAR) (:1171) -> mLastFrame = Frame(mCurrentFrame) (:718; the copy is kept aside so
        // the last frame stays the one with map points)
        std::vector<double> f_ctor, f_extract, f_search, f_copy;
        auto fallback = [&](bool record) {
            auto t0 = std::chrono::steady_clock::now();
            auto lap = [&t0]() {
                const auto t1 = std::chrono::steady_clock::now();
                const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
                t0 = t1;
                return ms;
            };
            T.mCurrentFrame = Frame(im1, T.mpORBextractorLeft);
            const double a = lap();
            T.mCurrentFrame.ExtractFeatures();
            const double b = lap();
            T.mCurrentFrame.SetPose(TCR * T.mLastFrame.mTcw);
            std::fill(C.mvpMapPoints.begin(), C.mvpMapPoints.end(), static_cast<MapPoint *>(nullptr));
            const int nm = T.MotionModel(15);
            const double c = lap();
            { Frame copy(T.mCurrentFrame); }
            const double d = lap();
            if (record) {
                f_ctor.push_back(a);
                f_extract.push_back(b);
                f_search.push_back(c);
                f_copy.push_back(d);
            }
            return nm;
        };
        {
            const int nm = fallback(false);
            int same = nm == wn && nm > 100;
            for (int i2 = 0; i2 < C.N && same; i2++) {
                MapPoint *exp = want[i2] >= 0 ? L.mvpMapPoints[src[want[i2]]] : nullptr;
                same = C.mvpMapPoints[i2] == exp;
            }
            CHECK(same, "whole fallback frame (Frame(im) -> ExtractFeatures -> SearchByProjection(mCurrentFrame, "
                        "mLastFrame, 15, MONOCULAR) -> Frame(mCurrentFrame)): %d matches (oracle %d)", nm, wn);
        }
        if (g_timing) {
            for (int i = 0; i < 4; i++) fallback(false);
            const double g = median_ms(30, [&] { fallback(true); });
            auto med = [](std::vector<double> v) {
                std::sort(v.begin(), v.end());
                return v[v.size() / 2];
            };
            std::vector<ygzo_kp> okf(4096);
            std::vector<uint8_t> odf(4096 * 32);
            const ygzo_mframe mfc = mframe(C, true);  // the frame the fallback left
            const double c = median_ms(10, [&] {
                ygzo_compute_pyramid(&o, im1.data, W, H, W, lp);
                ygzo_extract_orbslam(&o, lp, lw, lh, nullptr, 0, okf.data(), odf.data(), 4096);
                build_last();
                ygzo_search_projection_best(&mfc, q.data(), qd.data(), (int)q.size(), blocked.data(), 100, 1,
                                            want.data());
            });
            std::printf("TIMING fallback_frame dropin_ms %.4f oracle_ms %.4f frame_ctor_ms %.4f extract_ms %.4f "
                        "search_by_projection_ms %.4f last_frame_copy_ms %.4f\n",
                        g, c, med(f_ctor), med(f_extract), med(f_search), med(f_copy));
        }
    }

    // ---------------------------------------------------------------- SearchByProjection(F, local map points)
    {
        Frame &C = T.mCurrentFrame;
        for (int i = 0; i < C.N; i++) C.mvpMapPoints[i] = nullptr;
        T.mvpLocalMapPoints.clear();
        for (int i = 0; i < T.mLastFrame.N; i++) {
            MapPoint *pMP = &mps[i];
            const Vector3f x3Dc = C.mTcw * pMP->GetWorldPos();
            pMP->mbTrackInView = i % 9 != 4;
            pMP->mTrackProjX = C.fx * x3Dc[0] / x3Dc[2] + C.cx;
            pMP->mTrackProjY = C.fy * x3Dc[1] / x3Dc[2] + C.cy;
            pMP->mTrackProjXR = pMP->mTrackProjX - 30.f;
            pMP->mnTrackScaleLevel = T.mLastFrame.mvKeys[i].octave;
            pMP->mTrackViewCos = i % 2 ? 0.999f : 0.99f;
            T.mvpLocalMapPoints.push_back(pMP);
        }
        std::vector<ygzo_mquery> q;
        std::vector<uint8_t> qd;
        // the reference's per-point window set-up (ORBmatcher.cc:55-80), timed with the search
        auto build_local = [&] {
            q.clear();
            qd.clear();
            for (MapPoint *pMP : T.mvpLocalMapPoints) {
                const float r = (pMP->mTrackViewCos > 0.998 ? 2.5f : 4.0f) * 3.0f;
                const int lvl = pMP->mnTrackScaleLevel;
                ygzo_mquery Q{pMP->mTrackProjX, pMP->mTrackProjY, r * C.mvScaleFactors[lvl], pMP->mTrackProjXR, -1, -1,
                              0.f, (pMP->mbTrackInView && !pMP->isBad() ? YGZO_MQ_VALID : 0) | YGZO_MQ_STEREO |
                                       (pMP->Observations() > 0 ? YGZO_MQ_BLOCKS : 0)};
                q.push_back(Q);
                qd.insert(qd.end(), pMP->mDescriptor.data, pMP->mDescriptor.data + 32);
            }
        };
        build_local();
        std::vector<int32_t> want(C.N);
        const ygzo_mframe mf = mframe(C, true);
        const int wn = ygzo_search_projection_ratio(&mf, q.data(), qd.data(), (int)q.size(), nullptr, 0.8f, want.data());
        const int cnt = T.LocalPoints(3);
        int same = cnt == wn && cnt > 100;
        for (int i = 0; i < C.N && same; i++)
            same = C.mvpMapPoints[i] == (want[i] >= 0 ? T.mvpLocalMapPoints[want[i]] : nullptr);
        CHECK(same, "matcher.SearchByProjection(mCurrentFrame, mvpLocalMapPoints, th, false): %d (oracle %d)", cnt, wn);
        if (g_timing) {
            const double g = median_ms(50, [&] {
                for (int i = 0; i < C.N; i++) C.mvpMapPoints[i] = nullptr;
                T.LocalPoints(3);
            });
            const double c = median_ms(50, [&] {
                build_local();
                ygzo_search_projection_ratio(&mf, q.data(), qd.data(), (int)q.size(), nullptr, 0.8f, want.data());
            });
            std::printf("TIMING search_by_projection_local_map dropin_ms %.4f oracle_ms %.4f queries %zu\n", g, c,
                        q.size());
        }
    }

    // ---------------------------------------------------------------- SearchForInitialization
    {
        T.mInitialFrame = T.mLastFrame;
        T.mvbPrevMatched.clear();
        for (const cv::KeyPoint &kp : T.mInitialFrame.mvKeys) T.mvbPrevMatched.push_back(kp.pt);
        std::vector<float> prev;
        for (const cv::Point2f &p : T.mvbPrevMatched) {
            prev.push_back(p.x);
            prev.push_back(p.y);
        }
        std::vector<int32_t> want(T.mInitialFrame.N);
        const ygzo_mframe f1 = mframe(T.mInitialFrame, false), f2 = mframe(T.mCurrentFrame, false);
        const int wn = ygzo_search_for_initialization(&f1, &f2, prev.data(), 100, 0.9f, 1, want.data());
        const int nmatches = T.Initialization();
        int same = nmatches == wn && nmatches > 100 && (int)T.mvIniMatches.size() == T.mInitialFrame.N;
        for (int i = 0; i < T.mInitialFrame.N && same; i++)
            same = T.mvIniMatches[i] == want[i] && T.mvbPrevMatched[i].x == prev[2 * i] &&
                   T.mvbPrevMatched[i].y == prev[2 * i + 1];
        CHECK(same, "matcher.SearchForInitialization(mInitialFrame, mCurrentFrame, mvbPrevMatched, mvIniMatches, 100): "
                    "%d (oracle %d)", nmatches, wn);
    }

    // ---------------------------------------------------------------- SearchByBoW(pKF, F)
    {
        KeyFrame kf;
        kf.mvKeys = T.mLastFrame.mvKeys;
        kf.mDescriptors = T.mLastFrame.mDescriptors;
        for (int i = 0; i < T.mLastFrame.N; i++) kf.mvpMapPoints.push_back(T.mLastFrame.mvpMapPoints[i]);
        auto node_of = [](const uint8_t *d) { return (unsigned)((d[0] * 131u + d[5]) % 60u) * 7u + 3u; };
        for (int i = 0; i < T.mLastFrame.N; i++)
            kf.mFeatVec[node_of(T.mLastFrame.mDescriptors.data + 32 * i)].push_back(i);
        T.mCurrentFrame.mFeatVec.clear();
        for (int i = 0; i < T.mCurrentFrame.N; i++)
            T.mCurrentFrame.mFeatVec[node_of(T.mCurrentFrame.mDescriptors.data + 32 * i)].push_back(i);
        T.mpReferenceKF = &kf;
        auto csr = [](const DBoW2::FeatureVector &fv, std::vector<int32_t> &n, std::vector<int32_t> &p,
                      std::vector<int32_t> &f) {
            p.push_back(0);
            for (auto &e : fv) {
                n.push_back((int)e.first);
                for (unsigned x : e.second) f.push_back((int)x);
                p.push_back((int)f.size());
            }
        };
        std::vector<int32_t> kn, kp, kfe, fn, fp, ffe;
        csr(kf.mFeatVec, kn, kp, kfe);
        csr(T.mCurrentFrame.mFeatVec, fn, fp, ffe);
        std::vector<uint8_t> usable(kf.mvKeys.size());
        for (size_t i = 0; i < usable.size(); i++) usable[i] = kf.mvpMapPoints[i] && !kf.mvpMapPoints[i]->isBad();
        std::vector<int32_t> want(T.mCurrentFrame.N);
        const ygzo_mframe fk = mframe(T.mLastFrame, false), ff = mframe(T.mCurrentFrame, false);
        const int wn = ygzo_search_by_bow(&fk, &ff, usable.data(), (int)kn.size(), kn.data(), kp.data(), kfe.data(),
                                          (int)fn.size(), fn.data(), fp.data(), ffe.data(), 0.7f, 0, want.data());
        std::vector<MapPoint *> vpMapPointMatches;
        const int nmatches = T.ReferenceKF(vpMapPointMatches);
        int same = nmatches == wn && nmatches > 30 && (int)vpMapPointMatches.size() == T.mCurrentFrame.N;
        for (int i = 0; i < T.mCurrentFrame.N && same; i++)
            same = vpMapPointMatches[i] == (want[i] >= 0 ? kf.mvpMapPoints[want[i]] : nullptr);
        CHECK(same, "matcher.SearchByBoW(mpReferenceKF, mCurrentFrame, vpMapPointMatches): %d (oracle %d)", nmatches,
              wn);
    }

    // ---------------------------------------------------------------- Align2D
    {
        Frame *curr = &T.mCurrentFrame;
        int tried = 0, same = 0, conv = 0;
        for (int i = 0; i < curr->N && tried < 40; i += 7) {
            const cv::KeyPoint &k = curr->mvKeys[i];
            const int search_level = k.octave;
            const cv::Mat &img = curr->mvImagePyramid[search_level];
            const Vector2f px_curr(k.pt.x + 0.6f * curr->mvScaleFactors[search_level],
                                   k.pt.y - 0.4f * curr->mvScaleFactors[search_level]);
            const int u = (int)std::lround(k.pt.x * curr->mvInvScaleFactors[search_level]),
                      v = (int)std::lround(k.pt.y * curr->mvInvScaleFactors[search_level]);
            if (u < 8 || v < 8 || u >= img.cols - 8 || v >= img.rows - 8) continue;
            uint8_t _patch_with_border[100], _patch[64];
            for (int y = 0; y < 10; y++)
                for (int x = 0; x < 10; x++) _patch_with_border[y * 10 + x] = img.data[(v - 5 + y) * img.step[0] + u - 5 + x];
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) _patch[y * 8 + x] = _patch_with_border[(y + 1) * 10 + x + 1];
            tried++;
            Vector2f px_scaled = px_curr * curr->mvInvScaleFactors[search_level];
            bool success = ygz::Align2D(curr->mvImagePyramid[search_level], _patch_with_border, _patch, 10, px_scaled);
            float opx[2] = {px_curr[0] * curr->mvInvScaleFactors[search_level],
                            px_curr[1] * curr->mvInvScaleFactors[search_level]};
            const int ook = ygzo_align2d(img.data, img.cols, img.rows, (int)img.step[0], _patch_with_border, _patch, 10,
                                         opx);
            same += (int)success == ook && px_scaled[0] == opx[0] && px_scaled[1] == opx[1];
            conv += success;
        }
        CHECK(tried >= 20 && same == tried && conv > tried / 2,
              "ygz::Align2D(curr->mvImagePyramid[search_level], ...): %d / %d bit-exact with the oracle, %d converged",
              same, tried, conv);
    }

    // ---------------------------------------------------------------- SearchLocalPointsDirect + FindDirectProjection
    // NK keyframes of the plane: A = the last frame (identity pose), B, C, ... shifted images
    // (image shift (dx, dy) <=> T_cw translation (dx Z / fx, dy Z / fy, 0)); C is mpLastKeyFrame,
    // which SelectNearestKeyframe leaves out.  NK = 130 first: a local map larger than the
    // pyramid pool's soft capacity (96), whose keyframes a phase pins; then NK = 3, whose state
    // the FindDirectProjection checks below reuse.
    std::vector<KeyFrame> kfs;
    std::vector<Frame> kframes;
    std::vector<MapPoint> dm;
    std::vector<uint8_t *> rp;
    for (const int NK : {130, 3}) {
        kfs.clear();
        kframes.clear();
        kfs.resize(NK);
        kframes.reserve(NK);
        auto shift = [](int k, int c) {
            static const int s3[3][2] = {{0, 0}, {-1, 1}, {3, 2}};
            return k < 3 ? s3[k][c] : (c == 0 ? (k * 5) % 9 - 4 : (k * 3) % 7 - 3);
        };
        for (int k = 0; k < NK; k++) {
            cv::Mat kim = k == 0 ? im0 : synth(W, H, 7u, shift(k, 0), shift(k, 1));
            if (k >= 3) kim.data[k] ^= 0x5A;  // row 0 (no window reaches it): every keyframe's pyramid distinct
            kframes.push_back(Frame(kim, T.mpORBextractorLeft));
            kfs[k].mvImagePyramid = kframes[k].mvImagePyramid;  // shared, as KeyFrame.cc:257-260
            kfs[k].mvScaleFactors = kframes[k].mvScaleFactors;
            kfs[k].mTcw = SE3f(Eigen::Quaternionf(), Vector3f(shift(k, 0) * Z / Frame::fx, shift(k, 1) * Z / Frame::fy, 0.f));
            kfs[k].mnId = 10 + k;
        }
        T.mpLastKeyFrame = &kfs[2];
        // map points: the last frame's keypoints on the plane, plus a neighbour 0.6 px away after every
        // third one (neighbours share cells of the 5-px coverage grid)
        const Frame &L = T.mLastFrame;
        dm.clear();
        dm.reserve(2 * L.N);
        for (int i = 0; i < L.N; i++) {
            for (int c = 0; c < 1 + (i % 3 == 0); c++) {
                const cv::KeyPoint &kp = L.mvKeys[i];
                MapPoint mp;
                const float u = kp.pt.x + 0.6f * c, v = kp.pt.y - 0.4f * c;
                mp.mWorldPos = Vector3f((u - Frame::cx) / Frame::fx * Z, (v - Frame::cy) / Frame::fy * Z, Z);
                mp.mbBad = (dm.size() % 23) == 11;
                dm.push_back(mp);
            }
        }
        for (size_t j = 0; j < dm.size(); j++) {
            MapPoint &mp = dm[j];
            const int oc = (int)(j % 3);
            for (int k = 0; k < NK; k++) {
                if (k == 0 && j % 5 == 1) continue;  // observed by B / C only
                if (k == 1 && j % 4 == 2) continue;
                if (k >= 3 && (j / 2 + 7 * (size_t)k) % 26 != 0) continue;  // NK = 130: 5 more keyframes per point
                const Vector3f pc = kfs[k].mTcw * mp.mWorldPos;
                cv::KeyPoint kp(cv::Point2f(Frame::fx * pc[0] / pc[2] + Frame::cx, Frame::fy * pc[1] / pc[2] + Frame::cy),
                                31.f * kfs[k].mvScaleFactors[oc], -1, 0, oc);
                mp.mObservations[&kfs[k]] = kfs[k].mvKeys.size();
                kfs[k].mvKeys.push_back(kp);
            }
        }
        // the frame being tracked: no features yet (TrackLocalMapDirect, Tracking.cc:2194), pose = TCR
        T.mCurrentFrame = Frame(im1, T.mpORBextractorLeft);
        T.mCurrentFrame.SetPose(TCR);
        Frame &C = T.mCurrentFrame;
        const cv::Mat cur_level0 = C.mvImagePyramid[0];

        // expected: the oracle over the same filters and items (ORBmatcher.cc:1577-1582 inputs formed here)
        uint8_t *cp[YGZO_MAX_LEVELS];
        for (int l = 0; l < nl; l++) cp[l] = C.mvImagePyramid[l].data;
        rp.assign((size_t)NK * nl, nullptr);
        for (int k = 0; k < NK; k++)
            for (int l = 0; l < nl; l++) rp[k * nl + l] = kfs[k].mvImagePyramid[l].data;
        ygzo_cam ocam{Frame::fx, Frame::fy, Frame::cx, Frame::cy};
        struct Want {
            std::vector<cv::KeyPoint> keys;
            std::vector<MapPoint *> mps;
            std::vector<int> from;
            std::set<MapPoint *> cache;
            int local_runs = 0;
        };
        auto run_oracle_phase = [&](const std::vector<MapPoint *> &pts, int n_cache, int th, Want &w,
                                    std::vector<int> &status) {
            std::vector<int32_t> ip(1, 0), ri;
            std::vector<ygzo_kp> ok;
            std::vector<float> pt, proj;
            std::vector<ygzo_se3> tcr;
            std::vector<long> ids;
            for (MapPoint *mp : pts) {
                proj.push_back(mp->mTrackProjX);
                proj.push_back(mp->mTrackProjY);
                for (auto &ob : T.SelectNearestKeyframe(mp->GetObservations(), 5)) {
                    const SE3f pose_ref = ob.first->GetPose();
                    const Vector3f p = pose_ref * mp->GetWorldPos();
                    const SE3f Tcr = C.mTcw * pose_ref.inverse();
                    ri.push_back((int)(ob.first - &kfs[0]));
                    ok.push_back(*reinterpret_cast<const ygzo_kp *>(&ob.first->mvKeys[ob.second]));
                    for (int q = 0; q < 3; q++) pt.push_back(p[q]);
                    tcr.push_back(ygzo_se3{{Tcr.unit_quaternion().x(), Tcr.unit_quaternion().y(),
                                            Tcr.unit_quaternion().z(), Tcr.unit_quaternion().w()},
                                           {Tcr.translation()[0], Tcr.translation()[1], Tcr.translation()[2]}});
                    ids.push_back((long)ob.first->mnId);
                }
                ip.push_back((int32_t)ri.size());
            }
            const int n = (int)pts.size();
            std::vector<float> px(2 * n + 2);
            std::vector<int> m(n + 1);
            status.assign(n + 1, 0);
            int ran = 0;
            const int cs = ygzo_search_local_points_direct(&ocam, rp.data(), cp, lw, lh, nl, o.scale, o.inv_scale,
                                                           o.inv_sigma2[1], n_cache, n - n_cache, ip.data(), ri.data(),
                                                           ok.data(), pt.data(), tcr.data(), proj.data(), 20.f, 5, th,
                                                           px.data(), m.data(), status.data(), &ran);
            for (int i = 0; i < n; i++)
                if (status[i] == 1) {
                    w.keys.push_back(cv::KeyPoint(cv::Point2f(px[2 * i], px[2 * i + 1]), 7, -1, 0, 0));
                    w.mps.push_back(pts[i]);
                    w.from.push_back((int)ids[m[i]]);
                }
            return cs;
        };
        // Tracking.cc:2258-2410 restated over the oracle: cache filters, cache phase, mnCacheHitTh,
        // UpdateLocalMap, local filters, local phase
        auto expected = [&](const std::set<MapPoint *> &cache0, const std::vector<MapPoint *> &local, int th) {
            Want w;
            w.cache = cache0;
            std::vector<MapPoint *> pts;
            for (auto it = w.cache.begin(); it != w.cache.end();) {
                if ((*it)->isBad() || !C.isInFrustum(*it, 0.5)) { it = w.cache.erase(it); continue; }
                pts.push_back(*it);
                ++it;
            }
            std::vector<int> st;
            const int cnt = run_oracle_phase(pts, (int)pts.size(), th, w, st);
            for (size_t i = 0; i < pts.size(); i++)
                if (st[i] == 0) w.cache.erase(pts[i]);
            if (cnt > th) return w;
            w.local_runs = 1;
            pts.clear();
            for (MapPoint *mp : local) {
                if (w.cache.count(mp) || mp->isBad() || !C.isInFrustum(mp, 0.5)) continue;
                pts.push_back(mp);
            }
            const size_t before = w.mps.size();
            run_oracle_phase(pts, 0, th, w, st);
            for (size_t i = before; i < w.mps.size(); i++) w.cache.insert(w.mps[i]);
            return w;
        };
        std::set<MapPoint *> cache0;
        std::vector<MapPoint *> local;
        for (size_t j = 0; j < dm.size(); j++) {
            if (j % 2 == 0) cache0.insert(&dm[j]);
            local.push_back(&dm[j]);
        }
        for (int th : {1 << 30, 150}) {
            const Want w = expected(cache0, local, th);
            C.mvKeys.clear();
            C.mvpMapPoints.clear();
            C.mvDepth.clear();
            C.mvbOutlier.clear();
            C.mvMatchedFrom.clear();
            C.N = 0;
            T.mvpDirectMapPointsCache = cache0;
            T.mvpLocalMapPoints.clear();
            T.mvpNextLocalMapPoints = local;
            T.mnCacheHitTh = th;
            T.nUpdateLocalMap = 0;
            T.TrackLocalMapDirect();
            bool same = (size_t)C.N == w.keys.size() && C.mvKeys.size() == w.keys.size() &&
                        C.mvpMapPoints == w.mps && C.mvMatchedFrom == w.from &&
                        T.mvpDirectMapPointsCache == w.cache && T.nUpdateLocalMap == w.local_runs &&
                        (int)C.mvuRight.size() == C.N && C.mvDepth.size() == w.keys.size();
            for (size_t i = 0; same && i < w.keys.size(); i++)
                same = C.mvKeys[i].pt.x == w.keys[i].pt.x && C.mvKeys[i].pt.y == w.keys[i].pt.y &&
                       C.mvKeys[i].size == 7.f && C.mvKeys[i].angle == -1.f;
            CHECK(same && w.keys.size() > 100,
                  "SearchLocalPointsDirect() [%d keyframes, mnCacheHitTh %d]: %zu points tracked (oracle %zu), local "
                  "map %s, cache %zu -> %zu", NK, th, C.mvKeys.size(), w.keys.size(),
                  w.local_runs ? "searched" : "skipped", cache0.size(), T.mvpDirectMapPointsCache.size());
            if (NK > dropin::PyramidPool::soft_capacity() && th == 150)
                CHECK(dropin::PyramidPool::instance().peak() > dropin::PyramidPool::soft_capacity() &&
                          dropin::PyramidPool::instance().size() <= dropin::PyramidPool::soft_capacity(),
                      "  the pyramid pool grew past its soft capacity for the pinned keyframes (%d entries) and "
                      "shrank back once they were unpinned (%d)", dropin::PyramidPool::instance().peak(),
                      dropin::PyramidPool::instance().size());
            if (g_timing && th == 150 && NK == 3) {
                auto run = [&] {
                    C.mvKeys.clear();
                    C.mvpMapPoints.clear();
                    C.mvDepth.clear();
                    C.mvbOutlier.clear();
                    C.mvMatchedFrom.clear();
                    C.N = 0;
                    T.mvpDirectMapPointsCache = cache0;
                    T.mvpLocalMapPoints.clear();
                    T.mvpNextLocalMapPoints = local;
                    T.mnCacheHitTh = th;
                    T.nUpdateLocalMap = 0;
                    T.TrackLocalMapDirect();
                };
                const double g = median_ms(30, run);
                gpu::direct_stats() = gpu::DirectStats();
                for (int r = 0; r < 30; r++) run();
                const gpu::DirectStats ds = gpu::direct_stats();
                const double c = median_ms(5, [&] { (void)expected(cache0, local, th); });
                // split (means over 30 runs): C-ABI calls (H2D + kernels + D2H), pyramid-pool lookups
                std::printf("TIMING search_local_points_direct dropin_ms %.4f oracle_ms %.4f points %zu c_abi_ms %.4f "
                            "pool_ms %.4f calls_per_run %.1f\n", g, c, local.size() + cache0.size(), ds.call_ms / 30,
                            ds.pool_ms / 30, ds.calls / 30.0);
            }
        }
        if (NK == 3) {

        // ORBmatcher::FindDirectProjection, one pair at a time, against the oracle
        ORBmatcher matcher;
        int tried = 0, same = 0, conv = 0;
        for (size_t j = 0; j < dm.size() && tried < 40; j += 13) {
            MapPoint *mp = &dm[j];
            if (!C.isInFrustum(mp, 0.5)) continue;
            for (auto &ob : T.SelectNearestKeyframe(mp->GetObservations(), 5)) {
                Vector2f px_curr(mp->mTrackProjX, mp->mTrackProjY);
                int level = mp->mnTrackScaleLevel;
                const bool ok = matcher.FindDirectProjection(ob.first, &T.mCurrentFrame, mp, px_curr, level);
                const SE3f pose_ref = ob.first->GetPose();
                const Vector3f p = pose_ref * mp->GetWorldPos();
                const SE3f Tcr = C.mTcw * pose_ref.inverse();
                const ygzo_se3 ot{{Tcr.unit_quaternion().x(), Tcr.unit_quaternion().y(), Tcr.unit_quaternion().z(),
                                   Tcr.unit_quaternion().w()},
                                  {Tcr.translation()[0], Tcr.translation()[1], Tcr.translation()[2]}};
                const float pref[3] = {p[0], p[1], p[2]};
                float opx[2] = {mp->mTrackProjX, mp->mTrackProjY};
                int osl = 0;
                const int k = (int)(ob.first - &kfs[0]);
                const int ook = ygzo_find_direct_projection(
                    &ocam, &rp[k * nl], lw, lh, cp, lw, lh, nl, o.scale, o.inv_scale, o.inv_sigma2[1], &ot, pref,
                    reinterpret_cast<const ygzo_kp *>(&ob.first->mvKeys[ob.second]), opx, &osl);
                tried++;
                same += (int)ok == ook && level == osl && px_curr[0] == opx[0] && px_curr[1] == opx[1];
                conv += ok;
            }
        }
        CHECK(tried >= 20 && same == tried && conv > tried / 2,
              "matcher.FindDirectProjection(ob.first, &mCurrentFrame, mp, px_curr, level): %d / %d bit-exact, "
              "%d converged", same, tried, conv);
        (void)cur_level0;

        // ------------------------------------------------ whole direct frames in Tracking's call order
        // GrabImageMonocular's Frame(im) (Tracking.cc:390) -> TrackWithSparseAlignment: the pose from
        // the last frame (mVelocity = I, :2151), mpAlign->run (:2170-2171), SetPose(TCR *
        // mLastFrame.mTcw) (:2179) -> TrackLocalMapDirect's SearchLocalPointsDirect (:2191-2201) ->
        // for a keyframe, CreateNewKeyFrame's ExtractFeatures, DSO mode (:1535, Frame.cc:717-771:
        // N tracked points, no features yet) -> mLastFrame = Frame(mCurrentFrame) (:718).  The
        // frames alternate im1 / im0 and chain as in Tracking: each run() aligns against the copy
        // the previous frame left, whose points are the previous SearchLocalPointsDirect's.
        // The first frames are checked against the oracle step by step; then each kind is timed
        // beside the oracle's work on the same inputs (pyramid, SparseImgAlign, the search
        // restated above, ygzo_extract_dso).
        {
            const Frame saved_last = T.mLastFrame;
            const cv::Mat ims[2] = {im1, im0};
            ygzo_orb odso;
            ygzo_orb_init(&odso, 1000, 2.0f, nl, 20, 7, 0);
            auto reset_direct = [&] {
                T.mvpDirectMapPointsCache = cache0;
                T.mvpLocalMapPoints.clear();
                T.mvpNextLocalMapPoints = local;
                T.mnCacheHitTh = 150;
                T.nUpdateLocalMap = 0;
            };
            // SparseImageAlign.cc:57-128's inputs of the oracle, from the Frames' own members
            auto oracle_align = [&](const Frame &ref, const Frame &cur, ygzo_align_out &ao) {
                std::vector<float> xyz(3 * (size_t)ref.N, 0.f);
                std::vector<uint8_t> us(ref.N, 0);
                for (int i = 0; i < ref.N; i++) {
                    MapPoint *mp = ref.mvpMapPoints[i];
                    if (!mp || mp->isBad() || ref.mvbOutlier[i]) continue;
                    us[i] = 1;
                    const Vector3f p = ref.mTcw * mp->GetWorldPos();
                    for (int q = 0; q < 3; q++) xyz[3 * i + q] = p[q];
                }
                uint8_t *rpp[YGZO_MAX_LEVELS], *cpp[YGZO_MAX_LEVELS];
                for (int l = 0; l < nl; l++) {
                    rpp[l] = ref.mvImagePyramid[l].data;
                    cpp[l] = cur.mvImagePyramid[l].data;
                }
                const SE3f T0s = cur.mTcw * ref.mTcw.inverse();
                const ygzo_se3 T0{{T0s.unit_quaternion().x(), T0s.unit_quaternion().y(), T0s.unit_quaternion().z(),
                                   T0s.unit_quaternion().w()},
                                  {T0s.translation()[0], T0s.translation()[1], T0s.translation()[2]}};
                ygzo_sparse_align(rpp, cpp, lw, lh, o.inv_scale, &ocam,
                                  reinterpret_cast<const ygzo_kp *>(ref.mvKeys.data()), xyz.data(), us.data(), ref.N,
                                  nl - 1, 1, &T0, &ao);
            };
            std::vector<double> t_ctor, t_align, t_direct, t_kf, t_copy;
            std::vector<ygzo_kp> kf_exist;  // the last keyframe's tracked rows before its extraction
            int32_t kf_grid = -1;           // and the DSO grid state it started from
            auto stamp = [](std::chrono::steady_clock::time_point &t0) {
                const auto t1 = std::chrono::steady_clock::now();
                const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
                t0 = t1;
                return ms;
            };
            // one frame; check >= 0: compare every step with the oracle (frame number `check`)
            int bad = 0, steps = 0;
            size_t last_visible = 0;
            auto direct_frame = [&](int k, bool keyframe, bool check) {
                auto t0 = std::chrono::steady_clock::now();
                T.mCurrentFrame = Frame(ims[k & 1], T.mpORBextractorLeft);  // Tracking.cc:390
                const double a = stamp(t0);
                T.mCurrentFrame.SetPose(T.mLastFrame.mTcw);  // mVelocity * mLastFrame.mTcw, :2151
                ygzo_align_out ao;
                if (check) oracle_align(T.mLastFrame, T.mCurrentFrame, ao);
                t0 = std::chrono::steady_clock::now();
                SE3f TCRk;
                const size_t vis = T.SparseAlign(TCRk);  // :2170-2171
                const double b = stamp(t0);
                last_visible = vis;
                if (check) {
                    float err = 0.f;
                    const float gq[4] = {TCRk.unit_quaternion().x(), TCRk.unit_quaternion().y(),
                                         TCRk.unit_quaternion().z(), TCRk.unit_quaternion().w()};
                    for (int q = 0; q < 4; q++) err = std::fmax(err, std::fabs(gq[q] - ao.T.q[q]));
                    for (int q = 0; q < 3; q++) err = std::fmax(err, std::fabs(TCRk.translation()[q] - ao.T.t[q]));
                    bad += !(err <= 1e-4f && (int)vis == ao.n_visible && vis > 100);
                    steps++;
                }
                T.mCurrentFrame.SetPose(TCRk * T.mLastFrame.mTcw);  // :2179
                reset_direct();
                Want w;
                if (check) {
                    for (int l = 0; l < nl; l++) cp[l] = C.mvImagePyramid[l].data;
                    w = expected(cache0, local, 150);
                }
                t0 = std::chrono::steady_clock::now();
                T.TrackLocalMapDirect();  // :2201
                const double c = stamp(t0);
                if (check) {
                    bool same = C.mvKeys.size() == w.keys.size() && C.mvpMapPoints == w.mps && w.keys.size() > 100;
                    for (size_t i = 0; same && i < w.keys.size(); i++)
                        same = C.mvKeys[i].pt.x == w.keys[i].pt.x && C.mvKeys[i].pt.y == w.keys[i].pt.y;
                    bad += !same;
                    steps++;
                }
                double d = 0;
                if (keyframe) {
                    std::vector<ygzo_kp> ex(C.N), ok_(8192);
                    std::vector<uint8_t> odesc(8192 * 32);
                    std::memcpy(ex.data(), C.mvKeys.data(), sizeof(ygzo_kp) * C.N);
                    int32_t g0 = 0;
                    ygzfe_extractor_dso_grid(T.mpORBextractorLeft->handle(), &g0, nullptr);
                    kf_exist = ex;
                    kf_grid = g0;
                    t0 = std::chrono::steady_clock::now();
                    T.mCurrentFrame.ExtractFeatures();  // CreateNewKeyFrame, :1535 (DSO: N > 0, not extracted)
                    d = stamp(t0);
                    if (check) {
                        uint8_t *lpc[YGZO_MAX_LEVELS];
                        for (int l = 0; l < nl; l++) lpc[l] = C.mvImagePyramid[l].data;
                        odso.dso_grid = g0;
                        const int n = ygzo_extract_dso(&odso, lpc, lw, lh, ex.data(), (int)ex.size(), ok_.data(),
                                                       odesc.data(), 8192);
                        bad += !(n == C.N && n > (int)ex.size() &&
                                 std::memcmp(ok_.data(), C.mvKeys.data(), sizeof(ygzo_kp) * n) == 0 &&
                                 std::memcmp(odesc.data(), C.mDescriptors.data, (size_t)32 * n) == 0);
                        steps++;
                    }
                }
                t0 = std::chrono::steady_clock::now();
                T.mLastFrame = Frame(T.mCurrentFrame);  // :718
                const double e = stamp(t0);
                if (!check) {
                    t_ctor.push_back(a);
                    t_align.push_back(b);
                    t_direct.push_back(c);
                    t_kf.push_back(d);
                    t_copy.push_back(e);
                }
            };
            for (int k = 0; k < 4; k++) direct_frame(k, k == 3, true);
            CHECK(bad == 0, "whole direct frames (Frame(im) -> mpAlign->run -> SearchLocalPointsDirect [-> DSO "
                  "ExtractFeatures] -> mLastFrame = Frame(mCurrentFrame)), 4 chained frames: %d / %d steps == oracle "
                  "(last run() visible %zu)", steps - bad, steps, last_visible);
            if (g_timing) {
                auto med = [](std::vector<double> v) {
                    std::sort(v.begin(), v.end());
                    return v.empty() ? 0.0 : v[v.size() / 2];
                };
                for (int kind = 0; kind < 2; kind++) {
                    const bool kf = kind == 1;
                    t_ctor.clear(), t_align.clear(), t_direct.clear(), t_kf.clear(), t_copy.clear();
                    int k = 0;
                    for (int i = 0; i < 6; i++) direct_frame(k++, kf, false);  // warm
                    t_ctor.clear(), t_align.clear(), t_direct.clear(), t_kf.clear(), t_copy.clear();
                    const double g = median_ms(30, [&] { direct_frame(k++, kf, false); });
                    // the oracle's work on the same inputs: the pyramid, SparseImgAlign from the last
                    // frame the chain left, the search, and for a keyframe ygzo_extract_dso
                    std::vector<ygzo_kp> okk(8192);
                    std::vector<uint8_t> odk(8192 * 32);
                    for (int l = 0; l < nl; l++) cp[l] = C.mvImagePyramid[l].data;
                    const Frame last = T.mLastFrame;
                    const double c = median_ms(5, [&] {
                        ygzo_compute_pyramid(&o, ims[k & 1].data, W, H, W, lp);
                        ygzo_align_out ao;
                        oracle_align(last, T.mCurrentFrame, ao);
                        (void)expected(cache0, local, 150);
                        if (kf) {
                            odso.dso_grid = kf_grid;
                            ygzo_extract_dso(&odso, cp, lw, lh, kf_exist.data(), (int)kf_exist.size(), okk.data(),
                                             odk.data(), 8192);
                        }
                    });
                    std::printf("TIMING %s dropin_ms %.4f oracle_ms %.4f frame_ctor_ms %.4f run_ms %.4f "
                                "search_local_points_direct_ms %.4f extract_dso_ms %.4f last_frame_copy_ms %.4f\n",
                                kf ? "keyframe_frame" : "direct_frame", g, c, med(t_ctor), med(t_align), med(t_direct),
                                med(t_kf), med(t_copy));
                }
            }
            T.mLastFrame = saved_last;
            T.mCurrentFrame = Frame(im1, T.mpORBextractorLeft);
            T.mCurrentFrame.SetPose(TCR);
        }
        }
    }

    // ---------------------------------------------------------------- Frame.cc's §8f rows (Frame_gpu.inc)
    frame_rows();

    std::printf(fails ? "FAILED %d\n" : "OK\n", fails);
    return fails ? 1 : 0;
}
