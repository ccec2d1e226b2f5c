// tracking_demo.cpp — a Tracking.cc-shaped caller of the drop-in adapters
// (compat/ygz_compat.hpp).  It mirrors the reference's per-frame sequence:
//   extractor construction            Tracking.cc:255-261
//   Frame: ComputePyramid + ExtractORB Frame.cc:332-348, 807-813
//   matching inner loop               ORBmatcher.cc:1218-1350 (dense best/second)
//   TrackWithSparseAlignment          Tracking.cc:2145-2189 (SparseImgAlign(3,1).run)
// on a synthetic pair: frame 1 is frame 0 translated by (dx, dy) pixels, map
// points on a fronto-parallel plane at depth Z, so the true TCR translation is
// (-dx*Z/fx, -dy*Z/fy, 0).  Prints one line per check; exit 0 on success.
#include <cmath>
#include <cstdio>
#include <vector>

#include "ygz_compat.hpp"

static std::vector<uint8_t> synth(int W, int H, unsigned seed, int dx, int dy) {
    std::vector<uint8_t> img((size_t)W * H, 128);
    unsigned s = seed;
    auto rnd = [&](int n) { s = s * 1664525u + 1013904223u; return (int)((s >> 8) % (unsigned)n); };
    for (int r = 0; r < 900; r++) {
        const int x0 = rnd(W + 40) - 20, y0 = rnd(H + 40) - 20, w = 4 + rnd(40), h = 4 + rnd(40), v = rnd(256);
        for (int y = y0; y < y0 + h; y++)
            for (int x = x0; x < x0 + w; x++) {
                const int xx = x + dx, yy = y + dy;
                if (xx >= 0 && yy >= 0 && xx < W && yy < H) img[(size_t)yy * W + xx] = (uint8_t)v;
            }
    }
    return img;
}

int main() {
    const int W = 752, H = 480;
    const ygzfe_camera cam{458.654f, 457.296f, 367.215f, 248.375f};  // EuRoC.yaml:8-11
    const float Z = 3.0f;
    int fails = 0;
    try {
        ygz::ORBextractor extractor(1000, 2.0f, 4, 20, 7);  // EuRoC.yaml:32-45
        std::printf("levels %d scale %.1f features/level", extractor.GetLevels(), extractor.GetScaleFactor());
        for (int v : extractor.GetFeaturesPerLevel()) std::printf(" %d", v);
        std::printf("\n");

        const auto img0 = synth(W, H, 7u, 0, 0), img1 = synth(W, H, 7u, 2, -1);
        ygz::FramePyramid f0, f1;
        std::vector<ygz::KeyPoint> k0, k1;
        std::vector<uint8_t> d0, d1;
        extractor.ComputePyramid(f0, img0.data(), W, H, W);
        extractor(f0, k0, d0, ygz::ORBSLAM_KEYPOINT);
        extractor.ComputePyramid(f1, img1.data(), W, H, W);
        extractor(f1, k1, d1, ygz::ORBSLAM_KEYPOINT);
        std::printf("keypoints %zu %zu\n", k0.size(), k1.size());
        if (k0.size() < 300 || k1.size() < 300) fails++;

        ygz::ORBmatcher matcher(0.9f, true);
        std::vector<int> bi, bd, sd;
        matcher.SearchBest2(d1.data(), (int)k1.size(), d0.data(), (int)k0.size(), bi, bd, sd);
        int good = 0;
        for (size_t i = 0; i < k1.size(); i++)
            if (bd[i] <= ygz::ORBmatcher::TH_LOW && bd[i] < matcher.mfNNratio * sd[i]) good++;
        std::printf("matches(TH_LOW, ratio) %d; DescriptorDistance(d1[0], d0[bi0]) %d == %d\n", good,
                    ygz::ORBmatcher::DescriptorDistance(&d1[0], &d0[(size_t)bi[0] * 32]), bd[0]);
        if (good < 100 || ygz::ORBmatcher::DescriptorDistance(&d1[0], &d0[(size_t)bi[0] * 32]) != bd[0]) fails++;

        std::vector<float> xyz(3 * k0.size());
        std::vector<uint8_t> usable(k0.size(), 1);
        for (size_t i = 0; i < k0.size(); i++) {
            xyz[3 * i + 0] = (k0[i].pt.x - cam.cx) / cam.fx * Z;
            xyz[3 * i + 1] = (k0[i].pt.y - cam.cy) / cam.fy * Z;
            xyz[3 * i + 2] = Z;
        }
        ygz::SparseImgAlign align(3, 1);
        ygz::SE3 TCR;
        const size_t nvis = align.run(f0, f1, cam, k0, xyz.data(), usable.data(), TCR);
        const float tx = 2.0f * Z / cam.fx, ty = -1.0f * Z / cam.fy;
        std::printf("align visible %zu t (%.4f %.4f %.4f) expected (%.4f %.4f 0)\n", nvis, TCR.t[0], TCR.t[1],
                    TCR.t[2], tx, ty);
        if (nvis < 100 || std::fabs(TCR.t[0] - tx) > 2e-3f || std::fabs(TCR.t[1] - ty) > 2e-3f) fails++;
        // getFisherInformation() = H_ / (float)(5e-4 * 255 * 255) (SparseImageAlign.cc:51-55)
        const auto fisher = align.getFisherInformation();
        int fisher_bad = 0;
        for (int i = 0; i < 36; i++)
            fisher_bad += fisher[i] != align.hessian()[i] / (float)(5e-4 * 255 * 255);
        std::printf("fisher information H/32.5125: %s (I00 %.4g, H00 %.4g)\n", fisher_bad ? "WRONG" : "ok", fisher[0],
                    align.hessian()[0]);
        if (fisher_bad || !(align.hessian()[0] > 0.f)) fails++;
        // n_iter is ignored like the reference's (iterations[] overrides it, SparseImageAlign.cc:38-43)
        ygz::SparseImgAlign align30(3, 1, 30);
        ygz::SE3 TCR30;
        const size_t nvis30 = align30.run(f0, f1, cam, k0, xyz.data(), usable.data(), TCR30);
        std::printf("n_iter=30 ignored: visible %zu, same pose %d\n", nvis30, (int)(TCR30.t == TCR.t && TCR30.q == TCR.q));
        if (nvis30 != nvis || !(TCR30.t == TCR.t && TCR30.q == TCR.q)) fails++;

        // Align2D on level 0: the patch around frame 1's strongest level-0 corner,
        // started 0.7 / -0.5 px off
        const auto lv = f1.level(0);
        size_t best = 0;
        for (size_t i = 0; i < k1.size(); i++)
            if (k1[i].octave == 0 && k1[i].pt.x > 40 && k1[i].pt.y > 40 && k1[i].pt.x < W - 40 &&
                k1[i].pt.y < H - 40 && (k1[best].octave != 0 || k1[i].response > k1[best].response))
                best = i;
        const int u = (int)std::lround(k1[best].pt.x), v = (int)std::lround(k1[best].pt.y);
        uint8_t pb[100], p[64];
        for (int y = 0; y < 10; y++)
            for (int x = 0; x < 10; x++) pb[y * 10 + x] = lv[(size_t)(v - 5 + y) * W + (u - 5 + x)];
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) p[y * 8 + x] = pb[(y + 1) * 10 + (x + 1)];
        float px[2] = {u + 0.7f, v - 0.5f};
        const bool conv = ygz::Align2D(f1, 0, pb, p, 10, px);
        std::printf("Align2D converged %d px (%.3f %.3f) expected (%d %d)\n", (int)conv, px[0], px[1], u, v);
        if (!conv || std::fabs(px[0] - u) > 0.1f || std::fabs(px[1] - v) > 0.1f) fails++;

        // SearchLocalPointsDirect (Tracking.cc:2258-2410): frame 0 as the only keyframe,
        // every frame-0 keypoint a map point predicted 0.6 / -0.4 px off its true
        // position in frame 1; the batched search must land on the true shift
        ygz::DirectSearch ds;
        ygz::SE3 Tcr;
        Tcr.t = {tx, ty, 0.f};
        for (size_t i = 0; i < k0.size(); i++) {
            ds.add_point(k0[i].pt.x + 2.0f + 0.6f, k0[i].pt.y - 1.0f - 0.4f);
            ds.add_observation(0, k0[i], &xyz[3 * i], Tcr);
        }
        ds.run({&f0}, f1, cam);
        int hit = 0, close = 0, near = 0;
        for (int i = 0; i < ds.n_points(); i++) {
            if (!ds.matched(i)) continue;
            hit++;
            const float ex = std::fabs(ds.px(i)[0] - (k0[i].pt.x + 2.f)), ey = std::fabs(ds.px(i)[1] - (k0[i].pt.y - 1.f));
            close += ex < 0.1f && ey < 0.1f;
            near += ex < 0.5f && ey < 0.5f;
        }
        const auto outcome = ds.cache_pass(W, H);
        int kept = 0;
        for (auto o : outcome) kept += o == ygz::DirectSearch::kMatched;
        std::printf("direct search matched %d of %d, %d within 0.1 px, %d within 0.5 px; cache pass keeps %d\n", hit,
                    ds.n_points(), close, near, kept);
        if (hit < ds.n_points() / 2 || near < hit * 7 / 10 || close < hit / 2 || kept < 1 || kept > hit) fails++;

        // Stereo (Frame::ComputeStereoMatches, Frame.cc:509-682): the right image is the
        // left one moved 6 px left, so every match has disparity 6 and depth mbf / 6
        // (+-1 noise on the right image: with identical windows every SAD is 0 and the
        // reference's median cut, SAD >= 2.1 * median, drops all matches)
        auto imgR = synth(W, H, 7u, -6, 0);
        for (size_t i = 0; i < imgR.size(); i++) {
            const int v = imgR[i] + (int)(((uint32_t)i * 2654435761u) >> 30) - 1;
            imgR[i] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
        ygz::FramePyramid fR;
        std::vector<ygz::KeyPoint> kR;
        std::vector<uint8_t> dR;
        ygz::ORBextractor extractorRight(1000, 2.0f, 4, 20, 7);
        extractorRight.ComputePyramid(fR, imgR.data(), W, H, W);
        extractorRight(fR, kR, dR, ygz::ORBSLAM_KEYPOINT, false);
        const float mb = 0.11f, mbf = mb * cam.fx;
        std::vector<float> uRight, depth;
        ygz::ComputeStereoMatches(f0, fR, k0, d0, kR, dR, mb, mbf, uRight, depth);
        int nd = 0, good_d = 0;
        for (size_t i = 0; i < k0.size(); i++)
            if (depth[i] > 0) {
                nd++;
                good_d += std::fabs((k0[i].pt.x - uRight[i]) - 6.f) < 1.0f;  // sub-pixel disparity within 1 px
            }
        std::printf("stereo depths %d of %zu, %d with disparity 6 +- 1 px\n", nd, k0.size(), good_d);
        if (nd < (int)k0.size() / 5 || good_d < nd * 9 / 10) fails++;

        // ORBVocabulary (DBoW2) + Frame::ComputeBoW (Frame.cc:495-500) with a small
        // text vocabulary: 4 random words under the root
        const char *voc_path = "/tmp/ygzfe_demo_voc.txt";
        if (FILE *vf = std::fopen(voc_path, "w")) {
            std::fprintf(vf, "4 1  0 0\n");
            unsigned s = 11u;
            for (int n = 0; n < 4; n++) {
                std::fprintf(vf, "0 1 ");
                for (int b = 0; b < 32; b++) { s = s * 1664525u + 1013904223u; std::fprintf(vf, "%u ", (s >> 24) & 255u); }
                std::fprintf(vf, " %.3f\n", 0.5 + n);
            }
            std::fclose(vf);
        }
        ygz::ORBVocabulary voc;
        std::vector<std::pair<int, double>> bow;
        std::vector<std::pair<int, std::vector<unsigned>>> feat;
        const bool loaded = voc.loadFromTextFile(voc_path);
        if (loaded) voc.transform(d0.data(), (int)k0.size(), bow, feat, 4);
        double l1 = 0;
        size_t nfeat = 0;
        for (auto &b : bow) l1 += b.second;
        for (auto &f : feat) nfeat += f.second.size();
        std::printf("BoW: %zu words, L1 %.6f, %zu features in the FeatureVector\n", bow.size(), l1, nfeat);
        if (!loaded || bow.empty() || std::fabs(l1 - 1.0) > 1e-9 || nfeat != k0.size()) fails++;
    } catch (const std::exception &e) {
        std::printf("error: %s\n", e.what());
        return 2;
    }
    std::printf(fails ? "FAILED %d\n" : "OK\n", fails);
    return fails ? 1 : 0;
}
