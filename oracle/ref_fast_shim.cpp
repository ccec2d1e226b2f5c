// ref_fast_shim.cpp — extern "C" entry points over the reference's own
// Thirdparty/fast sources (compiled from /root/reference by oracle/Makefile
// into oracle/_ref/libfastref.so).  TEST INFRASTRUCTURE ONLY: used to produce
// and re-check the FAST-10 golden vectors (tests/golden/fast10_*.npz).
#include <stddef.h>
#include <stdint.h>
#include <vector>
#include <fast/fast.h>

extern "C" int ref_fast10_detect(const uint8_t *img, int w, int h, int stride, int barrier, int sse,
                                 int16_t *xs, int16_t *ys, int cap) {
    std::vector<fast::fast_xy> c;
    if (sse) fast::fast_corner_detect_10_sse2(img, w, h, stride, (short)barrier, c);
    else fast::fast_corner_detect_10(img, w, h, stride, (short)barrier, c);
    int n = (int)c.size();
    for (int i = 0; i < n && i < cap; i++) { xs[i] = c[i].x; ys[i] = c[i].y; }
    return n;
}

extern "C" void ref_fast10_score(const uint8_t *img, int stride, const int16_t *xs, const int16_t *ys,
                                 int n, int threshold, int *scores) {
    std::vector<fast::fast_xy> c;
    for (int i = 0; i < n; i++) c.push_back(fast::fast_xy(xs[i], ys[i]));
    std::vector<int> s;
    fast::fast_corner_score_10(img, stride, c, threshold, s);
    for (int i = 0; i < n; i++) scores[i] = s[i];
}

extern "C" int ref_fast10_nonmax(const int16_t *xs, const int16_t *ys, const int *scores, int n, int *keep) {
    std::vector<fast::fast_xy> c;
    std::vector<int> s(scores, scores + n), k;
    for (int i = 0; i < n; i++) c.push_back(fast::fast_xy(xs[i], ys[i]));
    fast::fast_nonmax_3x3(c, s, k);
    for (size_t i = 0; i < k.size(); i++) keep[i] = k[i];
    return (int)k.size();
}

// The reference library's whole FAST-10 pipeline (detect_sse2 + score + nonmax_3x3),
// `reps` times over one ROI, timed here so no Python call overhead is counted:
// returns the kept-corner count, *sec = mean seconds per pipeline.
#include <chrono>
extern "C" int ref_fast10_pipeline_bench(const uint8_t *img, int w, int h, int stride, int barrier, int reps,
                                         double *sec) {
    std::vector<fast::fast_xy> c;
    std::vector<int> s, k;
    int kept = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) {
        c.clear();
        fast::fast_corner_detect_10_sse2(img, w, h, stride, (short)barrier, c);
        fast::fast_corner_score_10(img, stride, c, barrier, s);
        fast::fast_nonmax_3x3(c, s, k);
        kept = (int)k.size();
    }
    const auto t1 = std::chrono::steady_clock::now();
    *sec = std::chrono::duration<double>(t1 - t0).count() / (reps > 0 ? reps : 1);
    return kept;
}
