// ref_arith_probe.cpp — TEST INFRASTRUCTURE: the floating-point expression
// shapes of the reference's rBRIEF sampling and Shi-Tomasi score, compiled by
// tests/test_cpu_ref_arith.py with the reference's own compiler flags
// (CMakeLists.txt:14,21: g++ -Wall -O3 -march=native -std=c++11).  It pins
// what that build does with them (glibc cosf/sinf via std::cos(float), FMA
// contraction of GET_VALUE and of the Shi-Tomasi discriminant) so the oracle's
// explicit restatement can be checked against the compiler, not assumed.
//
// The expressions keep the reference's operand order and types:
//   ORBextractor.cc:103,108-116  (factorPI, angle, a, b, GET_VALUE, cvRound)
//   ORBextractor.cc:1174-1186    (dx, dy sums, /(2.0*area), the 0.5*(...) root)
#include <cmath>
#include <cstdint>
#include <immintrin.h>

using namespace std;

namespace {
// cvRound(float) on x86-64 (OpenCV core/fast_math.hpp): SSE2 cvtss2si
inline int round_sse(float v) { return _mm_cvtss_si32(_mm_set_ss(v)); }
struct IPoint { int x, y; };
const float kDegToRad = (float)(M_PI / 180.f);
}  // namespace

extern "C" void probe_offsets(const int *pattern_xy, float angle_deg, int *dy, int *dx) {
    const IPoint *pt = reinterpret_cast<const IPoint *>(pattern_xy);
    float angle = (float)angle_deg * kDegToRad;
    float a = (float)cos(angle), b = (float)sin(angle);
    for (int j = 0; j < 512; ++j) {
        dy[j] = round_sse(pt[j].x * b + pt[j].y * a);
        dx[j] = round_sse(pt[j].x * a - pt[j].y * b);
    }
}

extern "C" void probe_sincos(const float *y, int n, float *s, float *c) {
    for (int i = 0; i < n; ++i) {
        float v = y[i];
        c[i] = (float)cos(v);
        s[i] = (float)sin(v);
    }
}

extern "C" float probe_shi_tomasi(const uint8_t *data, int stride, int rows, int cols, int u, int v) {
    float sxx = 0.0, syy = 0.0, sxy = 0.0;
    const int half = 4, box = 2 * half, area = box * box;
    const int x0 = u - half, x1 = u + half, y0 = v - half, y1 = v + half;
    if (x0 < 1 || x1 >= cols - 1 || y0 < 1 || y1 >= rows - 1) return 0.0;
    for (int y = y0; y < y1; ++y) {
        const uint8_t *l = data + stride * y + x0 - 1, *r = data + stride * y + x0 + 1;
        const uint8_t *t = data + stride * (y - 1) + x0, *b = data + stride * (y + 1) + x0;
        for (int x = 0; x < box; ++x, ++l, ++r, ++t, ++b) {
            float gx = *r - *l;
            float gy = *b - *t;
            sxx += gx * gx;
            syy += gy * gy;
            sxy += gx * gy;
        }
    }
    sxx = sxx / (2.0 * area);
    syy = syy / (2.0 * area);
    sxy = sxy / (2.0 * area);
    return 0.5 * (sxx + syy - sqrt((sxx + syy) * (sxx + syy) - 4 * (sxx * syy - sxy * sxy)));
}
