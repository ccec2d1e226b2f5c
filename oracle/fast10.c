/*
 * fast10.c — CPU restatement of Thirdparty/fast (libCVD FAST-10, YGZ-modified)
 * and of ORBextractor's DSO keypoint mode.
 * TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline); see ygz_oracle.h.
 *
 * The generated decision trees of fast_10.cpp / fast_10_score.cpp are
 * restated by their defining property (the FAST-ER trees are exact):
 *   corner(p, b)  <=>  >= 10 contiguous ring pixels (16-ring, wrapping) all
 *                       > p + b, or all < p - b;
 *   score(p, t)   =  max b >= t with corner(p, b)   (fast_10_score.cpp:21-3147:
 *                    b += min_diff until the test fails, return b - 1).
 * PINNED: tests/test_oracle_golden.py checks both against vectors produced by
 * the reference sources compiled in oracle/_ref.
 */
#include "ygz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#if defined(__AVX2__)
#include <immintrin.h>
#endif

/* fast_10.cpp:18-35 ring order */
static const int kRing[16][2] = {{0, 3},  {1, 3},  {2, 2},   {3, 1},   {3, 0},   {3, -1},
                                 {2, -2}, {1, -3}, {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                 {-3, 0}, {-3, 1}, {-2, 2},  {-1, 3}};

/* longest circular run of 1-bits in a 16-bit mask */
static int max_circular_run16(unsigned m) {
    if (m == 0xFFFFu) return 16;
    unsigned mm = m | (m << 16);
    int best = 0, run = 0;
    for (int i = 0; i < 32; i++) {
        if (mm & (1u << i)) { if (++run > best) best = run; }
        else run = 0;
    }
    return best > 16 ? 16 : best;
}

int ygzo_fast10_is_corner(const uint8_t *p, int stride, int barrier) {
    int v = p[0], cb = v + barrier, c_b = v - barrier;
    unsigned bright = 0, dark = 0;
    for (int k = 0; k < 16; k++) {
        int x = p[kRing[k][0] + kRing[k][1] * stride];
        if (x > cb) bright |= 1u << k;
        if (x < c_b) dark |= 1u << k;
    }
    return max_circular_run16(bright) >= 10 || max_circular_run16(dark) >= 10;
}

int ygzo_fast10_score(const uint8_t *p, int stride, int threshold) {
    /* closed form of the iterative barrier search: the largest b with a
     * 10-arc strictly beyond p +- b is (max over arcs of min margin) - 1. */
    int v = p[0], d[16];
    for (int k = 0; k < 16; k++) d[k] = p[kRing[k][0] + kRing[k][1] * stride] - v;
    int best = threshold;
    for (int s = 0; s < 16; s++) {
        int mnb = 1 << 20, mnd = 1 << 20;
        for (int k = 0; k < 10; k++) {
            int x = d[(s + k) & 15];
            if (x < mnb) mnb = x;
            if (-x < mnd) mnd = -x;
        }
        if (mnb - 1 > best) best = mnb - 1;
        if (mnd - 1 > best) best = mnd - 1;
    }
    return best;
}

int ygzo_fast10_detect_plain(const uint8_t *img, int w, int h, int stride, int barrier,
                             int16_t *xs, int16_t *ys, int cap) {
    int n = 0; /* YGZ scans every pixel of the ROI from (0,0) (fast_10.cpp:35-42) */
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++)
            if (ygzo_fast10_is_corner(img + (size_t)y * stride + x, stride, barrier)) {
                if (n < cap) { xs[n] = (int16_t)x; ys[n] = (int16_t)y; }
                n++;
            }
    return n;
}

/* The segment test on 16 consecutive pixels at once (GCC vector extensions,
 * int16 lanes: AVX2 / AVX-512 under -march=native), as the reference's own SSE2
 * detector works on 16 pixels per step (faster_corner_10_sse.cpp:24-183): the
 * compass points 0/4/8/12 screen the block (a 10-arc covers at least two
 * neighbouring compass points, so a pixel with no two of them beyond the
 * barrier on one side is no corner), then with e_k = ring_k - v the largest
 * 10-arc minimum of e (bright) and of -e (dark) by min / max doubling:
 * corner(b) <=> arcmax > b, and fast_corner_score_10's barrier search
 * (b += min_diff until the test fails, fast_10_score.cpp:21-3147) ends at
 * max(threshold, arcmax - 1).  Bit i of the mask = corner at p + i; arcmax[i]. */
typedef int16_t f10_i16x16 __attribute__((vector_size(32)));
typedef uint8_t f10_u8x16 __attribute__((vector_size(16)));
static inline f10_i16x16 f10_ld(const uint8_t *p) {
    f10_u8x16 b;
    memcpy(&b, p, 16);
    return __builtin_convertvector(b, f10_i16x16);
}
static inline int f10_any(f10_i16x16 m) {
    uint64_t q[4];
    memcpy(q, &m, 32);
    return (q[0] | q[1] | q[2] | q[3]) != 0;
}
static inline f10_i16x16 f10_min(f10_i16x16 a, f10_i16x16 b) { const f10_i16x16 m = a < b; return (a & m) | (b & ~m); }
static inline f10_i16x16 f10_max(f10_i16x16 a, f10_i16x16 b) { const f10_i16x16 m = a > b; return (a & m) | (b & ~m); }

static unsigned fast10_test16(const uint8_t *p, const int pix[16], int barrier, int16_t arcmax[16]) {
    const f10_i16x16 v = f10_ld(p);
    const f10_i16x16 lo = v - (int16_t)barrier, hi = v + (int16_t)barrier;
    f10_i16x16 e[16];
    for (int k = 0; k < 16; k += 4) e[k] = f10_ld(p + pix[k]);
    const f10_i16x16 b0 = e[0] > hi, b4 = e[4] > hi, b8 = e[8] > hi, b12 = e[12] > hi;
    const f10_i16x16 d0 = e[0] < lo, d4 = e[4] < lo, d8 = e[8] < lo, d12 = e[12] < lo;
    const f10_i16x16 scr = (b0 & b4) | (b4 & b8) | (b8 & b12) | (b12 & b0) | (d0 & d4) | (d4 & d8) | (d8 & d12) |
                           (d12 & d0);
    if (!f10_any(scr)) return 0u;
    for (int k = 0; k < 16; k++) {
        if (k & 3) e[k] = f10_ld(p + pix[k]);
        e[k] -= v;
    }
    f10_i16x16 n2[16], x2[16], n4[16], x4[16], n8[16], x8[16];
    for (int k = 0; k < 16; k++) { n2[k] = f10_min(e[k], e[(k + 1) & 15]); x2[k] = f10_max(e[k], e[(k + 1) & 15]); }
    for (int k = 0; k < 16; k++) { n4[k] = f10_min(n2[k], n2[(k + 2) & 15]); x4[k] = f10_max(x2[k], x2[(k + 2) & 15]); }
    for (int k = 0; k < 16; k++) { n8[k] = f10_min(n4[k], n4[(k + 4) & 15]); x8[k] = f10_max(x4[k], x4[(k + 4) & 15]); }
    f10_i16x16 bright = f10_min(n8[0], n2[8]), darkmin = f10_max(x8[0], x2[8]);
    for (int k = 1; k < 16; k++) {
        bright = f10_max(bright, f10_min(n8[k], n2[(k + 8) & 15]));
        darkmin = f10_min(darkmin, f10_max(x8[k], x2[(k + 8) & 15]));
    }
    const f10_i16x16 am = f10_max(bright, -darkmin);
    const f10_i16x16 c = (am > (int16_t)barrier) & scr;
    if (!f10_any(c)) return 0u;
    unsigned m = 0;
    for (int i = 0; i < 16; i++) {
        m |= (unsigned)(c[i] != 0) << i;
        arcmax[i] = am[i];
    }
    return m;
}

static void ring10_offsets(int stride, int pix[16]) {
    for (int k = 0; k < 16; k++) pix[k] = kRing[k][0] + kRing[k][1] * stride;
}

/* 0: the 16-pixel vector test (default), 1: the scalar one (test hook) */
static int g_fast10_scalar = 0;
void ygzo_fast10_force_scalar(int on) { g_fast10_scalar = on; }

#if defined(__AVX2__)
/* The compass screen on 32 pixels at once in unsigned-saturating bytes (the
 * reference's SSE2 detector screens in bytes too): bit i set when pixel p + i
 * has two neighbouring compass points both beyond v + b or both beyond v - b.
 * hi = v +sat b, lo = v -sat b are exact: a saturated bound cannot be passed. */
static inline uint32_t fast10_screen32(const uint8_t *p, const int pix[16], int barrier) {
    const __m256i v = _mm256_loadu_si256((const __m256i *)p);
    const __m256i b = _mm256_set1_epi8((char)barrier);
    const __m256i hi = _mm256_adds_epu8(v, b), lo = _mm256_subs_epu8(v, b);
    __m256i B[4], D[4];
    for (int k = 0; k < 4; k++) {
        const __m256i e = _mm256_loadu_si256((const __m256i *)(p + pix[4 * k]));
        B[k] = _mm256_subs_epu8(e, hi);  /* nonzero <=> e > hi */
        D[k] = _mm256_subs_epu8(lo, e);  /* nonzero <=> e < lo */
    }
    __m256i s = _mm256_min_epu8(B[0], B[1]);
    s = _mm256_max_epu8(s, _mm256_min_epu8(B[1], B[2]));
    s = _mm256_max_epu8(s, _mm256_min_epu8(B[2], B[3]));
    s = _mm256_max_epu8(s, _mm256_min_epu8(B[3], B[0]));
    s = _mm256_max_epu8(s, _mm256_min_epu8(D[0], D[1]));
    s = _mm256_max_epu8(s, _mm256_min_epu8(D[1], D[2]));
    s = _mm256_max_epu8(s, _mm256_min_epu8(D[2], D[3]));
    s = _mm256_max_epu8(s, _mm256_min_epu8(D[3], D[0]));
    return ~(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(s, _mm256_setzero_si256()));
}

/* The segment test and arcmax of 32 screened pixels in unsigned-saturating
 * bytes: bright margins b_k = ring_k -sat v, dark d_k = v -sat ring_k, the
 * largest 10-arc minimum of each by min doubling (2, 4, 8, then + 2).  The
 * saturation clamps arcmax at 0, and a corner needs arcmax > barrier >= 0, so
 * the corners and their arcmax are the int16 test's exactly (half the lanes'
 * work of fast10_test16 per pixel).  Bit i = corner at p + i; am[i] = arcmax. */
static inline uint32_t fast10_test32(const uint8_t *p, const int pix[16], int barrier, uint8_t am[32]) {
    const __m256i v = _mm256_loadu_si256((const __m256i *)p);
    __m256i b2[16], d2[16];
    {
        __m256i b[16], d[16];
        for (int k = 0; k < 16; k++) {
            const __m256i e = _mm256_loadu_si256((const __m256i *)(p + pix[k]));
            b[k] = _mm256_subs_epu8(e, v);
            d[k] = _mm256_subs_epu8(v, e);
        }
        for (int k = 0; k < 16; k++) {
            b2[k] = _mm256_min_epu8(b[k], b[(k + 1) & 15]);
            d2[k] = _mm256_min_epu8(d[k], d[(k + 1) & 15]);
        }
    }
    __m256i best = _mm256_setzero_si256();
    {
        __m256i b4[16], d4[16];
        for (int k = 0; k < 16; k++) {
            b4[k] = _mm256_min_epu8(b2[k], b2[(k + 2) & 15]);
            d4[k] = _mm256_min_epu8(d2[k], d2[(k + 2) & 15]);
        }
        for (int k = 0; k < 16; k++) {
            const __m256i b10 = _mm256_min_epu8(_mm256_min_epu8(b4[k], b4[(k + 4) & 15]), b2[(k + 8) & 15]);
            const __m256i d10 = _mm256_min_epu8(_mm256_min_epu8(d4[k], d4[(k + 4) & 15]), d2[(k + 8) & 15]);
            best = _mm256_max_epu8(best, _mm256_max_epu8(b10, d10));
        }
    }
    _mm256_storeu_si256((__m256i *)am, best);
    const __m256i over = _mm256_subs_epu8(best, _mm256_set1_epi8((char)barrier)); /* nonzero <=> am > barrier */
    return ~(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(over, _mm256_setzero_si256()));
}
#endif

/* corners of rows [y0, y1) x columns [3, w - 3) in raster order; arcmax per corner if am != NULL */
static int fast10_rows(const uint8_t *img, int w, int y0, int y1, int stride, int barrier, int16_t *xs, int16_t *ys,
                       int16_t *am, int cap) {
    int pix[16];
    ring10_offsets(stride, pix);
    int n = 0;
    for (int y = y0; y < y1; y++) {
        int x = 3;
        if (!g_fast10_scalar) {
#if defined(__AVX2__)
            for (; x + 32 <= w - 3; x += 32) {  /* 32 pixels screened, then tested, in bytes */
                const uint8_t *p = img + (size_t)y * stride + x;
                const uint32_t scr = fast10_screen32(p, pix, barrier);
                if (!scr) continue;
                uint8_t a[32];
                uint32_t m = fast10_test32(p, pix, barrier, a) & scr;
                while (m) {
                    const int i = __builtin_ctz(m);
                    m &= m - 1;
                    if (n < cap) {
                        xs[n] = (int16_t)(x + i); ys[n] = (int16_t)y;
                        if (am) am[n] = a[i];
                    }
                    n++;
                }
            }
#endif
            for (; x + 16 <= w - 3; x += 16) {  /* ring of lane 15: columns x + 12 .. x + 18 <= w - 1 */
                int16_t a[16];
                unsigned m = fast10_test16(img + (size_t)y * stride + x, pix, barrier, a);
                while (m) {
                    const int i = __builtin_ctz(m);
                    m &= m - 1;
                    if (n < cap) { xs[n] = (int16_t)(x + i); ys[n] = (int16_t)y; if (am) am[n] = a[i]; }
                    n++;
                }
            }
            if (x < w - 3 && w - 19 >= 3) {  /* the tail: one block ending at column w - 4 */
                const int xb = w - 19;
                int16_t a[16];
                unsigned m = fast10_test16(img + (size_t)y * stride + xb, pix, barrier, a) & (0xFFFFu << (x - xb));
                while (m) {
                    const int i = __builtin_ctz(m);
                    m &= m - 1;
                    if (n < cap) { xs[n] = (int16_t)(xb + i); ys[n] = (int16_t)y; if (am) am[n] = a[i]; }
                    n++;
                }
                x = w - 3;
            }
        }
        for (; x < w - 3; x++) {
            const uint8_t *p = img + (size_t)y * stride + x;
            if (ygzo_fast10_is_corner(p, stride, barrier)) {
                if (n < cap) {
                    xs[n] = (int16_t)x; ys[n] = (int16_t)y;
                    if (am) am[n] = (int16_t)(ygzo_fast10_score(p, stride, barrier) + 1);
                }
                n++;
            }
        }
    }
    return n;
}

int ygzo_fast10_detect_sse2(const uint8_t *img, int w, int h, int stride, int barrier,
                            int16_t *xs, int16_t *ys, int cap) {
    if (w < 22) return ygzo_fast10_detect_plain(img, w, h, stride, barrier, xs, ys, cap);
    if (h < 7) return 0;
    /* faster_corner_10_sse.cpp:24-183: rows [3,h-3), cols [3,w-3) */
    return fast10_rows(img, w, 3, h - 3, stride, barrier, xs, ys, NULL, cap);
}

/* fast_corner_detect_10_sse2 + fast_corner_score_10 + fast_nonmax_3x3 over one
 * ROI (the reference library's full FAST-10 pipeline): corners kept by the 3x3
 * non-maximum suppression (dropped if an 8-neighbour corner scores >= their
 * own, nonmax_3x3.cpp:17-112), raster order, with their scores.  The NMS reads
 * a dense score map of the ROI (-1 = no corner) instead of the reference's row
 * pointers: O(corners), same survivors. */
int ygzo_fast10_detect_score_nms(const uint8_t *img, int w, int h, int stride, int barrier, int16_t *xs,
                                 int16_t *ys, int *scores, int cap) {
    if (w < 22 || h < 7) return -1;
    /* per-thread scratch kept across calls: the score map stays all -1 between
     * calls (only the written corners are reset), so a call costs O(corners) on
     * top of the scan, with no page faults */
    static __thread int16_t *map = NULL, *cx = NULL;
    static __thread size_t map_n = 0, c_n = 0;
    const size_t npx = (size_t)w * h;
    if (map_n < npx) {
        free(map);
        map = (int16_t *)malloc(sizeof(int16_t) * npx);
        for (size_t i = 0; i < npx; i++) map[i] = -1;
        map_n = npx;
    }
    const size_t ncap = npx / 2 + 16;
    if (c_n < ncap) {
        free(cx);
        cx = (int16_t *)malloc(sizeof(int16_t) * 3 * ncap);
        c_n = ncap;
    }
    int16_t *cy = cx + ncap, *ca = cy + ncap;
    int nc = fast10_rows(img, w, 3, h - 3, stride, barrier, cx, cy, ca, (int)ncap);
    if (nc > (int)ncap) nc = (int)ncap;
    for (int k = 0; k < nc; k++) {
        const int s = ca[k] - 1 > barrier ? ca[k] - 1 : barrier;
        ca[k] = (int16_t)s;
        map[(size_t)cy[k] * w + cx[k]] = (int16_t)s;
    }
    int n = 0;
    for (int k = 0; k < nc; k++) {
        const int16_t *r = map + (size_t)cy[k] * w + cx[k];
        const int s = r[0];
        if (r[-1] >= s || r[1] >= s || r[-w - 1] >= s || r[-w] >= s || r[-w + 1] >= s || r[w - 1] >= s || r[w] >= s ||
            r[w + 1] >= s)
            continue;
        if (n < cap) { xs[n] = cx[k]; ys[n] = cy[k]; scores[n] = s; }
        n++;
    }
    for (int k = 0; k < nc; k++) map[(size_t)cy[k] * w + cx[k]] = -1;
    return n;
}

/* fast_nonmax_3x3 (nonmax_3x3.cpp:17-112): a corner is dropped if any
 * 8-neighbour corner has score >= its own.  Returns kept indices. */
int ygzo_fast10_nonmax(const int16_t *xs, const int16_t *ys, const int *scores, int n, int *keep) {
    int nk = 0;
    for (int i = 0; i < n; i++) {
        int drop = 0;
        for (int j = 0; j < n && !drop; j++) {
            if (j == i) continue;
            int dx = xs[j] - xs[i], dy = ys[j] - ys[i];
            if (dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1 && scores[j] >= scores[i]) drop = 1;
        }
        if (!drop) keep[nk++] = i;
    }
    return nk;
}

/* ShiTomasiScore (ORBextractor.cc:1152-1187): float accumulation in raster
 * order (exact: integer-valued sums < 2^24); the /(2.0*area) divisions are
 * exact powers of two.  The discriminant (:1186) is evaluated as the
 * reference's own build compiles it (g++ -std=c++11 -O3 -march=native,
 * CMakeLists.txt:14; C++ keeps -ffp-contract=fast): two fused multiply-subs,
 * disc = fma(s, s, -(4 * fma(dXX, dYY, -(dXY * dXY)))).
 * tests/test_cpu_ref_arith.py pins this against that compiler and flags. */
float ygzo_shi_tomasi(const uint8_t *img, int w, int h, int stride, int u, int v) {
    float dXX = 0.0f, dYY = 0.0f, dXY = 0.0f;
    const int half = 4, box = 8, area = 64;
    const int x_min = u - half, x_max = u + half, y_min = v - half, y_max = v + half;
    if (x_min < 1 || x_max >= w - 1 || y_min < 1 || y_max >= h - 1) return 0.0f;
    for (int y = y_min; y < y_max; ++y) {
        const uint8_t *row = img + (size_t)y * stride;
        for (int x = 0; x < box; ++x) {
            float dx = (float)(row[x_min + x + 1] - row[x_min + x - 1]);
            float dy = (float)(img[(size_t)(y + 1) * stride + x_min + x] - img[(size_t)(y - 1) * stride + x_min + x]);
            dXX += dx * dx;
            dYY += dy * dy;
            dXY += dx * dy;
        }
    }
    dXX = (float)(dXX / (2.0 * area));
    dYY = (float)(dYY / (2.0 * area));
    dXY = (float)(dXY / (2.0 * area));
    float s = dXX + dYY;
    float disc = fmaf(s, s, -(4.0f * fmaf(dXX, dYY, -(dXY * dXY))));
    return (float)(0.5 * (double)(dXX + dYY - sqrtf(disc)));
}

typedef struct { int16_t x, y; float s; int ord; } cscore;
static int cmp_cscore(const void *a, const void *b) {
    const cscore *p = (const cscore *)a, *q = (const cscore *)b;
    if (p->s != q->s) return p->s > q->s ? -1 : 1; /* descending score */
    return p->ord - q->ord;                          /* ties: detection order */
}

/* ComputeKeyPointsDSOSingleLevel (ORBextractor.cc:1275-1386).
 * std::sort (unstable) is replaced by a sort whose ties keep detection order. */
int ygzo_dso_single_level(ygzo_orb *o, uint8_t **levels, const int *lw, const int *lh,
                          ygzo_kp *exist, int n_exist, ygzo_kp *out, int cap) {
    const uint8_t *img = levels[0];
    const int w = lw[0], h = lh[0];
    uint8_t *occ = (uint8_t *)calloc((size_t)w * h, 1);
    for (int i = 0; i < n_exist; i++) {
        int yy = (int)lrintf(exist[i].y), xx = (int)lrintf(exist[i].x);
        if (yy >= 0 && yy < h && xx >= 0 && xx < w) occ[(size_t)yy * w + xx] = 255;
    }
    const int n = o->nfeatures;
    if (o->dso_grid < 0) o->dso_grid = (int)sqrt(1.0 * h * w / n);
    int cnt = 0, nout = 0;
    int16_t xs[4096], ys[4096];
    cscore cs[4096];
    while (cnt < n) {
        if (cnt > 0) {
            o->dso_grid -= 5;
            if (o->dso_grid < 7) { o->dso_grid = 7; break; }
        }
        nout = 0;
        const int g = o->dso_grid;
        const int rows = h / g, cols = w / g;
        cnt = 0;
        for (int k = 0; k < rows * cols; k++) {
            int nn = k / cols;
            if (nn == 0 || nn == rows - 1 || (k % cols) == 0 || (k + 1) % cols == 0) continue;
            int x_start = (k - nn * cols) * g, y_start = nn * g;
            const uint8_t *data = img + (size_t)y_start * w + x_start;
            int nc = ygzo_fast10_detect_sse2(data, g, g, w, 20, xs, ys, 4096);
            if (nc == 0) nc = ygzo_fast10_detect_sse2(data, g, g, w, 5, xs, ys, 4096);
            if (nc > 4096) nc = 4096;
            int ns = 0;
            for (int c = 0; c < nc; c++) {
                int x = xs[c] + x_start, y = ys[c] + y_start;
                if (x < 20 || y < 20 || x >= w - 20 || y >= h - 20) continue;
                if (occ[(size_t)y * w + x] == 255) continue;
                cs[ns].x = (int16_t)x; cs[ns].y = (int16_t)y;
                cs[ns].s = ygzo_shi_tomasi(img, w, h, w, x, y);
                if (isnan(cs[ns].s)) cs[ns].s = -3.4e38f; /* std::sort with NaN is undefined: NaN sorts last */
                cs[ns].ord = ns;
                ns++;
            }
            qsort(cs, ns, sizeof(cscore), cmp_cscore);
            int take = ns > 3 ? 3 : ns;
            for (int i = 0; i < take; i++) {
                ygzo_kp kp;
                kp.x = cs[i].x; kp.y = cs[i].y; kp.size = 7.f; kp.angle = -1.f;
                kp.response = 0.f; kp.octave = 0; kp.class_id = -1;
                kp.angle = ygzo_ic_angle(img, w, h, w, kp.x, kp.y, o->umax);
                if (nout < cap) out[nout] = kp;
                nout++;
                cnt++;
            }
        }
        if (cnt == 0) break; /* the reference loops forever on a corner-free image */
    }
    if (cnt > n) o->dso_grid += 5;
    for (int i = 0; i < n_exist; i++) {
        int oc = exist[i].octave;
        exist[i].angle = ygzo_ic_angle(levels[oc], lw[oc], lh[oc], lw[oc], exist[i].x * o->inv_scale[oc],
                                       exist[i].y * o->inv_scale[oc], o->umax);
    }
    free(occ);
    return nout;
}

/* ORBextractor::operator()(Frame*, ..., DSO_KEYPOINT) (ORBextractor.cc:1052-1127). */
int ygzo_extract_dso(ygzo_orb *o, uint8_t **levels, const int *lw, const int *lh,
                     ygzo_kp *existing, int n_existing, ygzo_kp *out_kps, uint8_t *out_desc,
                     int cap) {
    int capn = cap - n_existing > 0 ? cap - n_existing : 0;
    ygzo_kp *nk = (ygzo_kp *)malloc(sizeof(ygzo_kp) * (capn > 0 ? capn : 1));
    int nn = ygzo_dso_single_level(o, levels, lw, lh, existing, n_existing, nk, capn);
    int total = n_existing + nn;
    if (total > cap) { free(nk); return -1; }
    /* GaussianBlur of every level once (ORBextractor.cc:1079-1084), then the existing rows'
     * descriptors on their octave's blurred level (:1088-1099) and the new ones' on level 0 */
    uint8_t *blur[YGZO_MAX_LEVELS];
    for (int l = 0; l < o->nlevels; l++) {
        blur[l] = (uint8_t *)malloc((size_t)lw[l] * lh[l]);
        ygzo_gaussian_blur7(levels[l], lw[l], lh[l], lw[l], blur[l], lw[l], o->blur_variant);
    }
    for (int i = 0; i < n_existing; i++) {
        ygzo_kp t = existing[i];
        int oc = t.octave;
        t.x *= o->inv_scale[oc];
        t.y *= o->inv_scale[oc];
        ygzo_orb_descriptor(blur[oc], lw[oc], lh[oc], lw[oc], &t, out_desc + 32 * (size_t)i);
        out_kps[i] = existing[i];
    }
    for (int i = 0; i < nn; i++) {
        ygzo_orb_descriptor(blur[0], lw[0], lh[0], lw[0], &nk[i], out_desc + 32 * (size_t)(n_existing + i));
        out_kps[n_existing + i] = nk[i];
    }
    for (int l = 0; l < o->nlevels; l++) free(blur[l]);
    free(nk);
    return total;
}

/* ---------------- Hamming ---------------- */
/* DescriptorDistance (ORBmatcher.cc:1507-1523): popcount of 8 x u32 XOR. */
int ygzo_descriptor_distance(const uint8_t *a, const uint8_t *b) {
    int d = 0;
    for (int i = 0; i < 32; i += 4) {
        uint32_t x, y;
        memcpy(&x, a + i, 4);
        memcpy(&y, b + i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

void ygzo_hamming_best2(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *best_idx,
                        int32_t *best_dist, int32_t *second_dist) {
    for (int i = 0; i < nq; i++) {
        int b1 = 256 + 1, b2 = 256 + 1, bi = -1;
        for (int j = 0; j < nt; j++) {
            int d = ygzo_descriptor_distance(q + 32 * (size_t)i, t + 32 * (size_t)j);
            if (d < b1) { b2 = b1; b1 = d; bi = j; }
            else if (d < b2) b2 = d;
        }
        best_idx[i] = bi;
        best_dist[i] = b1;
        second_dist[i] = b2;
    }
}
