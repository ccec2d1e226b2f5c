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

int ygzo_fast10_detect_sse2(const uint8_t *img, int w, int h, int stride, int barrier,
                            int16_t *xs, int16_t *ys, int cap) {
    if (w < 22) return ygzo_fast10_detect_plain(img, w, h, stride, barrier, xs, ys, cap);
    if (h < 7) return 0;
    int n = 0; /* faster_corner_10_sse.cpp:24-183: rows [3,h-3), cols [3,w-3) */
    for (int y = 3; y < h - 3; y++)
        for (int x = 3; x < w - 3; x++)
            if (ygzo_fast10_is_corner(img + (size_t)y * stride + x, stride, barrier)) {
                if (n < cap) { xs[n] = (int16_t)x; ys[n] = (int16_t)y; }
                n++;
            }
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
    for (int i = 0; i < n_existing; i++) {
        ygzo_kp t = existing[i];
        int oc = t.octave;
        uint8_t *blur = (uint8_t *)malloc((size_t)lw[oc] * lh[oc]);
        ygzo_gaussian_blur7(levels[oc], lw[oc], lh[oc], lw[oc], blur, lw[oc], o->blur_variant);
        t.x *= o->inv_scale[oc];
        t.y *= o->inv_scale[oc];
        ygzo_orb_descriptor(blur, lw[oc], lh[oc], lw[oc], &t, out_desc + 32 * (size_t)i);
        out_kps[i] = existing[i];
        free(blur);
    }
    uint8_t *blur0 = (uint8_t *)malloc((size_t)lw[0] * lh[0]);
    ygzo_gaussian_blur7(levels[0], lw[0], lh[0], lw[0], blur0, lw[0], o->blur_variant);
    for (int i = 0; i < nn; i++) {
        ygzo_orb_descriptor(blur0, lw[0], lh[0], lw[0], &nk[i], out_desc + 32 * (size_t)(n_existing + i));
        out_kps[n_existing + i] = nk[i];
    }
    free(blur0);
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
