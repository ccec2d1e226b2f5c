/*
 * orb.c — CPU restatement of ORBextractor (ORB-SLAM octree mode).
 * TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline); see ygz_oracle.h.
 *
 * Build with -ffp-contract=off: every float expression below is evaluated as
 * written (no FMA contraction), which is the arithmetic the HIP kernels use.
 * Where the reference's own build (g++ -std=c++11 -O3 -march=native,
 * CMakeLists.txt:14) fuses a multiply-add, the restatement writes the fma
 * explicitly (rBRIEF sample coordinates; tests/test_cpu_ref_arith.py pins it).
 */
#include "ygz_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

static const int kPattern[256 * 4] = {
#include "../include/ygzfe_pattern.inc"
};

const int *ygzo_bit_pattern(void) { return kPattern; }

enum { PATCH_SIZE = 31, HALF_PATCH_SIZE = 15, EDGE_THRESHOLD = 19 };

/* cvRound: round half to even (SSE cvtss2si in the default MXCSR mode). */
static inline int cv_round_f(float v) { return (int)lrintf(v); }
static inline int cv_round_d(double v) { return (int)lrint(v); }
static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* ORBextractor::ORBextractor (ORBextractor.cc:412-470). */
void ygzo_orb_init(ygzo_orb *o, int nfeatures, float scale_factor, int nlevels, int ini_th,
                   int min_th, int blur_variant) {
    memset(o, 0, sizeof(*o));
    o->nfeatures = nfeatures;
    o->scale_factor = (double)scale_factor;
    o->nlevels = nlevels;
    o->ini_th = ini_th;
    o->min_th = min_th;
    o->blur_variant = blur_variant;
    o->scale[0] = 1.0f;
    o->sigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
        o->scale[i] = (float)((double)o->scale[i - 1] * o->scale_factor); /* :421 float*double */
        o->sigma2[i] = o->scale[i] * o->scale[i];
    }
    for (int i = 0; i < nlevels; i++) {
        o->inv_scale[i] = 1.0f / o->scale[i];
        o->inv_sigma2[i] = 1.0f / o->sigma2[i];
    }
    /* :435-445 feature budget per level */
    float factor = (float)(1.0 / o->scale_factor);
    float desired = (float)nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        o->feat_per_level[l] = cv_round_f(desired);
        sum += o->feat_per_level[l];
        desired *= factor;
    }
    o->feat_per_level[nlevels - 1] = nfeatures - sum > 0 ? nfeatures - sum : 0;
    /* :453-467 umax circle table */
    int vmax = (int)floorf(HALF_PATCH_SIZE * sqrtf(2.f) / 2 + 1);
    int vmin = (int)ceilf(HALF_PATCH_SIZE * sqrtf(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    int v, v0;
    for (v = 0; v <= vmax; ++v) o->umax[v] = cv_round_d(sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (o->umax[v0] == o->umax[v0 + 1]) ++v0;
        o->umax[v] = v0;
        ++v0;
    }
    o->dso_grid = -1;
}

void ygzo_level_sizes(const ygzo_orb *o, int W, int H, int *w, int *h) {
    for (int l = 0; l < o->nlevels; l++) {
        w[l] = cv_round_f((float)W * o->inv_scale[l]);
        h[l] = cv_round_f((float)H * o->inv_scale[l]);
    }
}

/*
 * cv::resize(src, dst, size, 0, 0, INTER_LINEAR) on CV_8UC1 (the call at
 * ORBextractor.cc:1139).  OpenCV promotes an exact x2 downscale to the
 * INTER_AREA fast path: dst = (a + b + c + d + 2) >> 2.  Otherwise the
 * fixed-point bilinear path with 11-bit coefficients; the vertical pass is
 * the scalar VResizeLinear/FixedPtCast rounding (b0*S0 + b1*S1 + 2^21) >> 22
 * for every pixel (SIMD builds of OpenCV round the bulk of a row through
 * (mulhi(S>>4,b) sums + 2) >> 2 instead: up to 1 LSB apart).
 */
void ygzo_resize(const uint8_t *src, int sw, int sh, int sstride, uint8_t *dst, int dw, int dh,
                 int dstride) {
    double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
    double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
    int iscale_x = (int)lrint(scale_x), iscale_y = (int)lrint(scale_y);
    int area_fast = fabs(scale_x - iscale_x) < DBL_EPSILON && fabs(scale_y - iscale_y) < DBL_EPSILON;
    if (area_fast && iscale_x == 2 && iscale_y == 2) {
        for (int y = 0; y < dh; y++) {
            const uint8_t *s0 = src + (size_t)(2 * y) * sstride, *s1 = s0 + sstride;
            uint8_t *d = dst + (size_t)y * dstride;
            for (int x = 0; x < dw; x++)
                d[x] = (uint8_t)((s0[2 * x] + s0[2 * x + 1] + s1[2 * x] + s1[2 * x + 1] + 2) >> 2);
        }
        return;
    }
    int *xofs = (int *)malloc(sizeof(int) * dw);
    short *ialpha = (short *)malloc(sizeof(short) * 2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        float c0 = 1.f - fx, c1 = fx;
        ialpha[2 * dx] = (short)clampi(cv_round_f(c0 * 2048), -32768, 32767);
        ialpha[2 * dx + 1] = (short)clampi(cv_round_f(c1 * 2048), -32768, 32767);
    }
    int *r0 = (int *)malloc(sizeof(int) * dw), *r1 = (int *)malloc(sizeof(int) * dw);
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)floorf(fy);
        fy -= sy;
        short b0 = (short)clampi(cv_round_f((1.f - fy) * 2048), -32768, 32767);
        short b1 = (short)clampi(cv_round_f(fy * 2048), -32768, 32767);
        int ya = clampi(sy, 0, sh - 1), yb = clampi(sy + 1, 0, sh - 1);
        const uint8_t *sa = src + (size_t)ya * sstride, *sb = src + (size_t)yb * sstride;
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (dx < xmax) {
                r0[dx] = sa[sx] * ialpha[2 * dx] + sa[sx + 1] * ialpha[2 * dx + 1];
                r1[dx] = sb[sx] * ialpha[2 * dx] + sb[sx + 1] * ialpha[2 * dx + 1];
            } else {
                r0[dx] = sa[sx] * 2048;
                r1[dx] = sb[sx] * 2048;
            }
        }
        uint8_t *d = dst + (size_t)dy * dstride;
        for (int dx = 0; dx < dw; dx++)
            d[dx] = (uint8_t)clampi((b0 * r0[dx] + b1 * r1[dx] + (1 << 21)) >> 22, 0, 255);
    }
    free(xofs); free(ialpha); free(r0); free(r1);
}

/* ComputePyramid (ORBextractor.cc:1129-1150) + Frame clone (Frame.cc:810-813). */
void ygzo_compute_pyramid(const ygzo_orb *o, const uint8_t *img, int W, int H, int stride,
                          uint8_t **levels) {
    int w[YGZO_MAX_LEVELS], h[YGZO_MAX_LEVELS];
    ygzo_level_sizes(o, W, H, w, h);
    for (int y = 0; y < H; y++) memcpy(levels[0] + (size_t)y * W, img + (size_t)y * stride, W);
    for (int l = 1; l < o->nlevels; l++)
        ygzo_resize(levels[l - 1], w[l - 1], h[l - 1], w[l - 1], levels[l], w[l], h[l], w[l]);
}

/* ------------------------------------------------------------------------ */
/* OpenCV FAST TYPE_9_16 (features2d/fast.cpp FAST_t<16>, cornerScore<16>):
 * the cv::FAST calls of ORBextractor.cc:765,768.                            */

static const int kRing16[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},  {3, -1},
                                   {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                   {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

static void ring_offsets(int stride, int pix[25]) {
    for (int k = 0; k < 16; k++) pix[k] = kRing16[k][0] + kRing16[k][1] * stride;
    for (int k = 16; k < 25; k++) pix[k] = pix[k - 16];
}

int ygzo_corner_score16(const uint8_t *ptr, int stride, int threshold) {
    int pix[25];
    ring_offsets(stride, pix);
    int v = ptr[0], d[25];
    for (int k = 0; k < 25; k++) d[k] = v - ptr[pix[k]];
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = d[k + 1] < d[k + 2] ? d[k + 1] : d[k + 2];
        if (d[k + 3] < a) a = d[k + 3];
        if (a <= a0) continue;
        for (int m = 4; m <= 8; m++) if (d[k + m] < a) a = d[k + m];
        int t = a < d[k] ? a : d[k];
        if (t > a0) a0 = t;
        t = a < d[k + 9] ? a : d[k + 9];
        if (t > a0) a0 = t;
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = d[k + 1] > d[k + 2] ? d[k + 1] : d[k + 2];
        for (int m = 3; m <= 5; m++) if (d[k + m] > b) b = d[k + m];
        if (b >= b0) continue;
        for (int m = 6; m <= 8; m++) if (d[k + m] > b) b = d[k + m];
        int t = b > d[k] ? b : d[k];
        if (t < b0) b0 = t;
        t = b > d[k + 9] ? b : d[k + 9];
        if (t < b0) b0 = t;
    }
    return -b0 - 1;
}

/* Segment test of FAST_t: >8 contiguous (of the 25-long wrapped ring) darker
 * than v-t, or brighter than v+t.  The opposite-pair screening in front is
 * FAST_t's own (fast.cpp: d = tab[p0] | tab[p8], &= the pairs 2/10, 4/12,
 * 6/14, then 1/9 .. 7/15): a necessary condition, so it only skips pixels the
 * full test rejects. */
static int fast9_test(const uint8_t *p, const int pix[25], int threshold) {
    int v = p[0];
    const int lo = v - threshold, hi = v + threshold;
#define YGZO_CLS(k) ((p[pix[k]] < lo ? 1 : 0) | (p[pix[k]] > hi ? 2 : 0))
    int d = YGZO_CLS(0) | YGZO_CLS(8);
    if (d == 0) return 0;
    d &= YGZO_CLS(2) | YGZO_CLS(10);
    d &= YGZO_CLS(4) | YGZO_CLS(12);
    d &= YGZO_CLS(6) | YGZO_CLS(14);
    if (d == 0) return 0;
    d &= YGZO_CLS(1) | YGZO_CLS(9);
    d &= YGZO_CLS(3) | YGZO_CLS(11);
    d &= YGZO_CLS(5) | YGZO_CLS(13);
    d &= YGZO_CLS(7) | YGZO_CLS(15);
#undef YGZO_CLS
    if (d == 0) return 0;
    int count = 0;
    if (d & 1) {
        for (int k = 0; k < 25; k++) {
            if (p[pix[k]] < lo) { if (++count > 8) return 1; }
            else count = 0;
        }
    }
    count = 0;
    if (d & 2) {
        for (int k = 0; k < 25; k++) {
            if (p[pix[k]] > hi) { if (++count > 8) return 1; }
            else count = 0;
        }
    }
    return 0;
}

/* The segment test on 16 consecutive pixels at once (GCC vector extensions:
 * int16 lanes, AVX2 / AVX-512 under -march=native), the form FAST_t's own SSE2
 * path takes: the compass points 0/4/8/12 screen the block, then the masks of
 * all 16 ring pixels and a run of 9 by doubling (runs of 2, 4, 8, then + 1).
 * Bit i of the result = fast9_test(p + i); the whole ring of every lane lies
 * inside the row window [p - 3, p + 18]. */
typedef int16_t ygzo_i16x16 __attribute__((vector_size(32)));
typedef uint8_t ygzo_u8x16 __attribute__((vector_size(16)));
static inline ygzo_i16x16 ld16(const uint8_t *p) {
    ygzo_u8x16 b;
    memcpy(&b, p, 16);
    return __builtin_convertvector(b, ygzo_i16x16);
}
static inline int any16(ygzo_i16x16 m) {
    uint64_t q[4];
    memcpy(q, &m, 32);
    return (q[0] | q[1] | q[2] | q[3]) != 0;
}
static inline ygzo_i16x16 vmin(ygzo_i16x16 a, ygzo_i16x16 b) {
    const ygzo_i16x16 m = a < b;
    return (a & m) | (b & ~m);
}
static inline ygzo_i16x16 vmax(ygzo_i16x16 a, ygzo_i16x16 b) {
    const ygzo_i16x16 m = a > b;
    return (a & m) | (b & ~m);
}
/* Also the 16 scores, cornerScore<16> in the closed form the GPU uses (checked
 * against ygzo_corner_score16 by tests/test_cpu_oracle_props.py): with
 * e_k = r_k - v, arcmax = max(max_k min e[k..k+8], max_k min -e[k..k+8]) by
 * min / max doubling; corner <=> arcmax > t, score = arcmax - 1. */
static unsigned fast9_test16(const uint8_t *p, const int pix[25], int threshold, int16_t score[16]) {
    const ygzo_i16x16 v = ld16(p);
    const ygzo_i16x16 lo = v - (int16_t)threshold, hi = v + (int16_t)threshold;
    ygzo_i16x16 e[16];
    for (int k = 0; k < 16; k += 4) e[k] = ld16(p + pix[k]);
    const ygzo_i16x16 scr = (((e[0] < lo) | (e[8] < lo)) & ((e[4] < lo) | (e[12] < lo))) |
                            (((e[0] > hi) | (e[8] > hi)) & ((e[4] > hi) | (e[12] > hi)));
    if (!any16(scr)) return 0u;
    for (int k = 0; k < 16; k++) {
        if (k & 3) e[k] = ld16(p + pix[k]);
        e[k] -= v;
    }
    ygzo_i16x16 n2[16], x2[16], n4[16], x4[16];
    for (int k = 0; k < 16; k++) { n2[k] = vmin(e[k], e[(k + 1) & 15]); x2[k] = vmax(e[k], e[(k + 1) & 15]); }
    for (int k = 0; k < 16; k++) { n4[k] = vmin(n2[k], n2[(k + 2) & 15]); x4[k] = vmax(x2[k], x2[(k + 2) & 15]); }
    ygzo_i16x16 bright = vmin(vmin(n4[0], n4[4]), e[8]), darkmin = vmax(vmax(x4[0], x4[4]), e[8]);
    for (int k = 1; k < 16; k++) {
        bright = vmax(bright, vmin(vmin(n4[k], n4[(k + 4) & 15]), e[(k + 8) & 15]));
        darkmin = vmin(darkmin, vmax(vmax(x4[k], x4[(k + 4) & 15]), e[(k + 8) & 15]));
    }
    const ygzo_i16x16 am = vmax(bright, -darkmin);
    const ygzo_i16x16 c = am > (int16_t)threshold;
    if (!any16(c)) return 0u;
    unsigned m = 0;
    for (int i = 0; i < 16; i++) {
        m |= (unsigned)(c[i] != 0) << i;
        score[i] = (int16_t)(am[i] - 1);
    }
    return m;
}

/* 0: the 16-pixel vector segment test (default), 1: scalar only (test hook) */
static int g_fast_scalar = 0;
void ygzo_fast9_force_scalar(int on) { g_fast_scalar = on; }

int ygzo_fast9_roi(const uint8_t *roi, int w, int h, int stride, int threshold, int16_t *xs,
                   int16_t *ys, uint8_t *scores, int cap) {
    if (threshold < 0) threshold = 0;
    if (threshold > 255) threshold = 255;
    int pix[25];
    ring_offsets(stride, pix);
    /* score map over the ROI, 0 where no corner (FAST_t's row buffers), and the
     * corner positions in raster order (the NMS visits only those) */
    uint8_t sc_stack[96 * 96];
    int32_t pos_stack[1024];
    const size_t npx = (size_t)w * h;
    uint8_t *sc = npx <= sizeof(sc_stack) ? sc_stack : (uint8_t *)malloc(npx);
    int32_t *pos = npx <= 1024 ? pos_stack : (int32_t *)malloc(sizeof(int32_t) * npx);
    memset(sc, 0, npx);
    int nc = 0;
    for (int y = 3; y < h - 3; y++) {
        int x = 3;
        if (!g_fast_scalar)
            for (; x + 16 <= w - 3; x += 16) {  /* ring of lane 15: columns x + 12 .. x + 18 <= w - 1 */
                const uint8_t *p = roi + (size_t)y * stride + x;
                int16_t s16[16];
                unsigned m = fast9_test16(p, pix, threshold, s16);
                while (m) {
                    const int i = __builtin_ctz(m);
                    m &= m - 1;
                    sc[(size_t)y * w + x + i] = (uint8_t)s16[i];
                    pos[nc++] = y * w + x + i;
                }
            }
        if (!g_fast_scalar && x < w - 3 && w - 19 >= 3) {  /* the tail: one block ending at column w - 4 */
            const int xb = w - 19;
            const uint8_t *p = roi + (size_t)y * stride + xb;
            int16_t s16[16];
            unsigned m = fast9_test16(p, pix, threshold, s16) & (0xFFFFu << (x - xb));
            while (m) {
                const int i = __builtin_ctz(m);
                m &= m - 1;
                sc[(size_t)y * w + xb + i] = (uint8_t)s16[i];
                pos[nc++] = y * w + xb + i;
            }
            x = w - 3;
        }
        for (; x < w - 3; x++) {
            const uint8_t *p = roi + (size_t)y * stride + x;
            if (fast9_test(p, pix, threshold)) {
                int s = ygzo_corner_score16(p, stride, threshold);
                sc[(size_t)y * w + x] = (uint8_t)s; /* uchar cast as in FAST_t */
                pos[nc++] = y * w + x;
            }
        }
    }
    /* nonmax: strictly greater than all 8 neighbours; raster order */
    int n = 0;
    for (int k = 0; k < nc; k++) {
        const uint8_t *r = sc + pos[k];
        const int s = r[0];
        if (!s) continue; /* a corner with score 0 can never survive the strict test */
        if (s > r[-1] && s > r[1] && s > r[-w - 1] && s > r[-w] && s > r[-w + 1] &&
            s > r[w - 1] && s > r[w] && s > r[w + 1]) {
            if (n < cap) {
                xs[n] = (int16_t)(pos[k] % w);
                ys[n] = (int16_t)(pos[k] / w);
                scores[n] = (uint8_t)s;
            }
            n++;
        }
    }
    if (pos != pos_stack) free(pos);
    if (sc != sc_stack) free(sc);
    return n;
}

/* ------------------------------------------------------------------------ */
/* DistributeOctTree (ORBextractor.cc:533-723) with ExtractorNode::DivideNode
 * (:479-531).  The std::list is a pool-backed doubly linked list; the node
 * "pointer" used as the sort tie-break (:656) is the node's creation order.  */

typedef struct onode {
    int x0, y0, x1, y1;       /* UL=(x0,y0) UR=(x1,y0) BL=(x0,y1) BR=(x1,y1) */
    int *keys, nkeys;         /* indices into the candidate array, in order */
    int no_more;
    int prev, next;           /* list links (-1 = none) */
    int seq;                  /* creation order = pointer order */
} onode;

typedef struct olist {
    onode *pool;
    int npool, cap;
    int head, size, seq;
} olist;

static int ol_new(olist *L, int x0, int y0, int x1, int y1) {
    if (L->npool == L->cap) {
        L->cap = L->cap ? 2 * L->cap : 64;
        L->pool = (onode *)realloc(L->pool, sizeof(onode) * L->cap);
    }
    onode *n = &L->pool[L->npool];
    n->x0 = x0; n->y0 = y0; n->x1 = x1; n->y1 = y1;
    n->keys = NULL; n->nkeys = 0; n->no_more = 0;
    n->prev = n->next = -1;
    n->seq = L->seq++;
    return L->npool++;
}

static void ol_push_front(olist *L, int id) {
    onode *n = &L->pool[id];
    n->prev = -1;
    n->next = L->head;
    if (L->head >= 0) L->pool[L->head].prev = id;
    L->head = id;
    L->size++;
}

/* returns the next node id (like list::erase) */
static int ol_erase(olist *L, int id) {
    onode *n = &L->pool[id];
    int nx = n->next;
    if (n->prev >= 0) L->pool[n->prev].next = n->next; else L->head = n->next;
    if (n->next >= 0) L->pool[n->next].prev = n->prev;
    L->size--;
    return nx;
}

static void divide_node(olist *L, int pid, const ygzo_kp *kps, int child[4]) {
    onode p = L->pool[pid]; /* copy: pool may be reallocated below */
    const int halfX = (int)ceilf((float)(p.x1 - p.x0) / 2);
    const int halfY = (int)ceilf((float)(p.y1 - p.y0) / 2);
    int mx = p.x0 + halfX, my = p.y0 + halfY;
    int bx[4][4] = {{p.x0, p.y0, mx, my}, {mx, p.y0, p.x1, my}, {p.x0, my, mx, p.y1}, {mx, my, p.x1, p.y1}};
    int *buf[4], cnt[4] = {0, 0, 0, 0};
    for (int c = 0; c < 4; c++) buf[c] = (int *)malloc(sizeof(int) * (p.nkeys > 0 ? p.nkeys : 1));
    for (int i = 0; i < p.nkeys; i++) {
        const ygzo_kp *kp = &kps[p.keys[i]];
        int c;
        if (kp->x < (float)mx) c = kp->y < (float)my ? 0 : 2;
        else c = kp->y < (float)my ? 1 : 3;
        buf[c][cnt[c]++] = p.keys[i];
    }
    for (int c = 0; c < 4; c++) {
        child[c] = -1;
        if (cnt[c] > 0) {
            int id = ol_new(L, bx[c][0], bx[c][1], bx[c][2], bx[c][3]);
            L->pool[id].keys = buf[c];
            L->pool[id].nkeys = cnt[c];
            L->pool[id].no_more = cnt[c] == 1;
            child[c] = id;
        } else {
            free(buf[c]);
        }
    }
}

typedef struct { int size, seq, id; } sizeptr;
static int cmp_sizeptr(const void *a, const void *b) {
    const sizeptr *x = (const sizeptr *)a, *y = (const sizeptr *)b;
    if (x->size != y->size) return x->size < y->size ? -1 : 1;
    return x->seq < y->seq ? -1 : (x->seq > y->seq);
}

int ygzo_distribute_octree(const ygzo_kp *keys, int n, int minX, int maxX, int minY, int maxY,
                           int N, ygzo_kp *out, int cap) {
    olist L = {0};
    L.head = -1;
    int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
    if (nIni < 1) nIni = 1; /* reference UB for w/h < 0.5 neutralised */
    const float hX = (float)(maxX - minX) / nIni;
    int *ini = (int *)malloc(sizeof(int) * nIni);
    /* push_back of the initial nodes: build then link in order */
    for (int i = 0; i < nIni; i++) {
        ini[i] = ol_new(&L, (int)(hX * (float)i), 0, (int)(hX * (float)(i + 1)), maxY - minY);
        L.pool[ini[i]].keys = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    }
    for (int i = nIni - 1; i >= 0; i--) ol_push_front(&L, ini[i]);
    for (int i = 0; i < n; i++) {
        int idx = (int)(keys[i].x / hX);
        if (idx >= nIni) idx = nIni - 1; /* not reachable for octree candidates */
        onode *nd = &L.pool[ini[idx]];
        nd->keys[nd->nkeys++] = i;
    }
    free(ini);
    for (int it = L.head; it >= 0;) {
        onode *nd = &L.pool[it];
        if (nd->nkeys == 1) { nd->no_more = 1; it = nd->next; }
        else if (nd->nkeys == 0) it = ol_erase(&L, it);
        else it = nd->next;
    }

    int finish = 0;
    sizeptr *vsp = NULL, *vprev = NULL;
    int nvsp = 0, capvsp = 0;
#define VSP_PUSH(sz, nid)                                                             \
    do {                                                                              \
        if (nvsp == capvsp) {                                                         \
            capvsp = capvsp ? 2 * capvsp : 64;                                        \
            vsp = (sizeptr *)realloc(vsp, sizeof(sizeptr) * capvsp);                  \
        }                                                                             \
        vsp[nvsp].size = (sz); vsp[nvsp].seq = L.pool[(nid)].seq; vsp[nvsp].id = (nid); \
        nvsp++;                                                                       \
    } while (0)

    while (!finish) {
        int prevSize = L.size;
        int nToExpand = 0;
        nvsp = 0;
        for (int it = L.head; it >= 0;) {
            if (L.pool[it].no_more) { it = L.pool[it].next; continue; }
            int ch[4];
            divide_node(&L, it, keys, ch);
            for (int c = 0; c < 4; c++) {
                if (ch[c] < 0) continue;
                ol_push_front(&L, ch[c]);
                if (L.pool[ch[c]].nkeys > 1) { nToExpand++; VSP_PUSH(L.pool[ch[c]].nkeys, ch[c]); }
            }
            it = ol_erase(&L, it);
        }
        if (L.size >= N || L.size == prevSize) {
            finish = 1;
        } else if (L.size + nToExpand * 3 > N) {
            while (!finish) {
                prevSize = L.size;
                int nprev = nvsp;
                vprev = (sizeptr *)realloc(vprev, sizeof(sizeptr) * (nprev > 0 ? nprev : 1));
                memcpy(vprev, vsp, sizeof(sizeptr) * nprev);
                nvsp = 0;
                qsort(vprev, nprev, sizeof(sizeptr), cmp_sizeptr);
                for (int j = nprev - 1; j >= 0; j--) {
                    int ch[4];
                    divide_node(&L, vprev[j].id, keys, ch);
                    for (int c = 0; c < 4; c++) {
                        if (ch[c] < 0) continue;
                        ol_push_front(&L, ch[c]);
                        if (L.pool[ch[c]].nkeys > 1) VSP_PUSH(L.pool[ch[c]].nkeys, ch[c]);
                    }
                    ol_erase(&L, vprev[j].id);
                    if (L.size >= N) break;
                }
                if (L.size >= N || L.size == prevSize) finish = 1;
            }
        }
    }
#undef VSP_PUSH
    int nout = 0;
    for (int it = L.head; it >= 0; it = L.pool[it].next) {
        const onode *nd = &L.pool[it];
        int best = nd->keys[0];
        float maxr = keys[best].response;
        for (int k = 1; k < nd->nkeys; k++)
            if (keys[nd->keys[k]].response > maxr) { best = nd->keys[k]; maxr = keys[best].response; }
        if (nout < cap) out[nout] = keys[best];
        nout++;
    }
    for (int i = 0; i < L.npool; i++) free(L.pool[i].keys);
    free(L.pool); free(vsp); free(vprev);
    return nout;
}

/* ComputeKeyPointsOctTree, one level (ORBextractor.cc:725-799). */
int ygzo_octree_level(const ygzo_orb *o, const uint8_t *lvl, int w, int h, int level,
                      ygzo_kp *out, int cap, int *n_candidates) {
    const float W = 30;
    const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
    const int maxBorderX = w - EDGE_THRESHOLD + 3, maxBorderY = h - EDGE_THRESHOLD + 3;
    const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    int ncand = 0, capc = 1024;
    ygzo_kp *cand = (ygzo_kp *)malloc(sizeof(ygzo_kp) * capc);
    if (nCols > 0 && nRows > 0) { /* nRows==0 divides by zero in the reference; no cells either way */
        const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
        int16_t xs[64 * 64], ys[64 * 64];
        uint8_t sc[64 * 64];
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(minBorderY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minBorderX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                int y0 = (int)iniY, x0 = (int)iniX, rh = (int)maxY - y0, rw = (int)maxX - x0;
                const uint8_t *roi = lvl + (size_t)y0 * w + x0;
                int capcell = (int)(sizeof(sc));
                int nc = ygzo_fast9_roi(roi, rw, rh, w, o->ini_th, xs, ys, sc, capcell);
                if (nc == 0) nc = ygzo_fast9_roi(roi, rw, rh, w, o->min_th, xs, ys, sc, capcell);
                for (int k = 0; k < nc; k++) {
                    if (ncand == capc) { capc *= 2; cand = (ygzo_kp *)realloc(cand, sizeof(ygzo_kp) * capc); }
                    ygzo_kp *kp = &cand[ncand++];
                    kp->x = (float)xs[k] + (float)(j * wCell);
                    kp->y = (float)ys[k] + (float)(i * hCell);
                    kp->size = 7.f; kp->angle = -1.f; kp->response = (float)sc[k];
                    kp->octave = 0; kp->class_id = -1;
                }
            }
        }
    }
    if (n_candidates) *n_candidates = ncand;
    int n = ygzo_distribute_octree(cand, ncand, minBorderX, maxBorderX, minBorderY, maxBorderY,
                                   o->feat_per_level[level], out, cap);
    free(cand);
    const int scaledPatchSize = (int)(PATCH_SIZE * o->scale[level]);
    for (int i = 0; i < n && i < cap; i++) {
        out[i].x += minBorderX;
        out[i].y += minBorderY;
        out[i].octave = level;
        out[i].size = (float)scaledPatchSize;
    }
    return n;
}

/* ------------------------------------------------------------------------ */
/* cv::fastAtan2 (core/mathfuncs: 7th-order polynomial, degrees in [0,360)). */
float ygzo_fast_atan2(float y, float x) {
    const float k = (float)(180 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    float ax = fabsf(x), ay = fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* IC_Angle (ORBextractor.cc:77-101).  Pixel reads are clamped to the image
 * (the reference reads out of bounds for keypoints nearer than 15 px to the
 * edge; never the case for octree/DSO keypoints). */
float ygzo_ic_angle(const uint8_t *img, int w, int h, int stride, float x, float y,
                    const int *umax) {
    int cx = cv_round_f(x), cy = cv_round_f(y);
#define PIX(yy, xx) img[(size_t)clampi((yy), 0, h - 1) * stride + clampi((xx), 0, w - 1)]
    int m01 = 0, m10 = 0;
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m10 += u * PIX(cy, cx + u);
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int vsum = 0, d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int vp = PIX(cy + v, cx + u), vm = PIX(cy - v, cx + u);
            vsum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * vsum;
    }
#undef PIX
    return ygzo_fast_atan2((float)m01, (float)m10);
}

/*
 * GaussianBlur(src, dst, Size(7,7), 2, 2, BORDER_REFLECT_101) on CV_8UC1
 * (ORBextractor.cc:1010,1083), as 8-bit fixed-point separable filtering:
 *   dst = sat8((sum_v k[v] * (sum_h k[h] * p) + 2^15) >> 16)
 * CV4 (bit-exact GaussianBlurFixedPoint, OpenCV >= 3.4.2/4.x): error-diffused
 * kernel [18,34,48,56,48,34,18]; CV3: cvRound(k*256) = [18,34,49,55,49,34,18]
 * with the FixedPtCastEx rounding of the scalar column filter.
 */
static const int kBlurCV4[7] = {18, 34, 48, 56, 48, 34, 18};
static const int kBlurCV3[7] = {18, 34, 49, 55, 49, 34, 18};

static inline int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

/* The two separable passes on 16-pixel vectors, as OpenCV's SIMD fixed-point
 * path runs them: the horizontal sums fit uint16 exactly (<= 257 * 255 = 65535),
 * the vertical sums int32 (<= 257 * 65535 + 32768 < 2^31).  Same integer sums as
 * the scalar form, so the same bytes.  Per-thread row scratch kept across calls. */
typedef uint16_t ygzo_u16x16 __attribute__((vector_size(32)));
typedef int32_t ygzo_i32x16 __attribute__((vector_size(64)));
void ygzo_gaussian_blur7(const uint8_t *src, int w, int h, int stride, uint8_t *dst,
                         int dstride, int variant) {
    const int *k = variant == YGZO_BLUR_CV3_ROUNDED ? kBlurCV3 : kBlurCV4;
    static __thread uint16_t *rows = NULL;
    static __thread size_t rows_n = 0;
    const size_t need = (size_t)w * h + 16;
    if (rows_n < need) {
        free(rows);
        rows = (uint16_t *)malloc(sizeof(uint16_t) * need);
        rows_n = need;
    }
    /* horizontal pass: border columns through reflect101, the interior on vectors */
    for (int y = 0; y < h; y++) {
        const uint8_t *s = src + (size_t)y * stride;
        uint16_t *r = rows + (size_t)y * w;
        for (int x = 0; x < w; x++) {
            if (x == 3 && w - 3 > 3) x = w - 3;  /* the interior is done below */
            int acc = 0;
            for (int t = 0; t < 7; t++) acc += k[t] * s[reflect101(x + t - 3, w)];
            r[x] = (uint16_t)acc;
        }
        int x = 3;
        for (; x + 16 <= w - 3; x += 16) {  /* symmetric kernel: k[t] = k[6 - t] */
            ygzo_u16x16 px[7];
            for (int t = 0; t < 7; t++) {
                ygzo_u8x16 b;
                memcpy(&b, s + x + t - 3, 16);
                px[t] = __builtin_convertvector(b, ygzo_u16x16);
            }
            const ygzo_u16x16 acc = (px[0] + px[6]) * (uint16_t)k[0] + (px[1] + px[5]) * (uint16_t)k[1] +
                                    (px[2] + px[4]) * (uint16_t)k[2] + px[3] * (uint16_t)k[3];
            memcpy(r + x, &acc, 32);
        }
        for (; x < w - 3; x++)
            r[x] = (uint16_t)(k[0] * s[x - 3] + k[1] * s[x - 2] + k[2] * s[x - 1] + k[3] * s[x] + k[4] * s[x + 1] +
                              k[5] * s[x + 2] + k[6] * s[x + 3]);
    }
    /* vertical pass: 7 row pointers (reflect101 at the top / bottom) */
    for (int y = 0; y < h; y++) {
        const uint16_t *rr[7];
        for (int t = 0; t < 7; t++) rr[t] = rows + (size_t)reflect101(y + t - 3, h) * w;
        uint8_t *o = dst + (size_t)y * dstride;
        int x = 0;
        for (; x + 16 <= w; x += 16) {
            ygzo_i32x16 v[7];
            for (int t = 0; t < 7; t++) {
                ygzo_u16x16 u;
                memcpy(&u, rr[t] + x, 32);
                v[t] = __builtin_convertvector(u, ygzo_i32x16);
            }
            ygzo_i32x16 acc = (v[0] + v[6]) * k[0] + (v[1] + v[5]) * k[1] + (v[2] + v[4]) * k[2] + v[3] * k[3];
            acc = (acc + 32768) >> 16;
            const ygzo_i32x16 big = acc > 255;  /* CV3's sum-257 kernel can reach 257 (saturate_cast) */
            acc = (acc & ~big) | (255 & big);
            const ygzo_u8x16 ob = __builtin_convertvector(acc, ygzo_u8x16);
            memcpy(o + x, &ob, 16);
        }
        for (; x < w; x++) {
            const int acc = k[0] * rr[0][x] + k[1] * rr[1][x] + k[2] * rr[2][x] + k[3] * rr[3][x] +
                            k[4] * rr[4][x] + k[5] * rr[5][x] + k[6] * rr[6][x];
            o[x] = (uint8_t)clampi((acc + 32768) >> 16, 0, 255);
        }
    }
}

/*
 * glibc's single-precision sin/cos (glibc >= 2.28: sysdeps/ieee754/flt-32
 * s_sinf.c / s_cosf.c / s_sincosf.c with sincosf.h and s_sincosf_data.c, the
 * double-evaluated "ARM optimized-routines" algorithm), restated for the
 * argument range rBRIEF uses: angle * pi/180 with angle = fastAtan2 in
 * [0, 360), i.e. |y| < 120 (the large-argument reduction is not needed).
 *   computeOrbDescriptor does `float angle; cos(angle), sin(angle)` under
 *   `using namespace std` (ORBextractor.cc:68-69, 108-109): std::cos(float) =
 *   cosf / sinf of the C library (g++ -O3 merges the pair into one sincosf
 *   call; sincosf_poly and sinf_poly are the same arithmetic).
 * Pinned to this image's glibc 2.35 (x86-64; the FMA and non-FMA ifunc
 * variants agree on [0, 2pi)): tests/test_cpu_ref_arith.py compares every
 * float in [0, 2pi) bit for bit with libm's cosf / sinf.
 */
typedef struct {
    double sign[4];               /* sign of the sine per quadrant */
    double hpi_inv, hpi;          /* 2/pi * 2^24 (no TOINT intrinsics on x86-64), pi/2 */
    double c0, c1, c2, c3, c4;    /* cosine polynomial */
    double s1, s2, s3;            /* sine polynomial */
} glibc_sincos_t;

static const glibc_sincos_t kSinCos[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0,
     0x1p0, -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0,
     -0x1p0, 0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
};

static inline uint32_t abstop12(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return (u >> 20) & 0x7ff;
}

/* sinf_poly (sincosf.h): odd n -> the cosine polynomial, even n -> the sine one */
static inline float glibc_sinf_poly(double x, double x2, const glibc_sincos_t *p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = p->s2 + x2 * p->s3;
        double x7 = x3 * x2;
        double s = x + x3 * p->s1;
        return (float)(s + x7 * s1);
    }
    double x4 = x2 * x2;
    double c2 = p->c3 + x2 * p->c4;
    double c1 = p->c0 + x2 * p->c1;
    double x6 = x4 * x2;
    double c = c1 + x4 * p->c2;
    return (float)(c + x6 * c2);
}

/* 4/pi bits, a sliding window of 24 words (s_sincosf_data.c __inv_pio4). */
static const uint32_t kInvPio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041,
};

/* reduce_large (sincosf.h): |y| >= 120, integer multiply by 4/pi bits. */
static inline double glibc_reduce_large(uint32_t xi, int *np) {
    const uint32_t *arr = &kInvPio4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = (uint64_t)(uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * 0x1.921FB54442D18p-62; /* pi * 2^-63 */
}

void ygzo_sincosf(float y, float *sinp, float *cosp) {
    const glibc_sincos_t *p = &kSinCos[0];
    double x = y;
    if (abstop12(y) >= abstop12(120.0f)) {
        if (!(fabsf(y) <= FLT_MAX)) { /* inf / nan: __math_invalidf */
            *sinp = *cosp = (y - y) / (y - y);
            return;
        }
        uint32_t xi;
        memcpy(&xi, &y, 4);
        int sign = xi >> 31, n;
        x = glibc_reduce_large(xi, &n);
        double s = p->sign[(n + sign) & 3];
        if ((n + sign) & 2) p = &kSinCos[1];
        *sinp = glibc_sinf_poly(x * s, x * x, p, n);
        *cosp = glibc_sinf_poly(x * s, x * x, p, n ^ 1);
        return;
    }
    if (abstop12(y) < abstop12((float)0x1.921FB54442D18p-1)) { /* |y| < pi/4 (top-12-bit compare) */
        if (abstop12(y) < abstop12(0x1p-12f)) {
            *sinp = y;
            *cosp = 1.0f;
            return;
        }
        double x2 = x * x;
        *sinp = glibc_sinf_poly(x, x2, p, 0);
        *cosp = glibc_sinf_poly(x, x2, p, 1);
        return;
    }
    /* reduce_fast: quadrant from the 2^24-prescaled product, truncating conversion */
    double r = x * p->hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * p->hpi;
    double s = p->sign[n & 3];
    if (n & 2) p = &kSinCos[1];
    *sinp = glibc_sinf_poly(x * s, x * x, p, n);
    *cosp = glibc_sinf_poly(x * s, x * x, p, n ^ 1);
}

/* Test hook: restated sincosf vs this process's libm sinf / cosf over the float
 * bit patterns [lo, hi); returns the number of inputs where either differs. */
int64_t ygzo_sincosf_sweep(uint32_t lo, uint32_t hi) {
    int64_t bad = 0;
    for (uint32_t u = lo; u < hi; u++) {
        float y, s, c;
        memcpy(&y, &u, 4);
        ygzo_sincosf(y, &s, &c);
        volatile float ls = sinf(y), lc = cosf(y);
        float lsv = ls, lcv = lc;
        bad += memcmp(&s, &lsv, 4) != 0 || memcmp(&c, &lcv, 4) != 0;
    }
    return bad;
}

/* Test hook: the 512 rotated sample offsets (row, column) GET_VALUE reads for
 * a keypoint angle (ORBextractor.cc:108-116), as ygzo_orb_descriptor forms them. */
void ygzo_orb_sample_offsets(float angle_deg, int *dy, int *dx) {
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float a, b;
    ygzo_sincosf(angle_deg * factorPI, &b, &a);
    for (int j = 0; j < 512; j++) {
        float px = (float)kPattern[2 * j], py = (float)kPattern[2 * j + 1];
        dy[j] = cv_round_f(fmaf(px, b, py * a));
        dx[j] = cv_round_f(fmaf(px, a, -(py * b)));
    }
}

/* computeOrbDescriptor (ORBextractor.cc:105-149).  (a, b) = glibc cosf / sinf
 * of the float angle (ygzo_sincosf above).  GET_VALUE (:114-116) as g++
 * -O3 -march=native compiles it: the first product fused into the add / sub,
 * y = fma(x, b, y*a), x = fma(x, a, -(y*b)); cvRound = round half even.
 * Sample coordinates are clamped to the image (out-of-bounds reads in the
 * reference are UB). */
void ygzo_orb_descriptor(const uint8_t *img, int w, int h, int stride, const ygzo_kp *kp,
                         uint8_t desc[32]) {
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float angle = kp->angle * factorPI;
    float a, b;
    ygzo_sincosf(angle, &b, &a);
    int cx = cv_round_f(kp->x), cy = cv_round_f(kp->y);
    const int *pat = kPattern;
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int k = 0; k < 8; k++) {
            const int *p = pat + (i * 8 + k) * 4;
            float px0 = (float)p[0], py0 = (float)p[1], px1 = (float)p[2], py1 = (float)p[3];
            int y0 = cy + cv_round_f(fmaf(px0, b, py0 * a)), x0 = cx + cv_round_f(fmaf(px0, a, -(py0 * b)));
            int y1 = cy + cv_round_f(fmaf(px1, b, py1 * a)), x1 = cx + cv_round_f(fmaf(px1, a, -(py1 * b)));
            int t0 = img[(size_t)clampi(y0, 0, h - 1) * stride + clampi(x0, 0, w - 1)];
            int t1 = img[(size_t)clampi(y1, 0, h - 1) * stride + clampi(x1, 0, w - 1)];
            val |= (t0 < t1) << k;
        }
        desc[i] = (uint8_t)val;
    }
}

/* ORBextractor::operator()(Frame*, ..., ORBSLAM_KEYPOINT) (ORBextractor.cc:1031-1127). */
int ygzo_extract_orbslam(ygzo_orb *o, uint8_t **levels, const int *lw, const int *lh,
                         const ygzo_kp *existing, int n_existing, ygzo_kp *out_kps,
                         uint8_t *out_desc, int cap) {
    int L = o->nlevels;
    ygzo_kp *lk[YGZO_MAX_LEVELS];
    int ln[YGZO_MAX_LEVELS];
    int total = n_existing;
    for (int l = 0; l < L; l++) {
        int bcap = o->feat_per_level[l] + 8;
        lk[l] = (ygzo_kp *)malloc(sizeof(ygzo_kp) * bcap);
        ln[l] = ygzo_octree_level(o, levels[l], lw[l], lh[l], l, lk[l], bcap, NULL);
        if (ln[l] > bcap) ln[l] = bcap; /* cannot happen: <= N + 3 */
        for (int i = 0; i < ln[l]; i++)  /* computeOrientation (:802-803) on the unblurred level */
            lk[l][i].angle = ygzo_ic_angle(levels[l], lw[l], lh[l], lw[l], lk[l][i].x, lk[l][i].y, o->umax);
        total += ln[l];
    }
    if (total > cap) {
        for (int l = 0; l < L; l++) free(lk[l]);
        return -1;
    }
    uint8_t *blur[YGZO_MAX_LEVELS];
    for (int l = 0; l < L; l++) {
        blur[l] = (uint8_t *)malloc((size_t)lw[l] * lh[l]);
        ygzo_gaussian_blur7(levels[l], lw[l], lh[l], lw[l], blur[l], lw[l], o->blur_variant);
    }
    for (int i = 0; i < n_existing; i++) { /* :1088-1099 */
        ygzo_kp t = existing[i];
        int oc = t.octave;
        t.x *= o->inv_scale[oc];
        t.y *= o->inv_scale[oc];
        ygzo_orb_descriptor(blur[oc], lw[oc], lh[oc], lw[oc], &t, out_desc + 32 * (size_t)i);
        out_kps[i] = existing[i];
    }
    int off = n_existing;
    for (int l = 0; l < L; l++) { /* :1102-1125 */
        for (int i = 0; i < ln[l]; i++) {
            ygzo_orb_descriptor(blur[l], lw[l], lh[l], lw[l], &lk[l][i], out_desc + 32 * (size_t)(off + i));
            ygzo_kp kp = lk[l][i];
            if (l != 0) { kp.x *= o->scale[l]; kp.y *= o->scale[l]; }
            out_kps[off + i] = kp;
        }
        off += ln[l];
    }
    for (int l = 0; l < L; l++) { free(lk[l]); free(blur[l]); }
    return total;
}
