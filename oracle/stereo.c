/*
 * stereo.c — CPU restatement of Frame::ComputeStereoMatches (Frame.cc:509-682)
 * and Frame::ComputeStereoFromRGBD (Frame.cc:684-700).
 * TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline); see ygz_oracle.h.
 *
 * Arithmetic follows the reference expression by expression:
 *   - row bands: maxr = ceil(y + r), minr = floor(y - r), r = 2 * scale[octave]
 *     (float), rows outside [0, nRows) are dropped (the reference indexes out
 *     of range there; keypoints never reach them);
 *   - the candidate list of a row is in right-keypoint order, best = first
 *     strict minimum below TH_HIGH = 100 (ORBmatcher.cc:36);
 *   - the 11x11 SAD windows are integer-valued floats (pixel minus the window
 *     centre), so every sum is exact; `round` is C round (half away from zero);
 *   - a window the reference would cut outside the level (cv::Mat::colRange /
 *     rowRange assertion) drops the keypoint here (documented deviation: the
 *     reference aborts);
 *   - `disparity = 0.01` / `bestuR = uL - 0.01` keep their double literals;
 *   - the final outlier cut keeps matches with SAD < 1.5f * 1.4f * median, the
 *     median being the SAD of element size/2 of the (SAD, index)-sorted list;
 *     with no match at all the reference reads an empty vector — no-op here.
 */
#include "ygz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static int popcnt32(uint32_t x) { return __builtin_popcount(x); }

static int desc_dist(const uint8_t *a, const uint8_t *b) {
    /* ORBmatcher::DescriptorDistance (ORBmatcher.cc:1507-1523) */
    int d = 0;
    for (int i = 0; i < 32; i += 4) {
        uint32_t x, y;
        memcpy(&x, a + i, 4);
        memcpy(&y, b + i, 4);
        d += popcnt32(x ^ y);
    }
    return d;
}

static int cmp_pair(const void *a, const void *b) {
    const int *x = (const int *)a, *y = (const int *)b;
    if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
    return x[1] < y[1] ? -1 : (x[1] > y[1]);
}

int ygzo_stereo_matches(uint8_t **left_levels, uint8_t **right_levels, const int *lw, const int *lh,
                        int nlevels, const float *scale, const float *inv_scale, const ygzo_kp *kl,
                        const uint8_t *dl, int nl, const ygzo_kp *kr, const uint8_t *dr, int nr, float mb,
                        float mbf, float *uRight, float *depth, int *sad_out) {
    (void)nlevels;
    for (int i = 0; i < nl; i++) {
        uRight[i] = -1.0f;
        depth[i] = -1.0f;
        if (sad_out) sad_out[i] = -1;
    }
    const int thOrbDist = (100 + 50) / 2;
    const int nRows = lh[0];
    /* vRowIndices as CSR, rows in right-keypoint order (Frame.cc:523-535) */
    int *cnt = (int *)calloc((size_t)nRows + 1, sizeof(int));
    for (int iR = 0; iR < nr; iR++) {
        const float kpY = kr[iR].y;
        const float r = 2.0f * scale[kr[iR].octave];
        const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) cnt[yi + 1]++;
    }
    for (int y = 0; y < nRows; y++) cnt[y + 1] += cnt[y];
    int *fill = (int *)malloc(sizeof(int) * ((size_t)nRows + 1));
    memcpy(fill, cnt, sizeof(int) * ((size_t)nRows + 1));
    int *rows = (int *)malloc(sizeof(int) * ((size_t)cnt[nRows] + 1));
    for (int iR = 0; iR < nr; iR++) {
        const float kpY = kr[iR].y;
        const float r = 2.0f * scale[kr[iR].octave];
        const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) rows[fill[yi]++] = iR;
    }
    const float minZ = mb, minD = 0;
    const float maxD = mbf / minZ;
    int *pairs = (int *)malloc(sizeof(int) * 2 * ((size_t)nl + 1));
    int np = 0;
    for (int iL = 0; iL < nl; iL++) {
        const ygzo_kp *kpL = &kl[iL];
        const int levelL = kpL->octave;
        const float vL = kpL->y, uL = kpL->x;
        if (!(vL >= 0.0f) || (int)vL >= nRows) continue;
        const int row = (int)vL;
        if (cnt[row + 1] == cnt[row]) continue;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = 100, bestIdxR = 0;
        const uint8_t *dL = dl + (size_t)iL * 32;
        for (int c = cnt[row]; c < cnt[row + 1]; c++) {
            const int iR = rows[c];
            const ygzo_kp *kpR = &kr[iR];
            if (kpR->octave < levelL - 1 || kpR->octave > levelL + 1) continue;
            const float uR = kpR->x;
            if (uR >= minU && uR <= maxU) {
                const int dist = desc_dist(dL, dr + (size_t)iR * 32);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist >= thOrbDist) continue;
        /* sub-pixel match by correlation (Frame.cc:589-658) */
        const float uR0 = kr[bestIdxR].x;
        const float scaleFactor = inv_scale[kpL->octave];
        const float scaleduL = roundf(kpL->x * scaleFactor);
        const float scaledvL = roundf(kpL->y * scaleFactor);
        const float scaleduR0 = roundf(uR0 * scaleFactor);
        const int w = 5, L = 5;
        const int W = lw[levelL], Hh = lh[levelL];
        const uint8_t *IL = left_levels[levelL], *IRimg = right_levels[levelL];
        const int r0 = (int)(scaledvL - w), c0 = (int)(scaleduL - w);
        if (r0 < 0 || r0 + 2 * w + 1 > Hh || c0 < 0 || c0 + 2 * w + 1 > W) continue; /* reference: assertion */
        const float iniu = scaleduR0 + L - w;
        const float endu = scaleduR0 + L + w + 1;
        if (iniu < 0 || endu >= W) continue;
        const int cr0 = (int)(scaleduR0 + -L - w);
        if (cr0 < 0 || (int)(scaleduR0 + L + w + 1) > W) continue; /* reference: assertion */
        const float cL = (float)IL[(size_t)(r0 + w) * W + c0 + w];
        int bestSad = 0x7fffffff, bestincR = 0;
        float vDists[11];
        for (int incR = -L; incR <= L; incR++) {
            const int cc = (int)(scaleduR0 + incR - w);
            const float cR = (float)IRimg[(size_t)(r0 + w) * W + cc + w];
            double acc = 0.0; /* cv::norm(NORM_L1) over CV_32F */
            for (int y = 0; y < 2 * w + 1; y++)
                for (int x = 0; x < 2 * w + 1; x++) {
                    const float a = (float)IL[(size_t)(r0 + y) * W + c0 + x] - cL;
                    const float b = (float)IRimg[(size_t)(r0 + y) * W + cc + x] - cR;
                    acc += fabs((double)a - (double)b);
                }
            const float dist = (float)acc;
            if (dist < (float)bestSad) {
                bestSad = (int)dist;
                bestincR = incR;
            }
            vDists[L + incR] = dist;
        }
        if (bestincR == -L || bestincR == L) continue;
        const float dist1 = vDists[L + bestincR - 1];
        const float dist2 = vDists[L + bestincR];
        const float dist3 = vDists[L + bestincR + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = scale[kpL->octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
        float disparity = (uL - bestuR);
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
                disparity = 0.01;
                bestuR = uL - 0.01;
            }
            depth[iL] = mbf / disparity;
            uRight[iL] = bestuR;
            if (sad_out) sad_out[iL] = bestSad;
            pairs[2 * np] = bestSad;
            pairs[2 * np + 1] = iL;
            np++;
        }
    }
    if (np > 0) {
        qsort(pairs, np, 2 * sizeof(int), cmp_pair);
        const float median = (float)pairs[2 * (np / 2)];
        const float thDist = 1.5f * 1.4f * median;
        for (int i = np - 1; i >= 0; i--) {
            if ((float)pairs[2 * i] < thDist) break;
            uRight[pairs[2 * i + 1]] = -1;
            depth[pairs[2 * i + 1]] = -1;
            if (sad_out) sad_out[pairs[2 * i + 1]] = -1;
        }
    }
    int kept = 0;
    for (int i = 0; i < nl; i++) kept += depth[i] > 0;
    free(cnt);
    free(fill);
    free(rows);
    free(pairs);
    return kept;
}

void ygzo_stereo_from_rgbd(const float *im_depth, int W, int H, int stride, const ygzo_kp *kps, int n, float mbf,
                           float *uRight, float *depth) {
    /* Frame::ComputeStereoFromRGBD (Frame.cc:684-700): imDepth.at<float>(v, u) with
     * float (v, u) converted to int; d > 0 -> depth d, uRight = u - mbf / d. */
    for (int i = 0; i < n; i++) {
        uRight[i] = -1;
        depth[i] = -1;
        const int v = (int)kps[i].y, u = (int)kps[i].x;
        if (v < 0 || v >= H || u < 0 || u >= W) continue;
        const float d = im_depth[(size_t)v * stride + u];
        if (d > 0) {
            depth[i] = d;
            uRight[i] = kps[i].x - mbf / d;
        }
    }
}
