/* undistort.c -- TEST INFRASTRUCTURE ONLY (the parity checker for the HIP
 * undistort path; never linked into the product).
 *
 * Frame::ComputeImagePyramid (Frame.cc:775-790) undistorts every frame before
 * the pyramid:
 *   cv::initUndistortRectifyMap(K, D, Mat(), K, size, CV_16SC2, map1, map2);
 *   cv::remap(img, out, map1, map2, cv::INTER_LINEAR);   // BORDER_CONSTANT, 0
 * K (Eigen Matrix3f, Tracking.cc:165-169) and D (CV_32F, Tracking.cc:171-199:
 * k1 k2 p1 p2 [k3] or k1..k6) are float values promoted to double by OpenCV.
 *
 * OpenCV is not in this image: this restates its scalar
 * (3.x) code path -- Matx33d::inv(DECOMP_LU) closed form for 3x3, the
 * incremental _x/_y/_w row walk, cvRound(u * INTER_TAB_SIZE) with
 * INTER_BITS = 5, and remapBilinear for CV_8U with the exact 15-bit bilinear
 * table (every (1-x)(1-y) weight is a multiple of 2^-10, so the table needs
 * no sum fix-up; the one entry OpenCV stores as {32767, 0, 0, 1} instead of
 * {32768, 0, 0, 0} -- short saturation then fix-up -- yields the same pixel,
 * (32767 a + b + 2^14) >> 15 == a for bytes a, b).  Parity unpinned against OpenCV itself. */
#include <math.h>
#include <stdint.h>

#include "ygz_oracle.h"

enum { INTER_BITS = 5, INTER_TAB_SIZE = 1 << INTER_BITS, COEF_BITS = 15 };

static double det3(const double a[9]) {
    return a[0] * (a[4] * a[8] - a[7] * a[5]) - a[1] * (a[3] * a[8] - a[6] * a[5]) +
           a[2] * (a[3] * a[7] - a[6] * a[4]);
}

/* saturate_cast<int>(double) = cvRound = cvtsd2si: round half to even, and
 * the x86 "integer indefinite" INT_MIN for NaN or anything out of range */
static int cv_round(double v) {
    const double r = rint(v);
    return (r >= -2147483648.0 && r <= 2147483647.0) ? (int)r : (int)0x80000000u;
}

/* Matx_FastInvOp<double, 3> (matx.hpp): cofactors times 1/det */
static void inv3(const double a[9], double b[9]) {
    double d = det3(a);
    d = 1. / d;
    b[0] = (a[4] * a[8] - a[5] * a[7]) * d;
    b[1] = (a[2] * a[7] - a[1] * a[8]) * d;
    b[2] = (a[1] * a[5] - a[2] * a[4]) * d;
    b[3] = (a[5] * a[6] - a[3] * a[8]) * d;
    b[4] = (a[0] * a[8] - a[2] * a[6]) * d;
    b[5] = (a[2] * a[3] - a[0] * a[5]) * d;
    b[6] = (a[3] * a[7] - a[4] * a[6]) * d;
    b[7] = (a[1] * a[6] - a[0] * a[7]) * d;
    b[8] = (a[0] * a[4] - a[1] * a[3]) * d;
}

void ygzo_undistort_map(const float cam[4], const float *dist, int ndist, int W, int H, int16_t *map1,
                        uint16_t *map2) {
    const double fx = cam[0], fy = cam[1], u0 = cam[2], v0 = cam[3];
    const double A[9] = {fx, 0, u0, 0, fy, v0, 0, 0, 1};
    double ir[9];
    inv3(A, ir); /* (Ar * R).inv() with Ar = K, R = I (the product is exact) */
    double k[14] = {0};
    for (int i = 0; i < ndist && i < 14; i++) k[i] = (double)dist[i];
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = k[4], k4 = k[5], k5 = k[6], k6 = k[7];
    const double s1 = k[8], s2 = k[9], s3 = k[10], s4 = k[11];
    for (int i = 0; i < H; i++) {
        double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
        for (int j = 0; j < W; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
            const double w = 1. / _w, x = _x * w, y = _y * w;
            const double x2 = x * x, y2 = y * y;
            const double r2 = x2 + y2, _2xy = 2 * x * y;
            const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            const double xd = (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2);
            const double yd = (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2);
            /* tilt matrix = I (tauX = tauY = 0): vecTilt = (xd, yd, 1), invProj = 1 */
            const double u = fx * 1. * xd + u0, v = fy * 1. * yd + v0;
            const int iu = cv_round(u * INTER_TAB_SIZE), iv = cv_round(v * INTER_TAB_SIZE);
            map1[2 * ((size_t)i * W + j)] = (int16_t)(iu >> INTER_BITS);
            map1[2 * ((size_t)i * W + j) + 1] = (int16_t)(iv >> INTER_BITS);
            map2[(size_t)i * W + j] = (uint16_t)((iv & (INTER_TAB_SIZE - 1)) * INTER_TAB_SIZE + (iu & (INTER_TAB_SIZE - 1)));
        }
    }
}

/* remapBilinear<FixedPtCast<int, uchar, 15>, RemapVec_8u, short> with
 * BORDER_CONSTANT (borderValue 0) */
void ygzo_remap_linear(const uint8_t *src, int W, int H, int sstride, const int16_t *map1, const uint16_t *map2,
                       int DW, int DH, uint8_t *dst, int dstride) {
    for (int y = 0; y < DH; y++)
        for (int x = 0; x < DW; x++) {
            const int sx = map1[2 * ((size_t)y * DW + x)], sy = map1[2 * ((size_t)y * DW + x) + 1];
            const int f = map2[(size_t)y * DW + x];
            const int tx = f & (INTER_TAB_SIZE - 1), ty = f >> INTER_BITS;
            /* initInterTab2D: itab[k1*2+k2] = cvRound(32768 * c_y[k1] * c_x[k2]), c = (1 - t/32, t/32) */
            const int w0 = (32 - ty) * (32 - tx) * 32, w1 = (32 - ty) * tx * 32;
            const int w2 = ty * (32 - tx) * 32, w3 = ty * tx * 32;
            int v0, v1, v2, v3;
            if ((unsigned)sx < (unsigned)(W - 1) && (unsigned)sy < (unsigned)(H - 1)) {
                const uint8_t *S = src + (size_t)sy * sstride + sx;
                v0 = S[0]; v1 = S[1]; v2 = S[sstride]; v3 = S[sstride + 1];
            } else if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
                dst[(size_t)y * dstride + x] = 0;
                continue;
            } else {
                const int x0 = sx, x1 = sx + 1, y0 = sy, y1 = sy + 1;
                const int ok_x0 = x0 >= 0 && x0 < W, ok_x1 = x1 >= 0 && x1 < W;
                const int ok_y0 = y0 >= 0 && y0 < H, ok_y1 = y1 >= 0 && y1 < H;
                v0 = ok_x0 && ok_y0 ? src[(size_t)y0 * sstride + x0] : 0;
                v1 = ok_x1 && ok_y0 ? src[(size_t)y0 * sstride + x1] : 0;
                v2 = ok_x0 && ok_y1 ? src[(size_t)y1 * sstride + x0] : 0;
                v3 = ok_x1 && ok_y1 ? src[(size_t)y1 * sstride + x1] : 0;
            }
            int val = (v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3 + (1 << (COEF_BITS - 1))) >> COEF_BITS;
            dst[(size_t)y * dstride + x] = (uint8_t)(val < 0 ? 0 : (val > 255 ? 255 : val));
        }
}

/* remapBilinear<Cast<float, float>, RemapNoVec, float> with BORDER_CONSTANT
 * (borderValue 0): the RGB-D depth image's undistortion (Frame.cc:799-804, the
 * same CV_16SC2 maps).  remap() takes the float weight table for every depth but
 * CV_8U (imgwarp.cpp: fixpt = depth == CV_8U); initInterTab2D's float entries are
 * c_y[k1] * c_x[k2] with c = (1 - t/32, t/32), exact in float.  The sum is
 * S00 w0 + S01 w1 + S10 w2 + S11 w3, left to right in float (no FMA contraction:
 * the scalar path of OpenCV's baseline x86-64 build; built -ffp-contract=off). */
void ygzo_remap_linear_f32(const float *src, int W, int H, int sstride, const int16_t *map1, const uint16_t *map2,
                           int DW, int DH, float *dst, int dstride) {
    for (int y = 0; y < DH; y++)
        for (int x = 0; x < DW; x++) {
            const int sx = map1[2 * ((size_t)y * DW + x)], sy = map1[2 * ((size_t)y * DW + x) + 1];
            const int f = map2[(size_t)y * DW + x];
            const int tx = f & (INTER_TAB_SIZE - 1), ty = f >> INTER_BITS;
            const float cx0 = 1.f - (float)tx * (1.f / INTER_TAB_SIZE), cx1 = (float)tx * (1.f / INTER_TAB_SIZE);
            const float cy0 = 1.f - (float)ty * (1.f / INTER_TAB_SIZE), cy1 = (float)ty * (1.f / INTER_TAB_SIZE);
            const float w0 = cy0 * cx0, w1 = cy0 * cx1, w2 = cy1 * cx0, w3 = cy1 * cx1;
            float v0, v1, v2, v3;
            if ((unsigned)sx < (unsigned)(W - 1) && (unsigned)sy < (unsigned)(H - 1)) {
                const float *S = src + (size_t)sy * sstride + sx;
                v0 = S[0]; v1 = S[1]; v2 = S[sstride]; v3 = S[sstride + 1];
            } else if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
                dst[(size_t)y * dstride + x] = 0.f;
                continue;
            } else {
                const int x0 = sx, x1 = sx + 1, y0 = sy, y1 = sy + 1;
                const int ok_x0 = x0 >= 0 && x0 < W, ok_x1 = x1 >= 0 && x1 < W;
                const int ok_y0 = y0 >= 0 && y0 < H, ok_y1 = y1 >= 0 && y1 < H;
                v0 = ok_x0 && ok_y0 ? src[(size_t)y0 * sstride + x0] : 0.f;
                v1 = ok_x1 && ok_y0 ? src[(size_t)y0 * sstride + x1] : 0.f;
                v2 = ok_x0 && ok_y1 ? src[(size_t)y1 * sstride + x0] : 0.f;
                v3 = ok_x1 && ok_y1 ? src[(size_t)y1 * sstride + x1] : 0.f;
            }
            dst[(size_t)y * dstride + x] = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3;
        }
}
