// undistort.hip — Frame::ComputeImagePyramid's undistortion (Frame.cc:775-790):
//   cv::initUndistortRectifyMap(K, D, I, K, size, CV_16SC2, map1, map2)
//   cv::remap(img, out, map1, map2, INTER_LINEAR)   (BORDER_CONSTANT, 0)
//
// k_undistort_map builds the fixed-point map once per camera.  OpenCV walks each
// row accumulating _x += ir[0] in double, so one thread owns one row and repeats
// exactly that sequence (-ffp-contract=off: no fused multiply-adds); the
// result is bit-identical to the restatement in oracle/undistort.c.
// k_remap_linear is the per-frame hot part: one thread per 4 output pixels;
// map1 (short2) / map2 (u16) reads are coalesced and reused across up to 8
// frames, the 2x2 source taps are gathers (the map is smooth, so they hit in
// cache), weights come from the exact 15-bit bilinear table
// w = 32 * (32 - tx | tx) * (32 - ty | ty).
#include "common.hpp"

namespace ygzfe {

struct UndistortParams {
    double fx, fy, u0, v0;
    double ir[9];
    double k[12];  // k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4
};

// cvRound (cvtsd2si): half to even, INT_MIN for NaN / out of range
__device__ __forceinline__ int cv_round(double v) {
    const double r = rint(v);
    return (r >= -2147483648.0 && r <= 2147483647.0) ? (int)r : (int)0x80000000u;
}

__global__ __launch_bounds__(64) void k_undistort_map(UndistortParams P, int W, int H, int16_t *__restrict__ map1,
                                                      uint16_t *__restrict__ map2) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= H) return;
    const double *ir = P.ir;
    const double k1 = P.k[0], k2 = P.k[1], p1 = P.k[2], p2 = P.k[3], k3 = P.k[4], k4 = P.k[5], k5 = P.k[6],
                 k6 = P.k[7];
    const double s1 = P.k[8], s2 = P.k[9], s3 = P.k[10], s4 = P.k[11];
    double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
    for (int j = 0; j < W; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
        const double w = 1. / _w, x = _x * w, y = _y * w;
        const double x2 = x * x, y2 = y * y;
        const double r2 = x2 + y2, _2xy = 2 * x * y;
        const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
        const double xd = (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2);
        const double yd = (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2);
        const double u = P.fx * 1. * xd + P.u0, v = P.fy * 1. * yd + P.v0;
        const int iu = cv_round(u * 32.0), iv = cv_round(v * 32.0);
        const size_t o = (size_t)i * W + j;
        map1[2 * o] = (int16_t)(iu >> 5);
        map1[2 * o + 1] = (int16_t)(iv >> 5);
        map2[o] = (uint16_t)((iv & 31) * 32 + (iu & 31));
    }
}

// one output pixel of remapBilinear<FixedPtCast<int, uchar, 15>> with BORDER_CONSTANT 0
__device__ __forceinline__ uint32_t remap_px(const uint8_t *__restrict__ S, int W, int H, int sstride, int sx, int sy,
                                             int f) {
    const int tx = f & 31, ty = f >> 5;
    int v0, v1, v2, v3;
    if ((unsigned)sx < (unsigned)(W - 1) && (unsigned)sy < (unsigned)(H - 1)) {
        const uint8_t *q = S + (size_t)sy * sstride + sx;
        v0 = q[0]; v1 = q[1]; v2 = q[sstride]; v3 = q[sstride + 1];
    } else if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
        return 0;
    } else {
        const bool ox0 = sx >= 0 && sx < W, ox1 = sx + 1 >= 0 && sx + 1 < W;
        const bool oy0 = sy >= 0 && sy < H, oy1 = sy + 1 >= 0 && sy + 1 < H;
        v0 = ox0 && oy0 ? S[(size_t)sy * sstride + sx] : 0;
        v1 = ox1 && oy0 ? S[(size_t)sy * sstride + sx + 1] : 0;
        v2 = ox0 && oy1 ? S[(size_t)(sy + 1) * sstride + sx] : 0;
        v3 = ox1 && oy1 ? S[(size_t)(sy + 1) * sstride + sx + 1] : 0;
    }
    const int w0 = (32 - ty) * (32 - tx) * 32, w1 = (32 - ty) * tx * 32;
    const int w2 = ty * (32 - tx) * 32, w3 = ty * tx * 32;
    // the weights sum to 2^15 and the taps are bytes: the result is already in [0, 255]
    return (uint32_t)((v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3 + (1 << 14)) >> 15);
}

// ---------------------------------------------------------------------------
// Tiled remap.  The map is smooth, so the source pixels one 64x16 output tile
// reads lie in a small box (at most 72x17 = 1224 B for EuRoC, 1440 B for
// TUM1).  The box of every tile is computed once with the map
// (k_remap_boxes).  A block owns one tile for kRemapFramesPerBlock frames:
//  - once per block, each thread turns its 4 map entries into 4 LDS tap
//    addresses and 4 bilinear weights per pixel; taps outside the image get
//    weight 0 and a clamped in-box address, so the BORDER_CONSTANT pixels take
//    the same straight-line code as the interior;
//  - the boxes of a group of 16/DW frames are loaded at once (coalesced
//    dwords through a range-checked buffer descriptor, DW per thread per
//    frame, all in flight together), staged into LDS, and each output pixel
//    is then 4 ds_read_u8 + 4 mul24 + a shift;
//  - lanes are columns (a tap read of a wave is ~64 consecutive LDS bytes,
//    free of bank conflicts) and each lane owns 4 rows; a DPP transpose in
//    each quad turns that into dword stores of 4 horizontal pixels.
// HBM traffic per frame: ~1.01 B/px read (box overlap) + 1 B/px written.
constexpr int kRemapTileW = 64, kRemapTileH = 16;  // 256 threads x 4 rows of one column
constexpr int kRemapLanesX = kRemapTileW / 4;      // (k_remap_boxes: 4 horizontal pixels per thread)
constexpr int kRemapFramesPerBlock = 16;  // 4, 8, 16, 32 measured: 85, 67, 60, 62 us per 256 frames
constexpr int kRemapLdsBytes = 16384;             // one group of boxes
constexpr int kRemapMaxBox = 4096;                // larger boxes gather from global memory

struct RemapBox { int x0, y0, w, h; };

// raw buffer descriptors: offsets at or past num_records load 0 / drop the store
constexpr uint32_t kOutOfRange = 0x80000000u;
constexpr int kRsrcFlags = 0x00020000;  // w, h == 0: no tap in the image; h < 0: too large for LDS

__global__ __launch_bounds__(256) void k_remap_boxes(int W, int H, const int16_t *__restrict__ map1,
                                                     RemapBox *__restrict__ boxes, int tiles_x) {
    __shared__ int red[4];
    const int t = threadIdx.x;
    const int X0 = (blockIdx.x % tiles_x) * kRemapTileW, Y0 = (blockIdx.x / tiles_x) * kRemapTileH;
    const int y = Y0 + t / kRemapLanesX, xb = X0 + (t % kRemapLanesX) * 4;
    int mnx = INT_MAX, mny = INT_MAX, mxx = INT_MIN, mxy = INT_MIN;
    if (y < H)
        for (int k = 0; k < 4; k++) {
            const int x = xb + k;
            if (x >= W) break;
            const size_t p = (size_t)y * W + x;
            const int sx = map1[2 * p], sy = map1[2 * p + 1];
            const int ax = max(sx, 0), bx = min(sx + 1, W - 1), ay = max(sy, 0), by = min(sy + 1, H - 1);
            if (ax <= bx && ay <= by) {
                mnx = min(mnx, ax); mxx = max(mxx, bx);
                mny = min(mny, ay); mxy = max(mxy, by);
            }
        }
    if (t < 4) red[t] = t < 2 ? INT_MAX : INT_MIN;
    __syncthreads();
    atomicMin(&red[0], mnx);
    atomicMin(&red[1], mny);
    atomicMax(&red[2], mxx);
    atomicMax(&red[3], mxy);
    __syncthreads();
    if (t == 0) {
        RemapBox b{0, 0, 0, 0};
        if (red[0] <= red[2]) {
            b.x0 = red[0] & ~3;  // dword-aligned columns
            b.y0 = red[1];
            b.w = ((red[2] + 1 - b.x0) + 3) & ~3;
            b.h = red[3] + 1 - red[1];
            if (b.w * b.h > kRemapMaxBox) b.h = -1;
        }
        boxes[blockIdx.x] = b;
    }
}

// 4x4 byte transpose across the 4 lanes of a quad: lane q enters with byte r
// = (row r, column q) and leaves with byte c = (row q, column c).  Step 1
// swaps bytes with lane q^1 (DPP quad_perm [1,0,3,2]), step 2 byte pairs with
// lane q^2 ([2,3,0,1]); v_perm picks the bytes with lane-parity selectors.
__device__ __forceinline__ uint32_t remap_quad_transpose(uint32_t d, uint32_t sel1, uint32_t sel2) {
    const uint32_t p = (uint32_t)__builtin_amdgcn_mov_dpp((int)d, 0xB1, 0xF, 0xF, false);
    const uint32_t e = __builtin_amdgcn_perm(d, p, sel1);
    const uint32_t r = (uint32_t)__builtin_amdgcn_mov_dpp((int)e, 0x4E, 0xF, 0xF, false);
    return __builtin_amdgcn_perm(e, r, sel2);
}

// VEC: W and the source/destination strides, pitches and bases are
// multiples of 4, so box rows load as dwords (the box never passes column W)
// and each thread's 4 transposed outputs store as one dword.  DW: box dwords per thread per
// frame (boxes up to DW KiB); G = 16 / DW frames per group.
template <bool VEC, int DW>
__global__ __launch_bounds__(256) void k_remap_tiles(const uint8_t *__restrict__ src, size_t src_pitch, int W, int H,
                                                     int sstride, const int16_t *__restrict__ map1,
                                                     const uint16_t *__restrict__ map2,
                                                     const RemapBox *__restrict__ boxes, int tiles_x,
                                                     uint8_t *__restrict__ dst, size_t dst_pitch, int dstride,
                                                     int n_images, int fpb) {
    constexpr int G = 16 / DW, kBox = DW * 1024;
    __shared__ __attribute__((aligned(16))) uint8_t s_box[kRemapLdsBytes];
    const int t = threadIdx.x;
    // adjacent tiles share source cache lines: keep them on one XCD's L2
    int tile, group;
    swizzled_block_2d(tile, group);
    const int X0 = (tile % tiles_x) * kRemapTileW, Y0 = (tile / tiles_x) * kRemapTileH;
    // lane = column, so one tap read of a wave is ~64 consecutive LDS bytes
    // of (mostly) one box row: no bank conflicts.  Each thread owns 4 rows of
    // its column; a quad of lanes transposes its 4x4 bytes before storing.
    const int x = X0 + (t & 63), y0 = Y0 + (t >> 6) * 4;
    const RemapBox B = boxes[tile];
    const int img0 = group * fpb;
    const int img1 = min(n_images, img0 + fpb);
    int sx[4], sy[4], f[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const bool on = x < W && y0 + k < H;
        const size_t p = on ? (size_t)(y0 + k) * W + x : 0;
        const uint32_t m = *as_global((const uint32_t *)(map1 + 2 * p));
        sx[k] = on ? (int)(int16_t)(m & 0xffff) : -8;  // off the image: no taps
        sy[k] = on ? (int)(int16_t)(m >> 16) : -8;
        f[k] = map2[p];
    }
    if (B.h < 0) return;  // box too large for LDS: k_remap_gather's tile
    // staging: dword i = t + 256 j of the box (row r, byte column c), as a
    // byte offset into the frame; dwords past the box get an offset beyond
    // the buffer's range, which the hardware turns into a 0 load
    const int bw = max(B.w, 4), bh = max(B.h, 1);
    const int nd = (B.w * B.h) >> 2, dpr = bw >> 2;
    const uint32_t src_bytes = (uint32_t)((H - 1) * sstride + W), dst_bytes = (uint32_t)((H - 1) * dstride + W);
    uint32_t boff[DW];
#pragma unroll
    for (int j = 0; j < DW; j++) {
        const int i = t + 256 * j;
        const int r = i / dpr, c = 4 * (i - r * dpr);
        boff[j] = i < nd ? (uint32_t)((B.y0 + r) * sstride + B.x0 + c) : kOutOfRange;
    }
    // after the quad transpose, lane q of a quad holds row y0 + q, columns
    // xq .. xq + 3; a dword store when all 4 are on the image (and VEC)
    const int q4 = t & 3, xq = x - q4, yq = y0 + q4;
    const int nq = yq < H ? max(0, min(4, W - xq)) : 0;
    const bool dvec = VEC && nq == 4;
    const uint32_t doff = (uint32_t)(yq * dstride + xq);
    // v_perm selectors of the two transpose steps (see remap_quad_transpose)
    const uint32_t sel1 = (q4 & 1) ? 0x07030501u : 0x02060004u;
    const uint32_t sel2 = (q4 & 2) ? 0x07060302u : 0x01000504u;
    // taps: (sum w' v + 2^9) >> 10 with w' = (32 - t)(32 - t') is OpenCV's
    // (sum w v + 2^14) >> 15 for its 15-bit table w = 32 w'
    uint32_t a[4][4], w[4][4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int tx = f[k] & 31, ty = f[k] >> 5;
        const int wx0 = sx[k] >= 0 && sx[k] < W ? 32 - tx : 0, wx1 = sx[k] + 1 >= 0 && sx[k] + 1 < W ? tx : 0;
        const int wy0 = sy[k] >= 0 && sy[k] < H ? 32 - ty : 0, wy1 = sy[k] + 1 >= 0 && sy[k] + 1 < H ? ty : 0;
        const int ax = sx[k] - B.x0, ay = sy[k] - B.y0;
        const int cx0 = min(max(ax, 0), bw - 1), cx1 = min(max(ax + 1, 0), bw - 1);
        const int cy0 = min(max(ay, 0), bh - 1) * bw, cy1 = min(max(ay + 1, 0), bh - 1) * bw;
        a[k][0] = cy0 + cx0; a[k][1] = cy0 + cx1; a[k][2] = cy1 + cx0; a[k][3] = cy1 + cx1;
        w[k][0] = wy0 * wx0; w[k][1] = wy0 * wx1; w[k][2] = wy1 * wx0; w[k][3] = wy1 * wx1;
    }
    for (int g0 = img0; g0 < img1; g0 += G) {
        const int ng = min(G, img1 - g0);
        uint32_t pf[G][DW];
#pragma unroll
        for (int q = 0; q < G; q++) {
            if (q >= ng) break;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void *)(src + (size_t)(g0 + q) * src_pitch), 0, src_bytes,
                                                  kRsrcFlags);
#pragma unroll
            for (int j = 0; j < DW; j++) {
                if (VEC) {
                    pf[q][j] = __builtin_amdgcn_raw_buffer_load_b32(rs, boff[j], 0, 0);
                } else {  // bytes: columns past the row end read the next row or 0; their weights are 0
                    pf[q][j] = 0;
                    for (int b = 0; b < 4; b++)
                        pf[q][j] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, boff[j] + b, 0, 0) << (8 * b);
                }
            }
        }
        if (g0 != img0) __syncthreads();  // the previous group's taps are read
#pragma unroll
        for (int q = 0; q < G; q++) {
            if (q >= ng) break;
#pragma unroll
            for (int j = 0; j < DW; j++)
                if (j * 256 < kBox / 4) *(uint32_t *)(s_box + q * kBox + 4 * (t + 256 * j)) = pf[q][j];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < G; q++) {
            if (q >= ng) break;
            const uint8_t *L = s_box + q * kBox;
            const __amdgpu_buffer_rsrc_t rd =
                __builtin_amdgcn_make_buffer_rsrc((void *)(dst + (size_t)(g0 + q) * dst_pitch), 0, dst_bytes,
                                                  kRsrcFlags);
            // every tap address is inside the box (off-image taps have weight 0),
            // so all 16 reads issue back to back
            uint32_t out = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t v = __umul24(w[k][0], L[a[k][0]]) + __umul24(w[k][1], L[a[k][1]]) +
                                   __umul24(w[k][2], L[a[k][2]]) + __umul24(w[k][3], L[a[k][3]]) + 512;
                out |= (v >> 10) << (8 * k);
            }
            out = remap_quad_transpose(out, sel1, sel2);
            if (dvec) {
                __builtin_amdgcn_raw_buffer_store_b32(out, rd, doff, 0, 0);
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(out >> (8 * k)), rd,
                                                         k < nq ? doff + k : kOutOfRange, 0, 0);
            }
        }
    }
}

// Tiles whose source box exceeds kRemapMaxBox (extreme distortion only):
// plain per-pixel gathers from global memory.  A separate kernel so that its
// registers do not limit the occupancy of k_remap_tiles.
__global__ __launch_bounds__(256) void k_remap_gather(const uint8_t *__restrict__ src, size_t src_pitch, int W, int H,
                                                      int sstride, const int16_t *__restrict__ map1,
                                                      const uint16_t *__restrict__ map2,
                                                      const RemapBox *__restrict__ boxes, int tiles_x,
                                                      uint8_t *__restrict__ dst, size_t dst_pitch, int dstride,
                                                      int n_images, int fpb) {
    const int tile = blockIdx.x;
    if (boxes[tile].h >= 0) return;
    const int t = threadIdx.x;
    const int xb = (tile % tiles_x) * kRemapTileW + (t % kRemapLanesX) * 4;
    const int y = (tile / tiles_x) * kRemapTileH + t / kRemapLanesX;
    const int img0 = blockIdx.y * fpb;
    const int img1 = min(n_images, img0 + fpb);
    if (y >= H) return;
    for (int k = 0; k < 4; k++) {
        const int x = xb + k;
        if (x >= W) break;
        const size_t p = (size_t)y * W + x;
        const int sx = map1[2 * p], sy = map1[2 * p + 1], f = map2[p];
        for (int im = img0; im < img1; im++)
            dst[(size_t)im * dst_pitch + (size_t)y * dstride + x] =
                (uint8_t)remap_px(src + (size_t)im * src_pitch, W, H, sstride, sx, sy, f);
    }
}

// Matx_FastInvOp<double, 3>: cofactors times 1/det (matches oracle/undistort.c)
static void inv3(const double a[9], double b[9]) {
    double d = a[0] * (a[4] * a[8] - a[7] * a[5]) - a[1] * (a[3] * a[8] - a[6] * a[5]) +
               a[2] * (a[3] * a[7] - a[6] * a[4]);
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

// The RGB-D depth image's undistortion (Frame.cc:799-804): the same maps, remap on
// CV_32F.  remapBilinear<Cast<float, float>> takes the float weight table
// (c_y * c_x, c = (1 - t/32, t/32), exact) and sums S00 w0 + S01 w1 + S10 w2 + S11 w3
// left to right in float (no contraction: -ffp-contract=off), BORDER_CONSTANT 0;
// oracle/undistort.c ygzo_remap_linear_f32.  One thread per output pixel, images
// along grid.y (map reads coalesced, the 2x2 taps cache-local: the map is smooth).
__global__ __launch_bounds__(256) void k_remap_f32(const float *__restrict__ src, size_t src_pitch, int W, int H,
                                                   int sstride, const int16_t *__restrict__ map1,
                                                   const uint16_t *__restrict__ map2, float *__restrict__ dst,
                                                   size_t dst_pitch, int dstride) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    const float *S0 = src + (size_t)blockIdx.z * src_pitch;
    const size_t o = (size_t)y * W + x;
    const uint32_t xy = reinterpret_cast<const uint32_t *>(map1)[o];
    const int sx = (int16_t)(xy & 0xFFFFu), sy = (int16_t)(xy >> 16);
    const int f = map2[o];
    const int tx = f & 31, ty = f >> 5;
    const float cx0 = 1.f - (float)tx * (1.f / 32), cx1 = (float)tx * (1.f / 32);
    const float cy0 = 1.f - (float)ty * (1.f / 32), cy1 = (float)ty * (1.f / 32);
    const float w0 = cy0 * cx0, w1 = cy0 * cx1, w2 = cy1 * cx0, w3 = cy1 * cx1;
    float v0, v1, v2, v3, r;
    if ((unsigned)sx < (unsigned)(W - 1) && (unsigned)sy < (unsigned)(H - 1)) {
        const float *S = S0 + (size_t)sy * sstride + sx;
        v0 = S[0];
        v1 = S[1];
        v2 = S[sstride];
        v3 = S[sstride + 1];
        r = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3;
    } else if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
        r = 0.f;
    } else {
        const bool ok_x0 = sx >= 0 && sx < W, ok_x1 = sx + 1 >= 0 && sx + 1 < W;
        const bool ok_y0 = sy >= 0 && sy < H, ok_y1 = sy + 1 >= 0 && sy + 1 < H;
        v0 = ok_x0 && ok_y0 ? S0[(size_t)sy * sstride + sx] : 0.f;
        v1 = ok_x1 && ok_y0 ? S0[(size_t)sy * sstride + sx + 1] : 0.f;
        v2 = ok_x0 && ok_y1 ? S0[(size_t)(sy + 1) * sstride + sx] : 0.f;
        v3 = ok_x1 && ok_y1 ? S0[(size_t)(sy + 1) * sstride + sx + 1] : 0.f;
        r = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3;
    }
    dst[(size_t)blockIdx.z * dst_pitch + (size_t)y * dstride + x] = r;
}

hipError_t launch_remap_f32(const float *src, size_t src_pitch, int W, int H, int sstride, const int16_t *map1,
                            const uint16_t *map2, float *dst, size_t dst_pitch, int dstride, int n_images,
                            hipStream_t st) {
    if (n_images <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_remap_f32, dim3((W + 63) / 64, (H + 3) / 4, n_images), dim3(256), 0, st, src, src_pitch, W,
                       H, sstride, map1, map2, dst, dst_pitch, dstride);
    return hipGetLastError();
}

hipError_t launch_undistort_map(const float cam[4], const float *dist, int ndist, int W, int H, int16_t *map1,
                                uint16_t *map2, hipStream_t st) {
    UndistortParams P;
    P.fx = cam[0];
    P.fy = cam[1];
    P.u0 = cam[2];
    P.v0 = cam[3];
    const double A[9] = {P.fx, 0, P.u0, 0, P.fy, P.v0, 0, 0, 1};
    inv3(A, P.ir);  // host: double, -ffp-contract=off like the kernel
    for (int i = 0; i < 12; i++) P.k[i] = i < ndist ? (double)dist[i] : 0.0;
    hipLaunchKernelGGL(k_undistort_map, dim3((H + 63) / 64), dim3(64), 0, st, P, W, H, map1, map2);
    return hipGetLastError();
}

int remap_tiles(int W, int H) { return ((W + kRemapTileW - 1) / kRemapTileW) * ((H + kRemapTileH - 1) / kRemapTileH); }

hipError_t launch_remap_boxes(int W, int H, const int16_t *map1, void *boxes, hipStream_t st) {
    const int tiles_x = (W + kRemapTileW - 1) / kRemapTileW;
    hipLaunchKernelGGL(k_remap_boxes, dim3(remap_tiles(W, H)), dim3(256), 0, st, W, H, map1, (RemapBox *)boxes,
                       tiles_x);
    return hipGetLastError();
}

hipError_t launch_remap_linear(const uint8_t *src, size_t src_pitch, int W, int H, int sstride, const int16_t *map1,
                               const uint16_t *map2, const void *boxes, int max_box, bool any_large, uint8_t *dst,
                               size_t dst_pitch, int dstride, int n_images, hipStream_t st) {
    if (n_images <= 0) return hipSuccess;
    // frames are addressed with 32-bit buffer offsets
    if ((size_t)(H - 1) * sstride + W >= kOutOfRange || (size_t)(H - 1) * dstride + W >= kOutOfRange)
        return hipErrorInvalidValue;
    const int tiles_x = (W + kRemapTileW - 1) / kRemapTileW;
    const int fpb = kRemapFramesPerBlock;
    const dim3 grid(remap_tiles(W, H), (n_images + fpb - 1) / fpb);
    const bool multi = n_images > 1;
    const bool vec = W % 4 == 0 && sstride % 4 == 0 && dstride % 4 == 0 && (!multi || src_pitch % 4 == 0) &&
                     (!multi || dst_pitch % 4 == 0) && ((uintptr_t)src & 3) == 0 && ((uintptr_t)dst & 3) == 0;
    const RemapBox *bx = (const RemapBox *)boxes;
#define YGZ_REMAP(V, D)                                                                                           \
    hipLaunchKernelGGL((k_remap_tiles<V, D>), grid, dim3(256), 0, st, src, src_pitch, W, H, sstride, map1, map2, bx, \
                       tiles_x, dst, dst_pitch, dstride, n_images, fpb)
    // max_box: the largest LDS-staged box (bytes); 1 or 2 KiB boxes stage 8 frames at once, larger ones 4
    if (vec) {
        if (max_box <= 2048) YGZ_REMAP(true, 2); else YGZ_REMAP(true, 4);
    } else {
        if (max_box <= 2048) YGZ_REMAP(false, 2); else YGZ_REMAP(false, 4);
    }
#undef YGZ_REMAP
    if (any_large)
        hipLaunchKernelGGL(k_remap_gather, grid, dim3(256), 0, st, src, src_pitch, W, H, sstride, map1, map2, bx,
                           tiles_x, dst, dst_pitch, dstride, n_images, fpb);
    return hipGetLastError();
}

}  // namespace ygzfe
