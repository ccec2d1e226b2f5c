// dso.hip — DSO_KEYPOINT mode (ComputeKeyPointsDSOSingleLevel,
// ORBextractor.cc:1275-1386) on gfx950: per grid cell FAST-10 (Thirdparty/fast
// semantics), Shi-Tomasi scoring (ORBextractor.cc:1152-1187) and top-3
// selection.  One 256-thread workgroup per cell; the host drives the
// grid-shrinking loop (it needs the total count between passes).
#include "common.hpp"

namespace ygzfe {

constexpr int kDsoHalo = 5;
constexpr int kDsoMaxGrid = 96;
constexpr int kDsoS = kDsoMaxGrid + 2 * kDsoHalo;

// longest circular run >= 10 of a 16-bit ring mask
__device__ __forceinline__ bool run10(uint32_t m16) {
    uint32_t x = m16 | (m16 << 16);
    uint32_t y = x & (x >> 1);
    y &= y >> 2;
    y &= y >> 4;
    y &= (x >> 8) & (x >> 9);
    return (y & 0xFFFFu) != 0;
}

// fast_10.cpp ring order (x, y): (0,3) (1,3) (2,2) (3,1) (3,0) (3,-1) (2,-2) (1,-3) (0,-3) ...
__device__ __forceinline__ bool fast10_corner(const uint8_t *p, int S, int b) {
    const int v = p[0], cb = v + b, c_b = v - b;
    const int r[16] = {p[3 * S],  p[1 + 3 * S],  p[2 + 2 * S],  p[3 + S],  p[3],  p[3 - S],
                       p[2 - 2 * S], p[1 - 3 * S], p[-3 * S], p[-1 - 3 * S], p[-2 - 2 * S], p[-3 - S],
                       p[-3], p[-3 + S], p[-2 + 2 * S], p[-1 + 3 * S]};
    uint32_t br = 0, dk = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        br |= (uint32_t)(r[k] > cb) << k;
        dk |= (uint32_t)(r[k] < c_b) << k;
    }
    return run10(br) || run10(dk);
}

// ShiTomasiScore on the LDS tile (pixel p = centre, stride S): float sums in raster order.
__device__ __forceinline__ float shi_tomasi(const uint8_t *p, int S) {
    float dXX = 0.f, dYY = 0.f, dXY = 0.f;
    for (int y = -4; y < 4; ++y)
        for (int x = -4; x < 4; ++x) {
            const uint8_t *q = p + y * S + x;
            const float dx = (float)(q[1] - q[-1]);
            const float dy = (float)(q[S] - q[-S]);
            dXX += dx * dx;
            dYY += dy * dy;
            dXY += dx * dy;
        }
    dXX = (float)(dXX / (2.0 * 64));
    dYY = (float)(dYY / (2.0 * 64));
    dXY = (float)(dXY / (2.0 * 64));
    const float s = dXX + dYY;
    // ORBextractor.cc:1186 as the reference's -O3 -march=native C++ build contracts it
    // (oracle/fast10.c ygzo_shi_tomasi): two fused multiply-subtracts
    const float disc = __builtin_fmaf(s, s, -(4.0f * __builtin_fmaf(dXX, dYY, -(dXY * dXY))));
    return (float)(0.5 * (double)(dXX + dYY - sqrtf(disc)));
}

// cell k of the grid; writes up to 3 keys (x | y << 16, level-0 px) sorted by
// descending score (NaN last, ties by scan order) and the count.
// Debug form (dbg_flags != null, ygzfe_debug_dso_cells): one pass of the cell's scan at
// `dbg_barrier` only, its corner flags written to dbg_flags[k][g * g] (cell-relative
// raster order, 0 outside the scanned region), no scoring -- the cell path's own
// segment-test output, compared with the reference's per-cell corner lists.
__global__ __launch_bounds__(256) void k_dso_cells(const uint8_t *__restrict__ img, int w, int h, int g,
                                                   const uint8_t *__restrict__ occ,
                                                   uint32_t *__restrict__ out_keys, int *__restrict__ out_cnt,
                                                   int dbg_barrier, uint8_t *__restrict__ dbg_flags) {
    __shared__ uint8_t s_img[kDsoS * kDsoS];
    __shared__ float s_sc[kDsoMaxGrid * kDsoMaxGrid];
    __shared__ int s_any;
    __shared__ unsigned long long s_best;
    const int rows = h / g, cols = w / g;
    const int k = blockIdx.x;
    const int nn = k / cols;
    if (dbg_flags) {
        for (int i = threadIdx.x; i < g * g; i += 256) dbg_flags[(size_t)k * g * g + i] = 0;
    } else if (threadIdx.x == 0) {
        out_cnt[k] = 0;
    }
    if (nn == 0 || nn == rows - 1 || (k % cols) == 0 || (k + 1) % cols == 0) return;
    const int x_start = (k - nn * cols) * g, y_start = nn * g;
    const int S = g + 2 * kDsoHalo;
    for (int i = threadIdx.x; i < S * S; i += 256) {
        const int yy = clampi(y_start - kDsoHalo + i / S, 0, h - 1);
        const int xx = clampi(x_start - kDsoHalo + i % S, 0, w - 1);
        s_img[i] = img[(size_t)yy * w + xx];
    }
    // scan region: plain detector (g < 22) covers the whole cell, SSE2 [3, g-3)
    const int lo = g < 22 ? 0 : 3, hi = g < 22 ? g : g - 3;
    const int span = hi > lo ? hi - lo : 0;
    __syncthreads();
    if (dbg_flags) {
        for (int i = threadIdx.x; i < span * span; i += 256) {
            const int cy = lo + i / span, cx = lo + i % span;
            dbg_flags[(size_t)k * g * g + cy * g + cx] =
                fast10_corner(s_img + (cy + kDsoHalo) * S + cx + kDsoHalo, S, dbg_barrier) ? 1 : 0;
        }
        return;
    }
    int barrier = 20;
    for (int pass = 0; pass < 2; pass++) {
        if (threadIdx.x == 0) s_any = 0;
        __syncthreads();
        int any = 0;
        for (int i = threadIdx.x; i < span * span; i += 256) {
            const int cy = lo + i / span, cx = lo + i % span;
            const bool c = fast10_corner(s_img + (cy + kDsoHalo) * S + cx + kDsoHalo, S, barrier);
            s_sc[cy * g + cx] = c ? 1.f : 0.f;  // corner flag for now
            any |= c;
        }
        if (any) atomicOr(&s_any, 1);
        __syncthreads();
        if (s_any) break;
        barrier = 5;
        __syncthreads();
    }
    if (!s_any) return;
    // filter + Shi-Tomasi; non-candidates get -inf, NaN maps to -inf too (sorts last)
    for (int i = threadIdx.x; i < span * span; i += 256) {
        const int cy = lo + i / span, cx = lo + i % span;
        float v = -INFINITY;
        if (s_sc[cy * g + cx] != 0.f) {
            const int x = cx + x_start, y = cy + y_start;
            if (!(x < 20 || y < 20 || x >= w - 20 || y >= h - 20) && occ[(size_t)y * w + x] != 255) {
                const float s = shi_tomasi(s_img + (cy + kDsoHalo) * S + cx + kDsoHalo, S);
                v = isnan(s) ? -INFINITY : s;
                if (v == -INFINITY) v = -3.4e38f;  // a candidate, ordered after every finite score
            }
        }
        s_sc[cy * g + cx] = v;
    }
    __syncthreads();
    int taken = 0;
    for (int r = 0; r < 3; r++) {
        if (threadIdx.x == 0) s_best = 0ull;
        __syncthreads();
        unsigned long long best = 0ull;
        for (int i = threadIdx.x; i < span * span; i += 256) {
            const int cy = lo + i / span, cx = lo + i % span;
            const float v = s_sc[cy * g + cx];
            if (v == -INFINITY) continue;
            // order-preserving float -> uint32, then prefer the lower scan index
            uint32_t u = __float_as_uint(v);
            u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
            const unsigned long long key = ((unsigned long long)u << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)i);
            best = key > best ? key : best;
        }
        for (int o = 32; o >= 1; o >>= 1) {
            const unsigned long long t = __shfl_xor(best, o, 64);
            best = t > best ? t : best;
        }
        if ((threadIdx.x & 63) == 0 && best) atomicMax(&s_best, best);
        __syncthreads();
        const unsigned long long b = s_best;
        if (!b) break;
        const int i = (int)(0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFu));
        const int cy = lo + i / span, cx = lo + i % span;
        if (threadIdx.x == 0) {
            out_keys[(size_t)k * 3 + r] = (uint32_t)(cx + x_start) | ((uint32_t)(cy + y_start) << 16);
            s_sc[cy * g + cx] = -INFINITY;
        }
        taken++;
        __syncthreads();
    }
    if (threadIdx.x == 0) out_cnt[k] = taken;
}

// compaction in cell order -> keypoints rows [row0, row0 + total)
__global__ __launch_bounds__(1024) void k_dso_finish(const uint32_t *__restrict__ keys,
                                                     const int *__restrict__ cnt, int ncells,
                                                     ygzfe_kp *__restrict__ kps, int row0,
                                                     int *__restrict__ total) {
    __shared__ int s_scan[1024];
    int base = 0;
    for (int c0 = 0; c0 < ncells; c0 += 1024) {
        const int c = c0 + threadIdx.x;
        const int n = c < ncells ? cnt[c] : 0;
        s_scan[threadIdx.x] = n;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const int v = threadIdx.x >= o ? s_scan[threadIdx.x - o] : 0;
            __syncthreads();
            s_scan[threadIdx.x] += v;
            __syncthreads();
        }
        const int pos = base + s_scan[threadIdx.x] - n;
        for (int j = 0; j < n; j++) {
            const uint32_t kk = keys[(size_t)c * 3 + j];
            ygzfe_kp kp;
            kp.x = (float)(kk & 0xFFFF);
            kp.y = (float)(kk >> 16);
            kp.size = 7.f;
            kp.angle = -1.f;
            kp.response = 0.f;
            kp.octave = 0;
            kp.class_id = -1;
            kps[row0 + pos + j] = kp;
        }
        base += s_scan[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = base;
}

__global__ void k_mark_occupancy(const ygzfe_kp *__restrict__ kps, int n, uint8_t *__restrict__ occ, int w,
                                 int h) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int x = (int)__builtin_rintf(kps[i].x), y = (int)__builtin_rintf(kps[i].y);
    if (x >= 0 && y >= 0 && x < w && y < h) occ[(size_t)y * w + x] = 255;
}

hipError_t launch_dso_occupancy(const ygzfe_kp *kps, int n, uint8_t *occ, int w, int h, hipStream_t st) {
    hipError_t e = hipMemsetAsync(occ, 0, (size_t)w * h, st);
    if (e != hipSuccess || n <= 0) return e;
    hipLaunchKernelGGL(k_mark_occupancy, dim3((n + 255) / 256), dim3(256), 0, st, kps, n, occ, w, h);
    return hipGetLastError();
}

hipError_t launch_dso_pass(const uint8_t *img, int w, int h, int g, const uint8_t *occ, uint32_t *keys, int *cnt,
                           hipStream_t st) {
    const int ncells = (h / g) * (w / g);
    if (ncells <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dso_cells, dim3(ncells), dim3(256), 0, st, img, w, h, g, occ, keys, cnt, 0,
                       (uint8_t *)nullptr);
    return hipGetLastError();
}

hipError_t launch_dso_cells_debug(const uint8_t *img, int w, int h, int g, int barrier, uint8_t *flags,
                                  hipStream_t st) {
    const int ncells = (h / g) * (w / g);
    if (ncells <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dso_cells, dim3(ncells), dim3(256), 0, st, img, w, h, g, (const uint8_t *)nullptr,
                       (uint32_t *)nullptr, (int *)nullptr, barrier, flags);
    return hipGetLastError();
}

hipError_t launch_dso_finish2(const uint32_t *keys, const int *cnt, int ncells, ygzfe_kp *kps, int row0,
                              int *total, hipStream_t st) {
    hipLaunchKernelGGL(k_dso_finish, dim3(1), dim3(1024), 0, st, keys, cnt, ncells, kps, row0, total);
    return hipGetLastError();
}

// Thirdparty/fast's fast_corner_detect_10 / _sse2 over caller ROIs (roi = x0, y0, w, h),
// the same segment test (fast10_corner) the DSO cells run.  Scan region per ROI:
// plain (variant 0) every pixel of the ROI (fast_10.cpp:35-42); SSE2 (variant 1)
// rows [3, h-3) x cols [3, w-3), a plain scan when w < 22 and nothing when h < 7
// (faster_corner_10_sse.cpp:24-202).  One 256-thread workgroup per ROI walks the
// region in raster order and appends corners in that order (the reference's
// vector order); counts may exceed cap (only the first cap are written).
__global__ __launch_bounds__(256) void k_fast10_rois(const uint8_t *__restrict__ img, int stride,
                                                     const int *__restrict__ rois, int barrier, int variant,
                                                     int16_t *__restrict__ out_xy, int cap,
                                                     int *__restrict__ counts) {
    __shared__ int s_wave[4];
    const int r = blockIdx.x;
    const int x0 = rois[4 * r], y0 = rois[4 * r + 1], w = rois[4 * r + 2], h = rois[4 * r + 3];
    int lo_x = 0, hi_x = w, lo_y = 0, hi_y = h;
    if (variant == 1 && w >= 22) {
        lo_x = 3, hi_x = w - 3, lo_y = 3, hi_y = h - 3;
        if (h < 7) hi_y = lo_y;
    }
    const int span = hi_x > lo_x ? hi_x - lo_x : 0;
    const int rows = hi_y > lo_y ? hi_y - lo_y : 0;
    const int total = span * rows;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int base = 0;
    for (int i0 = 0; i0 < total; i0 += 256) {
        const int i = i0 + threadIdx.x;
        int cx = 0, cy = 0;
        bool c = false;
        if (i < total) {
            cy = lo_y + i / span;
            cx = lo_x + i % span;
            c = fast10_corner(img + (size_t)(y0 + cy) * stride + (x0 + cx), stride, barrier);
        }
        const uint64_t m = __ballot(c);
        if (lane == 0) s_wave[wv] = __popcll(m);
        __syncthreads();
        int before = 0;
        for (int k = 0; k < wv; k++) before += s_wave[k];
        const int n_blk = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
        if (c) {
            const int pos = base + before + __popcll(m & ((1ull << lane) - 1ull));
            if (pos < cap) {
                out_xy[((size_t)r * cap + pos) * 2] = (int16_t)cx;
                out_xy[((size_t)r * cap + pos) * 2 + 1] = (int16_t)cy;
            }
        }
        base += n_blk;
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[r] = base;
}

hipError_t launch_fast10_rois(const uint8_t *img, int stride, const int *rois, int n_rois, int barrier,
                              int variant, int16_t *out_xy, int cap, int *counts, hipStream_t st) {
    if (n_rois <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fast10_rois, dim3(n_rois), dim3(256), 0, st, img, stride, rois, barrier, variant, out_xy,
                       cap, counts);
    return hipGetLastError();
}

}  // namespace ygzfe
