// common.hpp — shared definitions of the ygzfe HIP library (gfx950 only).
//
// Data layout in HBM:
//  * frame pyramid: one contiguous buffer of P = sum_l w_l*h_l bytes per frame,
//    level l at byte offset off[l], tight stride w_l (Frame::mvImagePyramid after
//    clone(), Frame.cc:810-813).  Batches stack frames at a fixed pitch P.
//  * blurred pyramid: same layout (GaussianBlur of every level,
//    ORBextractor.cc:1079-1084).
//  * FAST candidates: per (frame, cell) slot of cell_cap packed u32 keys
//    (x_rel:12 | y_rel:12 | score:8), in raster order, plus a count.
//  * octree output: per (frame, level) slot of sel_cap packed keys in
//    std::list order (ORBextractor.cc:707-720), plus a count.
//  * keypoints: ygzfe_kp rows (cv::KeyPoint layout) + 32-byte descriptors.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ygzfe.h"

namespace ygzfe {

constexpr int kMaxLevels = YGZFE_MAX_LEVELS;
constexpr int kBlurRows = 32;  // k_blur7 strip height (plan.cpp tiles the levels with it)
constexpr int kEdgeThreshold = 19;  // ORBextractor.cc:75
constexpr int kMinBorder = kEdgeThreshold - 3;
constexpr int kPatchSize = 31, kHalfPatch = 15;
constexpr int kMaxRoi = 72;          // max FAST cell ROI side (wCell <= 60, +6)

struct LevelDesc {
    int w, h;
    uint32_t off;        // byte offset of the level inside a frame pyramid
    int budget;          // mnFeaturesPerLevel
    int patch_size;      // scaledPatchSize (ORBextractor.cc:789)
    float scale, inv_scale;
    int cell_begin, ncells;
    int max_bx, max_by;  // maxBorderX / maxBorderY
    int n_ini;           // DistributeOctTree initial node count
    float hX;
    int sel_off, sel_cap;   // octree output slot inside a frame's selection buffer
    int cand_off, cand_cap; // candidate (key) scratch slot inside a frame
    int resize_mode;     // 0 = copy/none (level 0), 1 = area x2, 2 = bilinear
    int xtab_off, ytab_off;  // bilinear tables (ints) in the plan table buffer
    int xmax;
    int blur_tile_begin, blur_tiles_x, blur_tiles_y;
    int pyr_tile_begin;
    int fast_roi;        // largest FAST cell ROI side of this level
    int fast_rw, fast_rh;  // largest FAST cell ROI width / height of this level
};

struct CellDesc {
    int16_t x0, y0, rw, rh;   // ROI origin / size in level pixels
    int16_t offx, offy;       // j*wCell, i*hCell (key coordinates relative to minBorder)
    int16_t level, pad;
};

struct Plan {
    int W, H, nlevels;
    uint32_t pyr_bytes;       // P
    int ncells;               // total over levels
    int cell_cap;             // max NMS-surviving corners of any cell
    int sel_total;            // per-frame selection slots (sum of sel_cap)
    int cand_total;           // per-frame candidate slots
    int kp_cap;               // per-frame keypoint rows (sum over levels of sel_cap)
    int ini_th, min_th;
    int blur_variant;
    int blur_tiles;           // total blur tiles over levels
    int node_cap;             // octree node pool capacity (template instance)
    int fast_S;               // LDS row stride of a FAST cell ROI (max ROI side, multiple of 4)
    int umax[16];             // IC_Angle circle rows (ORBextractor.cc:453-467)
    LevelDesc lv[kMaxLevels];
};

// --------------------------------------------------------------------------
// device helpers

// Global-memory view of a pointer whose address space the compiler cannot
// infer (struct members, integer arithmetic): loads through it are global_load_*
// instead of flat_load_*, which also count against lgkmcnt and so serialise
// with LDS traffic.
template <class T>
using gptr_t = const __attribute__((address_space(1))) T *;
template <class T>
__device__ __forceinline__ gptr_t<T> as_global(const T *p) {
    return (gptr_t<T>)p;
}

// Diagnostic build only (make diag -> lib/libygzfe_diag.so): per-workgroup
// s_memrealtime (100 MHz, chip-synchronous) at kernel entry / exit, plus the
// XCC id, for dispatch / duration histograms (tools/diag_blocks.py).
#ifdef YGZ_STAMPS
#ifndef YGZ_STAMP_KERNEL
#define YGZ_STAMP_KERNEL 1  // 1 = k_orient_desc, 2 = k_fast_cells (level 0)
#endif
extern __device__ unsigned long long g_bstamps[1 << 20];
#define YGZ_BSTAMP_K(kern, slot)                                                                 \
    do {                                                                                          \
        if ((kern) != YGZ_STAMP_KERNEL) break;                                                    \
        const unsigned _b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);        \
        if (threadIdx.x == 0 && _b < (1u << 17))                                                   \
            g_bstamps[8 * _b + (slot)] = (slot) == 2 ? (unsigned long long)__builtin_amdgcn_s_getreg(   \
                                                           (20 << 0) | (0 << 6) | (3 << 11))      \
                                                     : __builtin_amdgcn_s_memrealtime();           \
    } while (0)
#define YGZ_BVAL_K(kern, slot, val)                                                              \
    do {                                                                                          \
        if ((kern) != YGZ_STAMP_KERNEL) break;                                                    \
        const unsigned _b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);        \
        if (threadIdx.x == 0 && _b < (1u << 17)) g_bstamps[8 * _b + (slot)] = (unsigned long long)(val); \
    } while (0)
#else
#define YGZ_BSTAMP_K(kern, slot) do {} while (0)
#define YGZ_BVAL_K(kern, slot, val) do {} while (0)
#endif

// Order LDS traffic between lanes of ONE wave: DS instructions of a wave
// execute in issue order, so only the compiler must not reorder them.  (A
// wavefront-scope fence would also emit s_waitcnt vmcnt(0) and stall on any
// global prefetch in flight.)
__device__ __forceinline__ void wave_lds_order() { __asm__ __volatile__("" ::: "memory"); }

// XCD-aware block order (cdna_hip_programming.md T1, bijective form): blocks
// dealt to one XCD (orig % 8) get one contiguous range of logical ids, so a
// frame's blocks share an L2.  A speed choice only; results never depend on it.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = orig & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (orig >> 3);
}

// logical (x, y) block coordinates of a 2D grid after the swizzle
__device__ __forceinline__ void swizzled_block_2d(int &bx, int &by) {
    const int orig = blockIdx.x + gridDim.x * blockIdx.y;
    const int id = xcd_swizzle(orig, gridDim.x * gridDim.y);
    bx = id % gridDim.x;
    by = id / gridDim.x;
}

__device__ __forceinline__ int lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

__device__ __forceinline__ int popc_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// cvRound on float: round half to even
__device__ __forceinline__ int cv_round(float v) { return (int)__builtin_rintf(v); }

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__host__ __device__ __forceinline__ uint32_t pack_key(int x, int y, int score) {
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)score << 24);
}
__host__ __device__ __forceinline__ int key_x(uint32_t k) { return (int)(k & 0xFFFu); }
__host__ __device__ __forceinline__ int key_y(uint32_t k) { return (int)((k >> 12) & 0xFFFu); }
__host__ __device__ __forceinline__ int key_score(uint32_t k) { return (int)(k >> 24); }

// cv::fastAtan2 (degrees): see oracle/orb.c ygzo_fast_atan2 for the restated formula.
__device__ __forceinline__ float fast_atan2_deg(float y, float x) {
    const float k = (float)(180 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float eps = (float)2.220446049250313e-16;
    float ax = fabsf(x), ay = fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

}  // namespace ygzfe

// --------------------------------------------------------------------------
// host-side error plumbing

namespace ygzfe {
void set_error(const char *fmt, ...);
}

// hipError_t-returning variant for launch helpers
#define YGZ_HIPR(call)                 \
    do {                               \
        hipError_t e_ = (call);        \
        if (e_ != hipSuccess) return e_; \
    } while (0)

#define YGZ_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ygzfe::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call,              \
                             hipGetErrorString(e_));                                   \
            return YGZFE_EHIP;                                                         \
        }                                                                              \
    } while (0)
