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
#ifndef YGZ_BLUR_ROWS
#define YGZ_BLUR_ROWS 32
#endif
constexpr int kBlurRows = YGZ_BLUR_ROWS;  // k_blur7 strip height (plan.cpp tiles the levels with it)
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
    // octree path codes (k_octree_paths): root bits, quadrant depth carried, and the
    // separable code tables in Plan::dtabs (code = X[x] | Y[y], key coordinates)
    int oct_rb, oct_dn, oct_xtab, oct_ytab;
};

struct alignas(16) CellDesc {
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
    const int32_t *dtabs;     // device copy of PlanHost::tabs (set at upload)
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
// ... and for stores: global_store_* (vmcnt only) instead of flat_store_*, which an
// LDS wait (lgkmcnt) would otherwise also wait on
template <class T>
using gmut_t = __attribute__((address_space(1))) T *;
template <class T>
__device__ __forceinline__ gmut_t<T> as_global_mut(T *p) {
    return (gmut_t<T>)p;
}
// a * b + c on 24-bit operands (v_mad_u32_u24, full rate); inline asm so the
// compiler cannot widen it into a quarter-rate v_mad_u64_u32
__device__ __forceinline__ uint32_t mad24(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm volatile("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// read-only data at a wave-uniform address through the scalar cache (constant
// address space: s_load, no vector-memory round trip)
template <class T>
using cptr_t = const __attribute__((address_space(4))) T *;
template <class T>
__device__ __forceinline__ T scalar_load(const T *p) {
    // dword-granular (s_load needs 4-B alignment; the records here are 4-B aligned)
    static_assert(sizeof(T) % 4 == 0, "scalar_load: dword-sized records only");
    struct W { uint32_t d[sizeof(T) / 4]; };
    return __builtin_bit_cast(T, *(cptr_t<W>)p);
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

// glibc's sinf / cosf for |y| < 120 (the rBRIEF angle, ORBextractor.cc:109
// std::cos(float) -> the C library's cosf): the double-evaluated polynomial of
// glibc >= 2.28 (sincosf.h), restated in oracle/orb.c ygzo_sincosf and pinned
// there bit for bit against this image's libm over [0, 2pi).  v_fma_f64 is not
// used: the file is built with -ffp-contract=off, as glibc's generic variant.
__device__ __forceinline__ float glibc_sinf_poly(double x, double x2, bool cos_branch, bool neg_cos) {
    if (!cos_branch) {
        const double x3 = x * x2;
        const double s1 = 0x1.1107605230bc4p-7 + x2 * -0x1.994eb3774cf24p-13;
        const double x7 = x3 * x2;
        const double s = x + x3 * -0x1.555545995a603p-3;
        return (float)(s + x7 * s1);
    }
    const double g = neg_cos ? -1.0 : 1.0;  // the table[1] cosine coefficients are negated (exact)
    const double x4 = x2 * x2;
    const double c2 = g * -0x1.6c087e89a359dp-10 + x2 * (g * 0x1.99343027bf8c3p-16);
    const double c1 = g * 0x1p0 + x2 * (g * -0x1.ffffffd0c621cp-2);
    const double x6 = x4 * x2;
    const double c = c1 + x4 * (g * 0x1.55553e1068f19p-5);
    return (float)(c + x6 * c2);
}

static __constant__ const uint32_t c_inv_pio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};

__device__ __forceinline__ void glibc_sincosf(float y, float &sinv, float &cosv) {
    const uint32_t top = (__float_as_uint(y) >> 20) & 0x7ffu;
    double x = y;
    if (top >= ((__float_as_uint(120.0f) >> 20) & 0x7ffu)) {  // never reached by octree angles
        if (!(fabsf(y) <= 3.40282347e38f)) {
            sinv = cosv = __builtin_nanf("");
            return;
        }
        // reduce_large: integer product with the 4/pi bit window (s_sincosf_data.c __inv_pio4)
        const uint32_t *kInvPio4 = c_inv_pio4;
        uint32_t xi = __float_as_uint(y);
        const int sign = (int)(xi >> 31);
        const int a = (xi >> 26) & 15, shift = (xi >> 23) & 7;
        xi = ((xi & 0xffffffu) | 0x800000u) << shift;
        uint64_t res0 = (uint64_t)(uint32_t)(xi * kInvPio4[a]);
        const uint64_t res1 = (uint64_t)xi * kInvPio4[a + 4];
        const uint64_t res2 = (uint64_t)xi * kInvPio4[a + 8];
        res0 = ((res2 >> 32) | (res0 << 32)) + res1;
        const uint64_t nq = (res0 + (1ull << 61)) >> 62;
        res0 -= nq << 62;
        x = (double)(int64_t)res0 * 0x1.921FB54442D18p-62;
        const int n = (int)nq, ns = n + sign;
        const double s = ((ns + 1) & 2) ? -1.0 : 1.0;
        const bool neg = (ns & 2) != 0;
        sinv = glibc_sinf_poly(x * s, x * x, (n & 1) != 0, neg);
        cosv = glibc_sinf_poly(x * s, x * x, (n & 1) == 0, neg);
        return;
    }
    if (top < ((__float_as_uint(0x1p-12f) >> 20) & 0x7ffu)) {
        sinv = y;
        cosv = 1.0f;
        return;
    }
    // |y| < pi/4 (glibc's first branch) is the n = 0 case of the reduction below: x * 2/pi
    // < 0.5 gives n = 0, x - 0 * pi/2 = x, sign +1 and table 0, so one path serves both.
    // Each polynomial is evaluated once, unsigned: the sine one is odd and the negated
    // cosine table (table 1) negates every coefficient, so sign and table come out as
    // exact float negations, and (n & 1) only swaps the two results.  (glibc_sinf_poly's
    // lane-dependent branches would otherwise run both polynomials twice per wave.)
    const double r = x * 0x1.45F306DC9C883p+23;  // reduce_fast: 2/pi * 2^24, truncating conversion
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * 0x1.921FB54442D18p0;
    const double x2 = x * x;
    const float sp = glibc_sinf_poly(x, x2, false, false), cp = glibc_sinf_poly(x, x2, true, false);
    const float ss = ((n + 1) & 2) ? -sp : sp;  // sign[n & 3] = {1, -1, -1, 1}
    const float cs = (n & 2) ? -cp : cp;        // table 1: the cosine coefficients negated
    sinv = (n & 1) ? cs : ss;
    cosv = (n & 1) ? ss : cs;
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
