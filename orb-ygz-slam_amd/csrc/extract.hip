// extract.hip — ORB extraction kernels for gfx950 (ORBSLAM_KEYPOINT mode).
//
// Stage            reference                               kernel
// pyramid          ORBextractor.cc:1129-1150               k_resize_area2 / k_resize_linear
// blur 7x7 s=2     ORBextractor.cc:1079-1084               k_blur7
// FAST-9 per cell  ORBextractor.cc:747-781 (+cv::FAST)     k_fast_cells
// octree           ORBextractor.cc:533-723, 783-798        k_octree_sort / k_octree_list
// angle + rBRIEF   ORBextractor.cc:77-149, 1101-1125       k_orient_desc / k_desc_existing
//
// Everything is batched over frames (grid.z / grid.y = frame) so one launch per
// stage serves a whole resident batch.  Bit-exactness with oracle/ is the
// contract: integer paths are exact, float expressions follow the reference's
// evaluation order and the library is built with -ffp-contract=off.
#include "common.hpp"

#include <algorithm>
#include <type_traits>

#include "plan.hpp"

namespace ygzfe {

__constant__ __attribute__((aligned(16))) int8_t c_pattern[1024];
// The same pattern as FP8 (OCP E4M3, gfx950's format): every coordinate is an integer with
// |v| <= 13, exact in E4M3 (3 mantissa bits hold every integer up to 16), so one
// v_cvt_pk_f32_fp8 turns a point's two bytes into its (x, y) floats: half the
// conversions of the int8 form (k_orient_desc)
__constant__ __attribute__((aligned(16))) uint8_t c_pattern_f8[1024];

#ifdef YGZ_STAMPS
__device__ unsigned long long g_bstamps[1 << 20];
extern "C" int ygzfe_diag_block_stamps(unsigned long long *out, int n) {
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bstamps), sizeof(unsigned long long) * (size_t)n);
    return 0;
}
#endif

// ---------------------------------------------------------------------------
// Pyramid

// OpenCV INTER_AREA fast path for an exact x2 downscale: (a+b+c+d+2)>>2.
__global__ __launch_bounds__(256) void k_resize_area2(uint8_t *__restrict__ pyr, uint32_t pitch,
                                                      const Plan *__restrict__ plan, int l) {
    const LevelDesc &S = plan->lv[l - 1];
    const LevelDesc &D = plan->lv[l];
    const int f = blockIdx.z;
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= D.w || y >= D.h) return;
    const uint8_t *s = pyr + (size_t)f * pitch + S.off + (size_t)(2 * y) * S.w + 2 * x;
    const int v = s[0] + s[1] + s[S.w] + s[S.w + 1] + 2;
    pyr[(size_t)f * pitch + D.off + (size_t)y * D.w + x] = (uint8_t)(v >> 2);
}

// The whole chain of exact x2 INTER_AREA levels 1..K in one pass: one lane per
// level-K pixel reads its 2^K x 2^K level-0 block (one 2^K-byte load per row,
// a wave's loads of a row are contiguous), forms every intermediate level in
// registers with the same (a+b+c+d+2)>>2 rounding, and writes each level's
// rows of the block (dword / ushort / byte stores).  Levels nest exactly
// (resize_mode 1 <=> w_{l-1} = 2 w_l, h_{l-1} = 2 h_l), so level 0 holds
// 2^K-aligned rows.
template <int K>
__global__ __launch_bounds__(256) void k_pyramid_area_chain(uint8_t *__restrict__ pyr, uint32_t pitch,
                                                            const Plan *__restrict__ plan) {
    constexpr int B = 1 << K;
    const LevelDesc &LK = plan->lv[K];
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= LK.w * LK.h) return;
    const int y = i / LK.w, x = i - y * LK.w;
    uint8_t *fr = pyr + (size_t)f * pitch;
    const int W0 = plan->lv[0].w;
    int v[B][B];
    const uint8_t *src = fr + (size_t)(B * y) * W0 + B * x;
#pragma unroll
    for (int r = 0; r < B; r++) {
        if constexpr (B == 8) {
            const uint2 q = *reinterpret_cast<const uint2 *>(src + (size_t)r * W0);
#pragma unroll
            for (int c = 0; c < 4; c++) { v[r][c] = (q.x >> (8 * c)) & 0xFF; v[r][4 + c] = (q.y >> (8 * c)) & 0xFF; }
        } else if constexpr (B == 4) {
            const uint32_t q = *reinterpret_cast<const uint32_t *>(src + (size_t)r * W0);
#pragma unroll
            for (int c = 0; c < 4; c++) v[r][c] = (q >> (8 * c)) & 0xFF;
        } else {
            const uint16_t q = *reinterpret_cast<const uint16_t *>(src + (size_t)r * W0);
            v[r][0] = q & 0xFF;
            v[r][1] = q >> 8;
        }
    }
#pragma unroll
    for (int l = 1; l <= K; l++) {
        const int n = B >> l;  // this level's block side
        const LevelDesc &D = plan->lv[l];
#pragma unroll
        for (int r = 0; r < n; r++) {
#pragma unroll
            for (int c = 0; c < n; c++)
                v[r][c] = (v[2 * r][2 * c] + v[2 * r][2 * c + 1] + v[2 * r + 1][2 * c] + v[2 * r + 1][2 * c + 1] + 2) >> 2;
            uint8_t *dst = fr + D.off + (size_t)(n * y + r) * D.w + n * x;
            if (n == 4)
                *reinterpret_cast<uint32_t *>(dst) =
                    (uint32_t)v[r][0] | ((uint32_t)v[r][1] << 8) | ((uint32_t)v[r][2] << 16) | ((uint32_t)v[r][3] << 24);
            else if (n == 2)
                *reinterpret_cast<uint16_t *>(dst) = (uint16_t)(v[r][0] | (v[r][1] << 8));
            else
                *dst = (uint8_t)v[r][0];
        }
    }
}

// OpenCV fixed-point INTER_LINEAR (11-bit coefficients), scalar rounding
// (b0*S0 + b1*S1 + 2^21) >> 22.  xtab[dx] = {sx, a0|a1<<16}, ytab[dy] = {ya, yb, b0|b1<<16}.
__global__ __launch_bounds__(256) void k_resize_linear(uint8_t *__restrict__ pyr, uint32_t pitch,
                                                       const Plan *__restrict__ plan,
                                                       const int *__restrict__ tabs, int l) {
    const LevelDesc &S = plan->lv[l - 1];
    const LevelDesc &D = plan->lv[l];
    const int f = blockIdx.z;
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= D.w || y >= D.h) return;
    const int *xt = tabs + D.xtab_off + 2 * x;
    const int *yt = tabs + D.ytab_off + 3 * y;
    const int sx = xt[0];
    const int a0 = (int)(int16_t)(xt[1] & 0xFFFF), a1 = (int)(int16_t)(xt[1] >> 16);
    const int b0 = (int)(int16_t)(yt[2] & 0xFFFF), b1 = (int)(int16_t)(yt[2] >> 16);
    const uint8_t *base = pyr + (size_t)f * pitch + S.off;
    const uint8_t *ra = base + (size_t)yt[0] * S.w, *rb = base + (size_t)yt[1] * S.w;
    int r0, r1;
    if (x < D.xmax) {
        r0 = ra[sx] * a0 + ra[sx + 1] * a1;
        r1 = rb[sx] * a0 + rb[sx + 1] * a1;
    } else {
        r0 = ra[sx] * 2048;
        r1 = rb[sx] * 2048;
    }
    const int v = (b0 * r0 + b1 * r1 + (1 << 21)) >> 22;
    pyr[(size_t)f * pitch + D.off + (size_t)y * D.w + x] = (uint8_t)clampi(v, 0, 255);
}

// Every INTER_LINEAR level from l0 on in one launch, one workgroup per frame (the
// batch path): level l is formed from level l-1 by the whole workgroup, four output
// pixels per thread per step, a barrier between levels.  The frame's levels
// (~1 MB for C4) stay in the CU's L1 / the XCD's L2 between levels.  A thread's four
// pixels x0..x0+3 need source bytes [sx0, sx3 + 1] of two rows, at most 9 bytes
// from the dword below sx0: three dword loads per row; same arithmetic as
// k_resize_linear.
__device__ __forceinline__ uint32_t pair_at(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t o) {
    // bytes o, o + 1 (o <= 8) of d2:d1:d0 in the low 16 bits
    const uint32_t lo = o < 4 ? d0 : (o < 8 ? d1 : d2), hi = o < 4 ? d1 : d2;
    return __builtin_amdgcn_alignbyte(hi, lo, o & 3u) & 0xFFFFu;
}

#ifndef YGZ_PYR_BATCH
#define YGZ_PYR_BATCH 4
#endif
constexpr int kPyrBatch = YGZ_PYR_BATCH;

__global__ __launch_bounds__(1024) void k_pyramid_linear_chain(uint8_t *__restrict__ pyr, uint32_t pitch,
                                                               const Plan *__restrict__ plan,
                                                               const int *__restrict__ tabs, int l0) {
    // the level's tables in LDS: x {sx, a0 | a1 << 16} (w <= 2048), y {ya, yb, b0 | b1 << 16} (h <= 2048)
    __shared__ int2 s_xt[2048];
    __shared__ int s_yt[3 * 2048];
    uint8_t *fr = pyr + (size_t)blockIdx.x * pitch;
    for (int l = l0; l < plan->nlevels; l++) {
        const LevelDesc &S = plan->lv[l - 1];
        const LevelDesc &D = plan->lv[l];
        for (int i = threadIdx.x; i < D.w; i += 1024)
            s_xt[i] = make_int2(tabs[D.xtab_off + 2 * i], tabs[D.xtab_off + 2 * i + 1]);
        for (int i = threadIdx.x; i < 3 * D.h; i += 1024) s_yt[i] = tabs[D.ytab_off + i];
        __syncthreads();  // tables in; level l - 1 complete (workgroup scope: one CU's L1)
        const int gw = (D.w + 3) >> 2, ng = gw * D.h;
        const uint8_t *src = fr + S.off;
        uint8_t *dst = fr + D.off;
        // kPyrBatch groups per thread per step: every source window of the step is loaded
        // before any of its stores (the compiler cannot hoist loads above stores that may
        // alias them).  Batches of 1, 4 and 8 measured equal, 0.285-0.288 ms / 256 frames
        // (profiles/r04_c4_pyramid_batch.txt): the load -> store round trip does not bind.
        for (int g0 = threadIdx.x; g0 < ng; g0 += 1024 * kPyrBatch) {
            uint4 wa[kPyrBatch], wb[kPyrBatch];
#pragma unroll
            for (int u = 0; u < kPyrBatch; u++) {
                const int g = g0 + 1024 * u;
                wa[u] = wb[u] = make_uint4(0u, 0u, 0u, 0u);
                if (g < ng) {
                    const int y = g / gw, x0 = (g - y * gw) * 4;
                    const int ya = s_yt[3 * y], yb = s_yt[3 * y + 1];
                    const uint32_t base = (uint32_t)s_xt[x0].x & ~3u;
                    const uint32_t sa = (uint32_t)((size_t)ya * S.w & 3), sb = (uint32_t)((size_t)yb * S.w & 3);
                    const uint32_t *ra = reinterpret_cast<const uint32_t *>(src + (size_t)ya * S.w + base - sa);
                    const uint32_t *rb = reinterpret_cast<const uint32_t *>(src + (size_t)yb * S.w + base - sb);
                    wa[u] = make_uint4(ra[0], ra[1], ra[2], ra[3]);
                    wb[u] = make_uint4(rb[0], rb[1], rb[2], rb[3]);
                }
            }
#pragma unroll
            for (int u = 0; u < kPyrBatch; u++) {
                const int g = g0 + 1024 * u;
                if (g >= ng) break;
                const int y = g / gw, x0 = (g - y * gw) * 4;
                const int ya = s_yt[3 * y], yb = s_yt[3 * y + 1], bw = s_yt[3 * y + 2];
                const int b0 = (int)(int16_t)(bw & 0xFFFF), b1 = (int)(int16_t)(bw >> 16);
                const int sx0 = s_xt[x0].x;
                const uint32_t base = (uint32_t)sx0 & ~3u;
                const uint32_t sa = (uint32_t)((size_t)ya * S.w & 3), sb = (uint32_t)((size_t)yb * S.w & 3);
                uint32_t out = 0u;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int x = x0 + i;
                    const int2 xt = s_xt[x < D.w ? x : x0];
                    const int sx = xt.x;
                    const int a0 = (int)(int16_t)(xt.y & 0xFFFF), a1 = (int)(int16_t)(xt.y >> 16);
                    // byte offsets of sx inside the dword windows of the two rows
                    const uint32_t oa = (uint32_t)(sx - (int)base) + sa, ob = (uint32_t)(sx - (int)base) + sb;
                    const uint32_t pa = oa < 8 ? pair_at(wa[u].x, wa[u].y, wa[u].z, oa) : pair_at(wa[u].y, wa[u].z, wa[u].w, oa - 4);
                    const uint32_t pb = ob < 8 ? pair_at(wb[u].x, wb[u].y, wb[u].z, ob) : pair_at(wb[u].y, wb[u].z, wb[u].w, ob - 4);
                    int r0, r1;
                    if (x < D.xmax) {
                        r0 = (int)(pa & 0xFF) * a0 + (int)(pa >> 8) * a1;
                        r1 = (int)(pb & 0xFF) * a0 + (int)(pb >> 8) * a1;
                    } else {
                        r0 = (int)(pa & 0xFF) * 2048;
                        r1 = (int)(pb & 0xFF) * 2048;
                    }
                    const int v = (b0 * r0 + b1 * r1 + (1 << 21)) >> 22;
                    out |= (uint32_t)clampi(v, 0, 255) << (8 * i);
                }
                uint8_t *o = dst + (size_t)y * D.w + x0;
                if (x0 + 4 <= D.w && (((uintptr_t)o & 3) == 0)) {
                    *reinterpret_cast<uint32_t *>(o) = out;
                } else {
                    for (int i = 0; i < 4 && x0 + i < D.w; i++) o[i] = (uint8_t)(out >> (8 * i));
                }
            }
        }
        __syncthreads();  // level l complete and the tables free before the next level
    }
}

// ---------------------------------------------------------------------------
// GaussianBlur 7x7 sigma=2, BORDER_REFLECT_101, 8-bit fixed point:
//   dst = sat8((sum_v k_v * (sum_h k_h * p) + 2^15) >> 16)
// One 256-thread workgroup per 64x16 output tile; the (16+6)x(64+6) source
// window and the horizontal sums live in LDS.

__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

// One wave per 256-column x kBlurRows-row strip, no LDS: lane owns 4 adjacent
// columns.  Each source row is read ONCE, as one dword per lane (a wave reads
// the 256 strip bytes with a single coalesced 256-B load; 3 more lanes fetch
// the dwords just left / right of the strip), and the 10-byte tap window
// [x-3, x+6] is assembled from the neighbouring lanes' dwords with DPP wave
// shifts.  The row index, its BORDER_REFLECT_101 mirror and the row address
// are wave-uniform (SGPRs).  Rows are prefetched kBlurAhead rows ahead.  The
// horizontal taps are two v_dot4_u32_u8 per pixel; the vertical taps slide
// over a 7-row register ring with 24-bit multiply-adds.  The first four
// columns (x < 4) and the last three (whose taps reach past the row) come out
// wrong; they are not stored by the main loop and are recomputed with
// BORDER_REFLECT_101 taps at the end.
#ifndef YGZ_BLUR_AHEAD
#define YGZ_BLUR_AHEAD 10  // rows in flight per wave
#endif
constexpr int kBlurAhead = YGZ_BLUR_AHEAD;

__device__ __forceinline__ void blur_hsum(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t o,
                                          uint32_t ka, uint32_t kb, uint32_t h[4]) {
    const uint32_t p0 = __builtin_amdgcn_alignbyte(w1, w0, o);
    const uint32_t p1 = __builtin_amdgcn_alignbyte(w2, w1, o);
    const uint32_t p2 = __builtin_amdgcn_alignbyte(w3, w2, o);
    h[0] = __builtin_amdgcn_udot4(p1, kb, __builtin_amdgcn_udot4(p0, ka, 0u, false), false);
#pragma unroll
    for (int j = 1; j < 4; j++)
        h[j] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(p2, p1, j), kb,
                                      __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(p1, p0, j), ka, 0u, false),
                                      false);
}

// exact 7x7 output at (x, y) with reflected taps (border columns, tiny levels)
__device__ __forceinline__ uint8_t blur_pixel_reflect(const uint8_t *__restrict__ src, int w, int h, int x, int y,
                                                      const int kk[7]) {
    int xs[7], acc = 0;
#pragma unroll
    for (int k = 0; k < 7; k++) xs[k] = reflect101(x - 3 + k, w);
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const uint8_t *row = src + (size_t)reflect101(y - 3 + r, h) * w;
        int hs = 0;
#pragma unroll
        for (int k = 0; k < 7; k++) hs += kk[k] * row[xs[k]];
        acc += kk[r] * hs;
    }
    return (uint8_t)min((acc + 32768) >> 16, 255);
}

// DPP whole-wave shifts by one lane (GFX9 wave_shl:1 / wave_shr:1): lane l
// receives lane l+1's / l-1's value; the lane shifted in from outside keeps 0
__device__ __forceinline__ uint32_t wave_from_next(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_from_prev(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}

struct BlurRow {
    uint32_t a;     // the lane's dword of the row (aligned)
    uint32_t halo;  // lane 0: dword left of the strip, lanes 1-2: the two right of it
    uint32_t o;     // row misalignment (row start & 3), wave-uniform
};

// Rows whose width is a multiple of 4 (every row dword-aligned: C2 levels
// 0-2): lane l's dword A_l holds columns x..x+3 and the tap window [x-3, x+6]
// is bytes 1..3 of A_{l-1}, A_l and bytes 0..2 of A_{l+1}.  The neighbours'
// dwords come by DPP wave shifts whose shifted-in lane keeps its own halo
// dword (lane 0: the dword left of the strip, lane 63: the one right of it).
// BORDER_REFLECT_101 is applied to the bytes themselves: at the left edge lane
// 0's left neighbour dword becomes (b4, b3, b2, b1); at the right edge the
// dword holding columns w..w+2 becomes (b[w-2], b[w-3], b[w-4]), so every
// output column, border ones included, comes out of the main loop.
// Loads and stores are buffer operations on the level (32-bit lane offsets,
// the row offset a scalar; reads past the level return 0 and are never used).
// Horizontal taps: the kernel shifted over the window bytes, 10 v_dot4_u32_u8
// per 4 pixels.  Vertical taps: the row sums (<= 255 * 256, 16 bits) of
// consecutive rows packed in pairs, three v_dot2_u32_u16 + one 24-bit
// multiply-add per pixel.
// The exact x2 INTER_AREA levels 1..K (K <= 3) of a level-0 strip, formed from the
// strip's own rows as the blur streams them (k_blur7's fused mode, the batch path of
// an all-area pyramid): lane l's dword holds columns x..x+3 of a row, so a row pair
// gives its two level-1 pixels, two row pairs its level-2 pixel and four the level-3
// pixel of the lane pair (l, l ^ 1) -- the (a + b + c + d + 2) >> 2 chain of
// k_pyramid_area_chain, level from level.  Strips are 256 columns x kBlurRows rows
// (multiples of 8), so every block lies inside one strip.
struct PyrFused {
    uint8_t *frame;   // the frame's pyramid (level 0 read by the blur, levels 1..K written here)
    int K;            // levels to form (0: none)
    uint32_t off[4];  // level offsets in the frame
    uint32_t w[4];    // level widths
    uint32_t prev;    // the previous (even) row's dword
    uint32_t l1;      // the lane's level-1 pair of the previous odd row (low: cols 0-1, high: 2-3)
    uint32_t l2;      // the lane's level-2 pixel of the previous level-2 row
};
#define YGZ_PYR_FUSED_ROW(P, raw, yy, x, store_lane, rs)                                                          \
    do {                                                                                                          \
        if ((yy) & 1) {                                                                                           \
            const uint32_t a_ = __builtin_amdgcn_udot4((raw), 0x00000101u, __builtin_amdgcn_udot4((P).prev, 0x00000101u, 2u, false), false) >> 2; \
            const uint32_t b_ = __builtin_amdgcn_udot4((raw), 0x01010000u, __builtin_amdgcn_udot4((P).prev, 0x01010000u, 2u, false), false) >> 2; \
            if (store_lane)                                                                                       \
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(a_ | (b_ << 8)), (rs),                            \
                    (P).off[1] + ((uint32_t)(yy) >> 1) * (P).w[1] + ((uint32_t)(x) >> 1), 0, 0);                   \
            if ((P).K >= 2 && ((yy) & 3) == 3) {                                                                  \
                const uint32_t l2_ = ((P).l1 & 0xFFu) + ((P).l1 >> 8) + a_ + b_ + 2u;                             \
                const uint32_t v2_ = l2_ >> 2;                                                                    \
                if (store_lane)                                                                                   \
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v2_, (rs),                                       \
                        (P).off[2] + ((uint32_t)(yy) >> 2) * (P).w[2] + ((uint32_t)(x) >> 2), 0, 0);               \
                if ((P).K >= 3 && ((yy) & 7) == 7) {                                                              \
                    const uint32_t t_ = (P).l2 + v2_;                                                             \
                    const uint32_t n_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t_, 0xB1, 0xF, 0xF, false); \
                    if ((store_lane) && ((x) & 7) == 0)                                                           \
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)((t_ + n_ + 2u) >> 2), (rs),                 \
                            (P).off[3] + ((uint32_t)(yy) >> 3) * (P).w[3] + ((uint32_t)(x) >> 3), 0, 0);           \
                }                                                                                                 \
                (P).l2 = v2_;                                                                                     \
            }                                                                                                     \
            (P).l1 = a_ | (b_ << 8);                                                                              \
        } else {                                                                                                  \
            (P).prev = (raw);                                                                                     \
        }                                                                                                         \
    } while (0)

template <bool CV3, bool PYR>
__device__ __forceinline__ void blur_strip_aligned(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, int w,
                                                   int hgt, int sx, int y0, int lane, PyrFused &pf) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    constexpr uint32_t k0 = 18, k1 = 34, k2 = CV3 ? 49 : 48, k3 = CV3 ? 55 : 56;
    const int x = sx + 4 * lane;
    const bool left_edge = sx == 0, right_edge = sx + 256 >= w;
    const uint32_t nbytes = (uint32_t)w * (uint32_t)hgt;
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, (int)nbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc((void *)dst, 0, (int)nbytes, 0x00020000);
    const uint32_t voff = (uint32_t)x;
    // halo: lane 0 the dword at x - 4 (ignored at the left edge), lane 63 the one at x + 4
    const uint32_t hoff = lane == 0 ? voff - 4u : voff + 4u;
    // shifted horizontal kernels: h[j] = dot4(p0, K0j) + dot4(p1, K1j) + dot4(p2, K2j)
    constexpr uint32_t K00 = k0 | (k1 << 8) | (k2 << 16) | (k3 << 24), K10 = k2 | (k1 << 8) | (k0 << 16);
    constexpr uint32_t K01 = K00 << 8, K11 = k3 | (k2 << 8) | (k1 << 16) | (k0 << 24);
    constexpr uint32_t K02 = (k0 << 16) | (k1 << 24), K12 = k2 | (k3 << 8) | (k2 << 16) | (k1 << 24), K22 = k0;
    constexpr uint32_t K03 = k0 << 24, K13 = k1 | (k2 << 8) | (k3 << 16) | (k2 << 24), K23 = k1 | (k0 << 8);
    // vertical pair kernels (low half = older row)
    const u16x2 V01 = {(unsigned short)k0, (unsigned short)k1}, V23 = {(unsigned short)k2, (unsigned short)k3};
    const u16x2 V21 = {(unsigned short)k2, (unsigned short)k1};
    struct Row {
        uint32_t a, halo;
    };
    auto fetch = [&](int r, Row &R) {
        const uint32_t so = (uint32_t)(reflect101(y0 + r - 3, hgt) * w);  // wave-uniform
        R.a = __builtin_amdgcn_raw_buffer_load_b32(rin, voff, so, 0);
        R.halo = __builtin_amdgcn_raw_buffer_load_b32(rin, hoff, so, 0);
    };
    Row buf[kBlurAhead];
#pragma unroll
    for (int r = 0; r < kBlurAhead; r++) fetch(r, buf[r]);
    // the lane holding columns w..w+2 (right edge inside the wave); lane 63's halo when w == sx + 256
    const bool fix_r = right_edge && x == w;
    const bool fix_halo = right_edge && lane == 63 && w == sx + 256;
    const bool store_lane = x < w;
    uint32_t prv[4] = {0u, 0u, 0u, 0u};  // row sums of the previous row
    uint32_t pr[5][4];                   // pr[m]: (row n-5+m-1, row n-5+m) packed, m = 0..4
    // the pyramid levels 1..K of this strip are written through the frame's buffer
    const __amdgpu_buffer_rsrc_t rpyr =
        __builtin_amdgcn_make_buffer_rsrc((void *)pf.frame, 0, PYR ? (int)(pf.off[pf.K] + pf.w[pf.K] * (uint32_t)(hgt >> pf.K)) : 0,
                                          0x00020000);
#pragma unroll
    for (int r = 0; r < kBlurRows + 6; r++) {
        Row cur = buf[r % kBlurAhead];
        if (r + kBlurAhead < kBlurRows + 6) fetch(r + kBlurAhead, buf[r % kBlurAhead]);
        if (PYR && r >= 3 && r < kBlurRows + 3 && y0 + r - 3 < hgt) {  // the strip's own rows (no reflection)
            const int yy = y0 + r - 3;
            YGZ_PYR_FUSED_ROW(pf, cur.a, yy, x, store_lane, rpyr);
        }
        uint32_t am1 = (uint32_t)__builtin_amdgcn_update_dpp((int)cur.halo, (int)cur.a, 0x138, 0xF, 0xF, false);
        if (right_edge) {
            if (fix_r) cur.a = __builtin_amdgcn_perm(cur.a, am1, 0x03000102u);
            if (fix_halo) cur.halo = __builtin_amdgcn_perm(cur.halo, cur.a, 0x03000102u);
        }
        const uint32_t ap1 = (uint32_t)__builtin_amdgcn_update_dpp((int)cur.halo, (int)cur.a, 0x130, 0xF, 0xF, false);
        if (left_edge && lane == 0) am1 = __builtin_amdgcn_perm(ap1, cur.a, 0x01020304u);
        const uint32_t p0 = __builtin_amdgcn_alignbyte(cur.a, am1, 1), p1 = __builtin_amdgcn_alignbyte(ap1, cur.a, 1);
        const uint32_t p2 = ap1 >> 8;
        uint32_t hs[4];
        hs[0] = __builtin_amdgcn_udot4(p1, K10, __builtin_amdgcn_udot4(p0, K00, 0u, false), false);
        hs[1] = __builtin_amdgcn_udot4(p1, K11, __builtin_amdgcn_udot4(p0, K01, 0u, false), false);
        hs[2] = __builtin_amdgcn_udot4(
            p2, K22, __builtin_amdgcn_udot4(p1, K12, __builtin_amdgcn_udot4(p0, K02, 0u, false), false), false);
        hs[3] = __builtin_amdgcn_udot4(
            p2, K23, __builtin_amdgcn_udot4(p1, K13, __builtin_amdgcn_udot4(p0, K03, 0u, false), false), false);
        const int y = y0 + r - 6;  // output row: taps rows y-3 .. y+3 = this row (n) and the six before
        if (r >= 6 && y < hgt && store_lane) {
            uint32_t pk = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                // rows (n-6, n-5), (n-4, n-3), (n-2, n-1) and n
                uint32_t acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, pr[0][j]), V01, 32768u, false);
                acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, pr[2][j]), V23, acc, false);
                acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, pr[4][j]), V21, acc, false);
                uint32_t v = (__umul24(k0, hs[j]) + acc) >> 16;
                if (CV3) v = min(v, 255u);  // CV3 taps sum to 257; CV4 (256 x 256) cannot exceed 255
                pk |= v << (8 * j);
            }
            __builtin_amdgcn_raw_buffer_store_b32(pk, rout, voff, (uint32_t)(y * w), 0);
        }
        // slide: pr[m] <- pr[m+1], pr[4] <- (row n-1, row n)
#pragma unroll
        for (int j = 0; j < 4; j++) {
#pragma unroll
            for (int m = 0; m < 4; m++) pr[m][j] = pr[m + 1][j];
            pr[4][j] = prv[j] | (hs[j] << 16);
            prv[j] = hs[j];
        }
    }
}

// 7 waves / SIMD (68 VGPRs, no spills; uncapped it took 74 and 6 waves) and 10
// rows ahead: the strips are load-latency bound (0-3 % faster than 6 / 6 on two
// boxes; 8 waves spill)
#ifndef YGZ_BLUR_EU
#define YGZ_BLUR_EU 7
#endif
#if YGZ_BLUR_EU > 0
#define YGZ_BLUR_ATTR __attribute__((amdgpu_waves_per_eu(YGZ_BLUR_EU)))
#else
#define YGZ_BLUR_ATTR
#endif
// Strips [task_begin, task_end) of the blur tiles (level order).  pyr_k > 0 (the batch
// path of an all-area pyramid, level-0 strips only): the strips also form pyramid
// levels 1..pyr_k (PyrFused), so the pyramid's own pass is not run.
template <bool PYR>  // PYR: the fused mode's launch (a separate kernel name for the profiles' stage split)
__global__ __launch_bounds__(256) YGZ_BLUR_ATTR void k_blur7(uint8_t *__restrict__ pyr,
                                               uint8_t *__restrict__ blur, uint32_t pitch,
                                               const Plan *__restrict__ plan, int task_begin, int task_end,
                                               int pyr_k) {
#ifndef YGZ_BLUR_SWZ
#define YGZ_BLUR_SWZ 1
#endif
    // one frame's strips on one XCD (swizzled_block_2d): the 6 halo rows a strip shares with
    // the band below are then read again from that XCD's L2, not from HBM (blur stage 3.29 ->
    // 3.21 ms per step; 48- and 64-row strips measured slower: profiles/r05/blur_xcd_strips)
    int bx = blockIdx.x, f = blockIdx.y;
    if (YGZ_BLUR_SWZ) swizzled_block_2d(bx, f);
    const int lane = threadIdx.x & 63;
    // wave-uniform strip index (readfirstlane: row indices, reflections and row
    // base addresses then live in SGPRs)
    int task = __builtin_amdgcn_readfirstlane(task_begin + bx * 4 + (threadIdx.x >> 6)), l = 0;
    if (task >= task_end) return;
    while (l + 1 < plan->nlevels && task >= plan->lv[l + 1].blur_tile_begin) l++;
    const LevelDesc &L = plan->lv[l];
    task -= L.blur_tile_begin;
    const int w = L.w, hgt = L.h;
    const int sx = (task % L.blur_tiles_x) * 256, x = sx + 4 * lane, y0 = (task / L.blur_tiles_x) * kBlurRows;
    const uint8_t *src = pyr + (size_t)f * pitch + L.off;
    uint8_t *dst = blur + (size_t)f * pitch + L.off;
    // kernels: CV4 [18,34,48,56,48,34,18] (default) / CV3 [18,34,49,55,49,34,18]
    const bool cv3 = plan->blur_variant == YGZFE_BLUR_CV3;
    const uint32_t k0 = 18, k1 = 34, k2 = cv3 ? 49 : 48, k3 = cv3 ? 55 : 56;
    const int kk[7] = {(int)k0, (int)k1, (int)k2, (int)k3, (int)k2, (int)k1, (int)k0};
    if (w >= 16 && (w & 3) == 0) {
        PyrFused pf;
        pf.frame = pyr + (size_t)f * pitch;
        pf.K = PYR && l == 0 ? pyr_k : 0;
        pf.prev = pf.l1 = pf.l2 = 0u;
        for (int k = 0; k < 4; k++) {
            pf.off[k] = k <= pf.K ? plan->lv[k].off : 0u;
            pf.w[k] = k <= pf.K ? (uint32_t)plan->lv[k].w : 0u;
        }
        if (pf.K > 0) {
            if (cv3) blur_strip_aligned<true, true>(src, dst, w, hgt, sx, y0, lane, pf);
            else blur_strip_aligned<false, true>(src, dst, w, hgt, sx, y0, lane, pf);
        } else {
            if (cv3) blur_strip_aligned<true, false>(src, dst, w, hgt, sx, y0, lane, pf);
            else blur_strip_aligned<false, false>(src, dst, w, hgt, sx, y0, lane, pf);
        }
        return;
    }
    if (w >= 16) {
        const uint32_t ka = k0 | (k1 << 8) | (k2 << 16) | (k3 << 24);
        const uint32_t kb = k2 | (k1 << 8) | (k0 << 16);
        // lanes whose dword is needed: bytes up to x + 6 of the last output lane
        // (reads stay within the level + the pyramid's 64-B tail padding)
        const bool need = x < w + 8;
        const int hoff = lane == 0 ? -4 : lane == 1 ? 256 : 260;  // halo dwords (relative to the strip start)
        const bool hneed = lane < 3 && (lane == 0 ? sx > 0 : sx + hoff < w + 8);
        auto fetch = [&](int r, BlurRow &R) {
            const int yy = reflect101(y0 + r - 3, hgt);
            const uint8_t *row = src + (size_t)yy * w;  // wave-uniform
            R.o = (uint32_t)((uintptr_t)row & 3u);
            const gptr_t<uint32_t> q = as_global(reinterpret_cast<const uint32_t *>(row - R.o + sx));
            R.a = need ? q[lane] : 0u;
            R.halo = hneed ? q[hoff >> 2] : 0u;
        };
        BlurRow buf[kBlurAhead];
#pragma unroll
        for (int r = 0; r < kBlurAhead; r++) fetch(r, buf[r]);
        const bool active = x < w;
        uint32_t ring[7][4];
#pragma unroll
        for (int r = 0; r < kBlurRows + 6; r++) {
            const BlurRow cur = buf[r % kBlurAhead];
            if (r + kBlurAhead < kBlurRows + 6) fetch(r + kBlurAhead, buf[r % kBlurAhead]);
            // A[l-1], A[l], A[l+1], A[l+2] (row dwords around the lane's own)
            const uint32_t hl = __builtin_amdgcn_readlane(cur.halo, 0);
            const uint32_t hr1 = __builtin_amdgcn_readlane(cur.halo, 1), hr2 = __builtin_amdgcn_readlane(cur.halo, 2);
            uint32_t am1 = wave_from_prev(cur.a);
            if (lane == 0) am1 = hl;
            uint32_t ap1 = wave_from_next(cur.a);
            if (lane == 63) ap1 = hr1;
            uint32_t ap2 = wave_from_next(ap1);
            if (lane == 63) ap2 = hr2;
            // taps [x-3, x+6] start o + 1 bytes into A[l-1] (o = 3: at A[l])
            uint32_t hs[4];
            if (cur.o == 3u)
                blur_hsum(cur.a, ap1, ap2, 0u, 0u, ka, kb, hs);
            else
                blur_hsum(am1, cur.a, ap1, ap2, cur.o + 1u, ka, kb, hs);
#pragma unroll
            for (int j = 0; j < 4; j++) {
#pragma unroll
                for (int k = 0; k < 6; k++) ring[k][j] = ring[k + 1][j];
                ring[6][j] = hs[j];
            }
            const int y = y0 + r - 6;
            if (r >= 6 && y < hgt && active) {
                uint32_t pk = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    // 24-bit multiplies (taps <= 56, tap-pair sums <= 2 * 255 * 256): v_mad_u32_u24
                    // at full rate instead of the quarter-rate v_mul_lo_u32 of a 32-bit product
                    const uint32_t acc = __umul24(k0, ring[0][j] + ring[6][j]) + __umul24(k1, ring[1][j] + ring[5][j]) +
                                         __umul24(k2, ring[2][j] + ring[4][j]) + __umul24(k3, ring[3][j]) + 32768u;
                    pk |= min(acc >> 16, 255u) << (8 * j);  // CV3 taps sum to 257
                }
                uint8_t *o = dst + (size_t)y * w + x;
                if (x >= 4 && x + 4 <= w - 3 && (((uintptr_t)o) & 3u) == 0) {
                    *reinterpret_cast<uint32_t *>(o) = pk;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (x + j >= 4 && x + j < w - 3) o[j] = (uint8_t)(pk >> (8 * j));
                }
            }
        }
    }
    // border columns (x < 4, x >= w - 3; every column when w < 16) of this strip
    const int ncol = w >= 16 ? 7 : w;
    const bool left = sx == 0, right = sx + 256 >= w;
    if (w >= 16 && !left && !right) return;
    const int nrows = min(kBlurRows, hgt - y0);
    for (int t = lane; t < ncol * nrows; t += 64) {
        const int cidx = t % ncol, r = t / ncol;
        const int xc = w >= 16 ? (cidx < 4 ? cidx : w - 7 + cidx) : cidx;
        if (w >= 16 && ((xc < 4 && !left) || (xc >= w - 3 && !right))) continue;
        const int y = y0 + r;
        dst[(size_t)y * w + xc] = blur_pixel_reflect(src, w, hgt, xc, y, kk);
    }
}

// ---------------------------------------------------------------------------
// Wave / workgroup scans (octree).

// Inclusive wave scan on DPP: Hillis-Steele inside each 16-lane row
// (row_shr:1,2,4,8; lanes shifted in from outside the row add 0), then
// row_bcast:15 / row_bcast:31 carry rows 0-1 / 0-2 into the rows above.
// Six DPP adds instead of six LDS-routed shuffles.
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// exclusive scan over the 256 threads of the block; *total = block sum
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int *red, int *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int incl = wave_incl_scan(v);
    if (lane == 63) red[w] = incl;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
        const int r = red[i];
        off += i < w ? r : 0;
        tot += r;
    }
    __syncthreads();
    *total = tot;
    return off + incl - v;
}

// ---------------------------------------------------------------------------
// FAST-9/16 + cornerScore<16> + 3x3 non-max suppression inside each cell ROI
// (ORBextractor.cc:747-781).

// Ring taps on a ROI tile of row stride S (compile time, so every ring tap is
// an immediate ds_read offset from q = centre - 3S - 3).
template <int S>
struct Ring {
    // Bresenham circle of radius 3 (cv::FAST order), offsets from q
    static constexpr int off(int k) {
        constexpr int dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
        constexpr int dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
        return (dy[k] + 3) * S + (dx[k] + 3);
    }
    static constexpr int kCentre = 3 * S + 3;
};

typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_s16x2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ uint32_t as_u32(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h16x2 as_h16x2(uint32_t v) { return __builtin_bit_cast(h16x2, v); }
__device__ __forceinline__ uint32_t as_u32(h16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// v_pk_minimum3_f16 / v_pk_maximum3_f16 (inputs here are never NaN: plain selection)
__device__ __forceinline__ h16x2 hmin3(h16x2 a, h16x2 b, h16x2 c) {
    return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ __forceinline__ h16x2 hmax3(h16x2 a, h16x2 b, h16x2 c) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}

// FAST-9 per cell (k_fast_cells): one cell ROI staged in LDS, phases A-D of
// fast_cell_item give cv::FAST's corners, scores and order per cell
// (ORBextractor.cc:747-781).

// a wave's per-cell LDS slice (16-B aligned): ROI tile S*R, score map S*R, pixel list
__host__ __device__ constexpr int fast_slice_bytes(int S, int R) {
    return (S * R + S * R + 2 * (S - 6) * (R - 6) + 15) / 16 * 16;
}
// The loads of the last YGZ_FAST_ROWS_ROI row groups are predicated on the ROI's rows (rh):
// rows past the ROI but inside the tile's R were fetched for nothing (level 0: 40-row tiles
// for 38-row ROIs).  FAST alone, counter traffic / algorithmic bytes: 1.46x with none, 1.38x
// with the last group, 1.36x with the last two, 1.35x with every group (+1.5 % time; the
// others within noise): profiles/r06/fast_rows_roi.txt
#ifndef YGZ_FAST_ROWS_ROI
#define YGZ_FAST_ROWS_ROI 2
#endif
template <int S, int R>
struct RoiStage {  // S: LDS row stride (>= ROI width), R: row capacity (>= ROI height)
    static constexpr int DW = S / 4, RPI = 64 / DW, NI = (R + RPI - 1) / RPI;
    uint32_t lo[NI], hi[NI];
    // Every lane loads its dword pair of rows rlane + k RPI unconditionally (rows past the
    // ROI, and columns past its width, land in tile bytes nothing reads; rows past the
    // level read 0 from the buffer); row k's offset is the lane's row-0 offset plus the
    // wave-uniform k RPI w, and its tile address an immediate offset.  Only the spare
    // lane (rlane == RPI) and rows past the tile's R are not stored.
    __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, uint32_t off0, int w, int rw, int rh, int lane) {
        const int rlane = lane / DW, dw = lane - rlane * DW;
        const uint32_t f0 = mad24((uint32_t)rlane, (uint32_t)w, off0) + 4u * (uint32_t)dw;
#pragma unroll
        for (int k = 0; k < NI; k++) {
            const uint32_t o = (f0 + (uint32_t)(k * RPI) * (uint32_t)w) & ~3u;
            lo[k] = hi[k] = 0u;
            if (stored(k, rlane) && (k + YGZ_FAST_ROWS_ROI < NI || k * RPI + rlane < rh)) {  // (a load used only under the store's condition is sunk past the others' waits)
                lo[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
                hi[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 4u, 0, 0);
            }
        }
    }
    static __device__ __forceinline__ bool stored(int k, int rlane) {
        return rlane < RPI && (k + 1 < NI || k * RPI + RPI <= R || k * RPI + rlane < R);
    }
    __device__ __forceinline__ void commit(uint8_t *img, uint32_t off0, int w, int rw, int rh, int lane) const {
        const int rlane = lane / DW, dw = lane - rlane * DW;
        const uint32_t f0 = mad24((uint32_t)rlane, (uint32_t)w, off0) + 4u * (uint32_t)dw;
        uint32_t *d = reinterpret_cast<uint32_t *>(img + rlane * S) + dw;
#pragma unroll
        for (int k = 0; k < NI; k++) {
            const uint32_t sh = (f0 + (uint32_t)(k * RPI) * (uint32_t)w) & 3u;
            if (stored(k, rlane)) d[k * RPI * DW] = __builtin_amdgcn_alignbyte(hi[k], lo[k], sh);
        }
        wave_lds_order();
    }
};

#if defined(__FAST_MATH__)
#error "the FAST kernels order ring bytes as f16 subnormals: build without fast-math (denormals kept)"
#endif

// The 4-point necessary test of 4 pixels (the bytes of C) at threshold th: a 9-arc
// holds a neighbouring pair of the compass points 0/4/8/12, so a corner has
// (T|B) & (L|R) beyond the threshold on one side.  T / B / Lw / Rw: the dwords of the
// pixels 3 up / 3 down / 3 left / 3 right.  Bit k: pixel k survives.
__device__ __forceinline__ uint32_t fast_screen4(uint32_t T, uint32_t B, uint32_t Lw, uint32_t Rw, uint32_t C,
                                                 int th) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const s16x2 t2 = {(short)th, (short)th};
    uint32_t sg[2];
#pragma unroll
    for (int hlf = 0; hlf < 2; hlf++) {
        // bright: (T|B) & (L|R) above v+t <=> min(max(T,B), max(L,R)) - v > t;
        // dark:   (T|B) & (L|R) below v-t <=> v - max(min(T,B), min(L,R)) > t;
        // sign of t - max(both) marks the survivors (v_pk_max/min_u16, bytes < 256)
        const uint32_t sel = hlf ? 0x0C030C01u : 0x0C020C00u;  // bytes 1,3 / 0,2 -> u16 lanes
        const u16x2 dT = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(T, T, sel));
        const u16x2 dB = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(B, B, sel));
        const u16x2 dL = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(Lw, Lw, sel));
        const u16x2 dR = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(Rw, Rw, sel));
        const u16x2 bv = __builtin_elementwise_min(__builtin_elementwise_max(dT, dB), __builtin_elementwise_max(dL, dR));
        const u16x2 dv = __builtin_elementwise_max(__builtin_elementwise_min(dT, dB), __builtin_elementwise_min(dL, dR));
        const s16x2 v = as_s16x2(__builtin_amdgcn_perm(C, C, sel));
        const s16x2 m = __builtin_elementwise_max(__builtin_bit_cast(s16x2, bv) - v, v - __builtin_bit_cast(s16x2, dv));
        sg[hlf] = as_u32(t2 - m);
    }
    return ((sg[0] >> 15) & 1u) | (((sg[1] >> 15) & 1u) << 1) | (((sg[0] >> 31) & 1u) << 2) |
           (((sg[1] >> 31) & 1u) << 3);
}

// The same test with per-lane packed thresholds (t01: pixels 0 / 2, t23: 1 / 3; a pixel
// outside the cell interior gets kFastNoTh, which no |m| <= 255 passes) and the two
// packed results returned as they are: pixel k survives iff its half of sg[k & 1] is
// negative (pixels 0 / 1: the low halves, 2 / 3: the high halves, so the 32-bit sign).
#ifndef YGZ_FAST_SG
#define YGZ_FAST_SG 1  // phase A: ballots straight from the packed signs (0: the 4-bit mask form)
#endif
constexpr uint32_t kFastNoTh = 0x3FFFu;
__device__ __forceinline__ void fast_screen4_sg(uint32_t T, uint32_t B, uint32_t Lw, uint32_t Rw, uint32_t C,
                                                uint32_t t01, uint32_t t23, uint32_t sg[2]) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int hlf = 0; hlf < 2; hlf++) {
        const uint32_t sel = hlf ? 0x0C030C01u : 0x0C020C00u;
        const u16x2 dT = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(T, T, sel));
        const u16x2 dB = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(B, B, sel));
        const u16x2 dL = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(Lw, Lw, sel));
        const u16x2 dR = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(Rw, Rw, sel));
        const u16x2 bv = __builtin_elementwise_min(__builtin_elementwise_max(dT, dB), __builtin_elementwise_max(dL, dR));
        const u16x2 dv = __builtin_elementwise_max(__builtin_elementwise_min(dT, dB), __builtin_elementwise_min(dL, dR));
        const s16x2 v = as_s16x2(__builtin_amdgcn_perm(C, C, sel));
        const s16x2 m = __builtin_elementwise_max(__builtin_bit_cast(s16x2, bv) - v, v - __builtin_bit_cast(s16x2, dv));
        sg[hlf] = as_u32(as_s16x2(hlf ? t23 : t01) - m);
    }
}

// Survivor / corner list entries: the pixel's byte offset row * S + col in the ROI tile
// (ring taps and score-map writes take it as it is; measured the same as row << 8 | col
// with a multiply per use, profiles/r05/fast_entry_offsets).
template <int S>
__device__ __forceinline__ uint32_t fast_entry(uint32_t row, uint32_t col) {
    return row * S + col;
}
template <int S>
__device__ __forceinline__ void fast_entry_xy(uint32_t e, int &x, int &y) {
    y = (int)(e / S);
    x = (int)e - y * S;
}

// Segment test and score of two survivors at once (list entries e, fast_entry, on a
// tile of row stride S), as packed pairs: with e[k] = r_k - v,
//   arcmax = max(max_k min(e[k..k+8]), max_k min(-e[k..k+8]))
// corner (FAST_t<16>: 9 contiguous ring pixels all > v+t or all < v-t) <=> arcmax > t,
// and then cornerScore<16> = max(t, arcmax) - 1 = arcmax - 1.  The min / max run on
// v_pk_minimum3_f16 / v_pk_maximum3_f16 over the ring bytes taken as f16 bit
// patterns (+0 and subnormals, ordered like the integers and selected exactly with f16
// denormals kept), and min / max commute with "- v".
template <int S>
__device__ __forceinline__ s16x2 fast_arcmax2(const uint8_t *img, uint32_t e0, uint32_t e1) {
    // ring bases q = centre - 3S - 3: every tap an immediate, non-negative ds_read offset
    uint32_t b0 = e0 - (3 * S + 3), b1 = e1 - (3 * S + 3);
    asm("" : "+v"(b0), "+v"(b1));  // taps off q (not off the centre): immediate offsets only
    const uint8_t *q0 = img + b0, *q1 = img + b1;
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    auto pair = [&](int o) {  // both survivors' bytes as the u16 halves
        u16x2 p;
        p.x = q0[o];
        p.y = q1[o];
        return __builtin_bit_cast(uint32_t, p);
    };
    const s16x2 vb = as_s16x2(pair(Ring<S>::kCentre));
    h16x2 e[16];
#pragma unroll
    for (int k = 0; k < 16; k++) e[k] = as_h16x2(pair(Ring<S>::off(k)));
    h16x2 w3[16];
    // bright: max_k min(e[k..k+8]) = max_k min3(w3[k], w3[k+3], w3[k+6]), w3 = min of 3
#pragma unroll
    for (int k = 0; k < 16; k++) w3[k] = hmin3(e[k], e[(k + 1) & 15], e[(k + 2) & 15]);
    h16x2 b9[16];
#pragma unroll
    for (int k = 0; k < 16; k++) b9[k] = hmin3(w3[k], w3[(k + 3) & 15], w3[(k + 6) & 15]);
    const h16x2 bright = hmax3(hmax3(hmax3(b9[0], b9[1], b9[2]), hmax3(b9[3], b9[4], b9[5]), hmax3(b9[6], b9[7], b9[8])),
                               hmax3(b9[9], b9[10], b9[11]), hmax3(hmax3(b9[12], b9[13], b9[14]), b9[15], b9[15]));
    // dark: max_k min(-e[k..k+8]) = -(min_k max(e[k..k+8]))
#pragma unroll
    for (int k = 0; k < 16; k++) w3[k] = hmax3(e[k], e[(k + 1) & 15], e[(k + 2) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++) b9[k] = hmax3(w3[k], w3[(k + 3) & 15], w3[(k + 6) & 15]);
    const h16x2 darkmin = hmin3(hmin3(hmin3(b9[0], b9[1], b9[2]), hmin3(b9[3], b9[4], b9[5]), hmin3(b9[6], b9[7], b9[8])),
                                hmin3(b9[9], b9[10], b9[11]), hmin3(hmin3(b9[12], b9[13], b9[14]), b9[15], b9[15]));
    const s16x2 bi = as_s16x2(as_u32(bright)) - vb, di = vb - as_s16x2(as_u32(darkmin));
    return __builtin_elementwise_max(bi, di);
}

// One (cell, frame) item on a wave whose ROI is already in LDS (row stride S), from
// threshold pass pass0 (0: iniThFAST then the minThFAST retry; 1: minThFAST only):
//   A  every interior pixel: the 4-point screen, 4 pixels per lane; survivors
//      compacted (ballot + mbcnt) into the list in raster order
//   BC survivors: segment test + score, corners compacted in place, scores into the map
//   D  corners: strict 3x3 non-max suppression, survivors -> the cell's list
// and the retry at minThFAST when no corner survives (ORBextractor.cc:765-770).
#ifndef YGZ_FAST_KO
#define YGZ_FAST_KO 0  // diagnostic knock-outs (tools/run_fast_phases.sh): 1 ROI staging only, 2 + A,
                       // 3 + BC, 4 + D (2-4: the first pass only, no retry); 0 the product
#endif
template <int S>
__device__ __forceinline__ void fast_cell_item(const Plan *__restrict__ plan, const CellDesc &cd, uint8_t *img,
                                               uint8_t *sc, uint16_t *list, uint32_t *__restrict__ out,
                                               int *__restrict__ cnt_out, int lane, int pass0) {
    const int rw = cd.rw, rh = cd.rh;
    const int iw = rw - 6, ih = rh - 6;
    int total = 0;
    for (int pass = pass0; pass < (YGZ_FAST_KO ? pass0 + 1 : 2); pass++) {
        const int th = pass == 0 ? plan->ini_th : plan->min_th;
        {
            uint4 *z = reinterpret_cast<uint4 *>(sc);
            const uint4 zero = {0u, 0u, 0u, 0u};
            const int nz = rh * S;
            for (int i = lane; i < nz / 16; i += 64) z[i] = zero;
            for (int i = (nz / 16) * 16 + lane; i < nz; i += 64) sc[i] = 0;
        }
        // A: 4 pixels per lane
        int na = 0;
        if (iw > 0 && ih > 0) {
            const int lpr = iw <= 32 ? 8 : (iw <= 64 ? 16 : 32);  // lanes per row (4 px each)
            const int rpc = 64 / lpr;                                  // rows per chunk
            const int j = lane & (lpr - 1), rr = lane / lpr;
#if YGZ_FAST_SG
            // per-lane packed thresholds: pixels past the interior's columns never pass
            const uint32_t thv = (uint32_t)th;
            const uint32_t tc01 = (4 * j + 0 < iw ? thv : kFastNoTh) | ((4 * j + 2 < iw ? thv : kFastNoTh) << 16);
            const uint32_t tc23 = (4 * j + 1 < iw ? thv : kFastNoTh) | ((4 * j + 3 < iw ? thv : kFastNoTh) << 16);
            // a row chunk of the interior; `full`: every row of the chunk is inside it (all but
            // the last chunk when rpc does not divide ih), so no per-row threshold select
            const uint32_t lane_off = (uint32_t)(rr * S + 4 * j);  // the lane's dword in a chunk's first row
            auto chunk = [&](int y0, bool full) {
                const int y = y0 + rr;
                // row addresses: the wave-uniform y0 S (SALU) plus the lane's offset
                const uint32_t o = (uint32_t)(y0 * S) + lane_off;
                const uint32_t *rt = reinterpret_cast<const uint32_t *>(img + o);
                const uint32_t *rc = reinterpret_cast<const uint32_t *>(img + o + 3 * S);
                const uint32_t *rb = reinterpret_cast<const uint32_t *>(img + o + 6 * S);
                const uint32_t D0 = rc[0], D1 = rc[1], D2 = rc[2];
                const uint32_t C = __builtin_amdgcn_alignbyte(D1, D0, 3);   // x .. x+3
                const uint32_t Rw = __builtin_amdgcn_alignbyte(D2, D1, 2);  // x+3 .. x+6
                const uint32_t Tw = __builtin_amdgcn_alignbyte(rt[1], rt[0], 3);
                const uint32_t Bw = __builtin_amdgcn_alignbyte(rb[1], rb[0], 3);
                const bool yin = full || y < ih;
                uint32_t sg[2];
                fast_screen4_sg(Tw, Bw, D0, Rw, C, yin ? tc01 : (kFastNoTh * 0x10001u), yin ? tc23 : (kFastNoTh * 0x10001u),
                                sg);
                // the low halves' signs as 32-bit signs: one v_cmp each, shared by the ballot and
                // the list write's exec mask (a 16-bit sign test compiles to two compares, one per
                // use; the opaque shift keeps it a 32-bit compare)
                uint32_t lo0 = sg[0] << 16, lo1 = sg[1] << 16;
                asm("" : "+v"(lo0), "+v"(lo1));
                const bool b0 = (int)lo0 < 0, b1 = (int)lo1 < 0;
                const bool b2 = (int)sg[0] < 0, b3 = (int)sg[1] < 0;
                const uint64_t M0 = __ballot(b0), M1 = __ballot(b1), M2 = __ballot(b2), M3 = __ballot(b3);
                // survivors in lanes below: one mbcnt chain (each step adds to the last)
                uint32_t pc = __builtin_amdgcn_mbcnt_lo((uint32_t)M0, (uint32_t)na);
                pc = __builtin_amdgcn_mbcnt_hi((uint32_t)(M0 >> 32), pc);
                pc = __builtin_amdgcn_mbcnt_lo((uint32_t)M1, pc);
                pc = __builtin_amdgcn_mbcnt_hi((uint32_t)(M1 >> 32), pc);
                pc = __builtin_amdgcn_mbcnt_lo((uint32_t)M2, pc);
                pc = __builtin_amdgcn_mbcnt_hi((uint32_t)(M2 >> 32), pc);
                pc = __builtin_amdgcn_mbcnt_lo((uint32_t)M3, pc);
                pc = __builtin_amdgcn_mbcnt_hi((uint32_t)(M3 >> 32), pc);
                na += __popcll(M0) + __popcll(M1) + __popcll(M2) + __popcll(M3);
                const uint32_t e = o + (uint32_t)(3 * S + 3);  // fast_entry<S>(y + 3, 4 j + 3)
                uint16_t *lp = list + pc;  // this lane's next list slot
                if (b0) *lp++ = (uint16_t)e;
                if (b1) *lp++ = (uint16_t)(e + 1u);
                if (b2) *lp++ = (uint16_t)(e + 2u);
                if (b3) *lp = (uint16_t)(e + 3u);
            };
            int y0 = 0;
            for (; y0 + rpc <= ih; y0 += rpc) chunk(y0, true);
            if (y0 < ih) chunk(y0, false);
#else
            uint32_t colmask = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) colmask |= (uint32_t)(4 * j + k < iw) << k;
            for (int y0 = 0; y0 < ih; y0 += rpc) {
                const int y = y0 + rr;
                const uint32_t *rt = reinterpret_cast<const uint32_t *>(img + y * S) + j;
                const uint32_t *rc = reinterpret_cast<const uint32_t *>(img + (y + 3) * S) + j;
                const uint32_t *rb = reinterpret_cast<const uint32_t *>(img + (y + 6) * S) + j;
                const uint32_t D0 = rc[0], D1 = rc[1], D2 = rc[2];
                const uint32_t C = __builtin_amdgcn_alignbyte(D1, D0, 3);   // x .. x+3
                const uint32_t Rw = __builtin_amdgcn_alignbyte(D2, D1, 2);  // x+3 .. x+6
                const uint32_t Tw = __builtin_amdgcn_alignbyte(rt[1], rt[0], 3);
                const uint32_t Bw = __builtin_amdgcn_alignbyte(rb[1], rb[0], 3);
                const uint32_t m = fast_screen4(Tw, Bw, D0, Rw, C, th) & (y < ih ? colmask : 0u);
                // survivors appended in raster order (lanes are row-major, bits in column order)
                const uint64_t M0 = __ballot(m & 1u), M1 = __ballot(m & 2u), M2 = __ballot(m & 4u), M3 = __ballot(m & 8u);
                int pos = na + popc_below(M0) + popc_below(M1) + popc_below(M2) + popc_below(M3);
                na += __popcll(M0) + __popcll(M1) + __popcll(M2) + __popcll(M3);
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if ((m >> k) & 1u) list[pos++] = (uint16_t)fast_entry<S>((uint32_t)(y + 3), (uint32_t)(4 * j + k + 3));
            }
#endif
        }
        if (YGZ_FAST_KO == 2) {
            total = na;
            break;
        }
        // BC: two survivors per lane (low half list[i], high half list[i+1]); corners
        // compacted in place in raster order (writes never pass the read front)
        int nc = 0;
        for (int i0 = 0; i0 < na; i0 += 128) {
            const int i = i0 + 2 * lane;
            const uint32_t pr = reinterpret_cast<const uint32_t *>(list)[i >> 1];  // list[i], list[i+1]
            const bool v0 = i < na, v1 = i + 1 < na;
            const uint32_t e0 = v0 ? (pr & 0xFFFFu) : fast_entry<S>(3u, 3u), e1 = v1 ? (pr >> 16) : fast_entry<S>(3u, 3u);
            const s16x2 am = fast_arcmax2<S>(img, e0, e1);
            const bool c0 = v0 && am.x > th, c1 = v1 && am.y > th;
            if (c0) sc[e0] = (uint8_t)(am.x - 1);
            if (c1) sc[e1] = (uint8_t)(am.y - 1);
            const uint64_t M0 = __ballot(c0), M1 = __ballot(c1);
            const int pos = nc + popc_below(M0) + popc_below(M1);
            if (c0) list[pos] = (uint16_t)e0;
            if (c1) list[pos + (c0 ? 1 : 0)] = (uint16_t)e1;
            nc += __popcll(M0) + __popcll(M1);
        }
        wave_lds_order();
        if (YGZ_FAST_KO == 3) {
            total = nc;
            break;
        }
        // D: strict 3x3 NMS over the corner list
        for (int i0 = 0; i0 < nc; i0 += 64) {
            const int i = i0 + lane;
            bool keep = false;
            int s = 0, x = 0, y = 0;
            if (i < nc) {
                fast_entry_xy<S>(list[i], x, y);
                const uint8_t *r = sc + (y - 1) * S + (x - 1);
                s = r[S + 1];
                // all nine reads in flight together (a short-circuit chain here
                // compiles to eight dependent LDS round trips)
                const uint32_t m0 = max(max((uint32_t)r[0], (uint32_t)r[1]), (uint32_t)r[2]);
                const uint32_t m1 = max(max((uint32_t)r[S], (uint32_t)r[S + 2]), (uint32_t)r[2 * S]);
                const uint32_t m2 = max((uint32_t)r[2 * S + 1], (uint32_t)r[2 * S + 2]);
                keep = (uint32_t)s > max(max(m0, m1), m2);
            }
            const uint64_t m = __ballot(keep);
            const int pos = total + popc_below(m);
            if (keep && pos < plan->cell_cap) out[pos] = pack_key(x + cd.offx, y + cd.offy, s);
            total += __popcll(m);
        }
        if (total > 0) break;
    }
    if (lane == 0) *cnt_out = min(total, plan->cell_cap);
}

// per-level ROI slice: the level's largest cell ROI, row stride a multiple of 4
// (>= 36), rows rounded up to 8 (>= 40)
static void fast_slice_shape(int rw, int rh, int &S, int &R) {
    S = rw <= 36 ? 36 : ((rw + 7) / 8) * 8;
    R = std::max(40, ((rh + 7) / 8) * 8);
}

// One wave per (cell, frame), kFastWaves per workgroup: the cell's ROI staged into the
// wave's LDS slice, then fast_cell_item.
// Waves (cells) per workgroup: 2.  Under the pipe schedule the smaller workgroups interleave
// with the other chunk's stages: headline +1.2 % over 4 waves in six alternating pass pairs (FAST
// alone ~0.7 % slower); 8 waves measured 6 % slower (profiles/r06/fast_waves/)
#ifndef YGZ_FAST_WAVES
#define YGZ_FAST_WAVES 2
#endif
constexpr int kFastWaves = YGZ_FAST_WAVES;
template <int S, int R>
__global__ __launch_bounds__(64 * kFastWaves) __attribute__((amdgpu_waves_per_eu(6))) void k_fast_cells(
    const uint8_t *__restrict__ pyr, uint32_t pitch, const Plan *__restrict__ plan,
    const CellDesc *__restrict__ cells, uint32_t *__restrict__ cellbuf, int *__restrict__ cellcnt, int cell_begin,
    int cell_end, int level, int *__restrict__ clear_flag) {
    extern __shared__ uint8_t s_dyn[];
    constexpr int slice = fast_slice_bytes(S, R);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // Block order (a traffic / speed choice; results never depend on it): runs of kRun
    // consecutive blocks (16 neighbouring cells) per XCD (block b runs on XCD b % 8), so
    // neighbouring cells' ROI halos come from one L2: HBM reads 1.29x the levels' bytes
    // instead of 2.07x in plain order, for +1 % time; whole frames per XCD read 0.87x but
    // ran 13 % slower (round 3)
    // Runs of kRun blocks = YGZ_FAST_RUN_CELLS cells whatever the workgroup size.  FAST alone
    // (1,024 C2 frames, 2-wave workgroups), counter traffic / algorithmic bytes and time: 8-cell
    // runs 1.59x / 0.548 ms, 16 cells 1.36x / 0.554 ms, 32 cells 1.16x / 0.534 ms; the headline
    // the same within noise (profiles/r06/fast_runs/)
#ifndef YGZ_FAST_RUN_CELLS
#define YGZ_FAST_RUN_CELLS 32
#endif
    constexpr int kRun = YGZ_FAST_RUN_CELLS / kFastWaves, kGroup = 8 * kRun;
    const int orig = blockIdx.x + gridDim.x * blockIdx.y, nwg = gridDim.x * gridDim.y;
    int lid = (orig / kGroup) * kGroup + (orig % 8) * kRun + (orig / 8) % kRun;
    if ((orig | (kGroup - 1)) >= nwg) lid = orig;  // the ragged tail keeps the plain order
    const int bx = lid % gridDim.x, f = lid / gridDim.x;
    const int c = cell_begin + bx * kFastWaves + wave;
    if (clear_flag && c == cell_begin && f == 0 && lane == 0) *clear_flag = 0;
    if (c >= cell_end) return;
    uint8_t *img = s_dyn + wave * slice;
    uint8_t *sc = img + S * R;
    uint16_t *list = reinterpret_cast<uint16_t *>(sc + S * R);
    const CellDesc cd = scalar_load(cells + c);
    const LevelDesc &L = plan->lv[level >= 0 ? level : cd.level];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(pyr + (size_t)f * pitch + L.off), 0, (int)((uint32_t)L.w * (uint32_t)L.h), 0x00020000);
    const uint32_t off0 = (uint32_t)cd.y0 * (uint32_t)L.w + (uint32_t)cd.x0;
    {
        RoiStage<S, R> st;
        st.issue(rs, off0, L.w, cd.rw, cd.rh, lane);
        st.commit(img, off0, L.w, cd.rw, cd.rh, lane);
    }
    if (YGZ_FAST_KO == 1) {  // staging only: one byte of the tile out, so the staging stays
        wave_lds_order();
        const uint32_t probe = (uint32_t)img[lane] + img[S * 8 + lane] + img[S * 20 + lane];  // < 2^10
        if (lane == 0) cellcnt[(size_t)f * plan->ncells + c] = (int)(probe >> 30);
        return;
    }
    fast_cell_item<S>(plan, cd, img, sc, list, cellbuf + ((size_t)f * plan->ncells + c) * plan->cell_cap,
                      cellcnt + (size_t)f * plan->ncells + c, lane, 0);
}


// ---------------------------------------------------------------------------
// Octree distribution by quadrant paths (DistributeOctTree, ORBextractor.cc:533-723
// with ExtractorNode::DivideNode :479-531).
//
// A node at depth d is the set of keys that share the first d quadrants of their
// path from the root column (the division midpoints, ORBextractor.cc:481-482, depend
// only on the node's bounds, so every key can walk its own path).  With the keys
// sorted by path code, every node of every depth is a contiguous run, and
// L_k = depth of the common prefix of sorted keys k-1 and k gives, for all depths at
// once (main loop, :585-640):
//   size(d)    = #{k : L_k < d}                      (nodes after pass d)
//   nexpand(d) = size(d) - #{k : max(L_k, L_k+1) < d} (nodes with > 1 key)
// so the pass P that ends the main loop follows from two histograms.  The list
// order after P passes is closed-form: push_front leaves, front to back, the nodes
// created at depth P, then the singletons created at P-1, P-2, ..., 0; within one
// creation depth e the order fo_e satisfies fo_0 = root ascending and fo_e =
// (parent in reverse fo_{e-1}, quadrant descending).  Storing the root field and the
// odd depths' quadrants complemented makes fo_e the ascending code order for odd e
// and its reverse for even e.  The final rounds (:641-676) divide the front nodes
// (those the last pass created) in (key count desc, list position asc) order -- the
// list position ascends with the std::sort tie-break taken as creation order
// descending, as in oracle/orb.c -- up to the first division that reaches N.
// tools/octree_proto.py checks this formulation against oracle/orb.c's list walk.

namespace oct {

// lanes whose db-bit value equals this lane's, among 'valid'
__device__ __forceinline__ uint64_t match_bits(uint32_t v, int db, uint64_t valid) {
    uint64_t m = valid;
    for (int b = 0; b < db; b++) {
        const bool bit = (v >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        m &= bit ? bal : ~bal;
    }
    return m;
}

__device__ __forceinline__ uint64_t lanes_below() { return (1ull << lane_id()) - 1ull; }

template <int NT>
constexpr int nwaves() { return NT / 64; }

// LDS of the list phase (from lsm): node lists, final-round scratch, then (kernel
// k_octree_list only) L of the sorted keys
template <int NC>
struct ListLayout {
    static constexpr int kNode = 0;                      // u32 [2][NC]: start | len << 16
    static constexpr int kDep = kNode + 8 * NC;          // u8  [2][NC]: depth | processed << 7
    static constexpr int kCk = (kDep + 2 * NC + 15) & ~15;  // u32 [NC + 4]: candidate sort keys
    static constexpr int kCe = kCk + 4 * NC + 16;        // u16 [NC]: children per candidate
    static constexpr int kCi = kCe + 2 * NC;             // u16 [NC]: inclusive children prefix
    static constexpr int kHs = kCi + 2 * NC;             // u16 [NC + 2]: sorted position of head r
    static constexpr int kNgr = kHs + 2 * NC + 4;        // u16 [NC]: list position -> head rank
    static constexpr int kLc = (kNgr + 2 * NC + 15) & ~15;
    static constexpr int bytes(int nl) { return kLc + nl + 16; }
};

// LDS of the sort phase: K | code0 | idx0 | {code1, idx1, hist}; the list phase of the
// global-scratch form uses the region from kU
template <int NC, int NK, int NT>
struct Layout {
    static constexpr int kK = 0;
    static constexpr int kCode0 = kK + 4 * NK;
    static constexpr int kIdx0 = kCode0 + 4 * NK;
    static constexpr int kU = (kIdx0 + 2 * NK + 15) & ~15;
    static constexpr int kCode1 = kU;
    static constexpr int kIdx1 = kCode1 + 4 * NK;
    static constexpr int kHist = (kIdx1 + 2 * NK + 15) & ~15;
    static constexpr int kSortEnd = kHist + 4 * 256 * nwaves<NT>();
    static constexpr int kListEnd = kU + ListLayout<NC>::bytes(0);
    static constexpr int kBytes = (kSortEnd > kListEnd ? kSortEnd : kListEnd);
};

struct Scal {
    int red[16];
    int wcnt[16][16];  // per wave: per-section head counts (sweep A)
    int whead[16];     // per wave: heads
    int hL[16], hM[16];  // histograms of L + 1 and max(L_k, L_k+1) + 1
    int s[8];
};

// One pass of an LSD radix sort over the wave-owned segment [s0, s1) (segments in
// wave order = array order, so each pass is stable): per-wave digit counts by
// ballot matching, one scan over (digit, wave), then the scatter.
template <int NT, typename CP, typename IP>
__device__ __forceinline__ void radix_pass(CP src_c, IP src_i, CP dst_c, IP dst_i, int s0, int s1, int sh,
                                           int db, uint32_t *hist, Scal &Sc) {
    constexpr int NW = nwaves<NT>();
    const int lane = lane_id(), w = threadIdx.x >> 6, nb = 1 << db;
    uint32_t *hw = hist + w * 256;
    for (int d = lane; d < nb; d += 64) hw[d] = 0u;
    for (int k0 = s0; k0 < s1; k0 += 64) {
        const int k = k0 + lane;
        const bool v = k < s1;
        const uint32_t dg = v ? (src_c[k] >> sh) & (uint32_t)(nb - 1) : 0u;
        const uint64_t peers = match_bits(dg, db, __ballot(v));
        if (v && (peers & lanes_below()) == 0) hw[dg] += (uint32_t)__popcll(peers);
    }
    __syncthreads();
    {
        const int d = threadIdx.x;  // NT >= 256 >= nb
        int s = 0;
        if (d < nb)
            for (int ww = 0; ww < NW; ww++) s += (int)hist[ww * 256 + d];
        int tot;
        const int base = block_excl_scan<NT>(d < nb ? s : 0, Sc.red, &tot);
        if (d < nb) {
            int run = base;
            for (int ww = 0; ww < NW; ww++) {
                const int c = (int)hist[ww * 256 + d];
                hist[ww * 256 + d] = (uint32_t)run;
                run += c;
            }
        }
    }
    __syncthreads();
    for (int k0 = s0; k0 < s1; k0 += 64) {
        const int k = k0 + lane;
        const bool v = k < s1;
        uint32_t c = 0u, dg = 0u;
        uint16_t ix = 0;
        if (v) {
            c = src_c[k];
            ix = src_i[k];
            dg = (c >> sh) & (uint32_t)(nb - 1);
        }
        const uint64_t peers = match_bits(dg, db, __ballot(v));
        const uint32_t base = v ? hw[dg] : 0u;
        if (v) {
            const uint64_t below = peers & lanes_below();
            const uint32_t dst = base + (uint32_t)__popcll(below);
            dst_c[dst] = c;
            dst_i[dst] = ix;
            if (below == 0) hw[dg] = base + (uint32_t)__popcll(peers);
        }
    }
    __syncthreads();
}

// radix_pass without the index array: one stable LSD pass of 32-bit codes
template <int NT>
__device__ __forceinline__ void radix_pass_codes(const uint32_t *src, uint32_t *dst, int s0, int s1, int sh, int db,
                                                 uint32_t *hist, Scal &Sc) {
    constexpr int NW = nwaves<NT>();
    const int lane = lane_id(), w = threadIdx.x >> 6, nb = 1 << db;
    uint32_t *hw = hist + w * 256;
    for (int d = lane; d < nb; d += 64) hw[d] = 0u;
    for (int k0 = s0; k0 < s1; k0 += 64) {
        const int k = k0 + lane;
        const bool v = k < s1;
        const uint32_t dg = v ? (src[k] >> sh) & (uint32_t)(nb - 1) : 0u;
        const uint64_t peers = match_bits(dg, db, __ballot(v));
        if (v && (peers & lanes_below()) == 0) hw[dg] += (uint32_t)__popcll(peers);
    }
    __syncthreads();
    {
        const int d = threadIdx.x;
        int sum = 0;
        if (d < nb)
            for (int ww = 0; ww < NW; ww++) sum += (int)hist[ww * 256 + d];
        int tot;
        const int base = block_excl_scan<NT>(d < nb ? sum : 0, Sc.red, &tot);
        if (d < nb) {
            int run = base;
            for (int ww = 0; ww < NW; ww++) {
                const int c = (int)hist[ww * 256 + d];
                hist[ww * 256 + d] = (uint32_t)run;
                run += c;
            }
        }
    }
    __syncthreads();
    for (int k0 = s0; k0 < s1; k0 += 64) {
        const int k = k0 + lane;
        const bool v = k < s1;
        uint32_t c = 0u, dg = 0u;
        if (v) {
            c = src[k];
            dg = (c >> sh) & (uint32_t)(nb - 1);
        }
        const uint64_t peers = match_bits(dg, db, __ballot(v));
        const uint32_t base = v ? hw[dg] : 0u;
        if (v) {
            const uint64_t below = peers & lanes_below();
            dst[base + (uint32_t)__popcll(below)] = c;
            if (below == 0) hw[dg] = base + (uint32_t)__popcll(peers);
        }
    }
    __syncthreads();
}

__device__ __forceinline__ int lcp_depth(uint32_t a, uint32_t b, int rb) {
    const uint32_t x = a ^ b;
    if (x == 0u) return 14;  // equal codes: not separated (Dn <= 14: flagged by the caller)
    const int lz = __clz((int)x);
    return lz < rb ? -1 : (lz - rb) >> 1;
}

// Sort phase of one (frame, level): the keys in candidate order into K, sorted by
// path code (code0 / idx0: codes and candidate indices in sorted order), L of the
// sorted keys into Lc (i8 [n + 1]); Sc.s[1] = keys not separated (never, for
// distinct pixels).  code1 / idx1: sort scratch.
template <int NC, int NK, int NT, int RB, typename KP, typename CP, typename IP, typename LP>
__device__ __forceinline__ void body_sort(const Plan *__restrict__ plan, const LevelDesc &L, int l, int f,
                                          uint8_t *smem, Scal &Sc, const uint32_t *__restrict__ cellbuf,
                                          const int *__restrict__ cellcnt, KP K, CP code0, IP idx0, CP code1,
                                          IP idx1, LP Lc, int n) {
    using Lay = Layout<NC, NK, NT>;
    constexpr int NW = nwaves<NT>();
    const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    // --- 1. vToDistributeKeys in cell order: every thread places its keys j = tid +
    //        NT u by branch-free binary searches over the cells' prefix (all steps of all
    //        its searches interleaved), then issues all their loads together
    {
        int *s_pref = reinterpret_cast<int *>(smem + Lay::kHist);
        int base = 0;
        for (int cb = 0; cb < L.ncells; cb += NT) {
            const int c = cb + tid;
            const int cnt = c < L.ncells ? cellcnt[(size_t)f * plan->ncells + L.cell_begin + c] : 0;
            int tot;
            const int ex = block_excl_scan<NT>(cnt, Sc.red, &tot);
            s_pref[tid] = ex;
            __syncthreads();
            const int nch = min(L.ncells - cb, NT);
            const uint32_t *cs0 = cellbuf + ((size_t)f * plan->ncells + L.cell_begin + cb) * plan->cell_cap;
            for (int j0 = 0; j0 < tot; j0 += NT * 8) {
                int cc[8];
#pragma unroll
                for (int u = 0; u < 8; u++) cc[u] = 0;
#pragma unroll
                for (int step = NT / 2; step >= 1; step >>= 1) {
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const int j = j0 + NT * u + tid, q = cc[u] + step;
                        if (q < nch && s_pref[q] <= j) cc[u] = q;
                    }
                }
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int j = j0 + NT * u + tid;
                    v[u] = j < tot ? cs0[(size_t)cc[u] * plan->cell_cap + (j - s_pref[cc[u]])] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int j = j0 + NT * u + tid;
                    if (j < tot) K[base + j] = v[u];
                }
            }
            base += tot;
            __syncthreads();
        }
    }
    if (l == 0) YGZ_BSTAMP_K(3, 3);
    // --- 2. path codes: root field (complemented) on top, then Dn quadrants of 2 bits,
    //        odd depths complemented; Dn levels separate any two pixels of the level
    const int rb = L.oct_rb, Dn = L.oct_dn;  // plan.cpp octree_code_tables
    const int bits = rb + 2 * Dn;
    const int passes = (bits + 7) >> 3;
    const int db = (bits + passes - 1) / passes;
    const int lowbit = 32 - passes * db;
    const int *xtab = plan->dtabs + L.oct_xtab, *ytab = plan->dtabs + L.oct_ytab;
    auto path_code = [&](uint32_t kk) -> uint32_t {
        return (uint32_t)as_global(xtab)[key_x(kk)] | (uint32_t)as_global(ytab)[key_y(kk)];
    };
    const int seg = (((n + NW - 1) / NW) + 63) & ~63;
    const int s0 = min(n, w * seg), s1 = min(n, s0 + seg);
    if constexpr (RB > 0) {
        // --- 3. sort by code (codes are distinct): counting sort on the top BB bits
        //        (NB = 4 NT buckets; one LDS atomic per key returns its slot), then each
        //        key's final place = its bucket's start + its rank among the bucket's
        //        keys (buckets hold a few keys: a depth-5 cell of the quadtree)
        constexpr int NB = 4 * NT;
        constexpr int BB = __builtin_ctz(NB);
        uint32_t *bcnt = reinterpret_cast<uint32_t *>(smem + Lay::kHist);
        static_assert(NB * 4 <= 4 * 256 * (NT / 64), "bucket counters fit the histogram region");
#pragma unroll
        for (int i = 0; i < 4; i++) bcnt[tid * 4 + i] = 0u;
        __syncthreads();
        for (int j = tid; j < n; j += NT) {
            const uint32_t c = path_code(K[j]);
            code0[j] = c;
            idx0[j] = (uint16_t)atomicAdd(&bcnt[c >> (32 - BB)], 1u);
        }
        __syncthreads();
        {
            const uint4 c4 = *reinterpret_cast<const uint4 *>(bcnt + 4 * tid);
            int tot;
            const int ex = block_excl_scan<NT>((int)(c4.x + c4.y + c4.z + c4.w), Sc.red, &tot);
            *reinterpret_cast<uint4 *>(bcnt + 4 * tid) =
                make_uint4((uint32_t)ex, (uint32_t)ex + c4.x, (uint32_t)ex + c4.x + c4.y,
                           (uint32_t)ex + c4.x + c4.y + c4.z);
        }
        __syncthreads();
        for (int j = tid; j < n; j += NT) {
            const uint32_t c = code0[j];
            const uint32_t p = bcnt[c >> (32 - BB)] + idx0[j];
            code1[p] = c;
            idx1[p] = (uint16_t)j;
        }
        __syncthreads();
        for (int p = tid; p < n; p += NT) {
            const uint32_t c = code1[p];
            const uint32_t b = c >> (32 - BB);
            const int st = (int)bcnt[b], en = b + 1 < (uint32_t)NB ? (int)bcnt[b + 1] : n;
            int rank = 0;
            for (int q = st; q < en; q++) rank += code1[q] < c;
            code0[st + rank] = c;
            idx0[st + rank] = idx1[p];
        }
        __syncthreads();
    } else {
        {
            CP c_out = (passes & 1) ? code1 : code0;  // the sort ends in buffer 0
            IP i_out = (passes & 1) ? idx1 : idx0;
            for (int j = tid; j < n; j += NT) {
                c_out[j] = path_code(K[j]);
                i_out[j] = (uint16_t)j;
            }
        }
        __syncthreads();
        // --- 3'. (more keys than the LDS holds) LSD radix sort in the global scratch
        uint32_t *hist = reinterpret_cast<uint32_t *>(smem + Lay::kHist);
        for (int p = 0; p < passes; p++) {
            const bool from1 = ((passes - p) & 1) != 0;
            radix_pass<NT>(from1 ? code1 : code0, from1 ? idx1 : idx0, from1 ? code0 : code1, from1 ? idx0 : idx1,
                           s0, s1, lowbit + p * db, db, hist, Sc);
        }
    }
    if (l == 0) YGZ_BSTAMP_K(3, 4);
    // --- 4. L_k = depth of the common prefix of sorted keys k-1 and k (-1: root differs)
    for (int k = tid; k <= n; k += NT) {
        int v = -1;
        if (k > 0 && k < n) {
            const uint32_t a = code0[k - 1], c = code0[k];
            v = lcp_depth(a, c, rb);
            if (v >= Dn || a == c) Sc.s[1] = 1;
        }
        Lc[k] = (int8_t)v;
    }
    __syncthreads();
}

// List phase of one (frame, level) after the sort: the main loop's pass count and
// list from the histograms of L, the final rounds, the retained keys.  Lc: L of the
// sorted keys (i8 [n + 1]); key_at(k) -> {key, candidate index} of sorted key k;
// lsm: ListLayout<NC> (L not in it).
#ifndef YGZ_OCT_SEGSCAN
#define YGZ_OCT_SEGSCAN 1  // the final rounds' scans over a contiguous run of items per thread (0: strided)
#endif
#ifndef YGZ_OCT_CAND_RADIX
#define YGZ_OCT_CAND_RADIX 1  // the final rounds' candidate order by radix passes (0: the rank sort)
#endif
template <int NC, int NT, typename LP, typename KF>
__device__ __forceinline__ void body_list(const Plan *__restrict__ plan, const LevelDesc &L, int l, int f,
                                          uint8_t *lsm, Scal &Sc, LP Lc, int n, int bad, KF key_at,
                                          uint32_t *__restrict__ sel, int *__restrict__ selcnt,
                                          int *__restrict__ err) {
    using Lay = ListLayout<NC>;
    constexpr int NW = nwaves<NT>();
    const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const int Dn = L.oct_dn;
    const int seg = (((n + NW - 1) / NW) + 63) & ~63;
    const int s0 = min(n, w * seg), s1 = min(n, s0 + seg);
    const int nch = (s1 - s0 + 63) / 64;
    if (l == 0) YGZ_BSTAMP_K(3, 7);
    if (tid < 16) {
        Sc.hL[tid] = 0;
        Sc.hM[tid] = 0;
    }
    if (YGZ_OCT_CAND_RADIX && tid == 0) Sc.s[2] = 0;
    __syncthreads();
    auto chunk_ab = [&](int i, int k, int &a, int &b) {
        (void)i;
        a = Lc[k];
        b = Lc[k + 1];
    };
    for (int i = 0; i < nch; i++) {
        const int k = s0 + 64 * i + lane;
        const bool v = k < s1;
        int a = 0, m = 0;
        if (v) {
            int a0, b0;
            chunk_ab(i, k, a0, b0);
            a = a0 + 1;
            m = (a0 > b0 ? a0 : b0) + 1;
        }
        const uint64_t valid = __ballot(v);
        const uint64_t pa = match_bits((uint32_t)a, 4, valid);
        if (v && (pa & lanes_below()) == 0) atomicAdd(&Sc.hL[a], __popcll(pa));
        const uint64_t pm = match_bits((uint32_t)m, 4, valid);
        if (v && (pm & lanes_below()) == 0) atomicAdd(&Sc.hM[m], __popcll(pm));
    }
    __syncthreads();
    // P: the pass that ends the main loop; final = the final rounds follow
    const int N = L.budget;
    int P = 0, final_round = 0;
    {
        int cL = Sc.hL[0], cM = Sc.hM[0];
        int prev = cL;
        for (int d = 1; d < 16; d++) {
            cL += Sc.hL[d];
            cM += Sc.hM[d];
            P = d;
            if (cL >= N || cL == prev) break;
            if (cL + 3 * (cL - cM) > N) { final_round = 1; break; }
            prev = cL;
        }
    }
    bad |= P >= Dn;
    // --- 5. the list after P passes: heads (L_k < P), sections e = min(m_k + 1, P)
    uint32_t *node = reinterpret_cast<uint32_t *>(lsm + Lay::kNode);
    uint8_t *ndep = lsm + Lay::kDep;
    uint16_t *hs = reinterpret_cast<uint16_t *>(lsm + Lay::kHs);
    uint16_t *ngr = reinterpret_cast<uint16_t *>(lsm + Lay::kNgr);
    auto chunk_sec = [&](int i, int k) -> int {
        int sec = -1;
        if (k < s1) {
            int a, b;
            chunk_ab(i, k, a, b);
            if (a < P) sec = min((a > b ? a : b) + 1, P);
        }
        return sec;
    };
    // sweep A: per wave, heads per section (lanes matched on their section; the run's
    // leader adds its count)
    if (tid < 16 * NW) (&Sc.wcnt[0][0])[tid] = 0;
    __syncthreads();
    {
        int wh = 0;
        for (int i = 0; i < nch; i++) {
            const int sec = chunk_sec(i, s0 + 64 * i + lane);
            const uint64_t hb = __ballot(sec >= 0);
            wh += __popcll(hb);
            const uint64_t peers = match_bits((uint32_t)(sec + 1), 4, hb);
            if (sec >= 0 && (peers & lanes_below()) == 0) Sc.wcnt[w][sec] += __popcll(peers);
        }
        if (lane == 0) Sc.whead[w] = wh;
    }
    __syncthreads();
    // section e (e <= P): its count, its list base (sections P..0 descending), and this
    // wave's running rank inside it (LDS, per wave)
    int nheads = 0, hbase = 0;
    for (int ww = 0; ww < NW; ww++) {
        const int h = Sc.whead[ww];
        hbase += ww < w ? h : 0;
        nheads += h;
    }
    int front0 = 0;
    {
        int scnt = 0, srun = 0;
        if (lane < 16)
            for (int ww = 0; ww < NW; ww++) {
                const int x = Sc.wcnt[ww][lane];
                srun += ww < w ? x : 0;
                scnt += x;
            }
        int acc = 0, sbase = 0;
        for (int e = 15; e >= 0; e--) {
            const int c = __builtin_amdgcn_readlane(scnt, e);
            sbase = lane == e ? acc : sbase;
            acc += c;
        }
        front0 = __builtin_amdgcn_readlane(scnt, P);
        __syncthreads();  // every wave has read wcnt
        if (lane < 16) {
            Sc.wcnt[w][lane] = srun;  // now: this wave's running rank in section lane
            if (w == 0) {
                Sc.hL[lane] = sbase;  // reused: section base / count
                Sc.hM[lane] = scnt;
            }
        }
        __syncthreads();
    }
    int overflow = bad || nheads > NC;
    if (!overflow) {
        int hr = hbase;
        for (int i = 0; i < nch; i++) {
            const int k = s0 + 64 * i + lane;
            const int sec = chunk_sec(i, k);
            const uint64_t hb = __ballot(sec >= 0);
            const int gr = hr + __popcll(hb & lanes_below());
            hr += __popcll(hb);
            const uint64_t peers = match_bits((uint32_t)(sec + 1), 4, hb);
            const int q = sec < 0 ? 0 : sec;
            const int r0 = Sc.wcnt[w][q];
            if (sec >= 0) {
                const uint64_t below = peers & lanes_below();
                const int rank = r0 + __popcll(below);
                if (below == 0) Sc.wcnt[w][q] = r0 + __popcll(peers);
                const int bse = Sc.hL[q], ce = Sc.hM[q];
                const int pos = bse + ((sec & 1) ? rank : ce - 1 - rank);
                hs[gr] = (uint16_t)k;
                ngr[pos] = (uint16_t)gr;
                ndep[pos] = (uint8_t)sec;
            }
        }
        if (tid == 0) hs[nheads] = (uint16_t)n;
    }
    __syncthreads();
    int size = nheads;
    if (!overflow) {
        for (int p = tid; p < size; p += NT) {
            const int gr = ngr[p];
            const int st = hs[gr];
            node[p] = (uint32_t)st | ((uint32_t)(hs[gr + 1] - st) << 16);
        }
    }
    __syncthreads();
    if (l == 0) YGZ_BSTAMP_K(3, 5);
    // --- 6. final rounds
    int cur = 0, front = front0;
    uint32_t *ck = reinterpret_cast<uint32_t *>(lsm + Lay::kCk);
    uint16_t *cev = reinterpret_cast<uint16_t *>(lsm + Lay::kCe);
    uint16_t *cin = reinterpret_cast<uint16_t *>(lsm + Lay::kCi);
    int guard = 0;
    while (final_round && !overflow) {
        const int prevSize = size;
        uint32_t *nd = node + cur * NC, *nn = node + (cur ^ 1) * NC;
        uint8_t *dd = ndep + cur * NC, *dn = ndep + (cur ^ 1) * NC;
        // candidates: front nodes with > 1 key, key (count desc, position asc)
        int nc = 0;
#if YGZ_OCT_SEGSCAN
        {   // a contiguous run of nodes per thread: one block scan for the whole front
            const int per = (front + NT - 1) / NT;
            const int b0 = min(front, tid * per), b1 = min(front, b0 + per);
            int cnt = 0;
            for (int p = b0; p < b1; p++) cnt += (nd[p] >> 16) > 1u ? 1 : 0;
            int tot;
            int o = block_excl_scan<NT>(cnt, Sc.red, &tot);
            for (int p = b0; p < b1; p++) {
                const uint32_t r = nd[p];
                if ((r >> 16) > 1u) {
                    ck[o++] = ((0xFFFFu - (r >> 16)) << 16) | (uint32_t)p;
                    if (YGZ_OCT_CAND_RADIX && (r >> 16) >= 256u) Sc.s[2] = 1;
                }
            }
            nc = tot;
        }
        if (false)
#endif
        for (int p0 = 0; p0 < front; p0 += NT) {
            const int p = p0 + tid;
            const uint32_t r = p < front ? nd[p] : 0u;
            const bool cand = p < front && (r >> 16) > 1u;
            int tot;
            const int ex = block_excl_scan<NT>(cand ? 1 : 0, Sc.red, &tot);
            if (cand) ck[nc + ex] = ((0xFFFFu - (r >> 16)) << 16) | (uint32_t)p;
            if (YGZ_OCT_CAND_RADIX && cand && (r >> 16) >= 256u) Sc.s[2] = 1;  // a node of >= 256 keys
            nc += tot;
        }
        if (tid < 4) ck[nc + tid] = 0xFFFFFFFFu;  // pad to a multiple of 4 (never smaller)
        __syncthreads();
#if YGZ_OCT_CAND_RADIX
        if constexpr (NW * 1024 <= 4 * NC) {
            // the candidates are in list-position order already, so (count desc, position asc)
            // is a stable sort on 0xFFFF - count: one 8-bit LSD pass (bits 16-23), a second
            // (bits 24-31) only when a node holds >= 256 keys
            uint32_t *tmp = reinterpret_cast<uint32_t *>(lsm + Lay::kCe);   // cev + cin: written after
            uint32_t *hist = reinterpret_cast<uint32_t *>(lsm + Lay::kHs);  // hs + ngr: free after step 5
            const int cseg = (((nc + NW - 1) / NW) + 63) & ~63;
            const int c0 = min(nc, w * cseg), c1 = min(nc, c0 + cseg);
            const bool big = Sc.s[2] != 0;
            radix_pass_codes<NT>(ck, tmp, c0, c1, 16, 8, hist, Sc);
            if (big) {
                radix_pass_codes<NT>(tmp, ck, c0, c1, 24, 8, hist, Sc);
            } else {
                for (int c = tid; c < nc; c += NT) ck[c] = tmp[c];
                __syncthreads();
            }
            if (tid == 0) Sc.s[2] = 0;
        } else
#endif
        {   // ascending by rank (distinct keys): one barrier, broadcast 16-B reads
            constexpr int kPer = (NC + NT - 1) / NT;
            uint32_t mine[kPer];
            int rk[kPer];
#pragma unroll
            for (int u = 0; u < kPer; u++) {
                mine[u] = tid + u * NT < nc ? ck[tid + u * NT] : 0xFFFFFFFFu;
                rk[u] = 0;
            }
#pragma unroll
            for (int u = 0; u < kPer; u++) {
                if (u * NT + w * 64 >= nc) break;  // wave-uniform: slots past the candidates skip
                for (int j = 0; j < nc; j += 4) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(ck + j);
                    rk[u] += (v.x < mine[u]) + (v.y < mine[u]) + (v.z < mine[u]) + (v.w < mine[u]);
                }
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kPer; u++)
                if (tid + u * NT < nc) ck[rk[u]] = mine[u];
            __syncthreads();
        }
        // children per candidate: 1 + #{k in the run : L_k == depth}, four L bytes per
        // LDS read (exact zero-byte test on L ^ depth)
        if (tid == 0) Sc.s[0] = nc;
        for (int c = tid; c < nc; c += NT) {
            const int p = (int)(ck[c] & 0xFFFFu);
            const uint32_t r = nd[p];
            const int st = (int)(r & 0xFFFFu), ln = (int)(r >> 16), dep = dd[p] & 0x7F;
            int e = 1;
            if constexpr (true) {
                const uint32_t rep = 0x01010101u * (uint32_t)dep;
                const int k0 = st + 1, k1 = st + ln;  // [k0, k1)
                for (int a = k0 & ~3; a < k1; a += 4) {
                    const uint32_t x = *reinterpret_cast<const uint32_t *>(Lc + a) ^ rep;
                    uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // 0x80 per zero byte
                    const int lo = k0 - a, hi = k1 - a;  // bytes [lo, hi) of this word count
                    if (lo > 0) z &= 0xFFFFFFFFu << (8 * lo);
                    if (hi < 4) z &= 0xFFFFFFFFu >> (8 * (4 - hi));
                    e += __popc(z);
                }
            }
            cev[c] = (uint16_t)e;
        }
        __syncthreads();
        // cut: first c with size + sum_{c' <= c} (e - 1) >= N; one scan carries both sums
#if YGZ_OCT_SEGSCAN
        {
            const int per = (nc + NT - 1) / NT;
            const int b0 = min(nc, tid * per), b1 = min(nc, b0 + per);
            int sE = 0, sD = 0;
            for (int c = b0; c < b1; c++) {
                const int e = (int)cev[c];
                sE += e;
                sD += e - 1;
            }
            int tot;
            const int ex = block_excl_scan<NT>((sE << 16) | sD, Sc.red, &tot);
            int runE = ex >> 16, runD = ex & 0xFFFF;
            bool hit = false;
            for (int c = b0; c < b1; c++) {
                const int e = (int)cev[c];
                runE += e;
                cin[c] = (uint16_t)runE;
                if (!hit && size + runD + (e - 1) >= N) {
                    atomicMin(&Sc.s[0], c);
                    hit = true;
                }
                runD += e - 1;
            }
        }
        if (false)
#endif
        {
            int carryE = 0, carryD = 0;
            for (int c0 = 0; c0 < nc; c0 += NT) {
                const int c = c0 + tid;
                const int e = c < nc ? (int)cev[c] : 0;
                int tot;
                const int ex = block_excl_scan<NT>(c < nc ? (e << 16) | (e - 1) : 0, Sc.red, &tot);
                const int exE = ex >> 16, exD = ex & 0xFFFF;
                if (c < nc) {
                    cin[c] = (uint16_t)(carryE + exE + e);
                    if (size + carryD + exD + (e - 1) >= N) atomicMin(&Sc.s[0], c);
                }
                carryE += tot >> 16;
                carryD += tot & 0xFFFF;
            }
        }
        __syncthreads();
        const int cstar = min(Sc.s[0], nc - 1);
        const int ctot = cstar >= 0 ? (int)cin[cstar] : 0;
        if (ctot + size - (cstar + 1) > NC) {
            overflow = 1;
            break;
        }
        // children of the divided nodes: group of c at ctot - cin[c], list-front order
        for (int c = tid; c <= cstar; c += NT) {
            const int p = (int)(ck[c] & 0xFFFFu);
            const uint32_t r = nd[p];
            const int st = (int)(r & 0xFFFFu), ln = (int)(r >> 16), dep = dd[p] & 0x7F;
            const int e = cev[c], g0 = ctot - (int)cin[c];
            const bool fwd = ((dep + 1) & 1) != 0;
            dd[p] = (uint8_t)(dep | 0x80);
            int i = 0, cs = st;
            for (int k = st + 1; k <= st + ln; k++) {
                if (k == st + ln || Lc[k] == dep) {
                    const int pos = g0 + (fwd ? i : e - 1 - i);
                    nn[pos] = (uint32_t)cs | ((uint32_t)(k - cs) << 16);
                    dn[pos] = (uint8_t)(dep + 1);
                    cs = k;
                    i++;
                }
            }
        }
        __syncthreads();
        // the other nodes keep their order behind the new front
#if YGZ_OCT_SEGSCAN
        {
            const int per = (size + NT - 1) / NT;
            const int b0 = min(size, tid * per), b1 = min(size, b0 + per);
            int cnt = 0;
            for (int p = b0; p < b1; p++) cnt += (dd[p] & 0x80) ? 0 : 1;
            int tot;
            int o = ctot + block_excl_scan<NT>(cnt, Sc.red, &tot);
            for (int p = b0; p < b1; p++) {
                if (!(dd[p] & 0x80)) {
                    nn[o] = nd[p];
                    dn[o] = dd[p];
                    o++;
                }
            }
        }
        if (false)
#endif
        {
            int carry = 0;
            for (int p0 = 0; p0 < size; p0 += NT) {
                const int p = p0 + tid;
                const bool keep = p < size && !(dd[p] & 0x80);
                int tot;
                const int ex = block_excl_scan<NT>(keep ? 1 : 0, Sc.red, &tot);
                if (keep) {
                    nn[ctot + carry + ex] = nd[p];
                    dn[ctot + carry + ex] = dd[p];
                }
                carry += tot;
            }
        }
        __syncthreads();
        size = ctot + size - (cstar + 1);
        front = ctot;
        cur ^= 1;
        if (size >= N || size == prevSize || ++guard > 64) break;
    }
    if (l == 0) YGZ_BSTAMP_K(3, 6);
    // --- 7. retained key per node (first maximum response in candidate order), list order
    uint32_t *out = sel + (size_t)f * plan->sel_total + L.sel_off;
    if (size > L.sel_cap) overflow = 1;
    if (!overflow) {
        const uint32_t *nd = node + cur * NC;
        for (int i = tid; i < size; i += NT) {
            const uint32_t r = nd[i];
            const int st = (int)(r & 0xFFFFu), ln = (int)(r >> 16);
            // the (score, -index) values are distinct, so the maximum does not depend on
            // the visiting order: four keys' loads in flight at a time
            uint32_t best = 0u, bkey = 0u;
            int k = st;
            for (; k + 4 <= st + ln; k += 4) {
                uint32_t kv[4], ix[4];
#pragma unroll
                for (int u = 0; u < 4; u++) key_at(k + u, kv[u], ix[u]);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t v = ((uint32_t)key_score(kv[u]) << 24) | (0xFFFFFFu - ix[u]);
                    bkey = v > best ? kv[u] : bkey;
                    best = v > best ? v : best;
                }
            }
            for (; k < st + ln; k++) {
                uint32_t kv, ix;
                key_at(k, kv, ix);
                const uint32_t v = ((uint32_t)key_score(kv) << 24) | (0xFFFFFFu - ix);
                bkey = v > best ? kv : bkey;
                best = v > best ? v : best;
            }
            out[i] = bkey;
        }
    }
    if (tid == 0) {
        selcnt[(size_t)f * plan->nlevels + l] = overflow ? 0 : size;
        if (overflow) atomicOr(err, 1);
    }
    if (l == 0) YGZ_BSTAMP_K(3, 1);
}

}  // namespace oct

// Work queues between the octree sort stages of one node-pool class (api.cpp zeroes
// the counters before each extraction): a task (f << 4 | l) whose level has more
// candidates than a stage's LDS holds is appended to the next stage's list.
struct OctQueue {
    int *cnt_in, *taken_in;
    const int *list_in;
    int *cnt_out, *list_out;
};

// Sorted-key scratch of a task in the candidate scratch: sorted keys Ks (u32 [C],
// candA), their candidate indices Is (u16 [C], candB) and L (i8 [C + 1], candB + 4 C).
struct OctScratch {
    uint32_t *Ks;
    uint16_t *Is;
    int8_t *Lg;
    __device__ OctScratch(const Plan *plan, const LevelDesc &L, uint32_t *candA, uint32_t *candB, int f) {
        const size_t slot = 2 * ((size_t)f * plan->cand_total + L.cand_off), C = (size_t)L.cand_cap;
        Ks = candA + slot;
        Is = reinterpret_cast<uint16_t *>(candB + slot);
        Lg = reinterpret_cast<int8_t *>(candB + slot + C);
    }
};

// Sort stage of one (frame, level) with keys, codes and indices in LDS (at most NK
// candidates): sorted keys, indices and L to the scratch, hdr = n + 1 | bad << 30
// (0: the task went on to a later stage).
template <int NC, int NK, int NT>
__device__ __forceinline__ void octree_sort_task(const Plan *__restrict__ plan, const uint32_t *__restrict__ cellbuf,
                                                 const int *__restrict__ cellcnt, uint32_t *__restrict__ candA,
                                                 uint32_t *__restrict__ candB, int *__restrict__ hdr, int f, int l,
                                                 const OctQueue &q, uint8_t *smem, oct::Scal &Sc) {
    using Lay = oct::Layout<NC, NK, NT>;
    const int tid = threadIdx.x;
    if (l == 0) YGZ_BSTAMP_K(3, 0);
    const LevelDesc &L = plan->lv[l];
    if (tid == 0) Sc.s[1] = 0;  // "not separated" flag (ordered by the scans' barriers)
    int part = 0;
    for (int c = tid; c < L.ncells; c += NT) part += cellcnt[(size_t)f * plan->ncells + L.cell_begin + c];
    int n;
    block_excl_scan<NT>(part, Sc.red, &n);
    const size_t t = (size_t)f * plan->nlevels + l;
    if (n > NK) {
        if (tid == 0) {
            hdr[t] = 0;
            q.list_out[atomicAdd(q.cnt_out, 1)] = (f << 4) | l;
        }
        return;
    }
    uint32_t *K = reinterpret_cast<uint32_t *>(smem + Lay::kK);
    uint32_t *c0 = reinterpret_cast<uint32_t *>(smem + Lay::kCode0);
    uint16_t *i0 = reinterpret_cast<uint16_t *>(smem + Lay::kIdx0);
    uint32_t *c1 = reinterpret_cast<uint32_t *>(smem + Lay::kCode1);
    uint16_t *i1 = reinterpret_cast<uint16_t *>(smem + Lay::kIdx1);
    static_assert(NK % NT == 0 && ((NK / NT) & (NK / NT - 1)) == 0, "NK = 64 x waves x a power of two");
    const OctScratch o(plan, L, candA, candB, f);
    oct::body_sort<NC, NK, NT, NK / NT>(plan, L, l, f, smem, Sc, cellbuf, cellcnt, K, c0, i0, c1, i1, o.Lg, n);
    for (int k = tid; k < n; k += NT) {
        const uint16_t ix = i0[k];
        o.Ks[k] = K[ix];
        o.Is[k] = ix;
    }
    if (tid == 0) hdr[t] = (n + 1) | (Sc.s[1] << 30);
}

// First sort stage: one workgroup per (frame, level) of the launch group.
template <int NC, int NK, int NT>
__global__ __launch_bounds__(NT) void k_octree_sort(const Plan *__restrict__ plan, const uint32_t *__restrict__ cellbuf,
                                                     const int *__restrict__ cellcnt, uint32_t *__restrict__ candA,
                                                     uint32_t *__restrict__ candB, int *__restrict__ hdr, int level0,
                                                     OctQueue q) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[oct::Layout<NC, NK, NT>::kBytes];
    __shared__ oct::Scal Sc;
    octree_sort_task<NC, NK, NT>(plan, cellbuf, cellcnt, candA, candB, hdr, blockIdx.x, level0 + blockIdx.y, q, smem,
                                 Sc);
}

// Later sort stages: a persistent grid takes the previous stage's overflow tasks.
template <int NC, int NK, int NT>
__global__ __launch_bounds__(NT) void k_octree_sort_q(const Plan *__restrict__ plan,
                                                       const uint32_t *__restrict__ cellbuf,
                                                       const int *__restrict__ cellcnt, uint32_t *__restrict__ candA,
                                                       uint32_t *__restrict__ candB, int *__restrict__ hdr, OctQueue q) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[oct::Layout<NC, NK, NT>::kBytes];
    __shared__ oct::Scal Sc;
    __shared__ int s_task;
    const int count = *q.cnt_in;
    while (true) {
        __syncthreads();  // the previous task's LDS reads are done
        if (threadIdx.x == 0) {
            const int i = atomicAdd(q.taken_in, 1);
            s_task = i < count ? q.list_in[i] : -1;
        }
        __syncthreads();
        const int t = s_task;
        if (t < 0) break;
        octree_sort_task<NC, NK, NT>(plan, cellbuf, cellcnt, candA, candB, hdr, t >> 4, t & 15, q, smem, Sc);
    }
}

// List phase of every sorted task of the launch group: L staged into LDS, the node
// lists in LDS (~31 KB at NC 1024: five workgroups per CU where the sort holds two).
template <int NC, int NT>
__global__ __launch_bounds__(NT) void k_octree_list(const Plan *__restrict__ plan, uint32_t *__restrict__ candA,
                                                     uint32_t *__restrict__ candB, const int *__restrict__ hdr,
                                                     uint32_t *__restrict__ sel, int *__restrict__ selcnt,
                                                     int *__restrict__ err, int level0) {
    using Lay = oct::ListLayout<NC>;
    __shared__ __attribute__((aligned(16))) uint8_t lsm[Lay::bytes(8192 + 4)];
    __shared__ oct::Scal Sc;
    const int f = blockIdx.x, l = level0 + blockIdx.y, tid = threadIdx.x;
    const int h = hdr[(size_t)f * plan->nlevels + l];
    if (h == 0) return;  // left to the global-scratch stage
    const int n = (h & 0x3FFFFFFF) - 1, bad = (h >> 30) & 1;
    const LevelDesc &L = plan->lv[l];
    const OctScratch o(plan, L, candA, candB, f);
    int8_t *Lc = reinterpret_cast<int8_t *>(lsm + Lay::kLc);
    for (int i = tid; i <= n >> 2; i += NT)
        reinterpret_cast<uint32_t *>(Lc)[i] = as_global(reinterpret_cast<const uint32_t *>(o.Lg))[i];
    // (body_list's first barrier publishes L)
    auto key_at = [&](int k, uint32_t &kv, uint32_t &ix) {
        kv = as_global(o.Ks)[k];
        ix = as_global(o.Is)[k];
    };
    oct::body_list<NC, NT>(plan, L, l, f, lsm, Sc, Lc, n, bad, key_at, sel, selcnt, err);
}

// Last stage (more keys than any LDS form holds: dense frames only): keys, codes and
// L in the candidate scratch (8 + 8 B per slot in candA / candB), LSD radix sort, then
// the list phase, in one workgroup.
template <int NC, int NT>
__global__ __launch_bounds__(NT) void k_octree_global(const Plan *__restrict__ plan,
                                                       const uint32_t *__restrict__ cellbuf,
                                                       const int *__restrict__ cellcnt, uint32_t *__restrict__ candA,
                                                       uint32_t *__restrict__ candB, uint32_t *__restrict__ sel,
                                                       int *__restrict__ selcnt, int *__restrict__ err, OctQueue q) {
    constexpr int NK = NT;  // no keys in LDS; the layout's union region holds the lists
    using Lay = oct::Layout<NC, NK, NT>;
    __shared__ __attribute__((aligned(16))) uint8_t smem[Lay::kBytes];
    __shared__ oct::Scal Sc;
    __shared__ int s_task;
    const int tid = threadIdx.x;
    const int count = *q.cnt_in;
    while (true) {
        __syncthreads();
        if (tid == 0) {
            const int i = atomicAdd(q.taken_in, 1);
            s_task = i < count ? q.list_in[i] : -1;
        }
        __syncthreads();
        const int t = s_task;
        if (t < 0) break;
        const int f = t >> 4, l = t & 15;
        const LevelDesc &L = plan->lv[l];
        if (tid == 0) Sc.s[1] = 0;
        int part = 0;
        for (int c = tid; c < L.ncells; c += NT) part += cellcnt[(size_t)f * plan->ncells + L.cell_begin + c];
        int n;
        block_excl_scan<NT>(part, Sc.red, &n);
        if (n > 65535) {  // u16 positions / run lengths
            if (tid == 0) {
                selcnt[(size_t)f * plan->nlevels + l] = 0;
                atomicOr(err, 1);
            }
            continue;
        }
        const size_t C = (size_t)L.cand_cap;
        uint32_t *A = candA + 2 * ((size_t)f * plan->cand_total + L.cand_off);
        uint32_t *B = candB + 2 * ((size_t)f * plan->cand_total + L.cand_off);
        uint16_t *i0 = reinterpret_cast<uint16_t *>(B + C);
        int8_t *Lg = reinterpret_cast<int8_t *>(B);  // L in code1's space once the sort is done with it
        oct::body_sort<NC, NK, NT, 0>(plan, L, l, f, smem, Sc, cellbuf, cellcnt, A, A + C, i0, B, i0 + C, Lg, n);
        auto key_at = [&](int k, uint32_t &kv, uint32_t &ix) {
            ix = i0[k];
            kv = A[ix];
        };
        oct::body_list<NC, NT>(plan, L, l, f, smem + Lay::kU, Sc, Lg, n, Sc.s[1], key_at, sel, selcnt, err);
    }
}


// ---------------------------------------------------------------------------
// Orientation (IC_Angle on the unblurred level, ORBextractor.cc:77-101) and
// steered BRIEF (computeOrbDescriptor on the blurred level, :105-149).
// One wave per keypoint; four per 256-thread workgroup.

struct KpJob {
    int x, y;        // integer centre at level scale (cvRound(pt))
    float angle;
};

__device__ __forceinline__ float ic_angle_wave(const uint8_t *img, int w, int h, int cx, int cy,
                                               const int *umax) {
    const int lane = threadIdx.x & 63;
    int m01 = 0, m10 = 0;
    if (lane < 31) {
        const int u = lane - 15, xx = clampi(cx + u, 0, w - 1);
        m10 = u * img[(size_t)clampi(cy, 0, h - 1) * w + xx];
        for (int v = 1; v <= 15; v++) {
            if (u < -umax[v] || u > umax[v]) continue;
            const int vp = img[(size_t)clampi(cy + v, 0, h - 1) * w + xx];
            const int vm = img[(size_t)clampi(cy - v, 0, h - 1) * w + xx];
            m01 += v * (vp - vm);
            m10 += u * (vp + vm);
        }
    }
    m01 = wave_sum_i(m01);
    m10 = wave_sum_i(m10);
    return fast_atan2_deg((float)m01, (float)m10);
}

// computeOrbDescriptor: lane l evaluates pairs 4l..4l+3; lanes 8w..8w+7 form word w.
__device__ __forceinline__ void orb_desc_wave(const uint8_t *img, int w, int h, int cx, int cy,
                                              float angle_deg, uint8_t *desc_out) {
    const int lane = threadIdx.x & 63;
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float ang = angle_deg * factorPI;
    float a, b;
    glibc_sincosf(ang, b, a);
    uint32_t nib = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int pi = (lane * 4 + k) * 4;
        const float px0 = (float)c_pattern[pi], py0 = (float)c_pattern[pi + 1];
        const float px1 = (float)c_pattern[pi + 2], py1 = (float)c_pattern[pi + 3];
        const int y0 = cy + cv_round(__builtin_fmaf(px0, b, py0 * a)), x0 = cx + cv_round(__builtin_fmaf(px0, a, -(py0 * b)));
        const int y1 = cy + cv_round(__builtin_fmaf(px1, b, py1 * a)), x1 = cx + cv_round(__builtin_fmaf(px1, a, -(py1 * b)));
        const int t0 = img[(size_t)clampi(y0, 0, h - 1) * w + clampi(x0, 0, w - 1)];
        const int t1 = img[(size_t)clampi(y1, 0, h - 1) * w + clampi(x1, 0, w - 1)];
        nib |= (uint32_t)(t0 < t1) << k;
    }
    uint32_t word = nib;
#pragma unroll
    for (int i = 1; i < 8; i++) word |= (uint32_t)__shfl_down((int)nib, i, 64) << (4 * i);
    if ((lane & 7) == 0) reinterpret_cast<uint32_t *>(desc_out)[lane >> 3] = word;
}

// 16-lane row reduction (DPP within a row; every lane of the row gets the sum)
__device__ __forceinline__ int row16_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);  // row_mirror
    return v;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) uint8_t lds_u8;
constexpr uint32_t kMagicBits = 0x4B000000u;  // bits of 2^23 (ulp 1 in [2^23, 2^24))
// LDS row of a staged keypoint window: the 13 dwords that hold the window's
// 37 bytes at any 16-B misalignment (o + 37 <= 52).  An odd dword stride puts
// 32 consecutive rows on 32 different banks (a 64-B stride folds every row onto
// two bank offsets); rows are 4-B aligned, so they are written as dwords.
// (A 44-B stride with each row stored from the dword holding the window's first
// byte fits 6 workgroups per CU: bit-exact, but 0.468 ms / 1024 frames at 5 waves
// / SIMD and 0.96 with the 6th wave's register spills, against 0.448 --
// profiles/r04_orient_patch44.txt.)
constexpr int kPatchStride = 52;
// slot per keypoint row: 37 rows, padded to 496 dwords (= 16 mod 32) so that the
// two keypoints of a 32-lane group read complementary bank sets in the IC pass
constexpr int kPatchBytes = 1984;
static_assert(37 * kPatchStride <= kPatchBytes && (kPatchBytes / 4) % 32 == 16, "patch slot");

__device__ __forceinline__ uint32_t patch_row_swz(uint32_t r) { return r * (uint32_t)kPatchStride; }

// A keypoint window (rows cy-R .. cy-R+NROWS-1) as 4 lanes x 16 B per row, each
// row the 64 B at ((img + (cy-R+r)*w + cx-R) & ~15): loaded into registers by
// load_window (so both windows of a keypoint are in flight together), written
// unshifted to LDS by store_window (tap (r, c) at P[r*64 + o(r) + c]).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));


template <int R, int NROWS>
struct Window {
    static constexpr int NK = (NROWS + 3) / 4;
    u32x4 v[NK];
    // frame: the frame's pyramid; c: byte offset of the centre pixel in it
    __device__ __forceinline__ void load(const uint8_t *frame, uint32_t w, uint32_t c, int s) {
        // 32-bit offsets (24-bit multiplies) added to the frame pointer once per row
        const uint32_t base = c - (uint32_t)R * w - (uint32_t)R;
        const uint32_t a0 = (uint32_t)(uintptr_t)frame & 15u;  // 0 unless a caller-bound buffer is unaligned
        const int j = s & 3, r0 = s >> 2;
#pragma unroll
        for (int k = 0; k < NK; k++) {  // rows past the window re-read its last row (not stored)
            const uint32_t o = ((mad24((uint32_t)min(r0 + 4 * k, NROWS - 1), w, base) + a0) & ~15u) - a0 + 16u * j;
            v[k] = as_global(reinterpret_cast<const u32x4 *>(frame + o))[0];
        }
    }
    // row r at 52 r: lane j of the row's four writes dwords 4j..4j+3 of the
    // row's aligned 64 B, only the first 13 (lane 3: one)
    __device__ __forceinline__ void store(uint8_t *P, int s) const {
        const int j = s & 3, r0 = s >> 2;
#pragma unroll
        for (int k = 0; k < NK; k++) {
            const int r = r0 + 4 * k;
            if (k + 1 < NK || r < NROWS) {
                uint32_t *d = reinterpret_cast<uint32_t *>(P + r * kPatchStride + 16 * j);
                d[0] = v[k].x;
                if (j < 3) {
                    d[1] = v[k].y;
                    d[2] = v[k].z;
                    d[3] = v[k].w;
                }
            }
        }
        wave_lds_order();
    }
};

// Keypoint rows of the octree selection (ORBextractor.cc:785-797): level-0
// coordinates (x, y) * scale, size = PATCH_SIZE * scale, response = FAST
// score, octave, class_id -1; angle is filled in by k_orient_desc.  Written
// as soon as the octree is done, so consumers of positions only (map-point
// snapshots, SparseImgAlign) need not wait for the descriptors.
// Beside each row: its orientation job {byte offset of the keypoint pixel in the
// frame's pyramid, level width | level << 16}, kOrientNone for selection slots
// past the frame's count, so k_orient_desc starts its window loads after one
// load (no per-level count prefix, plan lookup and key decode on its critical path).
constexpr uint32_t kOrientNone = 0xFFFFFFFFu;
__global__ __launch_bounds__(256) void k_emit_kps(const Plan *__restrict__ plan, const uint32_t *__restrict__ sel,
                                                  const int *__restrict__ selcnt, const int *__restrict__ n_existing,
                                                  ygzfe_kp *__restrict__ kps, int *__restrict__ counts, int row_cap,
                                                  uint2 *__restrict__ ojobs) {
    const int f = blockIdx.y;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int nl = plan->nlevels, sel_total = plan->sel_total;
    const int *sc = selcnt + (size_t)f * nl;
    const int ne = n_existing ? n_existing[f] : 0;
    int l = 0, pre = 0, acc = 0;
    for (int q = 0; q < nl; q++) {
        acc += sc[q];
        if (acc <= idx) { l = q + 1; pre = acc; }
    }
    if (idx == 0) counts[f] = ne + acc;
    if (l >= nl || ne + idx >= row_cap) {
        if (idx < sel_total) ojobs[(size_t)f * sel_total + idx] = make_uint2(kOrientNone, 0u);
        return;
    }
    const LevelDesc &L = plan->lv[l];
    const uint32_t key = sel[(size_t)f * sel_total + L.sel_off + (idx - pre)];
    const int cx = key_x(key) + kMinBorder, cy = key_y(key) + kMinBorder;
    ygzfe_kp kp;
    kp.x = (float)cx;
    kp.y = (float)cy;
    if (l != 0) { kp.x *= L.scale; kp.y *= L.scale; }
    kp.size = (float)L.patch_size;
    kp.angle = 0.f;
    kp.response = (float)key_score(key);
    kp.octave = l;
    kp.class_id = -1;
    kps[(size_t)f * row_cap + ne + idx] = kp;
    ojobs[(size_t)f * sel_total + idx] =
        make_uint2(L.off + (uint32_t)cy * (uint32_t)L.w + (uint32_t)cx, (uint32_t)L.w | ((uint32_t)l << 16));
}

// The IC window (31 rows from cy - 15) staged with the three aligned 16-B
// chunks a row needs (misalignment + 31 <= 46 B): chunk c = s + 16 k of the
// keypoint's 93 is row c / 3, chunk c % 3; row r at patch_row_swz(r) in LDS.
struct IcWindow {
    u32x4 v[6];
    __device__ __forceinline__ void load(const uint8_t *frame, uint32_t w, uint32_t c, int s) {
        const uint32_t base = c - 15u * w - 15u;
        const uint32_t a0 = (uint32_t)(uintptr_t)frame & 15u;
#pragma unroll
        for (int k = 0; k < 6; k++) {  // slots past chunk 92 re-read it (not stored)
            const uint32_t ch = min((uint32_t)(s + 16 * k), 92u), r = ch / 3u, j = ch - 3u * r;
            const uint32_t o = ((mad24(r, w, base) + a0) & ~15u) - a0 + 16u * j;
            v[k] = as_global(reinterpret_cast<const u32x4 *>(frame + o))[0];
        }
    }
    __device__ __forceinline__ void store(uint8_t *P, int s) const {
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const uint32_t ch = (uint32_t)(s + 16 * k), r = ch / 3u, j = ch - 3u * r;
            if (k < 5 || ch < 93u) {
                uint32_t *d = reinterpret_cast<uint32_t *>(P + patch_row_swz(r) + 16u * j);
                d[0] = v[k].x;
                d[1] = v[k].y;
                d[2] = v[k].z;
                d[3] = v[k].w;
            }
        }
        wave_lds_order();
    }
};

// New keypoints of the octree: rows n_existing + selection index.
// One 16-lane DPP row per keypoint (four per wave, sixteen per workgroup):
//   IC_Angle: lane s takes window rows 15 +- (s + 1) (lane 15: the centre row)
//   rBRIEF:   lane s evaluates pairs 16s..16s+15 (half of descriptor word s/2)
// Both windows are staged in LDS by 16-B aligned dwordx4 loads (4 lanes x 16 B
// per window row, kept unshifted: window row r starts at byte o(r) = (row
// address) & 15 of LDS row r); every tap is an LDS byte read.  Octree
// keypoints sit >= 19 px inside the level, so the 31x31 IC window and the
// 37x37 rotated-pattern window never leave it.
// (The rBRIEF taps gathered from the L1/L2-resident blurred level with only the IC window
// in LDS, six workgroups per CU, was bit-exact but 0.84 against 0.45 ms per 1,024 frames:
// 2.6x the TA busy cycles of the LDS form -- profiles/r05_orient_gather.txt.)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_orient_desc(const uint8_t *__restrict__ pyr,
                                                     const uint8_t *__restrict__ blur, uint32_t pitch,
                                                     const Plan *__restrict__ plan, const uint2 *__restrict__ ojobs,
                                                     const int *__restrict__ n_existing,
                                                     ygzfe_kp *__restrict__ kps, uint8_t *__restrict__ desc,
                                                     int row_cap) {
    __shared__ uint8_t s_patch[16][kPatchBytes];  // one 37x37 window per keypoint row
    // the pattern (c_pattern, 1 KB) staged once per workgroup; the IC row weights are
    // formed in registers from umax, so the workgroup's LDS is 32 KB (5 per CU)
    __shared__ uint4 s_const[64];
    int bx, f;
    swizzled_block_2d(bx, f);  // one frame's keypoints on one XCD: window lines shared in its L2
    const int lane = threadIdx.x & 63, s = lane & 15;
    const int idx = bx * 16 + (threadIdx.x >> 4);
    uint4 cst = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x < 64) cst = reinterpret_cast<const uint4 *>(c_pattern_f8)[threadIdx.x];
    const int sel_total = plan->sel_total;
    uint2 job = make_uint2(kOrientNone, 0u);
    if (idx < sel_total) job = ojobs[(size_t)f * sel_total + idx];
    const bool active = job.x != kOrientNone;
    // inactive rows load a dummy window at the start of the frame (unconditional
    // loads keep the wait counts static, so the barrier below waits only for the
    // constants, not for the windows in flight)
    const uint32_t c = active ? job.x : 18u * 64u + 18u, w = active ? job.y & 0xFFFFu : 64u;
    const uint8_t *fimg = pyr + (size_t)f * pitch;
    const uint8_t *fblur = blur + (size_t)f * pitch;
    uint8_t *P = s_patch[threadIdx.x >> 4];
    IcWindow wic;
    Window<18, 37> wdesc;
    wic.load(fimg, w, c, s);  // the rBRIEF window follows once the IC window is in LDS
    if (threadIdx.x < 64) s_const[threadIdx.x] = cst;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    wave_lds_order();
    if (!active) return;  // whole rows leave together
    // IC row weights of lane s's rows (|v| = s + 1; lane 15 the centre row): byte b of
    // the 32 is 1 / b where |b - 15| <= umax[|v|] (the disc), else 0
    uint32_t W0[8], W1[8];
    {
        const int um = plan->umax[s == 15 ? 0 : s + 1];
        const uint32_t M = (uint32_t)((2ull << (15 + um)) - (1ull << (15 - um)));  // bytes 15-um .. 15+um
#pragma unroll
        for (int k = 0; k < 8; k++) {
            W0[k] = (((M >> (4 * k)) & 15u) * 0x00204081u) & 0x01010101u;
            W1[k] = (W0[k] * 0xFFu) & (0x03020100u + 0x04040404u * (uint32_t)k);
        }
    }
    const int ne = n_existing ? n_existing[f] : 0;
    float angle;
    {
        wic.store(P, s);
        // in flight during the IC sums (issued beside the IC window's loads instead, one
        // load latency fewer per workgroup: 5.68 vs 5.44-5.57 ms per step, r05/orient_early)
        wdesc.load(fblur, w, c, s);
        // IC_Angle (ORBextractor.cc:77-101): lane s takes the window rows 15 +- (s+1)
        // (lane 15 the centre row).  Per row, with I the 31 row bytes (32nd
        // weighted 0): S0 = sum of I over the disc (dot4 with the 0/1 weights),
        // S1 = sum of (u + 15) I (dot4 with the u + 15 weights); then
        // m01 += v (S0(+v) - S0(-v)), m10 += S1 - 15 S0.  Integer sums: the
        // moments equal the reference's exactly.
        const uint32_t o0 = (uint32_t)(uintptr_t)fimg + c - 15u * w - 15u;
        auto row_sums = [&](int r, uint32_t &s0, uint32_t &s1) {
            const uint32_t o = mad24((uint32_t)r, w, o0) & 15u;  // window start inside LDS row r
            const uint32_t *d = reinterpret_cast<const uint32_t *>(P + patch_row_swz((uint32_t)r) + (o & ~3u));
            uint32_t dw[9];
#pragma unroll
            for (int k = 0; k < 9; k++) dw[k] = d[k];
            s0 = 0u;
            s1 = 0u;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t q = __builtin_amdgcn_alignbyte(dw[k + 1], dw[k], o & 3u);
                s0 = __builtin_amdgcn_udot4(q, W0[k], s0, false);
                s1 = __builtin_amdgcn_udot4(q, W1[k], s1, false);
            }
        };
        const int v = s == 15 ? 0 : s + 1;
        uint32_t s0p, s1p, s0m = 0u, s1m = 0u;
        row_sums(15 + v, s0p, s1p);
        if (s < 15) row_sums(15 - v, s0m, s1m);
        int m01 = v * ((int)s0p - (int)s0m);
        int m10 = (int)(s1p + s1m) - 15 * (int)(s0p + s0m);
        m01 = row16_sum(m01);
        m10 = row16_sum(m10);
        angle = fast_atan2_deg((float)m01, (float)m10);
    }
    // computeOrbDescriptor (ORBextractor.cc:105-149) on the blurred level
    int4 pat[4];  // 16 pairs x (x0, y0, x1, y1) FP8 (read after the IC pass: fewer live registers there)
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint4 u = s_const[s * 4 + q];
        pat[q] = make_int4((int)u.x, (int)u.y, (int)u.z, (int)u.w);
    }
    wave_lds_order();  // IC taps read before the window is replaced
    wdesc.store(P, s);
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float ca, sb;
    glibc_sincosf(angle * factorPI, sb, ca);  // the reference's std::cos(float) / std::sin(float) = glibc cosf / sinf
    // tap (dy, dx) at P + 52 r + o(r) + 18 + dx with r = 18 + dy, o(r) = (o0 + r w) & 15.
    // GET_VALUE's rotation in packed fp32 (the same IEEE products and fused sums
    // as the reference's -O3 -march=native build, oracle/orb.c ygzo_orb_descriptor);
    // cvRound as + 2^23 + K: the sum stays in [2^23, 2^24) (ulp 1) for |v| <= 18.4,
    // rounds half to even with an even K, and its bit pattern carries the integer:
    //   yb = bits(y + 2^23 + 64)     low bits 46 + r
    //   xb = bits(x + 2^23 + P + 64)
    //   o(r) = ((yb & 15) (w & 15) + c0) & 15 with c0 = (o0 - 46 w) & 15
    //   address = mad_u24(yb, 52, xb) + o(r) - kFix  (the low 24 bits of yb are 46 + r: bit 23
    //   of 2^23's exponent field is 0)
    const uint32_t o0 = (uint32_t)(uintptr_t)fblur + c - 18u * w - 18u;
    const uint32_t w16 = w & 15u;
    const uint32_t Pa = (uint32_t)(uintptr_t)(lds_u8 *)P;
    const uint32_t c0 = (o0 - 46u * w16) & 15u;
    const f32x2 magic = {__uint_as_float(kMagicBits + 64u), __uint_as_float(kMagicBits + Pa + 64u)};
    constexpr uint32_t kFix = kMagicBits + 46u * (uint32_t)kPatchStride + 64u - 18u;
    const f32x2 rot_a = {sb, ca}, rot_b = {ca, -sb};
    // rows whose width is a multiple of 16 (C2 level 0) start at the same offset o(r) = c0
    // in every LDS row: the tap address is then one mad24 and one add (a wave-uniform choice)
    const uint32_t cfix = c0 - kFix;
    auto descriptor = [&](auto aligned_rows) -> uint32_t {
        auto tap = [&](float px, float py) -> uint32_t {
            const f32x2 m = (f32x2){py, py} * rot_b;
            const f32x2 yx = __builtin_elementwise_fma((f32x2){px, px}, rot_a, m) + magic;
            const uint32_t yb = __float_as_uint(yx.x), xb = __float_as_uint(yx.y);
            const uint32_t a = mad24(yb, (uint32_t)kPatchStride, xb);
            if constexpr (decltype(aligned_rows)::value) {
                return (uint32_t)*(const lds_u8 *)(uintptr_t)(a + cfix);
            } else {
                const uint32_t o = (yb & 15u) * w16 + c0;
                return (uint32_t)*(const lds_u8 *)(uintptr_t)(a + (o & 15u) - kFix);
            }
        };
        uint32_t b = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int4 Pq = pat[q];
            uint32_t wd[4] = {(uint32_t)Pq.x, (uint32_t)Pq.y, (uint32_t)Pq.z, (uint32_t)Pq.w};
            // opaque per path: the pattern's conversions are not hoisted above the path choice
            // (both paths' 64 converted coordinates would be live there and spill)
            asm volatile("" : "+v"(wd[0]), "+v"(wd[1]), "+v"(wd[2]), "+v"(wd[3]));
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const f32x2 p0 = __builtin_amdgcn_cvt_pk_f32_fp8((int)wd[k], false);  // (x0, y0)
                const f32x2 p1 = __builtin_amdgcn_cvt_pk_f32_fp8((int)wd[k], true);   // (x1, y1)
                const uint32_t t0 = tap(p0.x, p0.y), t1 = tap(p1.x, p1.y);
                b |= (uint32_t)(t0 < t1) << (q * 4 + k);
            }
        }
        return b;
    };
    // (orientation stage 0.441 -> 0.435 ms / 1,024 frames, profiles/r05/orient_sincos_taps)
    const uint32_t bits = __ballot(w16 != 0u) == 0ull ? descriptor(std::true_type{}) : descriptor(std::false_type{});
    const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)bits, 0xB1, 0xF, 0xF, false);
    const int row = ne + idx;
    if ((s & 1) == 0)
        reinterpret_cast<uint32_t *>(desc + ((size_t)f * row_cap + row) * 32)[s >> 1] = bits | (other << 16);
    if (s == 0) kps[(size_t)f * row_cap + row].angle = angle;  // the rest of the row: k_emit_kps
}

// Existing keypoints (Frame::mvKeys of a direct-tracked frame): descriptor on
// the blurred level of their octave at pt * invScale (ORBextractor.cc:1088-1099).
// recompute_angle: DSO/FAST modes reset the angle by IC_Angle (:1383-1385).
__global__ __launch_bounds__(256) void k_desc_existing(const uint8_t *__restrict__ pyr,
                                                       const uint8_t *__restrict__ blur,
                                                       const Plan *__restrict__ plan,
                                                       ygzfe_kp *__restrict__ kps, uint8_t *__restrict__ desc,
                                                       int n, int recompute_angle) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= n) return;
    ygzfe_kp kp = kps[i];
    const int oc = clampi(kp.octave, 0, plan->nlevels - 1);
    const LevelDesc &L = plan->lv[oc];
    const float tx = kp.x * L.inv_scale, ty = kp.y * L.inv_scale;
    const int cx = cv_round(tx), cy = cv_round(ty);
    float angle = kp.angle;
    if (recompute_angle) angle = ic_angle_wave(pyr + L.off, L.w, L.h, cx, cy, plan->umax);
    orb_desc_wave(blur + L.off, L.w, L.h, cx, cy, angle, desc + (size_t)i * 32);
    if (lane == 0 && recompute_angle) kps[i].angle = angle;
}

// ---------------------------------------------------------------------------
// host launchers

// compute units of the current device (persistent grids are sized from it)
static int device_cus() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        return 256;
    return n;
}

// Arithmetic guard, run once per device before the first call (api.cpp
// ensure_device): the two bit-level tricks the kernels rest on, evaluated with this
// translation unit's own flags and helpers, so a build or mode change that breaks them
// (fast-math, f16 denormal flushing, a rounding mode other than nearest-even) fails
// every call instead of shifting corners or descriptor bits silently.
//   fails[0]: k_fast_cells' f16 ordering — bytes 0..255 as f16 bit patterns (+0 and
//             subnormals) must min / max exactly like the integers (hmin3 / hmax3);
//   fails[1]: k_orient_desc's cvRound — bits(v + 2^23 + 64) - bits(2^23 + 64) must be
//             round-half-even(v) over the taps' range |v| <= 18.4, incl. every .5.
__global__ __launch_bounds__(256) void k_arith_guard(uint32_t *__restrict__ fails) {
    const int a = blockIdx.x, b = threadIdx.x;
    const h16x2 ha = as_h16x2((uint32_t)a | ((uint32_t)b << 16)), hb = as_h16x2((uint32_t)b | ((uint32_t)a << 16));
    const uint32_t mn = as_u32(hmin3(ha, hb, hb)), mx = as_u32(hmax3(ha, ha, hb));
    const uint32_t lo = (uint32_t)min(a, b), hi = (uint32_t)max(a, b);
    if (mn != (lo | (lo << 16)) || mx != (hi | (hi << 16))) atomicAdd(&fails[0], 1u);
    if (a < 160) {  // v = (a - 80) / 4 + b / 1024: quarters, halves, and values between
        const float v = (float)(a - 80) * 0.25f + (float)b * (1.0f / 1024.0f);
        const float magic = __uint_as_float(kMagicBits + 64u);
        const int got = (int)(__float_as_uint(v + magic) - (kMagicBits + 64u));
        if (got != (int)__builtin_rintf(v)) atomicAdd(&fails[1], 1u);
    }
}

hipError_t run_arith_guard(uint32_t host_fails[2]) {
    uint32_t *d = nullptr;
    hipError_t e = hipMalloc(&d, 2 * sizeof(uint32_t));
    if (e != hipSuccess) return e;
    if ((e = hipMemset(d, 0, 2 * sizeof(uint32_t))) == hipSuccess) {
        hipLaunchKernelGGL(k_arith_guard, dim3(256), dim3(256), 0, 0, d);
        if ((e = hipGetLastError()) == hipSuccess)
            e = hipMemcpy(host_fails, d, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost);
    }
    (void)hipFree(d);
    return e;
}

hipError_t upload_pattern(const int *pat) {
    int8_t p8[1024];
    uint8_t f8[1024];
    for (int i = 0; i < 1024; i++) {
        p8[i] = (int8_t)pat[i];
        // OCP E4M3: sign, 4 exponent bits (bias 7), 3 mantissa bits; exact for |v| <= 16
        const int v = pat[i], a = v < 0 ? -v : v;
        if (a > 16) return hipErrorInvalidValue;
        int e = 0;
        while ((2 << e) <= a) e++;
        f8[i] = a == 0 ? 0 : (uint8_t)((v < 0 ? 0x80 : 0) | ((e + 7) << 3) | (((a << 3) >> e) & 7));
    }
    hipError_t err = hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), p8, sizeof(p8));
    if (err != hipSuccess) return err;
    return hipMemcpyToSymbol(HIP_SYMBOL(c_pattern_f8), f8, sizeof(f8));
}

hipError_t launch_pyramid(uint8_t *pyr, uint32_t pitch, const Plan &hp, const Plan *dp, const int *dtabs,
                          int nframes, hipStream_t st) {
    // levels 1..K exact x2 INTER_AREA (every C2 level): one fused pass
    int K = 0;
    while (K + 1 < hp.nlevels && K < 3 && hp.lv[K + 1].resize_mode == 1) K++;
    if (K > 0) {
        const int n = hp.lv[K].w * hp.lv[K].h;
        dim3 grid((n + 255) / 256, nframes);
        if (K == 3) hipLaunchKernelGGL(k_pyramid_area_chain<3>, grid, dim3(256), 0, st, pyr, pitch, dp);
        else if (K == 2) hipLaunchKernelGGL(k_pyramid_area_chain<2>, grid, dim3(256), 0, st, pyr, pitch, dp);
        else hipLaunchKernelGGL(k_pyramid_area_chain<1>, grid, dim3(256), 0, st, pyr, pitch, dp);
    }
    // a batch whose remaining levels are all INTER_LINEAR: one launch, a workgroup per
    // frame (a handful of frames keep the per-level launches, which spread each
    // level over the whole GPU)
    bool all_linear = K + 1 < hp.nlevels;
    for (int l = K + 1; l < hp.nlevels; l++)  // (four pixels span at most 16 source bytes up to 1.5 x)
        all_linear = all_linear && hp.lv[l].resize_mode == 2 && 2 * hp.lv[l - 1].w <= 3 * hp.lv[l].w &&
                     hp.lv[l].w <= 2048 && hp.lv[l].h <= 2048;
    if (all_linear && nframes >= 64) {
        hipLaunchKernelGGL(k_pyramid_linear_chain, dim3(nframes), dim3(1024), 0, st, pyr, pitch, dp, dtabs, K + 1);
        return hipGetLastError();
    }
    for (int l = K + 1; l < hp.nlevels; l++) {
        const LevelDesc &D = hp.lv[l];
        dim3 grid((D.w + 63) / 64, (D.h + 3) / 4, nframes);
        if (D.resize_mode == 1)
            hipLaunchKernelGGL(k_resize_area2, grid, dim3(256), 0, st, pyr, pitch, dp, l);
        else
            hipLaunchKernelGGL(k_resize_linear, grid, dim3(256), 0, st, pyr, pitch, dp, dtabs, l);
    }
    return hipGetLastError();
}

hipError_t launch_blur(const uint8_t *pyr, uint8_t *blur, uint32_t pitch, const Plan &hp, const Plan *dp,
                       int nframes, hipStream_t st) {
    hipLaunchKernelGGL(k_blur7<false>, dim3((hp.blur_tiles + 3) / 4, nframes), dim3(256), 0, st,
                       const_cast<uint8_t *>(pyr), blur, pitch, dp, 0, hp.blur_tiles, 0);
    return hipGetLastError();
}

// Levels 1..K of an all-area pyramid (every level >= 1 an exact x2 INTER_AREA, K <= 3)
// whose level 0 takes the aligned blur path: 0 when the plan does not qualify.
int pyramid_fusable(const Plan &hp) {
    const int K = hp.nlevels - 1;
    if (K < 1 || K > 3 || hp.lv[0].w < 16 || (hp.lv[0].w & 3) || kBlurRows % 8) return 0;
    for (int l = 1; l <= K; l++)
        if (hp.lv[l].resize_mode != 1) return 0;
    return K;
}

// The batch path's pyramid + level-0 blur in one pass (k_blur7 fused mode), then the
// blur of levels >= 1 on `st_rest` after it (caller orders st_rest after st_l0)
hipError_t launch_pyramid_blur0(uint8_t *pyr, uint8_t *blur, uint32_t pitch, const Plan &hp, const Plan *dp,
                                int nframes, hipStream_t st_l0) {
    const int K = pyramid_fusable(hp), n0 = hp.lv[0].blur_tiles_x * hp.lv[0].blur_tiles_y;
    hipLaunchKernelGGL(k_blur7<true>, dim3((n0 + 3) / 4, nframes), dim3(256), 0, st_l0, pyr, blur, pitch, dp, 0, n0, K);
    return hipGetLastError();
}
hipError_t launch_blur_rest(const uint8_t *pyr, uint8_t *blur, uint32_t pitch, const Plan &hp, const Plan *dp,
                            int nframes, hipStream_t st) {
    const int n0 = hp.lv[0].blur_tiles_x * hp.lv[0].blur_tiles_y, n = hp.blur_tiles - n0;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_blur7<false>, dim3((n + 3) / 4, nframes), dim3(256), 0, st, const_cast<uint8_t *>(pyr), blur,
                       pitch, dp, n0, hp.blur_tiles, 0);
    return hipGetLastError();
}

// the (S, R) instance of the per-cell slice for ROIs up to rw x rh
static void fast_shape_pick(int rw, int rh, int &S, int &R) {
    fast_slice_shape(rw, rh, S, R);
    if (S == 36 && R > 40) S = 40;
    if (!((S == 36 && R == 40) || (S == 40 && R <= 56))) S = R = std::max(S, R);
}
#define YGZ_FAST_SHAPES(X) X(36, 40) X(40, 40) X(40, 48) X(40, 56) X(48, 48) X(56, 56) X(64, 64) X(72, 72)

hipError_t launch_fast(const uint8_t *pyr, uint32_t pitch, const Plan &hp, const Plan *dp, const CellDesc *dcells,
                       uint32_t *cellbuf, int *cellcnt, int nframes, hipStream_t st0, const hipStream_t *lvl_streams,
                       int n_lvl_streams) {
    if (hp.ncells == 0) return hipSuccess;
    // one launch per level: the level's ROI shape sizes the LDS slices
    for (int l = 0; l < hp.nlevels; l++) {
        const LevelDesc &L = hp.lv[l];
        if (L.ncells == 0) continue;
        int S, R;
        fast_shape_pick(L.fast_rw, L.fast_rh, S, R);
        // level 0 on the caller's stream, the others spread over the given side streams
        const hipStream_t st = (l == 0 || !lvl_streams || n_lvl_streams <= 0) ? st0
                                                                                : lvl_streams[(l - 1) % n_lvl_streams];
        // Optional LDS floor per workgroup (a floor of 23,000 B caps the small-ROI levels at 7
        // workgroups/CU instead of 8, leaving slots to the other chunk's stages).  Round 5 under
        // the overlap schedule: floor 0 471k fps, 23000 485k, 26800 482k, 32000 463k.  Round 6
        // under the pipe schedule with this round's FAST: floor 0 runs FAST 1.5 % faster (7.00-7.09
        // vs 7.12-7.20 ms per step) and the headline within noise (+0.35 %), so no floor
        // (profiles/r06/lds_floor/).
#ifndef YGZ_FAST_LDS_MIN
#define YGZ_FAST_LDS_MIN 0
#endif
        const size_t lds = std::max<size_t>(kFastWaves * (size_t)fast_slice_bytes(S, R), YGZ_FAST_LDS_MIN);
        const dim3 grid((L.ncells + kFastWaves - 1) / kFastWaves, nframes);
#define YGZ_FAST(SS, RR)                                                                                        \
    if (S == SS && R == RR)                                                                                     \
        hipLaunchKernelGGL((k_fast_cells<SS, RR>), grid, dim3(64 * kFastWaves), lds, st, pyr, pitch, dp, dcells, \
                           cellbuf, cellcnt, L.cell_begin, L.cell_begin + L.ncells, l, nullptr);
        YGZ_FAST_SHAPES(YGZ_FAST)
#undef YGZ_FAST
    }
    return hipGetLastError();
}

// Every level's cells in ONE launch (the single-frame path: one frame's cells fill
// the GPU anyway, and three dependent launches cost three dispatch gaps): the
// slices of the largest ROI of any level.
hipError_t launch_fast_merged(const uint8_t *pyr, uint32_t pitch, const Plan &hp, const Plan *dp,
                              const CellDesc *dcells, uint32_t *cellbuf, int *cellcnt, int nframes, hipStream_t st,
                              int *clear_flag) {
    if (hp.ncells == 0) return hipSuccess;
    int rw = 0, rh = 0;
    for (int l = 0; l < hp.nlevels; l++) {
        if (hp.lv[l].ncells == 0) continue;
        rw = std::max(rw, hp.lv[l].fast_rw);
        rh = std::max(rh, hp.lv[l].fast_rh);
    }
    int S, R;
    fast_shape_pick(rw, rh, S, R);
    const size_t lds = kFastWaves * (size_t)fast_slice_bytes(S, R);
    const dim3 grid((hp.ncells + kFastWaves - 1) / kFastWaves, nframes);
#define YGZ_FAST(SS, RR)                                                                                        \
    if (S == SS && R == RR)                                                                                     \
        hipLaunchKernelGGL((k_fast_cells<SS, RR>), grid, dim3(64 * kFastWaves), lds, st, pyr, pitch, dp, dcells, \
                           cellbuf, cellcnt, 0, hp.ncells, -1, clear_flag);
    YGZ_FAST_SHAPES(YGZ_FAST)
#undef YGZ_FAST
    return hipGetLastError();
}

// node pool per level: budget + 4 nIni + 16 (plan.cpp), rounded up to a power of two
static int octree_nc(const LevelDesc &L) {
    const int need = L.budget + 4 * L.n_ini + 16;
    return need <= 256 ? 256 : need <= 512 ? 512 : need <= 1024 ? 1024 : 2048;
}

// threads per workgroup of the larger octree classes: the workgroup holds its
// LDS (two per CU) through a chain of barrier-separated passes, so more waves
// per workgroup shorten every pass's strided loops over keys and nodes
#ifndef YGZ_OCT_THREADS
#define YGZ_OCT_THREADS 512
#endif
constexpr int kOctThreads = YGZ_OCT_THREADS;
#ifndef YGZ_OCT_LIST_THREADS
#define YGZ_OCT_LIST_THREADS 256  // k_octree_list workgroup of the batched classes
#endif
constexpr int kOctListThreads = YGZ_OCT_LIST_THREADS;

// launch groups: runs of consecutive levels with one node-pool class (the class
// sequence can go back up, e.g. when the last level's remainder budget or a flipped
// n_ini moves it, so a plan may hold up to nlevels groups)
static int octree_groups(const Plan &hp) {
    int G = 0;
    for (int l = 0; l < hp.nlevels; G++) {
        const int nc = octree_nc(hp.lv[l]);
        while (l < hp.nlevels && octree_nc(hp.lv[l]) == nc) l++;
    }
    return G;
}
// queue words: 8 counters per launch group g at octq[8 g ..] (list i: count 2i, taken
// 2i + 1) in a head of max(64, 8 G) words; then 3 lists per group at
// octq[head + (3 g + i) T], T = frames x levels; then the per-task sort headers at
// octq[head + 3 G T + f levels + l]
static size_t oct_head(int G) { return (size_t)std::max(64, 8 * G); }
size_t octree_queue_ints(const Plan &hp, int nframes) {
    const int G = octree_groups(hp);
    return oct_head(G) + (size_t)(3 * G + 1) * nframes * hp.nlevels;
}

static hipError_t launch_octree_levels(int nc, const Plan *dp, const uint32_t *cellbuf, const int *cellcnt,
                                       uint32_t *candA, uint32_t *candB, uint32_t *sel, int *selcnt, int *err,
                                       int *octq, int g, int G, int T, int nframes, int l0, int nl,
                                       hipStream_t st, bool wide) {
    dim3 grid(nframes, nl);
    // sort stage 0: one workgroup per task, sized for the class's usual candidate count
    // (wide = one frame: 8,192 keys at once); stage 1: 4,096 keys in LDS (512 threads);
    // stage 2: 8,192 keys (1,024 threads, one workgroup per CU); stage 3: the
    // global-scratch form (sort + list); then the list phase of every LDS-sorted task
    int *cq = octq + 8 * g;
    int *lists = octq + oct_head(G) + (size_t)3 * g * T;
    int *hdr = octq + oct_head(G) + (size_t)3 * G * T;
    const OctQueue q0{nullptr, nullptr, nullptr, cq + 0, lists};
    const OctQueue q1{cq + 0, cq + 1, lists, cq + 2, lists + T};
    const OctQueue q2{cq + 2, cq + 3, lists + T, cq + 4, lists + 2 * T};
    const OctQueue q3{cq + 4, cq + 5, lists + 2 * T, nullptr, nullptr};
    const int tasks = nframes * nl;
#define YGZ_OCT_SORT0(NC, NK, NT)                                                                                 \
    hipLaunchKernelGGL((k_octree_sort<NC, NK, NT>), grid, dim3(NT), 0, st, dp, cellbuf, cellcnt, candA, candB, hdr, \
                       l0, q0)
#define YGZ_OCT_REST(NC, Q1)                                                                                      \
    do {                                                                                                          \
        if (Q1)                                                                                                   \
            hipLaunchKernelGGL((k_octree_sort_q<NC, 4096, 512>), dim3(std::min(tasks, 512)), dim3(512), 0, st, dp, \
                               cellbuf, cellcnt, candA, candB, hdr, q1);                                          \
        hipLaunchKernelGGL((k_octree_sort_q<NC, 8192, 1024>), dim3(std::min(tasks, NC >= 1024 ? 256 : 64)),      \
                           dim3(1024), 0, st, dp,                                                                 \
                           cellbuf, cellcnt, candA, candB, hdr, Q1 ? q2 : q1);                                    \
        hipLaunchKernelGGL((k_octree_global<NC, 512>), dim3(std::min(tasks, 64)), dim3(512), 0, st, dp, cellbuf,  \
                           cellcnt, candA, candB, sel, selcnt, err, Q1 ? q3 : q2);                                \
        hipLaunchKernelGGL((k_octree_list<NC, kOctListThreads>), grid, dim3(kOctListThreads), 0, st, dp, candA,   \
                           candB, hdr, sel, selcnt, err, l0);                                                     \
    } while (0)
    if (wide && nc <= 1024) {
        YGZ_OCT_SORT0(1024, 8192, 1024);
        // stage 0 overflows to list 0, which the global stage reads as its input
        hipLaunchKernelGGL((k_octree_global<1024, 512>), dim3(std::min(tasks, 256)), dim3(512), 0, st, dp, cellbuf,
                           cellcnt, candA, candB, sel, selcnt, err, q1);
        hipLaunchKernelGGL((k_octree_list<1024, 1024>), grid, dim3(1024), 0, st, dp, candA, candB, hdr, sel, selcnt,
                           err, l0);
    } else if (nc <= 256) {
        YGZ_OCT_SORT0(256, 1024, 256);
        YGZ_OCT_REST(256, true);
    } else if (nc <= 512) {
        YGZ_OCT_SORT0(512, 4096, 512);
        YGZ_OCT_REST(512, false);
    } else if (nc <= 1024) {
        YGZ_OCT_SORT0(1024, 4096, 512);
        YGZ_OCT_REST(1024, false);
    } else {
        YGZ_OCT_SORT0(2048, 4096, 512);
        YGZ_OCT_REST(2048, false);
    }
#undef YGZ_OCT_SORT0
#undef YGZ_OCT_REST
    return hipGetLastError();
}

// Levels grouped by node-pool class, each group one launch; groups after the
// first run on the side streams (fork after, join before the caller's next work).
hipError_t launch_octree(const Plan &hp, const Plan *dp, const uint32_t *cellbuf, const int *cellcnt,
                         uint32_t *candA, uint32_t *candB, uint32_t *sel, int *selcnt, int *err, int *octq,
                         int nframes, hipStream_t st, const hipStream_t *side, int nside, hipEvent_t fork,
                         const hipEvent_t *join, bool wide) {
    int l = 0, g = 0;
    const int G = octree_groups(hp);
    YGZ_HIPR(hipMemsetAsync(octq, 0, oct_head(G) * sizeof(int), st));  // queue counters
    if (wide) {  // one frame: every level in one launch chain when the node pools allow
        int ncmax = 0;
        for (int k = 0; k < hp.nlevels; k++) ncmax = std::max(ncmax, octree_nc(hp.lv[k]));
        if (ncmax <= 1024)
            return launch_octree_levels(1024, dp, cellbuf, cellcnt, candA, candB, sel, selcnt, err, octq, 0, G,
                                        nframes * hp.nlevels, nframes, 0, hp.nlevels, st, true);
    }
    if (side && nside > 0) YGZ_HIPR(hipEventRecord(fork, st));  // before the first group: the groups are independent
    while (l < hp.nlevels) {
        const int nc = octree_nc(hp.lv[l]);
        int e = l + 1;
        while (e < hp.nlevels && octree_nc(hp.lv[e]) == nc) e++;
        hipStream_t s = st;
        if (g > 0 && g - 1 < nside && side) {
            s = side[g - 1];
            YGZ_HIPR(hipStreamWaitEvent(s, fork, 0));
        }
        YGZ_HIPR(launch_octree_levels(nc, dp, cellbuf, cellcnt, candA, candB, sel, selcnt, err, octq, g, G,
                                      nframes * hp.nlevels, nframes, l, e - l, s, wide));
        if (s != st) YGZ_HIPR(hipEventRecord(join[g - 1], s));
        l = e;
        g++;
    }
    for (int k = 1; k < g && k - 1 < nside && side; k++) YGZ_HIPR(hipStreamWaitEvent(st, join[k - 1], 0));
    return hipSuccess;
}

hipError_t launch_orient_desc(const uint8_t *pyr, const uint8_t *blur, uint32_t pitch, const Plan &hp,
                              const Plan *dp, const uint2 *ojobs, const int *n_existing, ygzfe_kp *kps,
                              uint8_t *desc, int row_cap, int nframes, hipStream_t st) {
    const int max_new = hp.sel_total;
    hipLaunchKernelGGL(k_orient_desc, dim3((max_new + 15) / 16, nframes), dim3(256), 0, st, pyr, blur, pitch, dp,
                       ojobs, n_existing, kps, desc, row_cap);
    return hipGetLastError();
}

hipError_t launch_emit_kps(const Plan &hp, const Plan *dp, const uint32_t *sel, const int *selcnt,
                           const int *n_existing, ygzfe_kp *kps, int *counts, int row_cap, uint2 *ojobs, int nframes,
                           hipStream_t st) {
    hipLaunchKernelGGL(k_emit_kps, dim3((hp.sel_total + 255) / 256 + 1, nframes), dim3(256), 0, st, dp, sel, selcnt,
                       n_existing, kps, counts, row_cap, ojobs);
    return hipGetLastError();
}

hipError_t launch_desc_existing(const uint8_t *pyr, const uint8_t *blur, const Plan *dp, ygzfe_kp *kps,
                                uint8_t *desc, int n, int recompute_angle, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_desc_existing, dim3((n + 3) / 4), dim3(256), 0, st, pyr, blur, dp, kps, desc, n,
                       recompute_angle);
    return hipGetLastError();
}

}  // namespace ygzfe
