// extract.hip — ORB extraction kernels for gfx950 (ORBSLAM_KEYPOINT mode).
//
// Stage            reference                               kernel
// pyramid          ORBextractor.cc:1129-1150               k_resize_area2 / k_resize_linear
// blur 7x7 s=2     ORBextractor.cc:1079-1084               k_blur7
// FAST-9 per cell  ORBextractor.cc:747-781 (+cv::FAST)     k_fast_cells
// octree           ORBextractor.cc:533-723, 783-798        k_octree<NODE_CAP>
// angle + rBRIEF   ORBextractor.cc:77-149, 1101-1125       k_orient_desc / k_desc_existing
//
// Everything is batched over frames (grid.z / grid.y = frame) so one launch per
// stage serves a whole resident batch.  Bit-exactness with oracle/ is the
// contract: integer paths are exact, float expressions follow the reference's
// evaluation order and the library is built with -ffp-contract=off.
#include "common.hpp"

namespace ygzfe {

__constant__ int8_t c_pattern[1024];

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

__global__ __launch_bounds__(256) void k_blur7(const uint8_t *__restrict__ pyr,
                                               uint8_t *__restrict__ blur, uint32_t pitch,
                                               const Plan *__restrict__ plan) {
    constexpr int TW = 64, TH = 16, SW = TW + 6, SH = TH + 6;
    __shared__ uint8_t s_src[SH * SW];
    __shared__ int s_row[SH * TW];
    const int f = blockIdx.y;
    int tile = blockIdx.x, l = 0;
    while (l + 1 < plan->nlevels && tile >= plan->lv[l + 1].blur_tile_begin) l++;
    const LevelDesc &L = plan->lv[l];
    tile -= L.blur_tile_begin;
    const int tx0 = (tile % L.blur_tiles_x) * TW, ty0 = (tile / L.blur_tiles_x) * TH;
    const uint8_t *src = pyr + (size_t)f * pitch + L.off;
    for (int i = threadIdx.x; i < SH * SW; i += 256) {
        const int yy = reflect101(ty0 + i / SW - 3, L.h), xx = reflect101(tx0 + i % SW - 3, L.w);
        s_src[i] = src[(size_t)yy * L.w + xx];
    }
    __syncthreads();
    const int k0 = 18, k1 = 34;  // CV4 [18,34,48,56,48,34,18] / CV3 [18,34,49,55,49,34,18]
    const int k2 = plan->blur_variant == YGZFE_BLUR_CV3 ? 49 : 48;
    const int k3 = plan->blur_variant == YGZFE_BLUR_CV3 ? 55 : 56;
    for (int i = threadIdx.x; i < SH * TW; i += 256) {
        const uint8_t *p = s_src + (i / TW) * SW + (i % TW);
        s_row[i] = k0 * (p[0] + p[6]) + k1 * (p[1] + p[5]) + k2 * (p[2] + p[4]) + k3 * p[3];
    }
    __syncthreads();
    uint8_t *dst = blur + (size_t)f * pitch + L.off;
    for (int i = threadIdx.x; i < TH * TW; i += 256) {
        const int ry = i / TW, rx = i % TW;
        const int x = tx0 + rx, y = ty0 + ry;
        if (x >= L.w || y >= L.h) continue;
        const int *c = s_row + ry * TW + rx;
        const int acc = k0 * (c[0] + c[6 * TW]) + k1 * (c[TW] + c[5 * TW]) + k2 * (c[2 * TW] + c[4 * TW]) +
                        k3 * c[3 * TW];
        dst[(size_t)y * L.w + x] = (uint8_t)clampi((acc + 32768) >> 16, 0, 255);
    }
}

// ---------------------------------------------------------------------------
// FAST-9/16 + cornerScore<16> + 3x3 non-max suppression inside one cell ROI
// (ORBextractor.cc:747-781).  One 256-thread workgroup per (cell, frame).

__device__ __forceinline__ uint32_t run9(uint32_t m16) {
    uint32_t x = m16 | (m16 << 16);
    uint32_t y = x & (x >> 1);   // runs of 2
    y &= y >> 2;                 // 4
    y &= y >> 4;                 // 8
    y &= x >> 8;                 // 9
    return y & 0xFFFFu;
}

// ring offsets in the ROI tile (stride kMaxRoi)
__device__ __forceinline__ void ring_vals(const uint8_t *p, int d[16]) {
    constexpr int S = kMaxRoi;
    d[0] = p[3 * S];       d[1] = p[1 + 3 * S];  d[2] = p[2 + 2 * S];  d[3] = p[3 + S];
    d[4] = p[3];           d[5] = p[3 - S];      d[6] = p[2 - 2 * S];  d[7] = p[1 - 3 * S];
    d[8] = p[-3 * S];      d[9] = p[-1 - 3 * S]; d[10] = p[-2 - 2 * S]; d[11] = p[-3 - S];
    d[12] = p[-3];         d[13] = p[-3 + S];    d[14] = p[-2 + 2 * S]; d[15] = p[-1 + 3 * S];
}

// FAST_t segment test + cornerScore<16> closed form:
// score = max(t, max_arc9 min(v - r), max_arc9 min(r - v)) - 1 ; -1 if not a corner.
__device__ __forceinline__ int fast9_score(const uint8_t *p, int t) {
    int d[16];
    ring_vals(p, d);
    const int v = p[0];
    uint32_t dark = 0, bright = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        dark |= (uint32_t)(d[k] < v - t) << k;
        bright |= (uint32_t)(d[k] > v + t) << k;
    }
    if (!run9(dark) && !run9(bright)) return -1;
    int m2[16], best = t;
#pragma unroll
    for (int k = 0; k < 16; k++) m2[k] = min(v - d[k], v - d[(k + 1) & 15]);
    int m4[16];
#pragma unroll
    for (int k = 0; k < 16; k++) m4[k] = min(m2[k], m2[(k + 2) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int m9 = min(min(m4[k], m4[(k + 4) & 15]), v - d[(k + 8) & 15]);
        best = max(best, m9);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) m2[k] = min(d[k] - v, d[(k + 1) & 15] - v);
#pragma unroll
    for (int k = 0; k < 16; k++) m4[k] = min(m2[k], m2[(k + 2) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int m9 = min(min(m4[k], m4[(k + 4) & 15]), d[(k + 8) & 15] - v);
        best = max(best, m9);
    }
    return best - 1;
}

__global__ __launch_bounds__(256) void k_fast_cells(const uint8_t *__restrict__ pyr, uint32_t pitch,
                                                    const Plan *__restrict__ plan,
                                                    const CellDesc *__restrict__ cells,
                                                    uint32_t *__restrict__ cellbuf,
                                                    int *__restrict__ cellcnt) {
    constexpr int S = kMaxRoi;
    __shared__ uint8_t s_img[S * S];
    __shared__ uint8_t s_sc[S * S];
    __shared__ int s_scan[256];
    const int c = blockIdx.x, f = blockIdx.y;
    const CellDesc cd = cells[c];
    const LevelDesc &L = plan->lv[cd.level];
    const uint8_t *src = pyr + (size_t)f * pitch + L.off + (size_t)cd.y0 * L.w + cd.x0;
    const int rw = cd.rw, rh = cd.rh;
    for (int i = threadIdx.x; i < rw * rh; i += 256) {
        const int y = i / rw, x = i - y * rw;
        s_img[y * S + x] = src[(size_t)y * L.w + x];
    }
    const int iw = rw - 6, ih = rh - 6, n = iw > 0 && ih > 0 ? iw * ih : 0;
    const int per = (n + 255) / 256;
    uint32_t *out = cellbuf + ((size_t)f * plan->ncells + c) * plan->cell_cap;
    int total = 0;
    for (int pass = 0; pass < 2; pass++) {
        const int th = pass == 0 ? plan->ini_th : plan->min_th;
        for (int i = threadIdx.x; i < S * S; i += 256) s_sc[i] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += 256) {
            const int y = 3 + i / iw, x = 3 + i % iw;
            const int s = fast9_score(s_img + y * S + x, th);
            if (s >= 0) s_sc[y * S + x] = (uint8_t)s;
        }
        __syncthreads();
        // NMS + order-preserving compaction: thread t owns interior pixels [t*per, (t+1)*per)
        const int b = threadIdx.x * per, e = min(n, b + per);
        int cnt = 0;
        for (int i = b; i < e; i++) {
            const int y = 3 + i / iw, x = 3 + i % iw;
            const uint8_t *r = s_sc + y * S + x;
            const int s = r[0];
            cnt += s > 0 && s > r[-1] && s > r[1] && s > r[-S - 1] && s > r[-S] && s > r[-S + 1] &&
                   s > r[S - 1] && s > r[S] && s > r[S + 1];
        }
        s_scan[threadIdx.x] = cnt;
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan
            const int v = threadIdx.x >= o ? s_scan[threadIdx.x - o] : 0;
            __syncthreads();
            s_scan[threadIdx.x] += v;
            __syncthreads();
        }
        total = s_scan[255];
        int pos = s_scan[threadIdx.x] - cnt;
        for (int i = b; i < e; i++) {
            const int y = 3 + i / iw, x = 3 + i % iw;
            const uint8_t *r = s_sc + y * S + x;
            const int s = r[0];
            if (s > 0 && s > r[-1] && s > r[1] && s > r[-S - 1] && s > r[-S] && s > r[-S + 1] &&
                s > r[S - 1] && s > r[S] && s > r[S + 1]) {
                if (pos < plan->cell_cap) out[pos] = pack_key(x + cd.offx, y + cd.offy, s);
                pos++;
            }
        }
        __syncthreads();
        if (total > 0) break;
    }
    if (threadIdx.x == 0) cellcnt[(size_t)f * plan->ncells + c] = min(total, plan->cell_cap);
}

// ---------------------------------------------------------------------------
// Octree distribution (DistributeOctTree, ORBextractor.cc:533-723), one wave per
// (level, frame).  The std::list is a node pool in LDS with prev/next links;
// every list operation is executed uniformly by the whole wave.  Node key sets
// are contiguous segments of a key array; DivideNode is a stable 4-way
// partition of the segment into the other buffer of a ping-pong pair
// (ballot + mbcnt ranks), so keys keep their candidate order and "first max
// response wins" is preserved.  The std::sort tie-break on node pointers is
// the node creation order (seq), as in oracle/orb.c.

constexpr uint16_t NIL = 0xFFFF;

template <int NODE_CAP>
struct OctShared {
    uint32_t x0y0[NODE_CAP], x1y1[NODE_CAP], beg[NODE_CAP], cnt[NODE_CAP], seq[NODE_CAP];
    uint16_t prev[NODE_CAP], next[NODE_CAP], freel[NODE_CAP];
    uint64_t vsp[NODE_CAP], vprev[NODE_CAP];
};

template <int NODE_CAP>
struct OctState {
    OctShared<NODE_CAP> *s;
    uint32_t *A, *B;
    int head, size, seq, free_top, nvsp;
    int overflow;

    __device__ int alloc() {
        if (free_top == 0) { overflow = 1; return 0; }
        return s->freel[--free_top];
    }
    __device__ void push_front(int id) {
        s->prev[id] = NIL;
        s->next[id] = (uint16_t)head;
        if (head != NIL) s->prev[head] = (uint16_t)id;
        head = id;
        size++;
    }
    __device__ int erase(int id) {
        const int p = s->prev[id], nx = s->next[id];
        if (p != NIL) s->next[p] = (uint16_t)nx; else head = nx;
        if (nx != NIL) s->prev[nx] = (uint16_t)p;
        size--;
        s->freel[free_top++] = (uint16_t)id;
        return nx;
    }
    __device__ void vsp_push(int id) {
        if (nvsp >= NODE_CAP) { overflow = 1; return; }
        s->vsp[nvsp++] = ((uint64_t)s->cnt[id] << 40) | ((uint64_t)s->seq[id] << 16) | (uint64_t)id;
    }

    // ExtractorNode::DivideNode + push_front of the non-empty children (n1..n4);
    // returns the number of children with more than one key.
    __device__ int divide(int pid, bool record) {
        const int lane = threadIdx.x;
        const uint32_t a = s->x0y0[pid], b = s->x1y1[pid];
        const int x0 = (int)(a & 0xFFFF), y0 = (int)(a >> 16), x1 = (int)(b & 0xFFFF), y1 = (int)(b >> 16);
        const uint32_t bg = s->beg[pid];
        const int flag = (int)(bg >> 31), beg = (int)(bg & 0x7FFFFFFF), n = (int)s->cnt[pid];
        const int halfX = (int)ceilf((float)(x1 - x0) / 2), halfY = (int)ceilf((float)(y1 - y0) / 2);
        const int mx = x0 + halfX, my = y0 + halfY;
        const uint32_t *src = flag ? B : A;
        uint32_t *dst = flag ? A : B;
        int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
        if (n <= 64) {
            const bool act = lane < n;
            const uint32_t k = act ? src[beg + lane] : 0u;
            const int x = key_x(k), y = key_y(k);
            const int q = x < mx ? (y < my ? 0 : 2) : (y < my ? 1 : 3);
            const uint64_t m0 = __ballot(act && q == 0), m1 = __ballot(act && q == 1);
            const uint64_t m2 = __ballot(act && q == 2), m3 = __ballot(act && q == 3);
            c0 = __popcll(m0); c1 = __popcll(m1); c2 = __popcll(m2); c3 = __popcll(m3);
            const uint64_t mq = q == 0 ? m0 : q == 1 ? m1 : q == 2 ? m2 : m3;
            const int base = q == 0 ? 0 : q == 1 ? c0 : q == 2 ? c0 + c1 : c0 + c1 + c2;
            if (act) dst[beg + base + popc_below(mq)] = k;
        } else {
            for (int i = 0; i < n; i += 64) {
                const bool act = i + lane < n;
                const uint32_t k = act ? src[beg + i + lane] : 0u;
                const int x = key_x(k), y = key_y(k);
                const int q = x < mx ? (y < my ? 0 : 2) : (y < my ? 1 : 3);
                c0 += __popcll(__ballot(act && q == 0));
                c1 += __popcll(__ballot(act && q == 1));
                c2 += __popcll(__ballot(act && q == 2));
            }
            c3 = n - c0 - c1 - c2;
            int r0 = 0, r1 = c0, r2 = c0 + c1, r3 = c0 + c1 + c2;
            for (int i = 0; i < n; i += 64) {
                const bool act = i + lane < n;
                const uint32_t k = act ? src[beg + i + lane] : 0u;
                const int x = key_x(k), y = key_y(k);
                const int q = x < mx ? (y < my ? 0 : 2) : (y < my ? 1 : 3);
                const uint64_t m0 = __ballot(act && q == 0), m1 = __ballot(act && q == 1);
                const uint64_t m2 = __ballot(act && q == 2), m3 = __ballot(act && q == 3);
                const uint64_t mq = q == 0 ? m0 : q == 1 ? m1 : q == 2 ? m2 : m3;
                const int base = q == 0 ? r0 : q == 1 ? r1 : q == 2 ? r2 : r3;
                if (act) dst[beg + base + popc_below(mq)] = k;
                r0 += __popcll(m0); r1 += __popcll(m1); r2 += __popcll(m2); r3 += __popcll(m3);
            }
        }
        __syncthreads();  // partition stores visible to the wave before later reads
        const int cc[4] = {c0, c1, c2, c3};
        const int bx0[4] = {x0, mx, x0, mx}, by0[4] = {y0, y0, my, my};
        const int bx1[4] = {mx, x1, mx, x1}, by1[4] = {my, my, y1, y1};
        int off = 0, expand = 0;
        for (int q = 0; q < 4; q++) {
            if (cc[q] > 0) {
                const int id = alloc();
                s->x0y0[id] = (uint32_t)bx0[q] | ((uint32_t)by0[q] << 16);
                s->x1y1[id] = (uint32_t)bx1[q] | ((uint32_t)by1[q] << 16);
                s->beg[id] = (uint32_t)(beg + off) | ((uint32_t)(flag ^ 1) << 31);
                s->cnt[id] = (uint32_t)cc[q];
                s->seq[id] = (uint32_t)seq++;
                push_front(id);
                if (cc[q] > 1) {
                    expand++;
                    if (record) vsp_push(id);
                }
            }
            off += cc[q];
        }
        return expand;
    }
};

// bitonic sort of s->vprev[0..n) ascending (padded to a power of two with ~0)
template <int NODE_CAP>
__device__ void wave_sort_u64(uint64_t *v, int n) {
    int p2 = 1;
    while (p2 < n) p2 <<= 1;
    for (int i = n + threadIdx.x; i < p2; i += 64) v[i] = ~0ull;
    __syncthreads();
    for (int k = 2; k <= p2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < p2; i += 64) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = v[i], b = v[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) { v[i] = b; v[ixj] = a; }
                }
            }
            __syncthreads();
        }
}

template <int NODE_CAP>
__global__ __launch_bounds__(64) void k_octree(const Plan *__restrict__ plan,
                                               const uint32_t *__restrict__ cellbuf,
                                               const int *__restrict__ cellcnt,
                                               uint32_t *__restrict__ candA, uint32_t *__restrict__ candB,
                                               uint32_t *__restrict__ sel, int *__restrict__ selcnt,
                                               int *__restrict__ err) {
    __shared__ OctShared<NODE_CAP> sh;
    const int l = blockIdx.x, f = blockIdx.y, lane = threadIdx.x;
    const LevelDesc &L = plan->lv[l];
    uint32_t *A = candA + (size_t)f * plan->cand_total + L.cand_off;
    uint32_t *B = candB + (size_t)f * plan->cand_total + L.cand_off;
    // 1. gather the level's candidates in cell order into B (vToDistributeKeys)
    int n = 0;
    for (int cb = 0; cb < L.ncells; cb += 64) {
        const int c = cb + lane;
        const int cnt = c < L.ncells ? cellcnt[(size_t)f * plan->ncells + L.cell_begin + c] : 0;
        int incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        const int tot = __shfl(incl, 63, 64);
        const int excl = incl - cnt;
        const int m = min(64, L.ncells - cb);
        for (int k = 0; k < m; k++) {
            const int cc = __shfl(cnt, k, 64), base = n + __shfl(excl, k, 64);
            const uint32_t *cs = cellbuf + ((size_t)f * plan->ncells + L.cell_begin + cb + k) * plan->cell_cap;
            for (int i = lane; i < cc; i += 64) B[base + i] = cs[i];
        }
        n += tot;
    }
    __syncthreads();
    // 2. initial nodes (push_back order) and stable assignment keys -> node (x / hX)
    OctState<NODE_CAP> st;
    st.s = &sh; st.A = A; st.B = B;
    st.head = NIL; st.size = 0; st.seq = 0; st.nvsp = 0; st.overflow = 0;
    for (int i = lane; i < NODE_CAP; i += 64) sh.freel[i] = (uint16_t)(NODE_CAP - 1 - i);
    st.free_top = NODE_CAP;
    __syncthreads();
    const int nIni = L.n_ini;
    const float hX = L.hX;
    const int H0 = L.max_by - kMinBorder;
    int ini_ids[8];
    int ini_cnt[8];
    for (int i = 0; i < nIni; i++) ini_cnt[i] = 0;
    for (int i = 0; i < n; i += 64) {
        const bool act = i + lane < n;
        const uint32_t k = act ? B[i + lane] : 0u;
        int idx = (int)((float)key_x(k) / hX);
        idx = idx >= nIni ? nIni - 1 : idx;
        for (int q = 0; q < nIni; q++) ini_cnt[q] += __popcll(__ballot(act && idx == q));
    }
    {
        int run[8], off = 0;
        for (int q = 0; q < nIni; q++) { run[q] = off; off += ini_cnt[q]; }
        for (int i = 0; i < n; i += 64) {
            const bool act = i + lane < n;
            const uint32_t k = act ? B[i + lane] : 0u;
            int idx = (int)((float)key_x(k) / hX);
            idx = idx >= nIni ? nIni - 1 : idx;
            for (int q = 0; q < nIni; q++) {
                const uint64_t m = __ballot(act && idx == q);
                if (act && idx == q) A[run[q] + popc_below(m)] = k;
                run[q] += __popcll(m);
            }
        }
    }
    __syncthreads();
    {
        int off = 0;
        for (int i = 0; i < nIni; i++) {  // push_back: created in order; linked below
            const int id = st.alloc();
            ini_ids[i] = id;
            sh.x0y0[id] = (uint32_t)(int)(hX * (float)i);
            sh.x1y1[id] = (uint32_t)(int)(hX * (float)(i + 1)) | ((uint32_t)H0 << 16);
            sh.beg[id] = (uint32_t)off;
            sh.cnt[id] = (uint32_t)ini_cnt[i];
            sh.seq[id] = (uint32_t)st.seq++;
            off += ini_cnt[i];
        }
        for (int i = nIni - 1; i >= 0; i--) st.push_front(ini_ids[i]);
        for (int i = 0; i < nIni; i++)  // erase empty initial nodes (size-1 ones are bNoMore)
            if (ini_cnt[i] == 0) st.erase(ini_ids[i]);
    }
    __syncthreads();
    // 3. DistributeOctTree main loop
    const int N = L.budget;
    bool finish = false;
    while (!finish && !st.overflow) {
        const int prevSize = st.size;
        int nToExpand = 0;
        st.nvsp = 0;
        int it = st.head;
        while (it != NIL) {
            if (sh.cnt[it] == 1) { it = sh.next[it]; continue; }
            nToExpand += st.divide(it, true);
            it = st.erase(it);
            __syncthreads();
            if (st.overflow) break;
        }
        if (st.size >= N || st.size == prevSize) {
            finish = true;
        } else if (st.size + nToExpand * 3 > N) {
            while (!finish && !st.overflow) {
                const int prev2 = st.size;
                const int nprev = st.nvsp;
                for (int i = lane; i < nprev; i += 64) sh.vprev[i] = sh.vsp[i];
                __syncthreads();
                st.nvsp = 0;
                wave_sort_u64<NODE_CAP>(sh.vprev, nprev);
                for (int j = nprev - 1; j >= 0; j--) {
                    const int id = (int)(sh.vprev[j] & 0xFFFF);
                    st.divide(id, true);
                    st.erase(id);
                    __syncthreads();
                    if (st.size >= N || st.overflow) break;
                }
                if (st.size >= N || st.size == prev2) finish = true;
            }
        }
    }
    // 4. retain the best key per node, list order
    uint32_t *out = sel + (size_t)f * plan->sel_total + L.sel_off;
    int k = 0;
    for (int it = st.head; it != NIL && !st.overflow; it = sh.next[it]) {
        const uint32_t bg = sh.beg[it];
        const uint32_t *src = (bg >> 31) ? B : A;
        const int beg = (int)(bg & 0x7FFFFFFF), cnt = (int)sh.cnt[it];
        uint32_t best;
        if (cnt == 1) {
            best = src[beg];
        } else {
            uint32_t bestv = 0;  // (score << 24) | (0xFFFFFF - index): max = highest score, first index
            for (int i = lane; i < cnt; i += 64) {
                const uint32_t v = ((uint32_t)key_score(src[beg + i]) << 24) | (uint32_t)(0xFFFFFF - i);
                bestv = v > bestv ? v : bestv;
            }
            for (int o = 32; o >= 1; o >>= 1) {
                const uint32_t t = (uint32_t)__shfl_xor((int)bestv, o, 64);
                bestv = t > bestv ? t : bestv;
            }
            best = src[beg + (0xFFFFFF - (bestv & 0xFFFFFF))];
        }
        if (k < L.sel_cap) {
            if (lane == 0) out[k] = best;
        } else {
            st.overflow = 1;
        }
        k++;
    }
    if (lane == 0) {
        selcnt[(size_t)f * plan->nlevels + l] = min(k, L.sel_cap);
        if (st.overflow) atomicOr(err, 1);
    }
}

template __global__ void k_octree<512>(const Plan *, const uint32_t *, const int *, uint32_t *, uint32_t *,
                                       uint32_t *, int *, int *);
template __global__ void k_octree<1024>(const Plan *, const uint32_t *, const int *, uint32_t *, uint32_t *,
                                        uint32_t *, int *, int *);
template __global__ void k_octree<2048>(const Plan *, const uint32_t *, const int *, uint32_t *, uint32_t *,
                                        uint32_t *, int *, int *);

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
    const float a = (float)cos((double)ang), b = (float)sin((double)ang);
    uint32_t nib = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int pi = (lane * 4 + k) * 4;
        const float px0 = (float)c_pattern[pi], py0 = (float)c_pattern[pi + 1];
        const float px1 = (float)c_pattern[pi + 2], py1 = (float)c_pattern[pi + 3];
        const int y0 = cy + cv_round(px0 * b + py0 * a), x0 = cx + cv_round(px0 * a - py0 * b);
        const int y1 = cy + cv_round(px1 * b + py1 * a), x1 = cx + cv_round(px1 * a - py1 * b);
        const int t0 = img[(size_t)clampi(y0, 0, h - 1) * w + clampi(x0, 0, w - 1)];
        const int t1 = img[(size_t)clampi(y1, 0, h - 1) * w + clampi(x1, 0, w - 1)];
        nib |= (uint32_t)(t0 < t1) << k;
    }
    uint32_t word = nib;
#pragma unroll
    for (int i = 1; i < 8; i++) word |= (uint32_t)__shfl_down((int)nib, i, 64) << (4 * i);
    if ((lane & 7) == 0) reinterpret_cast<uint32_t *>(desc_out)[lane >> 3] = word;
}

// New keypoints of the octree: rows n_existing + prefix(level) + k.
__global__ __launch_bounds__(256) void k_orient_desc(const uint8_t *__restrict__ pyr,
                                                     const uint8_t *__restrict__ blur, uint32_t pitch,
                                                     const Plan *__restrict__ plan,
                                                     const uint32_t *__restrict__ sel,
                                                     const int *__restrict__ selcnt,
                                                     const int *__restrict__ n_existing,
                                                     ygzfe_kp *__restrict__ kps, uint8_t *__restrict__ desc,
                                                     int *__restrict__ counts, int row_cap) {
    const int f = blockIdx.y;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int idx = blockIdx.x * 4 + wave;
    const int *sc = selcnt + (size_t)f * plan->nlevels;
    const int ne = n_existing ? n_existing[f] : 0;
    int l = 0, pre = 0;
    while (l < plan->nlevels && idx >= pre + sc[l]) { pre += sc[l]; l++; }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int tot = 0;
        for (int q = 0; q < plan->nlevels; q++) tot += sc[q];
        counts[f] = ne + tot;
    }
    if (l >= plan->nlevels) return;
    const LevelDesc &L = plan->lv[l];
    const uint32_t key = sel[(size_t)f * plan->sel_total + L.sel_off + (idx - pre)];
    const int cx = key_x(key) + kMinBorder, cy = key_y(key) + kMinBorder;
    const float angle = ic_angle_wave(pyr + (size_t)f * pitch + L.off, L.w, L.h, cx, cy, plan->umax);
    const int row = ne + idx;
    if (row >= row_cap) return;
    orb_desc_wave(blur + (size_t)f * pitch + L.off, L.w, L.h, cx, cy, angle, desc + ((size_t)f * row_cap + row) * 32);
    if (lane == 0) {
        ygzfe_kp kp;
        kp.x = (float)cx;
        kp.y = (float)cy;
        if (l != 0) { kp.x *= L.scale; kp.y *= L.scale; }
        kp.size = (float)L.patch_size;
        kp.angle = angle;
        kp.response = (float)key_score(key);
        kp.octave = l;
        kp.class_id = -1;
        kps[(size_t)f * row_cap + row] = kp;
    }
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

hipError_t upload_pattern(const int *pat) {
    int8_t p8[1024];
    for (int i = 0; i < 1024; i++) p8[i] = (int8_t)pat[i];
    return hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), p8, sizeof(p8));
}

hipError_t launch_pyramid(uint8_t *pyr, uint32_t pitch, const Plan &hp, const Plan *dp, const int *dtabs,
                          int nframes, hipStream_t st) {
    for (int l = 1; l < hp.nlevels; l++) {
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
    hipLaunchKernelGGL(k_blur7, dim3(hp.blur_tiles, nframes), dim3(256), 0, st, pyr, blur, pitch, dp);
    return hipGetLastError();
}

hipError_t launch_fast(const uint8_t *pyr, uint32_t pitch, const Plan &hp, const Plan *dp, const CellDesc *dcells,
                       uint32_t *cellbuf, int *cellcnt, int nframes, hipStream_t st) {
    if (hp.ncells == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fast_cells, dim3(hp.ncells, nframes), dim3(256), 0, st, pyr, pitch, dp, dcells,
                       cellbuf, cellcnt);
    return hipGetLastError();
}

hipError_t launch_octree(const Plan &hp, const Plan *dp, const uint32_t *cellbuf, const int *cellcnt,
                         uint32_t *candA, uint32_t *candB, uint32_t *sel, int *selcnt, int *err, int nframes,
                         hipStream_t st) {
    dim3 grid(hp.nlevels, nframes);
    if (hp.node_cap <= 512)
        hipLaunchKernelGGL(k_octree<512>, grid, dim3(64), 0, st, dp, cellbuf, cellcnt, candA, candB, sel, selcnt, err);
    else if (hp.node_cap <= 1024)
        hipLaunchKernelGGL(k_octree<1024>, grid, dim3(64), 0, st, dp, cellbuf, cellcnt, candA, candB, sel, selcnt, err);
    else
        hipLaunchKernelGGL(k_octree<2048>, grid, dim3(64), 0, st, dp, cellbuf, cellcnt, candA, candB, sel, selcnt, err);
    return hipGetLastError();
}

hipError_t launch_orient_desc(const uint8_t *pyr, const uint8_t *blur, uint32_t pitch, const Plan &hp,
                              const Plan *dp, const uint32_t *sel, const int *selcnt, const int *n_existing,
                              ygzfe_kp *kps, uint8_t *desc, int *counts, int row_cap, int nframes,
                              hipStream_t st) {
    const int max_new = hp.sel_total;
    hipLaunchKernelGGL(k_orient_desc, dim3((max_new + 3) / 4, nframes), dim3(256), 0, st, pyr, blur, pitch, dp,
                       sel, selcnt, n_existing, kps, desc, counts, row_cap);
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
