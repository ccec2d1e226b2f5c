// match.hip — the tracking-path ORBmatcher searches (ORBmatcher.cc) on gfx950.
//
//   SearchByProjection(CurrentFrame, LastFrame, th, bMono, checkLevel)  :1218-1350  mode BEST
//   SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)  :1352-1469  mode BEST
//   SearchByProjection(F, vpMapPoints, th, checkLevel)                 :43-126     mode RATIO
//   SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, ws)    :375-478    mode INIT
//   SearchByBoW(pKF, F, vpMapPointMatches)                             :155-263    mode BOW
//   ComputeThreeMaxima                                                 :1471-1502
//
// The reference runs one query after another, and a query's candidates
// depend on the assignments of the queries before it (a keypoint matched to
// a MapPoint with observations is skipped later; SearchForInitialization
// skips keypoints already matched at an equal or smaller distance;
// SearchByBoW skips matched keypoints).  The work is split in two passes:
//
//  k_match_topk   one wave per query, all queries of all problems at once:
//                 the GetFeaturesInArea window (Frame.cc:424-481: the grid
//                 cell range, level filter, |dx| < r, |dy| < r; the stereo
//                 test of the projection searches) or the BoW node's feature
//                 list, every candidate's Hamming distance, and the K
//                 smallest (distance, candidate-order) keys — the order in
//                 which the reference's strict-< scan would rank them, so the
//                 first entry is its best, the next its second.
//  k_match_replay one wave per problem: the queries in the reference's order
//                 against the sequential state in LDS; per query the K
//                 entries' skip tests run in K lanes and a ballot gives the
//                 first / second surviving entry.  When the skips exhaust the
//                 K entries of a longer candidate list the wave re-scans that
//                 query's whole window under the current state, so the
//                 result never depends on K.  Then the rotation histogram
//                 votes (ComputeThreeMaxima) and the removals.
#include "kernels.hpp"

namespace ygzfe {

#ifdef YGZ_STAMPS  // diagnostic build: this file's kernels stamp into their own buffer
__device__ unsigned long long g_mstamps[1 << 20];
#define g_bstamps g_mstamps
extern "C" int ygzfe_diag_match_stamps(unsigned long long *out, int n) {
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mstamps), sizeof(unsigned long long) * (size_t)n);
    return 0;
}
#endif

constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS (Frame.h:27-28)
constexpr int kTopK = 8;      // per-lane list, and the entries the decisions keep in registers
constexpr int kTopList = 32;  // entries k_match_topk lists per query (J.topk stride)
// J.ncand[q] as k_match_topk writes it: candidates (bits 0-15) | valid | blocks | listed entries << 24
constexpr int kInfoValid = 1 << 22, kInfoBlocks = 1 << 23;
constexpr int kHisto = 30;                       // ORBmatcher::HISTO_LENGTH (ORBmatcher.cc:38)

// Frame::PosInGrid (Frame.cc:483-493): std::round(float), cell -1 when outside; and
// the grid as an index (Frame::mGrid, Frame.cc:412-422): the keypoints bucketed by
// cell (cell-major ix * rows + iy), cend[c] = end of cell c in cidx.  One workgroup,
// counting sort in LDS; the order inside a cell is immaterial (candidates are ranked
// by their (distance, cell, index) keys).
constexpr int kGridCells = kGridCols * kGridRows;  // 3072
__global__ __launch_bounds__(1024) void k_match_cells(const ygzfe_kp *__restrict__ kps, int n, float min_x,
                                                      float min_y, float inv_w, float inv_h,
                                                      int32_t *__restrict__ cell, int32_t *__restrict__ cend,
                                                      uint16_t *__restrict__ cidx) {
    __shared__ int cnt[kGridCells];
    __shared__ int s_sum[16];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    auto cell_of = [&](int i) -> int {
        const int px = (int)__builtin_roundf((kps[i].x - min_x) * inv_w);
        const int py = (int)__builtin_roundf((kps[i].y - min_y) * inv_h);
        return (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : (px << 8) | py;
    };
    for (int c = tid; c < kGridCells; c += 1024) cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        const int c = cell_of(i);
        cell[i] = c;
        if (c >= 0) atomicAdd(&cnt[(c >> 8) * kGridRows + (c & 0xFF)], 1);
    }
    __syncthreads();
    const int c0 = 3 * tid;
    const int a0 = cnt[c0], a1 = cnt[c0 + 1], a2 = cnt[c0 + 2], sum = a0 + a1 + a2;
    int incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) s_sum[wv] = incl;
    __syncthreads();
    int base = 0;
    for (int k = 0; k < wv; k++) base += s_sum[k];
    const int e0 = base + incl - sum + a0, e1 = e0 + a1, e2 = e1 + a2;  // ends of cells c0 .. c0 + 2
    cend[c0] = e0;
    cend[c0 + 1] = e1;
    cend[c0 + 2] = e2;
    cnt[c0] = e0;
    cnt[c0 + 1] = e1;
    cnt[c0 + 2] = e2;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {  // each cell filled from its end down
        const int c = cell_of(i);
        if (c >= 0) cidx[atomicSub(&cnt[(c >> 8) * kGridRows + (c & 0xFF)], 1) - 1] = (uint16_t)i;
    }
}

hipError_t launch_match_cells(const ygzfe_kp *kps, int n, float min_x, float min_y, float inv_w, float inv_h,
                              int32_t *cell, int32_t *cend, uint16_t *cidx, hipStream_t st) {
    hipLaunchKernelGGL(k_match_cells, dim3(1), dim3(1024), 0, st, kps, n, min_x, min_y, inv_w, inv_h, cell, cend,
                       cidx);
    return hipGetLastError();
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = shfl_xor_u64(v, m);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ int hamming32(const uint32_t q[8], const uint8_t *d) {
    const uint4 a = reinterpret_cast<const uint4 *>(d)[0], b = reinterpret_cast<const uint4 *>(d)[1];
    return __popc(q[0] ^ a.x) + __popc(q[1] ^ a.y) + __popc(q[2] ^ a.z) + __popc(q[3] ^ a.w) + __popc(q[4] ^ b.x) +
           __popc(q[5] ^ b.y) + __popc(q[6] ^ b.z) + __popc(q[7] ^ b.w);
}

// The window of GetFeaturesInArea (Frame.cc:429-449) in the reference's float arithmetic.
struct Window {
    int cx0, cx1, cy0, cy1;  // cell range (empty when cx0 > cx1)
    bool check_levels;
    int min_level, max_level;
    float x, y, r;
};

__device__ __forceinline__ Window make_window(const MatchJob &J, const ygzfe_match_query &q) {
    Window w;
    w.x = q.u;
    w.y = q.v;
    w.r = q.radius;
    w.min_level = q.min_level;
    w.max_level = q.max_level;
    w.check_levels = (q.min_level > 0) || (q.max_level >= 0);
    const float inv_w = J.inv_w, inv_h = J.inv_h;
    w.cx0 = max(0, (int)floorf((q.u - J.min_x - q.radius) * inv_w));
    w.cx1 = min(kGridCols - 1, (int)ceilf((q.u - J.min_x + q.radius) * inv_w));
    w.cy0 = max(0, (int)floorf((q.v - J.min_y - q.radius) * inv_h));
    w.cy1 = min(kGridRows - 1, (int)ceilf((q.v - J.min_y + q.radius) * inv_h));
    if (w.cx0 >= kGridCols || w.cx1 < 0 || w.cy0 >= kGridRows || w.cy1 < 0) w.cx0 = 1, w.cx1 = 0;
    return w;
}

// Is train keypoint j of cell (ix, iy) in the query's candidate list (window +
// level + stereo)?  Returns its candidate-order key (cell-major, then index) or ~0.
__device__ __forceinline__ uint32_t window_accept(const MatchJob &J, const Window &w, const ygzfe_match_query &q,
                                                  int j, int c) {
    const ygzfe_kp &kp = J.kps[j];
    if (w.check_levels) {
        if (kp.octave < w.min_level) return ~0u;
        if (w.max_level >= 0 && kp.octave > w.max_level) return ~0u;
    }
    const float dx = kp.x - w.x, dy = kp.y - w.y;
    if (!(fabsf(dx) < w.r && fabsf(dy) < w.r)) return ~0u;
    if ((q.flags & YGZFE_MQ_STEREO) && J.u_right && J.u_right[j] > 0) {
        const float er = fabsf(q.u_right - J.u_right[j]);
        if (er > q.radius) return ~0u;
    }
    return ((uint32_t)c << 16) | (uint32_t)j;  // GetFeaturesInArea order
}

// The window's cells' keypoints spread over the wave's lanes (64 cells at a time,
// their index ranges concatenated): fn(j, c) on each lane holding one.
template <class F>
__device__ __forceinline__ void for_window(const MatchJob &J, const Window &w, F fn) {
    const int lane = threadIdx.x & 63;
    if (w.cx0 > w.cx1) return;
    const int ncy = w.cy1 - w.cy0 + 1, ncell = (w.cx1 - w.cx0 + 1) * ncy;
    for (int cb = 0; cb < ncell; cb += 64) {
        int lo = 0, cnt = 0, c = 0;
        if (cb + lane < ncell) {
            const int k = cb + lane;
            c = (w.cx0 + k / ncy) * kGridRows + (w.cy0 + k % ncy);
            lo = c ? J.cend[c - 1] : 0;
            cnt = J.cend[c] - lo;
        }
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        const int total = __shfl(incl, 63, 64);
        for (int e0 = 0; e0 < total; e0 += 64) {
            const int e = e0 + lane;
            int src = 0;  // the lane holding e's cell: the first whose inclusive count exceeds e
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1)
                if (__shfl(incl, src + step - 1, 64) <= e) src += step;
            const int s_lo = __shfl(lo, src, 64), s_ex = __shfl(incl - cnt, src, 64), s_c = __shfl(c, src, 64);
            if (e < total) fn((int)J.cidx[s_lo + e - s_ex], s_c);
        }
    }
}

// key = dist << 52 | order << 20 | octave << 16 | train index (n <= 65535).  The
// candidate order is unique within a query, so the octave bits never decide a
// comparison; they spare the serial replay a dependent load per ratio test.
__device__ __forceinline__ uint64_t make_key(int dist, uint32_t order, int j, int octave) {
    return ((uint64_t)dist << 52) | ((uint64_t)order << 20) | ((uint64_t)(octave & 15) << 16) | (uint64_t)j;
}
__device__ __forceinline__ int key_train(uint64_t k) { return (int)(k & 0xFFFF); }
__device__ __forceinline__ int key_octave(uint64_t k) { return (int)((k >> 16) & 15); }

template <class Pred>
__device__ __forceinline__ void scan_query(const MatchJob &J, int q, const ygzfe_match_query &Q, const uint32_t qd[8],
                                           Pred skip, uint64_t L[kTopK], int &count) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kTopK; k++) L[k] = ~0ull;
    count = 0;
    auto consider = [&](int j, uint32_t order) {
        const int dist = hamming32(qd, J.desc + (size_t)j * 32);
        if (skip(j, dist)) return;
        count++;
        uint64_t key = make_key(dist, order, j, J.kps[j].octave);
#pragma unroll
        for (int k = 0; k < kTopK; k++) {  // sorted insertion, branch-free
            const uint64_t lo = key < L[k] ? key : L[k], hi = key < L[k] ? L[k] : key;
            L[k] = lo;
            key = hi;
        }
    };
    if (J.cand_ptr) {  // BoW node list: order = position in the node's feature vector
        const int b = J.cand_ptr[2 * q], e = J.cand_ptr[2 * q + 1];
        for (int p = b + lane; p < e; p += 64) consider(J.cand[p], (uint32_t)(p - b));
    } else {
        const Window w = make_window(J, Q);
        for_window(J, w, [&](int j, int c) {
            const uint32_t o = window_accept(J, w, Q, j, c);
            if (o != ~0u) consider(j, o);
        });
    }
}

__device__ __forceinline__ void load_qdesc(const MatchJob &J, int q, uint32_t qd[8]) {
    const int id = J.qid ? J.qid[q] : q;
    const uint4 *p = reinterpret_cast<const uint4 *>(J.qdesc + (size_t)id * 32);
    const uint4 a = p[0], b = p[1];
    qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
    qd[4] = b.x; qd[5] = b.y; qd[6] = b.z; qd[7] = b.w;
}

// k_match_topk: one wave per query, all queries at once.  Lanes collect the
// window's candidates (the frame's cell index, for_window) keeping their kTopK
// smallest keys; the kept keys go to LDS and each is ranked by counting the
// smaller ones (broadcast reads, no cross-lane reductions).  The first V ranks are
// exact: V counts the kept keys up to the smallest kTopK-th key of a lane that
// dropped candidates (its dropped ones are larger), capped at kTopList.
constexpr int kTopkWaves = 4;
__global__ __launch_bounds__(64 * kTopkWaves) void k_match_topk(const MatchJob J) {
    __shared__ uint64_t s_keys[kTopkWaves][64 * kTopK];
    const int q = __builtin_amdgcn_readfirstlane(blockIdx.x * kTopkWaves + (threadIdx.x >> 6));
    if (q >= J.nq) return;
    const int lane = threadIdx.x & 63;
    uint64_t *K = s_keys[threadIdx.x >> 6];
    const ygzfe_match_query Q = J.q[q];  // the query records may live in host memory (read once here)
    if (!(Q.flags & YGZFE_MQ_VALID)) {
        if (lane == 0) J.ncand[q] = 0;
        return;
    }
    if (lane == 0) J.qangle[q] = Q.angle;
    uint32_t qd[8];
    load_qdesc(J, q, qd);
    uint64_t L[kTopK];
    int count;
    scan_query(J, q, Q, qd, [](int, int) { return false; }, L, count);
    const int kept = min(count, kTopK);
    int off = kept;  // exclusive prefix of the kept counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(off, o, 64);
        if (lane >= o) off += v;
    }
    const int T = __shfl(off, 63, 64), total = wave_sum_i(count);
    off -= kept;
#pragma unroll
    for (int k = 0; k < kTopK; k++)
        if (k < kept) K[off + k] = L[k];
    uint64_t thr = ~0ull;  // keys above the smallest dropped-lane bound are not exact
    if (__ballot(count > kTopK)) thr = wave_min_u64(count > kTopK ? L[kTopK - 1] : ~0ull);
    wave_lds_order();
    int V = 0;
    for (int t0 = 0; t0 < T; t0 += 64) {
        const int t = t0 + lane;
        const uint64_t mine = t < T ? K[t] : ~0ull;
        int rank = 0;
        for (int u = 0; u < T; u++) rank += K[u] < mine;
        if (t < T && mine <= thr && rank < kTopList) J.topk[(size_t)q * kTopList + rank] = mine;
        V += __popcll(__ballot(t < T && mine <= thr));
    }
    V = min(V, kTopList);
    if (lane == 0) J.ncand[q] = total | kInfoValid | ((Q.flags & YGZFE_MQ_BLOCKS) ? kInfoBlocks : 0) | (V << 24);
}

// ComputeThreeMaxima (ORBmatcher.cc:1471-1502)
__device__ __forceinline__ void three_maxima(const int *h, int &ind1, int &ind2, int &ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    ind1 = ind2 = ind3 = -1;
    for (int i = 0; i < kHisto; i++) {
        const int s = h[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
}

// the rotation bin (ORBmatcher.cc:1318-1323): float rot, std::round(float)
__device__ __forceinline__ int rot_bin(float aq, float at) {
    const float factor = 1.0f / kHisto;
    float rot = aq - at;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)__builtin_roundf(rot * factor);
    if (bin == kHisto) bin = 0;
    return min(max(bin, 0), 63);
}

// LDS of k_match_replay: blocked [n], INIT's distance / match arrays, then (when the
// total stays under 64 KB) the train keypoints' angles and octaves
__host__ __device__ __forceinline__ size_t replay_lds_base(int n, int mode) {
    return (size_t)((n + 15) & ~15) + (mode == YGZFE_MATCH_INIT ? 4 * (size_t)((n + 7) & ~7) : 0);
}
__host__ __device__ __forceinline__ bool staged_kp_fits(int n, int mode) {
    return replay_lds_base(n, mode) + 5 * (size_t)((n + 3) & ~3) + 64 <= 65536;
}

// The serial replay, run by ONE wave (k_match_replay: INIT, jobs the resolve's LDS
// cannot hold, or YGZFE_MATCH_PASSES=0).
__device__ __forceinline__ void wave_sync() {
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void replay_serial(const MatchJob &J, uint8_t *lds, int mode, int th_dist, int check_ori,
                                           float nnratio, int stage_kv) {
    const auto g_train_out = as_global_mut(J.train_out), g_query_out = as_global_mut(J.query_out);
    const auto g_pushes = as_global_mut(J.pushes), g_nmatches = as_global_mut(J.nmatches);
    const auto g_ncand = as_global(J.ncand);
    const auto g_topk = as_global(J.topk);
    const auto g_kps = as_global(J.kps);
    const auto g_blocked0 = as_global(J.blocked0);
    const auto g_qid = as_global(J.qid);
    const int lane = threadIdx.x & 63;
    const int n = J.n_train;
    __shared__ int rot_count[64];
    uint8_t *blocked = lds;                                            // [n]
    uint16_t *mdist = reinterpret_cast<uint16_t *>(lds + ((n + 15) & ~15));  // INIT: vMatchedDistance (0xFFFF = INT_MAX)
    int16_t *m21 = reinterpret_cast<int16_t *>(mdist + ((n + 7) & ~7));      // INIT: vnMatches21
    // the train keypoints' octave and angle the per-query decisions read (LDS when it
    // fits: the replay is a serial chain, a global load per query is its latency)
    const size_t kv_off = ((n + 15) & ~15) + (mode == YGZFE_MATCH_INIT ? 4 * (size_t)((n + 7) & ~7) : 0);
    const bool kv_lds = stage_kv != 0;  // allocated for the launch's largest n (>= this job's)
    float *s_ang = reinterpret_cast<float *>(lds + kv_off);
    uint8_t *s_oct = lds + kv_off + 4 * (size_t)((n + 3) & ~3);
    for (int j = lane; j < n; j += 64) {
        blocked[j] = J.blocked0 ? g_blocked0[j] : 0;
        if (J.train_out) g_train_out[j] = -1;
        if (mode == YGZFE_MATCH_INIT) {
            mdist[j] = 0xFFFF;
            m21[j] = -1;
        }
        if (kv_lds) {
            s_ang[j] = g_kps[j].angle;
            s_oct[j] = (uint8_t)g_kps[j].octave;
        }
    }
    auto oct_of = [&](int j) -> int { return kv_lds ? (int)s_oct[j] : g_kps[j].octave; };
    auto ang_of = [&](int j) -> float { return kv_lds ? s_ang[j] : g_kps[j].angle; };
    if (mode == YGZFE_MATCH_INIT)
        for (int i = lane; i < J.nq; i += 64) g_query_out[i] = -1;
    rot_count[lane] = 0;
    wave_sync();
    int nmatches = 0, npush = 0, rescans = 0;
    const int need = mode == YGZFE_MATCH_BEST ? 1 : 2;
    // skip test of the reference's scan against the current state
    auto skip = [&](int j, int dist) -> bool {
        if (mode == YGZFE_MATCH_INIT) return (int)mdist[j] <= dist;  // vMatchedDistance[i2] <= dist (0xFFFF: INT_MAX)
        return blocked[j] != 0;
    };
    // Queries staged 64 at a time (lane i loads query b + i: flags, angle, candidate
    // count, top-K entries), double-buffered in LDS: the serial chain below then pays
    // LDS latencies only, the next block's global loads landing meanwhile.
    __shared__ uint64_t s_qe[2][64 * kTopK];
    struct Blk {
        int flags, cnt;
        float angle;
        uint64_t e[kTopK];
    };
    auto load_blk = [&](int b0) -> Blk {
        Blk r;
        const int q = b0 + lane;
        r.flags = 0;
        r.cnt = 0;
        r.angle = 0.f;
#pragma unroll
        for (int k = 0; k < kTopK; k++) r.e[k] = ~0ull;
        if (q < J.nq) {
            const int info = g_ncand[q];
            r.flags = (info & kInfoValid ? YGZFE_MQ_VALID : 0) | (info & kInfoBlocks ? YGZFE_MQ_BLOCKS : 0);
            r.angle = J.qangle[q];
            r.cnt = info & 0xFFFF;
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            const auto t = (gptr_t<v4u>)(J.topk + (size_t)q * kTopList);
#pragma unroll
            for (int k = 0; k < kTopK / 2; k++) {
                const v4u v = t[k];
                r.e[2 * k] = ((uint64_t)v.y << 32) | v.x;
                r.e[2 * k + 1] = ((uint64_t)v.w << 32) | v.z;
            }
        }
        return r;
    };
    auto store_blk = [&](int buf, const Blk &r) {
#pragma unroll
        for (int k = 0; k < kTopK; k++) s_qe[buf][lane * kTopK + k] = r.e[k];
        wave_lds_order();
    };
    Blk cur;
    if (J.nq > 0) {
        cur = load_blk(0);
        store_blk(0, cur);
    }
    for (int qb = 0; qb < J.nq; qb += 64) {
        const int buf = (qb >> 6) & 1;
        const bool more = qb + 64 < J.nq;
        Blk nxt;
        if (more) nxt = load_blk(qb + 64);  // in flight during this block
        const int qe = min(J.nq, qb + 64);
        // flags / counts / angles of the block by readlane (lane t holds query qb + t's);
        // the top-K entries by LDS reads issued one query ahead
        uint64_t Enext = lane < kTopK ? s_qe[buf][lane] : ~0ull;
    for (int q = qb; q < qe; q++) {
        const int t = q - qb;
        const uint64_t cE = Enext;
        if (q + 1 < qe) Enext = lane < kTopK ? s_qe[buf][(t + 1) * kTopK + lane] : ~0ull;
        const int cflags = __builtin_amdgcn_readlane(cur.flags, t), ccnt = __builtin_amdgcn_readlane(cur.cnt, t);
        if (!(cflags & YGZFE_MQ_VALID) || ccnt == 0) continue;
        const float cangle = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cur.angle), t));
        const int nk = min(ccnt, kTopK);
        int dist_l = (int)(cE >> 52), j_l = key_train(cE);
        const bool ok = lane < nk && !skip(j_l, dist_l);
        const uint64_t bal = __ballot(ok);
        uint64_t best = ~0ull, second = ~0ull;
        auto lane_key = [&](int from) -> uint64_t {  // uniform lane index: no LDS round trip
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cE, from);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(cE >> 32), from);
            return ((uint64_t)hi << 32) | lo;
        };
        if (__popcll(bal) >= need || ccnt <= kTopK) {
            if (bal) {
                best = lane_key(__builtin_ctzll(bal));
                const uint64_t rest = bal & (bal - 1);
                if (rest) second = lane_key(__builtin_ctzll(rest));
            }
        } else {  // the skips used up the K entries: re-scan this query under the current state
            rescans++;
            const ygzfe_match_query cq = J.q[q];
            uint32_t qd[8];
            load_qdesc(J, q, qd);
            uint64_t L[kTopK];
            int c2;
            scan_query(J, q, cq, qd, skip, L, c2);
            best = wave_min_u64(L[0]);
            if (L[0] == best) L[0] = L[1];
            second = wave_min_u64(L[0]);
        }
        const bool has1 = best != ~0ull, has2 = second != ~0ull;
        const int bj = key_train(best), bd = has1 ? (int)(best >> 52) : 256;
        const int sj = key_train(second), sdist = has2 ? (int)(second >> 52) : 256;
        const int id = J.qid ? g_qid[q] : q;
        int push_id = -1;
        if (mode == YGZFE_MATCH_BEST) {
            if (has1 && bd <= th_dist) {
                if (lane == 0) g_train_out[bj] = q;
                blocked[bj] = (cflags & YGZFE_MQ_BLOCKS) ? 1 : 0;
                nmatches++;
                push_id = bj;
            }
        } else if (mode == YGZFE_MATCH_RATIO) {
            const int bl = has1 ? key_octave(best) : -1, sl = has2 ? key_octave(second) : -1;
            if (has1 && bd <= 100 && !(bl == sl && bd > nnratio * sdist)) {
                if (lane == 0) g_train_out[bj] = q;
                blocked[bj] = (cflags & YGZFE_MQ_BLOCKS) ? 1 : 0;
                nmatches++;
            }
        } else if (mode == YGZFE_MATCH_INIT) {
            const int bdi = has1 ? bd : 0x7FFFFFFF, sdi = has2 ? sdist : 0x7FFFFFFF;
            if (has1 && bdi <= 50 && bdi < (float)sdi * nnratio) {
                const int old = m21[bj];
                if (old >= 0) {
                    if (lane == 0) g_query_out[old] = -1;
                    nmatches--;
                }
                if (lane == 0) g_query_out[q] = bj;
                m21[bj] = (int16_t)q;
                mdist[bj] = (uint16_t)bdi;
                nmatches++;
                push_id = q;
            }
        } else {  // BOW
            if (has1 && bd <= 50 && (float)bd < nnratio * (float)sdist) {
                if (lane == 0) g_train_out[bj] = id;
                blocked[bj] = 1;
                nmatches++;
                push_id = bj;
            }
        }
        if (push_id >= 0 && check_ori && mode != YGZFE_MATCH_RATIO) {  // histogram counted after the loop
            const int bin = rot_bin(cangle, ang_of(bj));
            if (lane == 0) g_pushes[npush] = (bin << 24) | push_id;
            npush++;
        }
        wave_lds_order();  // the LDS state updates precede the next query's reads (one wave: DS ops in order)
    }
        if (more) {
            store_blk(buf ^ 1, nxt);
            cur = nxt;
        }
    }
    if (check_ori && mode != YGZFE_MATCH_RATIO && npush > 0) {
        wave_sync();  // the pushes are visible to every lane
        for (int p = lane; p < npush; p += 64) atomicAdd(&rot_count[g_pushes[p] >> 24], 1);
        wave_sync();
        int i1, i2, i3;
        three_maxima(rot_count, i1, i2, i3);
        int removed = 0;
        for (int p = lane; p < npush; p += 64) {
            const int v = g_pushes[p], bin = v >> 24, pid = v & 0xFFFFFF;
            if (bin == i1 || bin == i2 || bin == i3) continue;
            if (mode == YGZFE_MATCH_BEST) {
                g_train_out[pid] = -2;
                removed++;
            } else if (mode == YGZFE_MATCH_BOW) {
                g_train_out[pid] = -1;
                removed++;
            } else if (g_query_out[pid] >= 0) {  // INIT
                g_query_out[pid] = -1;
                removed++;
            }
        }
        nmatches -= wave_sum_i(removed);
    }
    if (lane == 0) {
        g_nmatches[0] = nmatches;
        g_nmatches[1] = rescans;  // diagnostics: queries whose top-K list the skips exhausted
        g_nmatches[2] = -1;       // the serial replay decided
    }
}

__global__ __launch_bounds__(64) void k_match_replay(const MatchJob J, int mode, int th_dist, int check_ori,
                                                     float nnratio, int stage_kv) {
    extern __shared__ uint8_t lds[];
    replay_serial(J, lds, mode, th_dist, check_ori, nnratio, stage_kv);
}

// ---------------------------------------------------------------------------
// k_match_resolve<R>: the same sequential result, found in parallel.
//
// A query's decision depends on the state its candidates are in when the
// reference's loop reaches it, and that state is written only by earlier
// queries' matches: train keypoint j is skipped by query q iff the LAST query
// p < q that matched j set it (BEST / RATIO: p's MapPoint has observations —
// the test `mvpMapPoints[i2]->Observations() > 0`, ORBmatcher.cc:1290-1292 /
// :76-78; BoW: always, `vpMapPointMatches[realIdxF]` set, :210-211), else its
// initial state.  So decisions d_q = f_q(d_0 .. d_{q-1}) with f_q strictly
// causal, and the iteration d^{k+1}_q = f_q(d^k) (every query re-decided
// against the previous pass's decisions, all at once) has exactly one fixed
// point, the sequential result, reached after at most (longest chain of
// queries whose decisions feed each other) + 1 passes (4-13 on the test scenes).
//
// A pass: the matched queries are linked per train keypoint in LDS (atomic
// exchange into head[j]); each thread re-decides its R queries from their top-K
// entries (held in registers across passes, 4 B each), walking each entry's
// list for the latest chooser before the query.  A query whose skips exhaust
// the top-K entries of a longer candidate list (the serial path's re-scan) goes
// to a list that the 16 waves then work through, one query per wave: lanes over
// the query's GetFeaturesInArea cells (keypoints bucketed by cell in LDS on
// first need) or BoW node list, Hamming + state per candidate, a wave min for
// the best two.  A pass that changes no decision ends the loop.
// ---------------------------------------------------------------------------
constexpr int kResolveThreads = 1024, kResolveWaves = kResolveThreads / 64;
static_assert(kGridCells == 3 * kResolveThreads, "cell scan: 3 cells per thread");
constexpr uint32_t kNoEntry = 0xFFFFFFFFu;
constexpr uint16_t kChoiceNone = 0xFFFF, kChoicePending = 0xFFFE;

// LDS of the resolve: heads i32[2][n] | train angles f32[n] | link i16[nq] | choice u16[nq] |
// rq i16[nq] | q blocks u8[nq] | initial state u8[n]
__host__ __device__ __forceinline__ size_t resolve_lds_bytes(int n, int nq) {
    const size_t n2 = (size_t)((n + 1) & ~1), q2 = (size_t)((nq + 1) & ~1);
    return 12 * n2 + 6 * q2 + q2 + n2;
}
__host__ __device__ __forceinline__ size_t replay_lds_bytes(int n, int mode) {
    return replay_lds_base(n, mode) + (staged_kp_fits(n, mode) ? 5 * (size_t)((n + 3) & ~3) : 0) + 64;
}

// entry = dist << 20 | octave << 16 | train index (from a top-K key)
__device__ __forceinline__ uint32_t entry_of(uint64_t key) {
    return key == ~0ull ? kNoEntry : (uint32_t)((key >> 52) << 20) | (uint32_t)(key & 0xFFFFF);
}

template <int R>
__global__ __launch_bounds__(kResolveThreads) void k_match_resolve(const MatchJob J, int mode, int th_dist,
                                                                   int check_ori, float nnratio, int max_passes) {
    extern __shared__ uint8_t lds[];
    YGZ_BSTAMP_K(5, 0);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, n = J.n_train, nq = J.nq;
    const size_t n2 = (size_t)((n + 1) & ~1), q2 = (size_t)((nq + 1) & ~1);
    // pass k links into heads[k & 1]; the other buffer (read by pass k - 1) is cleared meanwhile
    int32_t *heads = reinterpret_cast<int32_t *>(lds);       // [2][n] latest linked chooser of j
    float *tang = reinterpret_cast<float *>(heads + 2 * n2);  // [n]  train keypoint angles (rotation check)
    int16_t *link = reinterpret_cast<int16_t *>(tang + n2);  // [nq] next chooser of the same j
    uint16_t *choice = reinterpret_cast<uint16_t *>(link + q2);   // [nq] matched train index / none
    int16_t *rq = reinterpret_cast<int16_t *>(choice + q2);  // [nq] this pass's re-scan queries
    uint8_t *qbl = reinterpret_cast<uint8_t *>(rq + q2);     // [nq] a match by q blocks its keypoint
    uint8_t *bl0 = qbl + q2;                                 // [n]  initial skip state
    __shared__ int s_rot[kHisto + 2];
    __shared__ int s_sum[kResolveWaves];
    __shared__ int s_nrq[2], s_chg[2];  // per pass parity: pass k resets pass k + 1's
    const auto g_ncand = as_global(J.ncand);
    const auto g_blocked0 = as_global(J.blocked0);
    const auto g_kps = as_global(J.kps);
    const auto g_topk = as_global(J.topk);
    const int need = mode == YGZFE_MATCH_BEST ? 1 : 2;
    // the thread's queries q = tid + 1024 r: candidate count (-1: not valid), listed
    // entries, angle, and the first kTopK entries
    int qcnt[R], qlist[R];
    float qang[R];
    uint32_t E[R][kTopK];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int q = tid + kResolveThreads * r;
        qcnt[r] = -1;
        qlist[r] = 0;
        qang[r] = 0.f;
        if (q < nq) {
            const int nc = g_ncand[q];
            qang[r] = J.qangle[q];
            qcnt[r] = (nc & kInfoValid) ? (nc & 0xFFFF) : -1;
            qlist[r] = (uint32_t)nc >> 24;
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            const auto t = (gptr_t<v4u>)(J.topk + (size_t)q * kTopList);
#pragma unroll
            for (int k = 0; k < kTopK / 2; k++) {
                const v4u v = t[k];
                E[r][2 * k] = entry_of(((uint64_t)v.y << 32) | v.x);
                E[r][2 * k + 1] = entry_of(((uint64_t)v.w << 32) | v.z);
            }
            choice[q] = kChoiceNone;
            qbl[q] = mode == YGZFE_MATCH_BOW ? 1 : ((nc & kInfoBlocks) ? 1 : 0);
        }
    }
    const bool ori = check_ori && mode != YGZFE_MATCH_RATIO;
    for (int j = tid; j < n; j += kResolveThreads) {
        heads[j] = -1;
        heads[n2 + j] = -1;
        bl0[j] = J.blocked0 ? g_blocked0[j] : 0;
        if (ori) tang[j] = g_kps[j].angle;
    }
    if (tid == 0) s_nrq[0] = s_nrq[1] = s_chg[0] = s_chg[1] = 0;
    if (tid < kHisto + 2) s_rot[tid] = 0;
    // the state query q sees keypoint j in: set by the latest chooser before q
    const int32_t *head = heads;
    auto blocked_at = [&](int j, int q) -> bool {
        int last = -1;
        for (int p = head[j]; p >= 0; p = link[p])
            if (p < q && p > last) last = p;
        return (last >= 0 ? qbl[last] : bl0[j]) != 0;
    };
    // blocked entries among the first nk register entries of query (r, q), as a bit mask:
    // every entry's head and initial state read at once, list walks only where linked
    auto blocked_mask = [&](const uint32_t (&e)[kTopK], int nk, int q) -> uint32_t {
        int hk[kTopK];
        uint8_t b0[kTopK];
#pragma unroll
        for (int k = 0; k < kTopK; k++) {
            const int j = (int)(e[k] & 0xFFFF);
            hk[k] = k < nk ? head[j] : -1;
            b0[k] = k < nk ? bl0[j] : 0;
        }
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < kTopK; k++) {
            int last = -1;
            for (int p = hk[k]; p >= 0; p = link[p])
                if (p < q && p > last) last = p;
            m |= (uint32_t)((last >= 0 ? qbl[last] : b0[k]) != 0) << k;
        }
        return m;
    };
    auto rule = [&](uint32_t best, uint32_t second) -> int {  // the mode's acceptance test
        const bool has1 = best != kNoEntry, has2 = second != kNoEntry;
        const int bd = has1 ? (int)(best >> 20) : 256, sdist = has2 ? (int)(second >> 20) : 256;
        bool ok;
        if (mode == YGZFE_MATCH_BEST) {
            ok = has1 && bd <= th_dist;
        } else if (mode == YGZFE_MATCH_RATIO) {
            const int bl = has1 ? (int)((best >> 16) & 15) : -1, sl = has2 ? (int)((second >> 16) & 15) : -1;
            ok = has1 && bd <= 100 && !(bl == sl && bd > nnratio * sdist);
        } else {  // BOW
            ok = has1 && bd <= 50 && (float)bd < nnratio * (float)sdist;
        }
        return ok ? (int)(best & 0xFFFF) : kChoiceNone;
    };
    // the serial path's re-scan by one wave: every candidate under the current state
    auto wave_rescan = [&](int q) -> int {
        const ygzfe_match_query Q = J.q[q];
        uint32_t qd[8];
        load_qdesc(J, q, qd);
        uint64_t b1 = ~0ull, b2 = ~0ull;
        auto consider = [&](int j, uint32_t order) {
            if (blocked_at(j, q)) return;
            const uint64_t key = make_key(hamming32(qd, J.desc + (size_t)j * 32), order, j, g_kps[j].octave);
            if (key < b1) {
                b2 = b1;
                b1 = key;
            } else if (key < b2) {
                b2 = key;
            }
        };
        if (J.cand_ptr) {
            const int b = J.cand_ptr[2 * q], e = J.cand_ptr[2 * q + 1];
            for (int p = b + lane; p < e; p += 64) consider(J.cand[p], (uint32_t)(p - b));
        } else {
            const Window w = make_window(J, Q);
            for_window(J, w, [&](int j, int c) {
                const uint32_t o = window_accept(J, w, Q, j, c);
                if (o != ~0u) consider(j, o);
            });
        }
        const uint64_t best = wave_min_u64(b1);
        if (b1 == best) b1 = b2;  // keys are unique: one lane pops
        const uint64_t second = wave_min_u64(b1);
        return rule(entry_of(best), entry_of(second));
    };
    __syncthreads();
    YGZ_BSTAMP_K(5, 1);
    int pass = 0;
    bool converged = false;
    // the fixed point is reached within nq + 1 passes (query k is final after pass k + 1);
    // max_passes only bounds a broken invariant, reported as status -1
    while (pass < max_passes) {
        const int b = pass & 1;
        int32_t *hb = heads + (b ? n2 : 0), *ho = heads + (b ? 0 : n2);
        head = hb;
        if (pass > 0) {  // link the previous pass's matches per keypoint (hb was cleared last pass)
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int q = tid + kResolveThreads * r;
                if (q < nq) {
                    const int c = choice[q];
                    if (c != kChoiceNone) link[q] = (int16_t)atomicExch(&hb[c], q);
                }
            }
            __syncthreads();
            if (pass == 1) YGZ_BSTAMP_K(5, 6);
        }
        for (int j = tid; j < n; j += kResolveThreads) ho[j] = -1;  // next pass's lists
        int changed = 0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int q = tid + kResolveThreads * r;
            if (qcnt[r] <= 0) continue;  // invalid, past nq, or no candidate: never matches
            uint32_t best = kNoEntry, second = kNoEntry;
            int found = 0;
            const int nk = min(qlist[r], kTopK);
#pragma unroll
            for (int k = 0; k < kTopK; k++) {  // in order, stopping at the decision (fewest instructions)
                if (k >= nk || found >= need) break;
                const uint32_t e = E[r][k];
                if (blocked_at((int)(e & 0xFFFF), q)) continue;
                if (found == 0) best = e;
                else second = e;
                found++;
            }
            for (int k = kTopK; k < qlist[r] && found < need; k++) {  // the listed entries past the registers
                const uint32_t e = entry_of(g_topk[(size_t)q * kTopList + k]);
                if (blocked_at((int)(e & 0xFFFF), q)) continue;
                if (found == 0) best = e;
                else second = e;
                found++;
            }
            if (found < need && qcnt[r] > qlist[r]) {
                rq[atomicAdd(&s_nrq[b], 1)] = (int16_t)q;  // decided below by a wave
                continue;
            }
            const int c = rule(best, second);
            changed |= c != choice[q];
            choice[q] = (uint16_t)c;  // lists are not rebuilt until the next pass: no reader sees this
        }
        if (changed) s_chg[b] = 1;
        __syncthreads();
        if (pass == 1) YGZ_BSTAMP_K(5, 7);
        const int nrq = s_nrq[b];
        if (nrq > 0) {
            changed = 0;
            for (int i = wv; i < nrq; i += kResolveWaves) {
                const int q = rq[i];
                const int c = wave_rescan(q);
                if (lane == 0) {
                    changed |= c != choice[q];
                    choice[q] = (uint16_t)c;
                }
            }
            if (changed) s_chg[b] = 1;
            __syncthreads();
        }
        pass++;
        if (pass == 1) YGZ_BSTAMP_K(5, 3);
        const bool any = s_chg[b] != 0;
        // the parity-(b ^ 1) flags were last read in the previous pass, before this pass's
        // first barrier; the next pass writes them only after its link barrier
        if (tid == 0) s_chg[b ^ 1] = s_nrq[b ^ 1] = 0;
        if (!any) {
            converged = true;
            break;
        }
    }
    YGZ_BSTAMP_K(5, 4);
    if (!converged) {
        if (tid == 0) as_global_mut(J.nmatches)[2] = -1;  // the host reports the error
        return;
    }
    // outputs, each written once (J.train_out / J.nmatches may be page-locked host memory):
    // the rotation check's removals are marked in the spare head buffer first
    int32_t *removed_at = head == heads ? heads + n2 : heads;  // all -1 (cleared in the last pass)
    int matched = 0, bins[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int q = tid + kResolveThreads * r;
        bins[r] = -1;
        if (q >= nq) continue;
        const int c = choice[q];
        if (c == kChoiceNone) continue;
        matched++;
        if (ori) {
            bins[r] = rot_bin(qang[r], tang[c]);
            atomicAdd(&s_rot[bins[r]], 1);
        }
    }
    __syncthreads();
    int removed = 0;
    if (ori) {
        int i1, i2, i3;
        three_maxima(s_rot, i1, i2, i3);
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int bin = bins[r];
            if (bin < 0 || bin == i1 || bin == i2 || bin == i3) continue;
            removed_at[choice[tid + kResolveThreads * r]] = 1;
            removed++;
        }
    }
    // diagnostics: queries whose top-K list the final state exhausts (the serial path's re-scans)
    int nrescan = 0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int q = tid + kResolveThreads * r;
        if (qcnt[r] <= kTopK) continue;
        nrescan += __popc(~blocked_mask(E[r], kTopK, q) & 0xFFu) < need;
    }
    const int net = wave_sum_i(matched - removed), nr = wave_sum_i(nrescan);
    if (lane == 0) s_sum[wv] = net | (nr << 20);
    __syncthreads();
    // train_out[j]: the last query that matched j (the final lists), -2 / -1 where removed
    const auto g_train_out = as_global_mut(J.train_out);
    const auto g_qid = as_global(J.qid);
    if (J.train_out)
        for (int j = tid; j < n; j += kResolveThreads) {
            int last = -1;
            for (int p = head[j]; p >= 0; p = link[p]) last = max(last, p);
            int v = last < 0 ? -1 : (mode == YGZFE_MATCH_BOW && J.qid ? g_qid[last] : last);
            if (removed_at[j] >= 0) v = mode == YGZFE_MATCH_BEST ? -2 : -1;
            g_train_out[j] = v;
        }
    if (tid == 0) {
        int tot = 0, totr = 0;
        for (int k = 0; k < kResolveWaves; k++) {
            tot += s_sum[k] & 0xFFFFF;
            totr += s_sum[k] >> 20;
        }
        const auto g_nm = as_global_mut(J.nmatches);
        g_nm[0] = tot;
        g_nm[1] = totr;
        g_nm[2] = pass;
    }
    YGZ_BSTAMP_K(5, 5);
}

bool match_resolves(int n_train, int nq, int mode, int max_passes) {
    return max_passes > 0 && mode != YGZFE_MATCH_INIT && resolve_fits(n_train, nq);
}

bool resolve_fits(int n_train, int nq) {
    return nq <= 4 * kResolveThreads && n_train <= 65533 && resolve_lds_bytes(n_train, nq) <= 65536;
}

hipError_t launch_match(const MatchJob &J, int mode, int th_dist, int check_ori, float nnratio, int max_passes,
                        hipStream_t st) {
    if (J.nq > 0)
        hipLaunchKernelGGL(k_match_topk, dim3((J.nq + kTopkWaves - 1) / kTopkWaves), dim3(64 * kTopkWaves), 0, st, J);
    const int n = J.n_train, nq = J.nq;
    const int stage_kv = (int)staged_kp_fits(n, mode);
    // INIT's skip state is a distance and a re-match unmatches the previous query: serial only
    const int R = nq <= kResolveThreads ? 1 : nq <= 2 * kResolveThreads ? 2 : 4;
    if (match_resolves(n, nq, mode, max_passes)) {
        auto k = R == 1 ? k_match_resolve<1> : R == 2 ? k_match_resolve<2> : k_match_resolve<4>;
        hipLaunchKernelGGL(k, dim3(1), dim3(kResolveThreads), resolve_lds_bytes(n, nq), st, J, mode, th_dist,
                           check_ori, nnratio, nq + 2);
    } else {
        hipLaunchKernelGGL(k_match_replay, dim3(1), dim3(64), replay_lds_bytes(n, mode), st, J, mode, th_dist,
                           check_ori, nnratio, stage_kv);
    }
    return hipGetLastError();
}

}  // namespace ygzfe
