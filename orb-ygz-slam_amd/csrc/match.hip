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

constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS (Frame.h:27-28)
constexpr int kTopK = 8;
constexpr int kHisto = 30;                       // ORBmatcher::HISTO_LENGTH (ORBmatcher.cc:38)

// Frame::PosInGrid (Frame.cc:483-493): std::round(float), cell -1 when outside
__global__ __launch_bounds__(256) void k_match_cells(const ygzfe_kp *__restrict__ kps, int n, float min_x,
                                                     float min_y, float inv_w, float inv_h,
                                                     int32_t *__restrict__ cell) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int px = (int)__builtin_roundf((kps[i].x - min_x) * inv_w);
    const int py = (int)__builtin_roundf((kps[i].y - min_y) * inv_h);
    cell[i] = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : (px << 8) | py;
}

hipError_t launch_match_cells(const ygzfe_kp *kps, int n, float min_x, float min_y, float inv_w, float inv_h,
                              int32_t *cell, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_match_cells, dim3((n + 255) / 256), dim3(256), 0, st, kps, n, min_x, min_y, inv_w, inv_h,
                       cell);
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

// Is train keypoint j in the query's candidate list (window + level + stereo)?
// Returns its candidate-order key (cell-major, then index) or ~0.
__device__ __forceinline__ uint32_t window_order(const MatchJob &J, const Window &w, const ygzfe_match_query &q,
                                                 int j) {
    const int c = J.cell[j];
    if (c < 0) return ~0u;
    const int ix = c >> 8, iy = c & 0xFF;
    if (ix < w.cx0 || ix > w.cx1 || iy < w.cy0 || iy > w.cy1) return ~0u;
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
    return ((uint32_t)(ix * kGridRows + iy) << 16) | (uint32_t)j;  // GetFeaturesInArea order
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
        if (w.cx0 <= w.cx1)
            for (int j = lane; j < J.n_train; j += 64) {
                const uint32_t o = window_order(J, w, Q, j);
                if (o != ~0u) consider(j, o);
            }
    }
}

__device__ __forceinline__ void load_qdesc(const MatchJob &J, int q, uint32_t qd[8]) {
    const int id = J.qid ? J.qid[q] : q;
    const uint4 *p = reinterpret_cast<const uint4 *>(J.qdesc + (size_t)id * 32);
    const uint4 a = p[0], b = p[1];
    qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
    qd[4] = b.x; qd[5] = b.y; qd[6] = b.z; qd[7] = b.w;
}

// wave-merge of the lanes' sorted lists: the K smallest keys, ascending, in lanes 0..K-1
__device__ __forceinline__ uint64_t merge_topk(uint64_t L[kTopK]) {
    const int lane = threadIdx.x & 63;
    uint64_t mine = ~0ull;
#pragma unroll
    for (int e = 0; e < kTopK; e++) {
        const uint64_t m = wave_min_u64(L[0]);
        if (lane == e) mine = m;
        if (L[0] == m && m != ~0ull) {  // keys are unique: one lane pops
#pragma unroll
            for (int k = 0; k + 1 < kTopK; k++) L[k] = L[k + 1];
            L[kTopK - 1] = ~0ull;
        }
    }
    return mine;
}

__global__ __launch_bounds__(256) void k_match_topk(const MatchJob *__restrict__ jobs, int max_q) {
    const MatchJob &J = jobs[blockIdx.y];
    const int q = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (q >= J.nq) return;
    const int lane = threadIdx.x & 63;
    const ygzfe_match_query Q = J.q[q];
    if (!(Q.flags & YGZFE_MQ_VALID)) {
        if (lane == 0) J.ncand[q] = 0;
        return;
    }
    uint32_t qd[8];
    load_qdesc(J, q, qd);
    uint64_t L[kTopK];
    int count;
    scan_query(J, q, Q, qd, [](int, int) { return false; }, L, count);
    count = wave_sum_i(count);
    const uint64_t mine = merge_topk(L);
    if (lane < kTopK) J.topk[(size_t)q * kTopK + lane] = mine;
    if (lane == 0) J.ncand[q] = count;
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

// ---------------------------------------------------------------------------
// k_match_resolve: the same sequential result, found in parallel.
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
// queries whose decisions feed each other) + 1 passes (4-5 on the test scenes).
// A pass: the matched queries are linked per train keypoint in LDS (atomic
// exchange into head[j]); each query walks its top-K entries in order and, for
// each, the entry's list for the latest chooser before it.  A pass that changes
// no decision ends the loop.
//
// A query whose skips exhaust its top-K entries of a longer candidate list needs
// its whole candidate list under the current state (the serial path's re-scan).
// Once the passes settle with such queries present, the train keypoints are
// bucketed by grid cell in LDS (counting sort) and the passes continue with
// those queries scanning their GetFeaturesInArea cells (or BoW node list) in
// their own thread.  If the pass budget runs out the status word hands the job
// to k_match_replay (the serial replay from scratch); otherwise the outputs are
// written here and k_match_replay exits on entry.
// ---------------------------------------------------------------------------
constexpr int kResolveThreads = 1024;
constexpr int kGridCells = kGridCols * kGridRows;  // 3072 = 3 per thread
static_assert(kGridCells == 3 * kResolveThreads, "cell scan: 3 cells per thread");
__host__ __device__ __forceinline__ size_t resolve_lds_bytes(int n, int nq) {
    return 4 * (size_t)n + 8 * (size_t)nq + 4 * (size_t)kGridCells + 2 * (size_t)((n + 1) & ~1) +
           (size_t)((nq + 3) & ~3);
}

__global__ __launch_bounds__(kResolveThreads) void k_match_resolve(const MatchJob *__restrict__ jobs, int mode,
                                                                   int th_dist, int check_ori, float nnratio,
                                                                   int max_passes) {
    extern __shared__ uint8_t lds[];
    const MatchJob J = jobs[blockIdx.x];
    const int tid = threadIdx.x, n = J.n_train, nq = J.nq;
    int32_t *head = reinterpret_cast<int32_t *>(lds);       // [n]  latest linked chooser of j
    int32_t *link = head + n;                               // [nq] next chooser of the same j
    int32_t *choice = link + nq;                            // [nq] matched train index, -1 none, -2 re-scan
    int32_t *cend = choice + nq;                            // [cells] end of each cell's keypoints in sidx
    uint16_t *sidx = reinterpret_cast<uint16_t *>(cend + kGridCells);             // [n] keypoints by cell
    uint8_t *qbl = reinterpret_cast<uint8_t *>(sidx + ((n + 1) & ~1));            // [nq] q's match blocks
    __shared__ int s_rot[kHisto + 2];
    __shared__ int s_sum[16];
    const auto g_topk = as_global(J.topk);
    const auto g_ncand = as_global(J.ncand);
    const auto g_q = as_global(J.q);
    const auto g_blocked0 = as_global(J.blocked0);
    const auto g_kps = as_global(J.kps);
    const int need = mode == YGZFE_MATCH_BEST ? 1 : 2;
    for (int q = tid; q < nq; q += kResolveThreads) {
        choice[q] = -1;
        qbl[q] = mode == YGZFE_MATCH_BOW ? 1 : ((g_q[q].flags & YGZFE_MQ_BLOCKS) ? 1 : 0);
    }
    for (int j = tid; j < n; j += kResolveThreads) head[j] = -1;
    // the state query q sees keypoint j in: set by the latest chooser before q
    auto blocked_at = [&](int j, int q) -> bool {
        int last = -1;
        for (int p = head[j]; p >= 0; p = link[p])
            if (p < q && p > last) last = p;
        return last >= 0 ? qbl[last] != 0 : (J.blocked0 ? g_blocked0[j] != 0 : false);
    };
    // the serial path's re-scan, in one thread: the whole candidate list under the state
    auto rescan = [&](int q, uint64_t &best, uint64_t &second) {
        const ygzfe_match_query Q = J.q[q];
        uint32_t qd[8];
        load_qdesc(J, q, qd);
        best = second = ~0ull;
        auto consider = [&](int j, uint32_t order) {
            if (blocked_at(j, q)) return;
            const uint64_t key = make_key(hamming32(qd, J.desc + (size_t)j * 32), order, j, g_kps[j].octave);
            if (key < best) {
                second = best;
                best = key;
            } else if (key < second) {
                second = key;
            }
        };
        if (J.cand_ptr) {
            const int b = J.cand_ptr[2 * q], e = J.cand_ptr[2 * q + 1];
            for (int p = b; p < e; p++) consider(J.cand[p], (uint32_t)(p - b));
        } else {
            const Window w = make_window(J, Q);
            for (int ix = w.cx0; ix <= w.cx1; ix++)
                for (int iy = w.cy0; iy <= w.cy1; iy++) {
                    const int c = ix * kGridRows + iy;
                    for (int t = c ? cend[c - 1] : 0; t < cend[c]; t++) {
                        const int j = sidx[t];
                        const uint32_t o = window_order(J, w, Q, j);
                        if (o != ~0u) consider(j, o);
                    }
                }
        }
    };
    // query q's decision against the chooser lists of the previous pass
    auto decide = [&](int q, bool full) -> int {
        const int flags = g_q[q].flags, cnt = g_ncand[q];
        if (!(flags & YGZFE_MQ_VALID) || cnt == 0) return -1;
        const int nk = min(cnt, kTopK);
        uint64_t best = ~0ull, second = ~0ull;
        int found = 0;
        for (int k = 0; k < nk && found < need; k++) {
            const uint64_t e = g_topk[(size_t)q * kTopK + k];
            if (blocked_at(key_train(e), q)) continue;
            if (found == 0) best = e;
            else second = e;
            found++;
        }
        if (found < need && cnt > kTopK) {
            if (!full) return -2;
            rescan(q, best, second);
        }
        const bool has1 = best != ~0ull, has2 = second != ~0ull;
        const int bd = has1 ? (int)(best >> 52) : 256, sdist = has2 ? (int)(second >> 52) : 256;
        bool ok;
        if (mode == YGZFE_MATCH_BEST) {
            ok = has1 && bd <= th_dist;
        } else if (mode == YGZFE_MATCH_RATIO) {
            const int bl = has1 ? key_octave(best) : -1, sl = has2 ? key_octave(second) : -1;
            ok = has1 && bd <= 100 && !(bl == sl && bd > nnratio * sdist);
        } else {  // BOW
            ok = has1 && bd <= 50 && (float)bd < nnratio * (float)sdist;
        }
        return ok ? key_train(best) : -1;
    };
    // keypoints bucketed by cell (cell-major ix * rows + iy), for the re-scans
    auto build_cells = [&]() {
        for (int c = tid; c < kGridCells; c += kResolveThreads) cend[c] = 0;
        __syncthreads();
        for (int j = tid; j < n; j += kResolveThreads) {
            const int c = J.cell[j];
            if (c >= 0) atomicAdd(&cend[(c >> 8) * kGridRows + (c & 0xFF)], 1);
        }
        __syncthreads();
        const int c0 = 3 * tid;
        const int a0 = cend[c0], a1 = cend[c0 + 1], a2 = cend[c0 + 2], sum = a0 + a1 + a2;
        const int lane = tid & 63, wv = tid >> 6;
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
        const int start = base + incl - sum;  // exclusive start of cell c0
        cend[c0] = start;                     // starts for now; the scatter advances them to ends
        cend[c0 + 1] = start + a0;
        cend[c0 + 2] = start + a0 + a1;
        __syncthreads();
        for (int j = tid; j < n; j += kResolveThreads) {
            const int c = J.cell[j];
            if (c >= 0) sidx[atomicAdd(&cend[(c >> 8) * kGridRows + (c & 0xFF)], 1)] = (uint16_t)j;
        }
        __syncthreads();
    };
    __syncthreads();
    int pass = 0;
    bool converged = false, full = false;
    while (pass < max_passes) {
        if (pass > 0) {  // link the previous pass's matches per keypoint
            for (int j = tid; j < n; j += kResolveThreads) head[j] = -1;
            __syncthreads();
            for (int q = tid; q < nq; q += kResolveThreads) {
                const int c = choice[q];
                if (c >= 0) link[q] = atomicExch(&head[c], q);
            }
            __syncthreads();
        }
        int changed = 0, pending = 0;
        for (int q = tid; q < nq; q += kResolveThreads) {
            const int c = decide(q, full);
            changed |= c != choice[q];
            pending |= c == -2;
            choice[q] = c;  // lists are not rebuilt until the next pass: no reader sees this
        }
        pass++;
        if (!__syncthreads_or(changed)) {
            if (!__syncthreads_or(pending)) {
                converged = true;
                break;
            }
            build_cells();  // settled with re-scans outstanding: the next passes do them
            full = true;
        }
    }
    if (!converged) {
        if (tid == 0) as_global_mut(J.nmatches)[2] = -1;  // k_match_replay takes the job
        return;
    }
    // outputs: train_out[j] = the last query that matched j
    const auto g_train_out = as_global_mut(J.train_out);
    const auto g_qid = as_global(J.qid);
    for (int j = tid; j < n; j += kResolveThreads) {
        int last = -1;
        for (int p = head[j]; p >= 0; p = link[p]) last = max(last, p);
        if (J.train_out) g_train_out[j] = last < 0 ? -1 : (mode == YGZFE_MATCH_BOW && J.qid ? g_qid[last] : last);
    }
    if (tid < kHisto + 2) s_rot[tid] = 0;
    __syncthreads();
    int matched = 0, nrescan = 0;
    const bool ori = check_ori && mode != YGZFE_MATCH_RATIO;
    for (int q = tid; q < nq; q += kResolveThreads) {
        const int c = choice[q];
        if (c < 0) continue;
        matched++;
        if (ori) atomicAdd(&s_rot[rot_bin(g_q[q].angle, g_kps[c].angle)], 1);
    }
    __syncthreads();
    int removed = 0;
    if (ori) {
        int i1, i2, i3;
        three_maxima(s_rot, i1, i2, i3);
        for (int q = tid; q < nq; q += kResolveThreads) {
            const int c = choice[q];
            if (c < 0) continue;
            const int bin = rot_bin(g_q[q].angle, g_kps[c].angle);
            if (bin == i1 || bin == i2 || bin == i3) continue;
            if (J.train_out) g_train_out[c] = mode == YGZFE_MATCH_BEST ? -2 : -1;
            removed++;
        }
    }
    if (full)  // diagnostics: the queries whose top-K list the final state exhausts
        for (int q = tid; q < nq; q += kResolveThreads) {
            const int cnt = g_ncand[q];
            if (!(g_q[q].flags & YGZFE_MQ_VALID) || cnt <= kTopK) continue;
            int found = 0;
            for (int k = 0; k < kTopK && found < need; k++)
                found += !blocked_at(key_train(g_topk[(size_t)q * kTopK + k]), q);
            nrescan += found < need;
        }
    const int net = wave_sum_i(matched - removed), nr = wave_sum_i(nrescan);
    __syncthreads();  // s_sum reused
    if ((tid & 63) == 0) s_sum[tid >> 6] = net | (nr << 20);
    __syncthreads();
    if (tid == 0) {
        int tot = 0, totr = 0;
        for (int k = 0; k < kResolveThreads / 64; k++) {
            tot += s_sum[k] & 0xFFFFF;
            totr += s_sum[k] >> 20;
        }
        const auto g_nm = as_global_mut(J.nmatches);
        g_nm[0] = tot;
        g_nm[1] = totr;
        g_nm[2] = pass;
    }
}

__global__ __launch_bounds__(64) void k_match_replay(const MatchJob *__restrict__ jobs, int mode, int th_dist,
                                                     int check_ori, float nnratio, int stage_kv, int resolved_first) {
    extern __shared__ uint8_t lds[];
    // the job's fields in registers: the loop's global stores could otherwise alias the
    // job record and force a reload of every field (a scalar-load latency per query)
    const MatchJob J = jobs[blockIdx.x];
    if (resolved_first && as_global(J.nmatches)[2] >= 0) return;  // k_match_resolve wrote the outputs
    const auto g_train_out = as_global_mut(J.train_out), g_query_out = as_global_mut(J.query_out);
    const auto g_pushes = as_global_mut(J.pushes), g_nmatches = as_global_mut(J.nmatches);
    const auto g_q = as_global(J.q);
    const auto g_ncand = as_global(J.ncand);
    const auto g_topk = as_global(J.topk);
    const auto g_kps = as_global(J.kps);
    const auto g_blocked0 = as_global(J.blocked0);
    const auto g_qid = as_global(J.qid);
    const int lane = threadIdx.x;
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
    __syncthreads();
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
            r.flags = g_q[q].flags;
            r.angle = g_q[q].angle;
            r.cnt = g_ncand[q];
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            const auto t = (gptr_t<v4u>)(J.topk + (size_t)q * kTopK);
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
        __threadfence_block();
        __syncthreads();  // the pushes are visible to every lane
        for (int p = lane; p < npush; p += 64) atomicAdd(&rot_count[g_pushes[p] >> 24], 1);
        __syncthreads();
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

hipError_t launch_match(const MatchJob *d_jobs, int njobs, int max_q, int max_train, int mode, int th_dist,
                        int check_ori, float nnratio, int max_passes, hipStream_t st) {
    if (njobs <= 0) return hipSuccess;
    if (max_q > 0)
        hipLaunchKernelGGL(k_match_topk, dim3((max_q + 3) / 4, njobs), dim3(256), 0, st, d_jobs, max_q);
    // INIT's skip state is a distance, and a re-match unmatches the previous query: serial only
    const size_t rl = resolve_lds_bytes(max_train, max_q);
    const bool resolve = max_passes > 0 && mode != YGZFE_MATCH_INIT && rl <= 65536;
    if (resolve)
        hipLaunchKernelGGL(k_match_resolve, dim3(njobs), dim3(kResolveThreads), rl, st, d_jobs, mode, th_dist,
                           check_ori, nnratio, max_passes);
    const size_t lds = replay_lds_base(max_train, mode) +
                       (staged_kp_fits(max_train, mode) ? 5 * (size_t)((max_train + 3) & ~3) : 0) + 64;
    hipLaunchKernelGGL(k_match_replay, dim3(njobs), dim3(64), lds, st, d_jobs, mode, th_dist, check_ori, nnratio,
                       (int)staged_kp_fits(max_train, mode), (int)resolve);
    return hipGetLastError();
}

}  // namespace ygzfe
