// bow.hip — DBoW2 TemplatedVocabulary::transform for Frame::ComputeBoW
// (Frame.cc:495-500) on gfx950.
//
// Vocabulary in HBM (VocabDev): per node its children as a CSR slot range
// [child_ptr[n], child_ptr[n+1]) and, per slot, the child's node id and its
// 32-byte descriptor stored in slot order, so the k children of a node are k
// consecutive 32-byte rows (one coalesced read per level).  word_id / weight
// (double, DBoW2's WordValue) per node.
//
// k_bow_transform: 16 lanes per descriptor (16 descriptors per 256-thread
// workgroup, blockIdx.y = frame).  Per level the lanes take one child each,
// key = (FORB::distance << 8) | child slot, and a 16-lane min gives the first
// strict minimum — TemplatedVocabulary.h:1259-1270's `d < best_d` from the
// first child.  The descent stops at a node without children (isLeaf());
// the node reached at level L - levelsup is the FeatureVector node.
//
// k_bow_vectors: one 1024-thread workgroup per frame builds the BowVector and
// FeatureVector of TemplatedVocabulary::transform(features, v, fv, levelsup)
// (:1150-1212): bitonic sort of (word, feature) keys in LDS; per word run the
// value is w folded c times in feature order (addWeight; addIfNotExist keeps
// w); DotProduct scoring divides TF / TF_IDF values by v.size(); the others
// normalise (BowVector.cpp:62-84) with the norm summed sequentially in word
// order, as std::map iteration does.  The FeatureVector is the (node,
// feature)-sorted list of the same features.
#include "common.hpp"
#include "kernels.hpp"

namespace ygzfe {

constexpr int kBowLanes = 16;

__global__ __launch_bounds__(256) void k_bow_transform(VocabDev V, const uint8_t *__restrict__ desc,
                                                       size_t desc_pitch, const int *__restrict__ counts,
                                                       int n_static, int levelsup, int32_t *__restrict__ word_out,
                                                       double *__restrict__ weight_out,
                                                       int32_t *__restrict__ nid_out, size_t out_pitch) {
    const int f = blockIdx.y;
    const int n = counts ? counts[f] : n_static;
    const int i = blockIdx.x * (256 / kBowLanes) + (threadIdx.x / kBowLanes);
    const int sub = threadIdx.x & (kBowLanes - 1);
    if (i >= n) return;  // whole 16-lane group
    const uint4 *fp = (const uint4 *)(desc + (size_t)f * desc_pitch + (size_t)i * 32);
    const uint4 a0 = fp[0], a1 = fp[1];
    const int nid_level = V.L - levelsup;
    int nid = 0;
    int node = 0, level = 0;
    for (int guard = 0; guard < V.n_nodes; guard++) {
        const int b = V.child_ptr[node], e = V.child_ptr[node + 1];
        if (e == b) break;  // isLeaf()
        uint32_t key = 0xFFFFFFFFu;
        for (int c = sub; c < e - b; c += kBowLanes) {
            const uint4 *dp = (const uint4 *)(V.slot_desc + (size_t)(b + c) * 32);
            const uint4 b0 = dp[0], b1 = dp[1];
            const int d = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                          __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
            key = min(key, ((uint32_t)d << 8) | (uint32_t)c);
        }
#pragma unroll
        for (int o = kBowLanes / 2; o >= 1; o >>= 1) key = min(key, (uint32_t)__shfl_xor((int)key, o, 64));
        node = V.slot_node[b + (int)(key & 0xFFu)];
        ++level;
        if (level == nid_level) nid = node;
    }
    if (sub == 0) {
        const size_t o = (size_t)f * out_pitch + i;
        word_out[o] = V.word_id[node];
        weight_out[o] = V.weight[node];
        nid_out[o] = nid;
    }
}

hipError_t launch_bow_transform(const VocabDev &V, const uint8_t *desc, size_t desc_pitch, const int *counts,
                                int n_max, int n_frames, int levelsup, int32_t *word, double *weight, int32_t *nid,
                                size_t out_pitch, hipStream_t st) {
    if (n_max <= 0 || n_frames <= 0) return hipSuccess;
    const int per = 256 / kBowLanes;
    hipLaunchKernelGGL(k_bow_transform, dim3((n_max + per - 1) / per, n_frames), dim3(256), 0, st, V, desc,
                       desc_pitch, counts, n_max, levelsup, word, weight, nid, out_pitch);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
constexpr int kBowSortMax = kBowMaxFeatures;  // keys sorted in LDS per frame (64 KB)

__device__ void bow_bitonic(uint64_t *s, int P) {
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < P; t += blockDim.x) {
                const int p = t ^ j;
                if (p > t) {
                    const uint64_t a = s[t], b = s[p];
                    const bool up = (t & k) == 0;
                    if ((a > b) == up) {
                        s[t] = b;
                        s[p] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// The same sort for P <= blockDim.x (one key per thread, the usual frame): the key stays in
// a register; stages whose partner lies in the same wave (j < 64) exchange by lane
// shuffles with no barrier, the others through LDS (two barriers).  Same network, same
// result as bow_bitonic.
__device__ void bow_bitonic_reg(uint64_t *s, int P) {
    const int t = threadIdx.x;
    uint64_t key = t < P ? s[t] : ~0ull;
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            uint64_t b;
            if (j >= 64) {
                __syncthreads();  // the previous LDS stage's reads are done
                if (t < P) s[t] = key;
                __syncthreads();
                b = t < P ? s[t ^ j] : ~0ull;
            } else {
                const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)key, j, 64);
                const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(key >> 32), j, 64);
                b = ((uint64_t)hi << 32) | lo;
            }
            const bool up = (t & k) == 0, lower = t < (t ^ j);
            key = (lower == up) ? (key < b ? key : b) : (key < b ? b : key);
        }
    __syncthreads();
    if (t < P) s[t] = key;
    __syncthreads();
}

// exclusive scan of one int per thread over the workgroup (1024 threads)
__device__ int bow_block_scan(int v, int *s_tmp, int *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_tmp[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int w = 0; w < nw; w++) {
            const int t = s_tmp[w];
            s_tmp[w] = acc;
            acc += t;
        }
        s_tmp[nw] = acc;
    }
    __syncthreads();
    const int r = s_tmp[wave] + x - v;
    *total = s_tmp[nw];
    __syncthreads();
    return r;
}

// Two workgroups per frame: even blocks the BowVector, odd blocks the FeatureVector (they
// share nothing but the inputs, so the FeatureVector's sort runs beside the BowVector's
// sort, fold and ordered norm instead of after them).
__global__ __launch_bounds__(1024) void k_bow_vectors(const int *__restrict__ counts, int n_static,
                                                      const int32_t *__restrict__ word_in,
                                                      const double *__restrict__ weight_in,
                                                      const int32_t *__restrict__ nid_in, size_t in_pitch,
                                                      int weighting, int scoring, int32_t *__restrict__ bow_words,
                                                      double *__restrict__ bow_values, int *__restrict__ n_words,
                                                      int32_t *__restrict__ fv_nodes, int32_t *__restrict__ fv_feats,
                                                      int *__restrict__ n_fv, size_t out_pitch) {
    __shared__ uint64_t s_key[kBowSortMax];
    __shared__ int s_tmp[17];
    __shared__ double s_norm;
    const int f = blockIdx.x >> 1;
    const bool feature_vector = blockIdx.x & 1;
    const int n = counts ? counts[f] : n_static;
    const int32_t *wi = word_in + (size_t)f * in_pitch;
    const double *wv = weight_in + (size_t)f * in_pitch;
    const int32_t *ni = nid_in + (size_t)f * in_pitch;
    int P = 1;
    while (P < n) P <<= 1;
    if (feature_vector) {
        // FeatureVector: (node, feature) in map order, of the features that are not stopped
        int32_t *fn = fv_nodes + (size_t)f * out_pitch;
        int32_t *ff = fv_feats + (size_t)f * out_pitch;
        int m = 0;
        for (int t = threadIdx.x; t < P; t += blockDim.x) {
            const bool ok = t < n && wv[t] > 0;
            m += ok;
            s_key[t] = ok ? (((uint64_t)(uint32_t)ni[t] << 32) | (uint32_t)t) : ~0ull;
        }
        int m_total;
        (void)bow_block_scan(m, s_tmp, &m_total);
        if (P <= (int)blockDim.x) bow_bitonic_reg(s_key, P);
        else bow_bitonic(s_key, P);
        for (int j = threadIdx.x; j < m_total; j += blockDim.x) {
            fn[j] = (int32_t)(s_key[j] >> 32);
            ff[j] = (int32_t)(uint32_t)s_key[j];
        }
        if (threadIdx.x == 0) n_fv[f] = m_total;
        return;
    }
    int32_t *bw = bow_words + (size_t)f * out_pitch;
    double *bv = bow_values + (size_t)f * out_pitch;
    // (word, feature) keys of the features that are not stopped (weight > 0)
    for (int t = threadIdx.x; t < P; t += blockDim.x)
        s_key[t] = (t < n && wv[t] > 0) ? (((uint64_t)(uint32_t)wi[t] << 32) | (uint32_t)t) : ~0ull;
    __syncthreads();
    if (P <= (int)blockDim.x) bow_bitonic_reg(s_key, P);
    else bow_bitonic(s_key, P);
    const bool tf = weighting == 0 || weighting == 1;  // TF_IDF, TF
    const bool must = scoring != 5;                     // all but DOT_PRODUCT
    const bool l2 = scoring == 1;
    // run heads -> output positions (each thread owns a contiguous chunk of at most
    // kBowSortMax / 1024 keys; their folded values are kept in registers)
    constexpr int kMaxChunk = (kBowSortMax + 1023) / 1024;
    const int chunk = (P + blockDim.x - 1) / blockDim.x;
    const int t0 = threadIdx.x * chunk;
    int heads = 0;
    for (int j = t0; j < t0 + chunk && j < P; j++) {
        const uint64_t k = s_key[j];
        if (k != ~0ull && (j == 0 || (s_key[j - 1] >> 32) != (k >> 32))) heads++;
    }
    int nw_total;
    const int pos0 = bow_block_scan(heads, s_tmp, &nw_total);
    double vals[kMaxChunk];
    int pos = pos0, h = 0;
    for (int j = t0; j < t0 + chunk && j < P; j++) {
        const uint64_t k = s_key[j];
        if (k == ~0ull || (j > 0 && (s_key[j - 1] >> 32) == (k >> 32))) continue;
        const double w = wv[(uint32_t)k];
        double v = w;
        if (tf)
            for (int r = j + 1; r < P && s_key[r] != ~0ull && (s_key[r] >> 32) == (k >> 32); r++) v += w;
        bw[pos] = (int32_t)(k >> 32);
#pragma unroll
        for (int u = 0; u < kMaxChunk; u++)
            if (u == h) vals[u] = v;
        h++;
        pos++;
    }
    __syncthreads();  // every key read: the values go into the sorted keys' LDS
    // the values in LDS (over the keys, no longer read): the norm's ordered sum (one thread,
    // the reference's order) and the scaling read LDS, not global memory
    double *s_val = reinterpret_cast<double *>(s_key);
#pragma unroll
    for (int u = 0; u < kMaxChunk; u++)
        if (u < h) s_val[pos0 + u] = vals[u];
    __syncthreads();
    if (must) {
        if (threadIdx.x == 0) {
            // the sum in word order, as std::map iteration does; the LDS reads of 16 values
            // are issued together ahead of their adds (one LDS latency per 16, not per value)
            double norm = 0.0;
            int j = 0;
            for (; j + 16 <= nw_total; j += 16) {
                double t[16];
#pragma unroll
                for (int u = 0; u < 16; u++) t[u] = s_val[j + u];
#pragma unroll
                for (int u = 0; u < 16; u++) norm += l2 ? t[u] * t[u] : fabs(t[u]);
            }
            for (; j < nw_total; j++) norm += l2 ? s_val[j] * s_val[j] : fabs(s_val[j]);
            if (l2) norm = sqrt(norm);
            s_norm = norm;
        }
        __syncthreads();
        const double norm = s_norm;
        for (int j = threadIdx.x; j < nw_total; j += blockDim.x) bv[j] = norm > 0.0 ? s_val[j] / norm : s_val[j];
    } else {
        const double nd = (double)nw_total;  // DOT_PRODUCT: TF / TF_IDF values divided by v.size()
        for (int j = threadIdx.x; j < nw_total; j += blockDim.x) bv[j] = tf ? s_val[j] / nd : s_val[j];
    }
    if (threadIdx.x == 0) n_words[f] = nw_total;
}

hipError_t launch_bow_vectors(const int *counts, int n_static, int n_frames, const int32_t *word, const double *weight,
                              const int32_t *nid, size_t in_pitch, int weighting, int scoring, int32_t *bow_words,
                              double *bow_values, int *n_words, int32_t *fv_nodes, int32_t *fv_feats, int *n_fv,
                              size_t out_pitch, hipStream_t st) {
    if (n_frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_bow_vectors, dim3(2 * n_frames), dim3(1024), 0, st, counts, n_static, word, weight, nid, in_pitch,
                       weighting, scoring, bow_words, bow_values, n_words, fv_nodes, fv_feats, n_fv, out_pitch);
    return hipGetLastError();
}

}  // namespace ygzfe
