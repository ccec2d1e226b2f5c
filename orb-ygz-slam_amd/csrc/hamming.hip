// hamming.hip — ORBmatcher Hamming search on gfx950.
//
// DescriptorDistance (ORBmatcher.cc:1507-1523) = popcount(a XOR b) over 256 bits.
// Dense best/second-best: the inner candidate loops of SearchByProjection /
// SearchForInitialization / SearchByBoW (ORBmatcher.cc:43-126,375-478,1218-1350)
// keep `dist < bestDist` (first index wins on ties) and the second best.
// A query descriptor lives in 8 VGPRs of its lane; train descriptors are
// staged through LDS in 1024-row tiles (32 KiB) shared by the workgroup and
// read as broadcasts, 4 rows per step.
#include "common.hpp"

namespace ygzfe {

constexpr int kHamTile = 1024;

__device__ __forceinline__ void best2_update(int d, int j, int &b1, int &b2, int &bi) {
    if (d < b1) { b2 = b1; b1 = d; bi = j; }
    else if (d < b2) b2 = d;
}

__device__ __forceinline__ int ham256(const uint32_t a[8], const uint4 &v0, const uint4 &v1) {
    int d = __popc(a[0] ^ v0.x);
    d = __popc(a[1] ^ v0.y) + d;
    d = __popc(a[2] ^ v0.z) + d;
    d = __popc(a[3] ^ v0.w) + d;
    d = __popc(a[4] ^ v1.x) + d;
    d = __popc(a[5] ^ v1.y) + d;
    d = __popc(a[6] ^ v1.z) + d;
    d = __popc(a[7] ^ v1.w) + d;
    return d;
}

// A workgroup serves 64 queries (one per lane); its 4 waves scan the four
// contiguous quarters of the train set (4x the waves of a query-per-thread
// layout), then the partial results merge in train order: best = smallest b1,
// earliest quarter on ties (so the first minimum index wins, as in the
// sequential loop); second = min(winner's b2, the other quarters' b1) -- the
// sequential b2 is the smallest distance over all trains but the winner.
constexpr int kQPB = 64;

__device__ void hamming_block(const uint8_t *__restrict__ q, int nq, const uint8_t *__restrict__ t, int nt,
                              int32_t *__restrict__ bi_out, int32_t *__restrict__ bd_out,
                              int32_t *__restrict__ sd_out, int qblock) {
    __shared__ uint4 s_t[kHamTile * 2];
    __shared__ int s_part[4][3][kQPB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int qi = qblock * kQPB + lane;
    uint32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (qi < nq) {
        const uint4 *qp = reinterpret_cast<const uint4 *>(q + (size_t)qi * 32);
        const uint4 u0 = qp[0], u1 = qp[1];
        a[0] = u0.x; a[1] = u0.y; a[2] = u0.z; a[3] = u0.w;
        a[4] = u1.x; a[5] = u1.y; a[6] = u1.z; a[7] = u1.w;
    }
    int b1 = 257, b2 = 257, bi = -1;
    for (int t0 = 0; t0 < nt; t0 += kHamTile) {
        const int m = min(kHamTile, nt - t0);
        __syncthreads();
        const uint4 *tp = reinterpret_cast<const uint4 *>(t + (size_t)t0 * 32);
        for (int i = threadIdx.x; i < m * 2; i += blockDim.x) s_t[i] = tp[i];
        __syncthreads();
        const int qlen = (m + 3) >> 2, jb = wave * qlen, je = min(m, jb + qlen);  // this wave's quarter
        int j = jb;
        for (; j + 4 <= je; j += 4) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = s_t[2 * j + u];
#pragma unroll
            for (int u = 0; u < 4; u++) best2_update(ham256(a, v[2 * u], v[2 * u + 1]), t0 + j + u, b1, b2, bi);
        }
        for (; j < je; j++) best2_update(ham256(a, s_t[2 * j], s_t[2 * j + 1]), t0 + j, b1, b2, bi);
        // merge this tile's quarters in order into wave 0's running result
        s_part[wave][0][lane] = b1;
        s_part[wave][1][lane] = b2;
        s_part[wave][2][lane] = bi;
        __syncthreads();
        if (wave == 0) {
#pragma unroll
            for (int w = 1; w < 4; w++) {
                const int c1 = s_part[w][0][lane], c2 = s_part[w][1][lane], ci = s_part[w][2][lane];
                if (c1 < b1) { b2 = min(b1, c2); b1 = c1; bi = ci; }
                else b2 = min(b2, c1);
            }
        } else {
            b1 = 257; b2 = 257; bi = -1;
        }
    }
    if (wave == 0 && qi < nq) {
        bi_out[qi] = bi;
        bd_out[qi] = b1;
        sd_out[qi] = b2;
    }
}

__global__ __launch_bounds__(256) void k_hamming_best2(const uint8_t *__restrict__ q, int nq,
                                                       const uint8_t *__restrict__ t, int nt,
                                                       int32_t *__restrict__ bi, int32_t *__restrict__ bd,
                                                       int32_t *__restrict__ sd) {
    hamming_block(q, nq, t, nt, bi, bd, sd, blockIdx.x);
}

// batched: pair p matches the descriptors of frame qframe[p] against frame
// tframe[p] of a batch (rows [0, counts[f]) of a [F][row_cap][32] array);
// outputs at [p][row_cap].
__global__ __launch_bounds__(256) void k_hamming_best2_pairs(const uint8_t *__restrict__ desc,
                                                             const int32_t *__restrict__ counts, int row_cap,
                                                             const int32_t *__restrict__ qframe,
                                                             const int32_t *__restrict__ tframe,
                                                             int32_t *__restrict__ bi, int32_t *__restrict__ bd,
                                                             int32_t *__restrict__ sd) {
    const int p = blockIdx.y;
    const int qf = qframe[p], tf = tframe[p];
    const int nq = counts[qf], nt = counts[tf];
    if ((int)(blockIdx.x * kQPB) >= nq) return;
    hamming_block(desc + (size_t)qf * row_cap * 32, nq, desc + (size_t)tf * row_cap * 32, nt,
                  bi + (size_t)p * row_cap, bd + (size_t)p * row_cap, sd + (size_t)p * row_cap, blockIdx.x);
}

// CSR candidate distances: dist[k] for k in [row_ptr[i], row_ptr[i+1]) of query i.
__global__ __launch_bounds__(256) void k_hamming_csr(const uint8_t *__restrict__ q, int nq,
                                                     const uint8_t *__restrict__ t,
                                                     const int32_t *__restrict__ row_ptr,
                                                     const int32_t *__restrict__ cand, int32_t *__restrict__ dist) {
    const int i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= nq) return;
    const uint4 *qp = reinterpret_cast<const uint4 *>(q + (size_t)i * 32);
    const uint4 u0 = qp[0], u1 = qp[1];
    for (int k = row_ptr[i] + lane; k < row_ptr[i + 1]; k += 64) {
        const uint4 *tp = reinterpret_cast<const uint4 *>(t + (size_t)cand[k] * 32);
        const uint4 v0 = tp[0], v1 = tp[1];
        dist[k] = __popc(u0.x ^ v0.x) + __popc(u0.y ^ v0.y) + __popc(u0.z ^ v0.z) + __popc(u0.w ^ v0.w) +
                  __popc(u1.x ^ v1.x) + __popc(u1.y ^ v1.y) + __popc(u1.z ^ v1.z) + __popc(u1.w ^ v1.w);
    }
}

hipError_t launch_hamming_best2(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *bi, int32_t *bd,
                                int32_t *sd, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_hamming_best2, dim3((nq + kQPB - 1) / kQPB), dim3(256), 0, st, q, nq, t, nt, bi, bd, sd);
    return hipGetLastError();
}

hipError_t launch_hamming_best2_pairs(const uint8_t *desc, const int32_t *counts, int row_cap, int npairs,
                                      const int32_t *qframe, const int32_t *tframe, int32_t *bi, int32_t *bd,
                                      int32_t *sd, hipStream_t st) {
    if (npairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_hamming_best2_pairs, dim3((row_cap + kQPB - 1) / kQPB, npairs), dim3(256), 0, st,
                       desc, counts,
                       row_cap, qframe, tframe, bi, bd, sd);
    return hipGetLastError();
}

hipError_t launch_hamming_csr(const uint8_t *q, int nq, const uint8_t *t, const int32_t *row_ptr,
                              const int32_t *cand, int32_t *dist, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_hamming_csr, dim3((nq + 3) / 4), dim3(256), 0, st, q, nq, t, row_ptr, cand, dist);
    return hipGetLastError();
}

}  // namespace ygzfe
