// stereo.hip — Frame::ComputeStereoMatches (Frame.cc:509-682) and
// Frame::ComputeStereoFromRGBD (Frame.cc:684-700) on gfx950.
//
// k_stereo_match: one wave per left keypoint, 4 per workgroup, blockIdx.y =
// stereo pair.  (1) Row-band Hamming: the 64 lanes stride over the right
// keypoints; a right keypoint is a candidate of left row int(vL) when that row
// lies in its band [floor(y - 2 s_o), ceil(y + 2 s_o)] (the reference's
// vRowIndices table, Frame.cc:523-535), its octave is within +-1 and its x in
// [uL - mbf/mb, uL].  Per lane the running key (dist << 16 | iR) keeps the
// smallest distance with the smallest index — the reference's candidate loop
// in iR order with `dist < bestDist` from TH_HIGH — and one wave min merges
// the lanes.  (2) When bestDist < (TH_HIGH + TH_LOW) / 2, the 11 sliding 11x11
// SAD windows at the left octave: lane t (< 121, two per lane) sums one row of
// one window, all in integers (the reference's centred float windows hold
// integers, so every sum is exact); lanes 0..10 add the rows of their window
// and a wave min of (sad << 8 | window) gives the first strict minimum.
// (3) Lane 0 does the parabola fit, disparity and depth in float exactly as
// written (no contraction, IEEE division).
//
// k_stereo_filter: one workgroup per pair applies the median outlier cut
// (Frame.cc:671-681): the median = the (n/2)-th smallest winning SAD, found by
// a two-round 8-bit radix select over LDS histograms; every match with
// SAD >= 1.5f * 1.4f * median is dropped.
#include "common.hpp"
#include "kernels.hpp"

namespace ygzfe {

constexpr int kStereoWaves = 4;

__global__ __launch_bounds__(256) void k_stereo_match(const StereoJob *__restrict__ jobs, StereoLevels lv, float mb,
                                                      float mbf) {
    __shared__ int s_sad[kStereoWaves][128];
    const StereoJob J = jobs[blockIdx.y];
    const int nl = *J.n_left, nr = *J.n_right;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int iL = blockIdx.x * kStereoWaves + wave;
    if (iL >= nl) return;  // wave-uniform
    const ygzfe_kp kpL = J.left_kps[iL];
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int nRows = lv.h[0];
    float out_u = -1.0f, out_d = -1.0f;
    int out_sad = -1;
    const float minD = 0;
    const float maxD = mbf / mb;
    const float minU = uL - maxD, maxU = uL - minD;
    int bestDist = 100;
    int bestIdxR = 0;
    if (vL >= 0.0f && (int)vL < nRows && !(maxU < 0)) {
        const int row = (int)vL;
        const uint4 *dl = (const uint4 *)(J.left_desc + (size_t)iL * 32);
        const uint4 a0 = dl[0], a1 = dl[1];
        uint32_t key = 0xFFFFFFFFu;
        for (int j = lane; j < nr; j += 64) {
            const ygzfe_kp kpR = J.right_kps[j];
            const float r = 2.0f * lv.scale[kpR.octave];
            const int maxr = (int)ceilf(kpR.y + r), minr = (int)floorf(kpR.y - r);
            if (row < minr || row > maxr) continue;
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float uR = kpR.x;
            if (!(uR >= minU && uR <= maxU)) continue;
            const uint4 *dr = (const uint4 *)(J.right_desc + (size_t)j * 32);
            const uint4 b0 = dr[0], b1 = dr[1];
            const int dist = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                             __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
            if (dist < 100) key = min(key, ((uint32_t)dist << 16) | (uint32_t)j);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) key = min(key, (uint32_t)__shfl_xor((int)key, o, 64));
        if (key != 0xFFFFFFFFu) {
            bestDist = (int)(key >> 16);
            bestIdxR = (int)(key & 0xFFFFu);
        }
    }
    const int thOrbDist = (100 + 50) / 2;
    if (bestDist < thOrbDist) {  // wave-uniform
        const float uR0 = J.right_kps[bestIdxR].x;
        const float scaleFactor = lv.inv_scale[levelL];
        const float scaleduL = roundf(kpL.x * scaleFactor);
        const float scaledvL = roundf(kpL.y * scaleFactor);
        const float scaleduR0 = roundf(uR0 * scaleFactor);
        const int w = 5, L = 5;
        const int W = lv.w[levelL], Hh = lv.h[levelL];
        const int r0 = (int)(scaledvL - w), c0 = (int)(scaleduL - w);
        const float iniu = scaleduR0 + L - w;
        const float endu = scaleduR0 + L + w + 1;
        const int cr0 = (int)(scaleduR0 + -L - w);
        // windows the reference would cut outside the level abort it (cv::Mat
        // range assertions): dropped here, as in the oracle
        const bool inside = !(r0 < 0 || r0 + 2 * w + 1 > Hh || c0 < 0 || c0 + 2 * w + 1 > W) &&
                            !(iniu < 0 || endu >= W) && !(cr0 < 0 || (int)(scaleduR0 + L + w + 1) > W);
        if (inside) {
            const uint8_t *IL = J.left_pyr + lv.off[levelL];
            const uint8_t *IR = J.right_pyr + lv.off[levelL];
            const int cL = IL[(size_t)(r0 + w) * W + c0 + w];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int t = lane + 64 * h;
                if (t < 121) {
                    const int win = t / 11, y = t - win * 11;
                    const int cc = cr0 + win;
                    const int cR = IR[(size_t)(r0 + w) * W + cc + w];
                    const uint8_t *pl = IL + (size_t)(r0 + y) * W + c0;
                    const uint8_t *pr = IR + (size_t)(r0 + y) * W + cc;
                    int s = 0;
#pragma unroll
                    for (int x = 0; x < 11; x++) s += abs(((int)pl[x] - cL) - ((int)pr[x] - cR));
                    s_sad[wave][t] = s;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            int wsum = 0;
            if (lane < 11)
#pragma unroll
                for (int y = 0; y < 11; y++) wsum += s_sad[wave][lane * 11 + y];
            uint32_t k = lane < 11 ? (((uint32_t)wsum << 8) | (uint32_t)lane) : 0xFFFFFFFFu;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) k = min(k, (uint32_t)__shfl_xor((int)k, o, 64));
            const int bestincR = (int)(k & 0xFFu) - L;
            const int bestSad = (int)(k >> 8);
            if (bestincR != -L && bestincR != L) {
                const float dist1 = (float)__shfl(wsum, L + bestincR - 1, 64);
                const float dist2 = (float)__shfl(wsum, L + bestincR, 64);
                const float dist3 = (float)__shfl(wsum, L + bestincR + 1, 64);
                const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                if (!(deltaR < -1 || deltaR > 1)) {
                    float bestuR = lv.scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
                    float disparity = (uL - bestuR);
                    if (disparity >= minD && disparity < maxD) {
                        if (disparity <= 0) {
                            disparity = 0.01f;
                            bestuR = (float)((double)uL - 0.01);
                        }
                        out_d = mbf / disparity;
                        out_u = bestuR;
                        out_sad = bestSad;
                    }
                }
            }
        }
    }
    if (lane == 0) {
        J.u_right[iL] = out_u;
        J.depth[iL] = out_d;
        J.sad[iL] = out_sad;
    }
}

__global__ __launch_bounds__(256) void k_stereo_filter(const StereoJob *__restrict__ jobs) {
    __shared__ int s_hist[256];
    __shared__ int s_sel[2];
    const StereoJob J = jobs[blockIdx.x];
    const int nl = *J.n_left;
    const int tid = threadIdx.x;
    // n = number of matches
    s_hist[tid] = 0;
    __syncthreads();
    int cnt = 0;
    for (int i = tid; i < nl; i += 256) cnt += J.sad[i] >= 0;
    atomicAdd(&s_hist[0], cnt);
    __syncthreads();
    const int np = s_hist[0];
    __syncthreads();
    if (np == 0) return;  // the reference reads an empty vector here (UB): no-op
    int k = np / 2;       // median = SAD of element np/2 of the sorted list
    int prefix = 0;
#pragma unroll 1
    for (int round = 0; round < 2; round++) {
        s_hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < nl; i += 256) {
            const int v = J.sad[i];
            if (v < 0) continue;
            if (round == 1 && (v >> 8) != prefix) continue;
            atomicAdd(&s_hist[round == 0 ? (v >> 8) & 0xFF : v & 0xFF], 1);
        }
        __syncthreads();
        if (tid == 0) {
            int acc = 0, b = 0;
            for (; b < 256; b++) {
                if (acc + s_hist[b] > k) break;
                acc += s_hist[b];
            }
            s_sel[0] = b;
            s_sel[1] = k - acc;
        }
        __syncthreads();
        const int b = s_sel[0];
        k = s_sel[1];
        prefix = round == 0 ? b : ((prefix << 8) | b);
        __syncthreads();
    }
    const float median = (float)prefix;
    const float thDist = 1.5f * 1.4f * median;
    for (int i = tid; i < nl; i += 256) {
        const int v = J.sad[i];
        if (v >= 0 && !((float)v < thDist)) {
            J.u_right[i] = -1.0f;
            J.depth[i] = -1.0f;
            J.sad[i] = -1;
        }
    }
}

// batch jobs: pair p = (left frame left_idx[p], right frame right_idx[p]) of one batch
__global__ void k_build_stereo_jobs(int n, const uint8_t *pyr, size_t pyr_pitch, const ygzfe_kp *kps,
                                    const uint8_t *desc, const int *counts, int kp_cap, const int32_t *left_idx,
                                    const int32_t *right_idx, float *u_right, float *depth, int *sad,
                                    StereoJob *jobs) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int l = left_idx[p], r = right_idx[p];
    StereoJob J;
    J.left_pyr = pyr + (size_t)l * pyr_pitch;
    J.right_pyr = pyr + (size_t)r * pyr_pitch;
    J.left_kps = kps + (size_t)l * kp_cap;
    J.right_kps = kps + (size_t)r * kp_cap;
    J.left_desc = desc + (size_t)l * kp_cap * 32;
    J.right_desc = desc + (size_t)r * kp_cap * 32;
    J.n_left = counts + l;
    J.n_right = counts + r;
    J.u_right = u_right + (size_t)p * kp_cap;
    J.depth = depth + (size_t)p * kp_cap;
    J.sad = sad + (size_t)p * kp_cap;
    jobs[p] = J;
}

hipError_t launch_stereo(const StereoJob *jobs, int n_pairs, int max_left, const StereoLevels &lv, float mb, float mbf,
                         hipStream_t st) {
    if (n_pairs <= 0 || max_left <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_stereo_match, dim3((max_left + kStereoWaves - 1) / kStereoWaves, n_pairs), dim3(256), 0, st,
                       jobs, lv, mb, mbf);
    hipLaunchKernelGGL(k_stereo_filter, dim3(n_pairs), dim3(256), 0, st, jobs);
    return hipGetLastError();
}

hipError_t launch_build_stereo_jobs(int n, const uint8_t *pyr, size_t pyr_pitch, const ygzfe_kp *kps,
                                    const uint8_t *desc, const int *counts, int kp_cap, const int32_t *left_idx,
                                    const int32_t *right_idx, float *u_right, float *depth, int *sad,
                                    StereoJob *jobs, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_build_stereo_jobs, dim3((n + 255) / 256), dim3(256), 0, st, n, pyr, pyr_pitch, kps, desc,
                       counts, kp_cap, left_idx, right_idx, u_right, depth, sad, jobs);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ComputeStereoFromRGBD (Frame.cc:684-700): d = imDepth.at<float>(int v, int u);
// d > 0 -> mvDepth = d, mvuRight = u - mbf / d
__global__ __launch_bounds__(256) void k_stereo_rgbd(const float *__restrict__ im_depth, size_t depth_pitch, int W,
                                                     int H, int stride, const ygzfe_kp *__restrict__ kps,
                                                     int kp_pitch, const int *__restrict__ n_ptr, int n_static,
                                                     float mbf, float *__restrict__ u_right,
                                                     float *__restrict__ depth) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = n_ptr ? n_ptr[f] : n_static;
    if (i >= n) return;
    const ygzfe_kp kp = kps[(size_t)f * kp_pitch + i];
    const float *img = im_depth + (size_t)f * depth_pitch;
    float ur = -1.0f, dd = -1.0f;
    const int v = (int)kp.y, u = (int)kp.x;
    if (v >= 0 && v < H && u >= 0 && u < W) {
        const float d = img[(size_t)v * stride + u];
        if (d > 0) {
            dd = d;
            ur = kp.x - mbf / d;
        }
    }
    u_right[(size_t)f * kp_pitch + i] = ur;
    depth[(size_t)f * kp_pitch + i] = dd;
}

hipError_t launch_stereo_rgbd(const float *im_depth, size_t depth_pitch, int W, int H, int stride,
                              const ygzfe_kp *kps, int kp_pitch, const int *n_ptr, int n_max, int n_frames, float mbf,
                              float *u_right, float *depth, hipStream_t st) {
    if (n_max <= 0 || n_frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_stereo_rgbd, dim3((n_max + 255) / 256, n_frames), dim3(256), 0, st, im_depth, depth_pitch, W,
                       H, stride, kps, kp_pitch, n_ptr, n_max, mbf, u_right, depth);
    return hipGetLastError();
}

}  // namespace ygzfe
