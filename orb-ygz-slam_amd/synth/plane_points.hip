// plane_points.hip -- synthetic-scene helper for bench.py (not product code).
// Stand-in for Tracking's map-point snapshot xyz_ref = T_ref * P_w
// (Tracking.cc:2145-2189): every keypoint of reference frame i is
// back-projected onto the synthetic plane Z_w = plane_z, i.e. along the
// camera ray d = ((x - cx) / fx, (y - cy) / fy, 1) to depth
// lam = (plane_z - cz_i) / (r3_i . d).  One fused pass instead of a chain of
// elementwise torch kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void k_plane_points(const float *__restrict__ kps, int kp_stride_f, int cap,
                                                      int n_frames, float fx, float fy, float cx, float cy,
                                                      const float *__restrict__ r3, const float *__restrict__ cz,
                                                      float plane_z, float *__restrict__ xyz) {
    const int i = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
    if (i >= n_frames || j >= cap) return;
    const float *k = kps + ((size_t)i * cap + j) * kp_stride_f;
    const float dx = (k[0] - cx) / fx, dy = (k[1] - cy) / fy;
    const float lam = (plane_z - cz[i]) / (r3[3 * i] * dx + r3[3 * i + 1] * dy + r3[3 * i + 2]);
    float *o = xyz + ((size_t)i * cap + j) * 3;
    o[0] = dx * lam;
    o[1] = dy * lam;
    o[2] = lam;
}

extern "C" int ygzs_plane_points(const float *d_kps, int kp_stride_f, int cap, int n_frames, const float cam[4],
                                 const float *d_r3, const float *d_cz, float plane_z, float *d_xyz, void *stream) {
    if (n_frames <= 0) return 0;
    hipLaunchKernelGGL(k_plane_points, dim3((cap + 255) / 256, n_frames), dim3(256), 0, (hipStream_t)stream, d_kps,
                       kp_stride_f, cap, n_frames, cam[0], cam[1], cam[2], cam[3], d_r3, d_cz, plane_z, d_xyz);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
