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

// Device renderer of the bench's synthetic sequence (same scene as synth.c
// ygzs_render_plane: pinhole camera T_cw looking at the textured plane
// Z_w = plane_z, bilinear texture lookup in double), so a rank renders its
// shard of the 13,728-frame C5 sequence straight into the batch's level-0
// slots instead of rendering on the host and uploading.  Per-pixel noise
// U{-amp..amp} from a splitmix64 hash of (seed, pixel): every frame distinct.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ void qrot_d(const double q[4], const double v[3], double o[3]) {
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    for (int i = 0; i < 3; i++) uv[i] *= 2;
    const double c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    for (int i = 0; i < 3; i++) o[i] = v[i] + q[3] * uv[i] + c[i];
}

__global__ __launch_bounds__(256) void k_render_plane(const uint8_t *__restrict__ tex, int TW, int TH, double texel,
                                                      double plane_z, float fx, float fy, float cx, float cy,
                                                      const float *__restrict__ q_cw, const float *__restrict__ t_cw,
                                                      const uint64_t *__restrict__ seeds, int W, int H, int amp,
                                                      uint8_t *__restrict__ out, size_t pitch) {
    const int f = blockIdx.y;
    const int pix = blockIdx.x * 256 + threadIdx.x;
    if (pix >= W * H) return;
    const int x = pix % W, y = pix / W;
    const double qi[4] = {-q_cw[4 * f], -q_cw[4 * f + 1], -q_cw[4 * f + 2], q_cw[4 * f + 3]};
    const double mt[3] = {-t_cw[3 * f], -t_cw[3 * f + 1], -t_cw[3 * f + 2]};
    double C[3], dw[3];
    qrot_d(qi, mt, C);
    const double dc[3] = {(x - (double)cx) / fx, (y - (double)cy) / fy, 1.0};
    qrot_d(qi, dc, dw);
    int val = 0;
    if (fabs(dw[2]) >= 1e-12) {
        const double lam = (plane_z - C[2]) / dw[2];
        if (lam > 0) {
            const double tx = (C[0] + lam * dw[0]) / texel + TW * 0.5, ty = (C[1] + lam * dw[1]) / texel + TH * 0.5;
            const int ix = (int)floor(tx), iy = (int)floor(ty);
            if (ix >= 0 && iy >= 0 && ix < TW - 1 && iy < TH - 1) {
                const double ax = tx - ix, ay = ty - iy;
                const uint8_t *p = tex + (size_t)iy * TW + ix;
                const double v = (1 - ax) * (1 - ay) * p[0] + ax * (1 - ay) * p[1] + (1 - ax) * ay * p[TW] +
                                 ax * ay * p[TW + 1];
                val = (int)floor(v + 0.5);
            }
        }
    }
    if (amp > 0) val += (int)(mix64(seeds[f] * 0x100000000ull + (uint64_t)pix) % (uint64_t)(2 * amp + 1)) - amp;
    out[(size_t)f * pitch + pix] = (uint8_t)(val < 0 ? 0 : (val > 255 ? 255 : val));
}

extern "C" int ygzs_render_plane_device(const uint8_t *d_tex, int TW, int TH, double texel, double plane_z,
                                        const float cam[4], const float *d_q, const float *d_t,
                                        const uint64_t *d_seeds, int n_frames, int W, int H, int amp,
                                        uint8_t *d_out, size_t pitch, void *stream) {
    if (n_frames <= 0) return 0;
    hipLaunchKernelGGL(k_render_plane, dim3((W * H + 255) / 256, n_frames), dim3(256), 0, (hipStream_t)stream, d_tex,
                       TW, TH, texel, plane_z, cam[0], cam[1], cam[2], cam[3], d_q, d_t, d_seeds, W, H, amp, d_out,
                       pitch);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
