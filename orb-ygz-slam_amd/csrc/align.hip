// align.hip — direct alignment kernels for gfx950.
//
//  * k_sparse_align: SparseImgAlign::run (SparseImageAlign.cc:20-49) with
//    precomputeReferencePatches (:57-128), computeResiduals (:130-231), the
//    Gauss-Newton loop of NLSSolver_impl.hpp:18-91, LDLT solve (:233-238) and
//    T <- T * exp(-x) (:240-244).  One 256-thread workgroup per frame pair runs
//    every level and iteration; the (feature, pixel) residual terms are spread
//    over the workgroup and H / Jres / chi2 are reduced with wave shuffles +
//    LDS.  The reduction order differs from the reference's sequential sum,
//    so poses agree within 1e-4, not bitwise.
//  * k_align2d: Align2D (Align.cc:8-105), one lane per patch, sequential float
//    order as the reference -> bit-exact with oracle/.
//  * k_find_direct: FindDirectProjection (ORBmatcher.cc:1573-1602) =
//    GetWarpAffineMatrix + GetBestSearchLevel + WarpAffine + Align2D, one lane
//    per (map point, keyframe) item.
#include "kernels.hpp"

namespace ygzfe {

// ------------------------------------------------------------------ SE3f
struct SE3 {
    float q[4], t[3];
};

__device__ __forceinline__ void quat_mul(const float a[4], const float b[4], float o[4]) {
    const float x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    const float y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    const float z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    const float w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}

__device__ __forceinline__ void quat_rotate(const float q[4], const float v[3], float o[3]) {
    float uv0 = q[1] * v[2] - q[2] * v[1];
    float uv1 = q[2] * v[0] - q[0] * v[2];
    float uv2 = q[0] * v[1] - q[1] * v[0];
    uv0 += uv0; uv1 += uv1; uv2 += uv2;
    o[0] = v[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
    o[1] = v[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
    o[2] = v[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
}

__device__ __forceinline__ void se3_act(const SE3 &T, const float p[3], float o[3]) {
    float r[3];
    quat_rotate(T.q, p, r);
    o[0] = r[0] + T.t[0]; o[1] = r[1] + T.t[1]; o[2] = r[2] + T.t[2];
}

__device__ void se3_mul(const SE3 &a, const SE3 &b, SE3 &out) {
    float r[3], q[4];
    quat_rotate(a.q, b.t, r);
    const float t0 = a.t[0] + r[0], t1 = a.t[1] + r[1], t2 = a.t[2] + r[2];
    quat_mul(a.q, b.q, q);
    const float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; i++) out.q[i] = q[i] / n;
    out.t[0] = t0; out.t[1] = t1; out.t[2] = t2;
}

__device__ void quat_to_mat(const float q[4], float R[9]) {
    const float tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const float twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const float txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const float tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// Sophus SE3::exp (se3.hpp:407-428), SO3::expAndTheta (so3.hpp:426-455)
__device__ void se3_exp(const float a[6], SE3 &out) {
    const float eps = 1e-5f;
    const float w0 = a[3], w1 = a[4], w2 = a[5];
    const float theta_sq = w0 * w0 + w1 * w1 + w2 * w2;
    const float theta = sqrtf(theta_sq);
    const float half_theta = 0.5f * theta;
    float imag, real;
    if (theta < eps) {
        const float theta_po4 = theta_sq * theta_sq;
        imag = 0.5f - (float)(1.0 / 48.0) * theta_sq + (float)(1.0 / 3840.0) * theta_po4;
        real = 1.f - 0.5f * theta_sq + (float)(1.0 / 384.0) * theta_po4;
    } else {
        imag = sinf(half_theta) / theta;
        real = cosf(half_theta);
    }
    const float q[4] = {imag * w0, imag * w1, imag * w2, real};
    const float O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    float V[9];
    if (theta < eps) {
        quat_to_mat(q, V);
    } else {
        float O2[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                O2[i * 3 + j] = O[i * 3 + 0] * O[0 * 3 + j] + O[i * 3 + 1] * O[1 * 3 + j] + O[i * 3 + 2] * O[2 * 3 + j];
        const float c1 = (1.f - cosf(theta)) / theta_sq;
        const float c2 = (theta - sinf(theta)) / (theta_sq * theta);
        for (int i = 0; i < 9; i++) V[i] = ((i % 4 == 0) ? 1.f : 0.f) + c1 * O[i] + c2 * O2[i];
    }
    for (int i = 0; i < 3; i++) out.t[i] = V[i * 3 + 0] * a[0] + V[i * 3 + 1] * a[1] + V[i * 3 + 2] * a[2];
    for (int i = 0; i < 4; i++) out.q[i] = q[i];
}

// Eigen LDLT (diagonal pivoting, lower-triangle transpositions), solve with
// |D_i| <= FLT_MIN treated as 0.  Same algorithm as oracle/align.c.
__device__ void ldlt_solve6(const float Hin[36], const float b[6], float x[6]) {
    float A[36];
    int perm[6];
    for (int i = 0; i < 36; i++) A[i] = Hin[i];
    for (int i = 0; i < 6; i++) perm[i] = i;
    for (int k = 0; k < 6; k++) {
        int piv = k;
        float big = fabsf(A[k * 6 + k]);
        for (int i = k + 1; i < 6; i++)
            if (fabsf(A[i * 6 + i]) > big) { big = fabsf(A[i * 6 + i]); piv = i; }
        if (piv != k) {
            for (int j = 0; j < k; j++) { const float t = A[k * 6 + j]; A[k * 6 + j] = A[piv * 6 + j]; A[piv * 6 + j] = t; }
            for (int i = piv + 1; i < 6; i++) { const float t = A[i * 6 + k]; A[i * 6 + k] = A[i * 6 + piv]; A[i * 6 + piv] = t; }
            { const float t = A[k * 6 + k]; A[k * 6 + k] = A[piv * 6 + piv]; A[piv * 6 + piv] = t; }
            for (int i = k + 1; i < piv; i++) { const float t = A[i * 6 + k]; A[i * 6 + k] = A[piv * 6 + i]; A[piv * 6 + i] = t; }
            const int t = perm[k]; perm[k] = perm[piv]; perm[piv] = t;
        }
        float tmp[6];
        for (int j = 0; j < k; j++) tmp[j] = A[j * 6 + j] * A[k * 6 + j];
        float s = 0.f;
        for (int j = 0; j < k; j++) s += A[k * 6 + j] * tmp[j];
        A[k * 6 + k] -= s;
        for (int i = k + 1; i < 6; i++) {
            float t = 0.f;
            for (int j = 0; j < k; j++) t += A[i * 6 + j] * tmp[j];
            A[i * 6 + k] -= t;
        }
        const float akk = A[k * 6 + k];
        if (k == 0 && akk == 0.f) {
            for (int i = 0; i < 6; i++) perm[i] = i;
            break;
        }
        if (akk != 0.f)
            for (int i = k + 1; i < 6; i++) A[i * 6 + k] /= akk;
    }
    float y[6];
    for (int i = 0; i < 6; i++) y[i] = b[perm[i]];
    for (int i = 0; i < 6; i++) {
        float s = y[i];
        for (int j = 0; j < i; j++) s -= A[i * 6 + j] * y[j];
        y[i] = s;
    }
    for (int i = 0; i < 6; i++) {
        const float d = A[i * 6 + i];
        y[i] = fabsf(d) > 1.17549435e-38f ? y[i] / d : 0.f;
    }
    for (int i = 5; i >= 0; i--) {
        float s = y[i];
        for (int j = i + 1; j < 6; j++) s -= A[j * 6 + i] * y[j];
        y[i] = s;
    }
    for (int i = 0; i < 6; i++) x[perm[i]] = y[i];
}

__device__ __forceinline__ float wmul(double a, double b) { return (float)(a * b); }

// ------------------------------------------------------------------ sparse align
constexpr int kPA = 16;    // patch_area_
constexpr int kRed = 29;   // 21 (upper H) + 6 (Jres) + chi2 + count

size_t sparse_align_scratch_floats(int n) { return (size_t)n * kPA * 7 + (size_t)n; }

__global__ __launch_bounds__(256) void k_sparse_align(AlignLevels lv, ygzfe_camera cam,
                                                      const AlignJob *__restrict__ jobs, float *__restrict__ scratch,
                                                      size_t scratch_per_job,
                                                      ygzfe_align_result *__restrict__ out) {
    __shared__ float s_red[4][kRed];
    __shared__ SE3 s_T, s_old;
    __shared__ float s_chi2, s_H[36];
    __shared__ int s_stop, s_break, s_nmeas;
    const AlignJob job = jobs[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = job.n;
    float *patch = scratch + blockIdx.x * scratch_per_job;
    float *jac = patch + (size_t)n * kPA;
    float *vis = jac + (size_t)n * kPA * 6;
    if (tid == 0) {
        for (int i = 0; i < 4; i++) s_T.q[i] = job.T_init.q[i];
        for (int i = 0; i < 3; i++) s_T.t[i] = job.T_init.t[i];
        s_chi2 = 1e10f;
        s_stop = 0;
        s_nmeas = 0;
        for (int i = 0; i < 36; i++) s_H[i] = 0.f;
    }
    for (int i = tid; i < n; i += 256) vis[i] = 0.f;
    __syncthreads();
    if (n <= 0) {
        if (tid == 0) {
            ygzfe_align_result r;
            for (int i = 0; i < 4; i++) r.T_cur_ref.q[i] = s_T.q[i];
            for (int i = 0; i < 3; i++) r.T_cur_ref.t[i] = s_T.t[i];
            r.n_visible = 0;
            r.chi2 = s_chi2;
            for (int i = 0; i < 36; i++) r.H[i] = 0.f;
            out[blockIdx.x] = r;
        }
        return;
    }
    const int border = 3;
    for (int level = job.max_level; level >= job.min_level; level--) {
        const int W = lv.w[level], H = lv.h[level];
        const float scale = lv.inv_scale[level];
        const uint8_t *rimg = job.ref_pyr + lv.off[level];
        const uint8_t *cimg = job.cur_pyr + lv.off[level];
        // precomputeReferencePatches: (feature, pixel) per thread
        for (int e = tid; e < n * kPA; e += 256) {
            const int i = e >> 4, pc = e & 15;
            float *J = jac + (size_t)e * 6;
            bool ok = job.usable[i] != 0;
            const float u_ref = job.kps[i].x * scale, v_ref = job.kps[i].y * scale;
            const int ui = (int)floorf(u_ref), vi = (int)floorf(v_ref);
            if (ok && (ui - border < 0 || vi - border < 0 || ui + border >= W || vi + border >= H)) ok = false;
            if (!ok) {
                for (int k = 0; k < 6; k++) J[k] = 0.f;
                continue;
            }
            if (pc == 0) vis[i] = 1.f;
            const float x = job.xyz[3 * i], y = job.xyz[3 * i + 1], z = job.xyz[3 * i + 2];
            const float z_inv = (float)(1. / (double)z);
            const float z_inv_2 = z_inv * z_inv;
            float fj[12];
            fj[0] = -z_inv; fj[1] = 0.f; fj[2] = x * z_inv_2; fj[3] = y * fj[2];
            fj[4] = (float)(-(1.0 + (double)(x * fj[2]))); fj[5] = y * z_inv;
            fj[6] = 0.f; fj[7] = -z_inv; fj[8] = y * z_inv_2; fj[9] = (float)(1.0 + (double)(y * fj[8]));
            fj[10] = -fj[3]; fj[11] = -x * z_inv;
            const float su = u_ref - ui, sv = v_ref - vi;
            const float wtl = wmul(1.0 - su, 1.0 - sv), wtr = wmul(su, 1.0 - sv);
            const float wbl = wmul(1.0 - su, sv), wbr = wmul(su, sv);
            const int py = pc >> 2, px = pc & 3;
            const int s = W;
            const uint8_t *p = rimg + (size_t)(vi + py - 2) * s + (ui + px - 2);
            patch[e] = wtl * p[0] + wtr * p[1] + wbl * p[s] + wbr * p[s + 1];
            const float dx = 0.5f * ((wtl * p[1] + wtr * p[2] + wbl * p[s + 1] + wbr * p[s + 2]) -
                                     (wtl * p[-1] + wtr * p[0] + wbl * p[s - 1] + wbr * p[s]));
            const float dy = 0.5f * ((wtl * p[s] + wtr * p[1 + s] + wbl * p[s * 2] + wbr * p[s * 2 + 1]) -
                                     (wtl * p[-s] + wtr * p[1 - s] + wbl * p[0] + wbr * p[1]));
            const float fs = cam.fx * scale;
            for (int k = 0; k < 6; k++) J[k] = (dx * fj[k] + dy * fj[6 + k]) * fs;
        }
        if (tid == 0) s_old = s_T;
        __syncthreads();
        for (int it = 0; it < 10; it++) {
            const SE3 T = s_T;
            float acc[kRed];
            for (int k = 0; k < kRed; k++) acc[k] = 0.f;
            for (int e = tid; e < n * kPA; e += 256) {
                const int i = e >> 4, pc = e & 15;
                if (vis[i] == 0.f) continue;
                float pc3[3];
                se3_act(T, job.xyz + 3 * i, pc3);
                const float u = (cam.fx * pc3[0] / pc3[2] + cam.cx) * scale;
                const float v = (cam.fy * pc3[1] / pc3[2] + cam.cy) * scale;
                const int ui = (int)floorf(u), vi = (int)floorf(v);
                if (ui < 0 || vi < 0 || ui - border < 0 || vi - border < 0 || ui + border >= W || vi + border >= H)
                    continue;
                const float su = u - ui, sv = v - vi;
                const float wtl = wmul(1.0 - su, 1.0 - sv), wtr = wmul(su, 1.0 - sv);
                const float wbl = wmul(1.0 - su, sv), wbr = wmul(su, sv);
                const int py = pc >> 2, px = pc & 3;
                const uint8_t *p = cimg + (size_t)(vi + py - 2) * W + (ui + px - 2);
                const float ic = wtl * p[0] + wtr * p[1] + wbl * p[W] + wbr * p[W + 1];
                const float res = ic - patch[e];
                const float *J = jac + (size_t)e * 6;
                float j[6];
                for (int k = 0; k < 6; k++) j[k] = J[k];
                int m = 0;
                for (int r = 0; r < 6; r++)
                    for (int c = r; c < 6; c++) acc[m++] += j[r] * j[c];
                for (int r = 0; r < 6; r++) acc[21 + r] -= j[r] * res;
                acc[27] += res * res;
                acc[28] += 1.f;
            }
            for (int k = 0; k < kRed; k++) acc[k] = wave_sum_f(acc[k]);
            if (lane == 0)
                for (int k = 0; k < kRed; k++) s_red[wave][k] = acc[k];
            __syncthreads();
            if (tid == 0) {
                float r[kRed];
                for (int k = 0; k < kRed; k++) r[k] = (s_red[0][k] + s_red[1][k]) + (s_red[2][k] + s_red[3][k]);
                float Hm[36], b[6], x[6];
                int m = 0;
                for (int rr = 0; rr < 6; rr++)
                    for (int c = rr; c < 6; c++) { Hm[rr * 6 + c] = r[m]; Hm[c * 6 + rr] = r[m]; m++; }
                for (int k = 0; k < 6; k++) b[k] = r[21 + k];
                const int nmeas = (int)r[28];
                const float new_chi2 = r[27] / (float)nmeas;
                for (int k = 0; k < 36; k++) s_H[k] = Hm[k];
                s_nmeas = nmeas;
                ldlt_solve6(Hm, b, x);
                if (isnan(x[0])) s_stop = 1;
                s_break = 0;
                if ((it > 0 && (double)new_chi2 > 1.2 * (double)s_chi2) || s_stop) {
                    s_T = s_old;
                    s_break = 1;
                } else {
                    float mx[6];
                    for (int k = 0; k < 6; k++) mx[k] = -x[k];
                    SE3 E, Tn;
                    se3_exp(mx, E);
                    se3_mul(s_T, E, Tn);
                    s_old = s_T;
                    s_T = Tn;
                    s_chi2 = new_chi2;
                    float nm = -1.f;
                    for (int k = 0; k < 6; k++) nm = fabsf(x[k]) > nm ? fabsf(x[k]) : nm;
                    if (nm <= 0.000001f) s_break = 1;
                }
            }
            __syncthreads();
            if (s_break) break;
        }
        __syncthreads();
    }
    if (tid == 0) {
        ygzfe_align_result r;
        for (int i = 0; i < 4; i++) r.T_cur_ref.q[i] = s_T.q[i];
        for (int i = 0; i < 3; i++) r.T_cur_ref.t[i] = s_T.t[i];
        r.n_visible = s_nmeas / kPA;
        r.chi2 = s_chi2;
        for (int i = 0; i < 36; i++) r.H[i] = s_H[i];
        out[blockIdx.x] = r;
    }
}

hipError_t launch_sparse_align(const AlignLevels &lv, const ygzfe_camera &cam, const AlignJob *jobs, int njobs,
                               float *scratch, size_t scratch_per_job, ygzfe_align_result *out, hipStream_t st) {
    if (njobs <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sparse_align, dim3(njobs), dim3(256), 0, st, lv, cam, jobs, scratch, scratch_per_job, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------ Align2D
__device__ void inverse3(const float m[9], float r[9]) {
#define M(i, j) m[(i) * 3 + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    const float c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
    const float det = c0 * M(0, 0) + c1 * M(1, 0) + c2 * M(2, 0);
    const float inv = 1.f / det;
    r[0] = c0 * inv; r[1] = c1 * inv; r[2] = c2 * inv;
    r[3] = COF(0, 1) * inv; r[4] = COF(1, 1) * inv; r[5] = COF(2, 1) * inv;
    r[6] = COF(0, 2) * inv; r[7] = COF(1, 2) * inv; r[8] = COF(2, 2) * inv;
#undef COF
#undef M
}

__device__ int align2d_lane(const uint8_t *cur, int w, int h, const uint8_t *rpb, const uint8_t *rp, int n_iter,
                            float *px) {
    const int hp = 4, ps = 8, step = 10;
    float rdx[64], rdy[64], H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int y = 0; y < ps; ++y)
        for (int x = 0; x < ps; ++x) {
            const uint8_t *it = rpb + (y + 1) * step + 1 + x;
            const float J0 = (float)(0.5 * (it[1] - it[-1]));
            const float J1 = (float)(0.5 * (it[step] - it[-step]));
            const float J[3] = {J0, J1, 1.f};
            rdx[y * 8 + x] = J0;
            rdy[y * 8 + x] = J1;
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) H[r * 3 + c] += J[r] * J[c];
        }
    float Hi[9];
    inverse3(H, Hi);
    float mean_diff = 0.f, u = px[0], v = px[1];
    const float min_upd2 = (float)(0.03 * 0.03);
    int converged = 0;
    for (int iter = 0; iter < n_iter; ++iter) {
        const int ur = (int)floorf(u), vr = (int)floorf(v);
        if (ur < hp || vr < hp || ur >= w - hp || vr >= h - hp) break;
        if (isnan(u) || isnan(v)) return 0;
        const float sx = u - ur, sy = v - vr;
        const float wTL = wmul(1.0 - sx, 1.0 - sy), wTR = wmul(sx, 1.0 - sy);
        const float wBL = wmul(1.0 - sx, sy), wBR = wmul(sx, sy);
        float Jr0 = 0.f, Jr1 = 0.f, Jr2 = 0.f;
        for (int y = 0; y < ps; ++y) {
            const uint8_t *it = cur + (size_t)(vr + y - hp) * w + ur - hp;
            for (int x = 0; x < ps; ++x, ++it) {
                const float sp = wTL * it[0] + wTR * it[1] + wBL * it[w] + wBR * it[w + 1];
                const float res = sp - rp[y * 8 + x] + mean_diff;
                Jr0 -= res * rdx[y * 8 + x];
                Jr1 -= res * rdy[y * 8 + x];
                Jr2 -= res;
            }
        }
        const float u0 = Hi[0] * Jr0 + Hi[1] * Jr1 + Hi[2] * Jr2;
        const float u1 = Hi[3] * Jr0 + Hi[4] * Jr1 + Hi[5] * Jr2;
        const float u2 = Hi[6] * Jr0 + Hi[7] * Jr1 + Hi[8] * Jr2;
        u += u0;
        v += u1;
        mean_diff += u2;
        if (u0 * u0 + u1 * u1 < min_upd2) { converged = 1; break; }
    }
    px[0] = u;
    px[1] = v;
    return converged;
}

__global__ __launch_bounds__(256) void k_align2d(const uint8_t *__restrict__ img, int w, int h, int n,
                                                 const uint8_t *__restrict__ pwb, const uint8_t *__restrict__ p,
                                                 int n_iter, float *__restrict__ px, uint8_t *__restrict__ conv) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float q[2] = {px[2 * i], px[2 * i + 1]};
    const int ok = align2d_lane(img, w, h, pwb + (size_t)i * 100, p + (size_t)i * 64, n_iter, q);
    px[2 * i] = q[0];
    px[2 * i + 1] = q[1];
    conv[i] = (uint8_t)ok;
}

hipError_t launch_align2d(const uint8_t *img, int w, int h, int n, const uint8_t *pwb, const uint8_t *p,
                          int n_iter, float *px, uint8_t *conv, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_align2d, dim3((n + 255) / 256), dim3(256), 0, st, img, w, h, n, pwb, p, n_iter, px, conv);
    return hipGetLastError();
}

// ------------------------------------------------------------------ FindDirectProjection
__global__ __launch_bounds__(256) void k_find_direct(const uint8_t *const *__restrict__ ref_pyrs, AlignLevels rlv,
                                                     const uint8_t *__restrict__ cur_pyr, AlignLevels clv,
                                                     int nlevels, const float *__restrict__ scale,
                                                     float inv_sigma2_1, ygzfe_camera cam, int n,
                                                     const int32_t *__restrict__ ref_index,
                                                     const ygzfe_kp *__restrict__ kps, const float *__restrict__ pts,
                                                     const ygzfe_se3 *__restrict__ Tcr, float *__restrict__ px_io,
                                                     int32_t *__restrict__ level_out, uint8_t *__restrict__ ok_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ygzfe_kp kp = kps[i];
    SE3 T;
    for (int k = 0; k < 4; k++) T.q[k] = Tcr[i].q[k];
    for (int k = 0; k < 3; k++) T.t[k] = Tcr[i].t[k];
    const float pt[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
    const int oc = clampi(kp.octave, 0, nlevels - 1);
    // GetWarpAffineMatrix (ORBmatcher.cc:1525-1547)
    const float depth = pt[2], ls = scale[oc];
    const float du_x = kp.x + 4.f * ls, du_y = kp.y + 0.f * ls;
    const float dv_x = kp.x + 0.f * ls, dv_y = kp.y + 4.f * ls;
    const float pdu[3] = {(du_x - cam.cx) * depth / cam.fx, (du_y - cam.cy) * depth / cam.fy, depth};
    const float pdv[3] = {(dv_x - cam.cx) * depth / cam.fx, (dv_y - cam.cy) * depth / cam.fy, depth};
    float c[3], cu[3], cv[3];
    se3_act(T, pt, c);
    se3_act(T, pdu, cu);
    se3_act(T, pdv, cv);
    const float pc0 = cam.fx * c[0] / c[2] + cam.cx, pc1 = cam.fy * c[1] / c[2] + cam.cy;
    const float pu0 = cam.fx * cu[0] / cu[2] + cam.cx, pu1 = cam.fy * cu[1] / cu[2] + cam.cy;
    const float pv0 = cam.fx * cv[0] / cv[2] + cam.cx, pv1 = cam.fy * cv[1] / cv[2] + cam.cy;
    const float A0 = (pu0 - pc0) / 4, A2 = (pu1 - pc1) / 4, A1 = (pv0 - pc0) / 4, A3 = (pv1 - pc1) / 4;
    // GetBestSearchLevel (ORBmatcher.h:226-238)
    int sl = 0;
    float D = A0 * A3 - A2 * A1;
    while (D > 3.0f && sl < nlevels - 1) { sl += 1; D *= inv_sigma2_1; }
    level_out[i] = sl;
    // WarpAffine 10x10 (ORBmatcher.cc:1549-1571)
    const uint8_t *rimg = ref_pyrs[ref_index[i]] + rlv.off[oc];
    const int rw = rlv.w[oc], rh = rlv.h[oc];
    const float det = A0 * A3 - A2 * A1;
    const float inv = 1.f / det;
    const float R00 = A3 * inv, R01 = -A1 * inv, R10 = -A2 * inv, R11 = A0 * inv;
    const float prx = kp.x / scale[oc], pry = kp.y / scale[oc];
    uint8_t pb[100], pp[64];
    for (int y = 0; y < 10; y++)
        for (int x = 0; x < 10; x++) {
            const float ppx = (float)(x - 5) * scale[sl], ppy = (float)(y - 5) * scale[sl];
            const float qx = (R00 * ppx + R01 * ppy) + prx;
            const float qy = (R10 * ppx + R11 * ppy) + pry;
            uint8_t val = 0;
            if (!(qx < 0 || qy < 0 || qx >= rw - 1 || qy >= rh - 1)) {
                const double X = qx, Y = qy;
                const double xx = X - floor(X), yy = Y - floor(Y);
                const uint8_t *d = rimg + (size_t)(int)Y * rw + (int)X;
                val = (uint8_t)((1 - xx) * (1 - yy) * d[0] + xx * (1 - yy) * d[1] + (1 - xx) * yy * d[rw] +
                                xx * yy * d[rw + 1]);
            }
            pb[y * 10 + x] = val;
        }
    for (int y = 1; y < 9; ++y)
        for (int x = 0; x < 8; ++x) pp[(y - 1) * 8 + x] = pb[y * 10 + 1 + x];
    const float is = 1.0f / scale[sl];
    (void)is;
    float q[2] = {px_io[2 * i] * clv.inv_scale[sl], px_io[2 * i + 1] * clv.inv_scale[sl]};
    const int ok = align2d_lane(cur_pyr + clv.off[sl], clv.w[sl], clv.h[sl], pb, pp, 10, q);
    px_io[2 * i] = q[0] * scale[sl];
    px_io[2 * i + 1] = q[1] * scale[sl];
    ok_out[i] = (uint8_t)ok;
}

hipError_t launch_find_direct(const uint8_t *const *ref_pyrs, const AlignLevels &ref_lv, const uint8_t *cur_pyr,
                              const AlignLevels &cur_lv, int nlevels, const float *scale, float inv_sigma2_1,
                              const ygzfe_camera &cam, int n, const int32_t *ref_index, const ygzfe_kp *kp_ref,
                              const float *pt_ref, const ygzfe_se3 *T_cr, float *px, int32_t *level, uint8_t *ok,
                              hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_find_direct, dim3((n + 255) / 256), dim3(256), 0, st, ref_pyrs, ref_lv, cur_pyr, cur_lv,
                       nlevels, scale, inv_sigma2_1, cam, n, ref_index, kp_ref, pt_ref, T_cr, px, level, ok);
    return hipGetLastError();
}

}  // namespace ygzfe
