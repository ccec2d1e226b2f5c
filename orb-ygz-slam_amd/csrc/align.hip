// align.hip — direct alignment kernels for gfx950.
//
//  * k_sparse_align: SparseImgAlign::run (SparseImageAlign.cc:20-49) with
//    precomputeReferencePatches (:57-128), computeResiduals (:130-231), the
//    Gauss-Newton loop of NLSSolver_impl.hpp:18-91, LDLT solve (:233-238) and
//    T <- T * exp(-x) (:240-244).  One 1024-thread workgroup per frame pair runs
//    every level and iteration (wave 0 solves, waves 1..15 own one feature per
//    lane); H / Jres / chi2 are reduced with DPP / permlane wave steps + one LDS
//    pass, and while no feature leaves the level a step is x = H_vis^-1 Jres with
//    the inverse formed once per level.  The reduction order differs from the
//    reference's sequential sum, so poses agree within 1e-4, not bitwise
//    (SURVEY.md §8a row a12).
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

// se3_mul with the quaternion normalised by one rsqrt (the solver wave's
// pose update; 1-ulp differences are inside the 1e-4 pose parity)
__device__ __forceinline__ void se3_mul_fast(const SE3 &a, const SE3 &b, SE3 &out) {
#pragma clang fp contract(fast)  // solver wave: fused products (rounding-level, pose parity 1e-4)
    float r[3], q[4];
    quat_rotate(a.q, b.t, r);
    const float t0 = a.t[0] + r[0], t1 = a.t[1] + r[1], t2 = a.t[2] + r[2];
    quat_mul(a.q, b.q, q);
    const float inv = __builtin_amdgcn_rsqf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; i++) out.q[i] = q[i] * inv;
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

// Row-major upper-triangle index of (i, j): the lane order of the H components
// (lane 8 + hpack6) in the solver wave.
__device__ __forceinline__ int hpack6(int i, int j) {
    const int a = i < j ? i : j, c = i < j ? j : i;
    return a * 6 - ((a * (a - 1)) >> 1) + (c - a);
}

template <int K>
__device__ __forceinline__ bool ldlt6_step_nopiv(float (&A)[36]) {
#pragma clang fp contract(fast)  // solver wave: fused products (rounding-level, pose parity 1e-4)
    float tmp[6];
#pragma unroll
    for (int j = 0; j < K; j++) tmp[j] = A[j * 6 + j] * A[K * 6 + j];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < K; j++) s += A[K * 6 + j] * tmp[j];
    A[K * 6 + K] -= s;
#pragma unroll
    for (int i = K + 1; i < 6; i++) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < K; j++) t += A[i * 6 + j] * tmp[j];
        A[i * 6 + K] -= t;
    }
    const float akk = A[K * 6 + K];
    if (K == 0 && akk == 0.f) return false;  // Eigen: a zero first pivot ends the factorization
    if (akk != 0.f) {
        const float r = __builtin_amdgcn_rcpf(akk);
#pragma unroll
        for (int i = K + 1; i < 6; i++) A[i * 6 + K] *= r;
    }
    return true;
}

// H = J^T J is symmetric positive semi-definite, for which LDL^T needs no
// pivoting to be backward stable: this variant factors H in place (no pivot
// search, no permutation), straight-line code on wave-uniform values.  Against
// Eigen's diagonally pivoted LDLT the solution differs by rounding only (pose
// parity is 1e-4).  The zero rules are Eigen's: a zero first pivot leaves the
// factorization, |D_i| <= FLT_MIN gives y_i = 0 (an all-zero H solves to x = 0).
__device__ __forceinline__ void ldlt_solve6_nopiv(float r, float x[6]) {
#pragma clang fp contract(fast)  // solver wave: fused products (rounding-level, pose parity 1e-4)
    const int ri = __float_as_int(r);
    float A[36], y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        y[i] = __int_as_float(__builtin_amdgcn_readlane(ri, i));
#pragma unroll
        for (int j = i; j < 6; j++) {
            const float v = __int_as_float(__builtin_amdgcn_readlane(ri, 8 + hpack6(i, j)));
            A[i * 6 + j] = v;
            A[j * 6 + i] = v;
        }
    }
    if (ldlt6_step_nopiv<0>(A)) {
        ldlt6_step_nopiv<1>(A);
        ldlt6_step_nopiv<2>(A);
        ldlt6_step_nopiv<3>(A);
        ldlt6_step_nopiv<4>(A);
        ldlt6_step_nopiv<5>(A);
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        float t = y[i];
#pragma unroll
        for (int j = 0; j < i; j++) t -= A[i * 6 + j] * y[j];
        y[i] = t;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        const float dd = A[i * 6 + i];
        y[i] = fabsf(dd) > 1.17549435e-38f ? y[i] * __builtin_amdgcn_rcpf(dd) : 0.f;
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        float t = y[i];
#pragma unroll
        for (int j = i + 1; j < 6; j++) t -= A[j * 6 + i] * y[j];
        y[i] = t;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = y[i];
}

// The level's fixed H_vis (no feature out of bounds: H = H_vis exactly) solved once
// per level for the six unit vectors: lane c (< 6) runs ldlt_solve6_nopiv's
// factorization and substitutions on H_vis with y = e_c and keeps column c of
// M = H_vis^-1 (the same zero rules, so x = M b is the LDLT solve of b up to
// rounding); every iteration then costs a 6x6 matrix-vector product.  `hv` holds
// H_vis in lanes 8 + hpack6(i, j) (ldlt_solve6_nopiv's layout).  Column c goes to
// Mw[r * 6 + c].
__device__ __forceinline__ void ldlt6_inverse_cols(float hv, int lane, float *Mw) {
#pragma clang fp contract(fast)  // solver: fused products (rounding-level, pose parity 1e-4)
    const int ri = __float_as_int(hv);
    float A[36], y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        y[i] = lane == i ? 1.f : 0.f;
#pragma unroll
        for (int j = i; j < 6; j++) {
            const float v = __int_as_float(__builtin_amdgcn_readlane(ri, 8 + hpack6(i, j)));
            A[i * 6 + j] = v;
            A[j * 6 + i] = v;
        }
    }
    if (ldlt6_step_nopiv<0>(A)) {
        ldlt6_step_nopiv<1>(A);
        ldlt6_step_nopiv<2>(A);
        ldlt6_step_nopiv<3>(A);
        ldlt6_step_nopiv<4>(A);
        ldlt6_step_nopiv<5>(A);
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        float t = y[i];
#pragma unroll
        for (int j = 0; j < i; j++) t -= A[i * 6 + j] * y[j];
        y[i] = t;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        const float dd = A[i * 6 + i];
        y[i] = fabsf(dd) > 1.17549435e-38f ? y[i] * __builtin_amdgcn_rcpf(dd) : 0.f;
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        float t = y[i];
#pragma unroll
        for (int j = i + 1; j < 6; j++) t -= A[j * 6 + i] * y[j];
        y[i] = t;
    }
    if (lane < 6) {
#pragma unroll
        for (int r = 0; r < 6; r++) Mw[r * 6 + lane] = y[r];
    }
}

// Eigen's diagonally pivoted LDLT (lower-triangle transpositions; |D_i| <=
// FLT_MIN gives 0), the algorithm of oracle/align.c, with every array index a
// compile-time constant (pivot swaps and the permutation applied through
// selects) so the 6x6 system stays in VGPRs: the generic (> 960 features) path.
__device__ __forceinline__ void ldlt_solve6_reg(const float Hin[36], const float b[6], float x[6]) {
    float A[36];
    int perm[6];
#pragma unroll
    for (int i = 0; i < 36; i++) A[i] = Hin[i];
#pragma unroll
    for (int i = 0; i < 6; i++) perm[i] = i;
    bool stopped = false;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        if (stopped) break;
        int piv = k;
        float big = fabsf(A[k * 6 + k]);
#pragma unroll
        for (int i = k + 1; i < 6; i++)
            if (fabsf(A[i * 6 + i]) > big) { big = fabsf(A[i * 6 + i]); piv = i; }
#pragma unroll
        for (int p = k + 1; p < 6; p++) {
            if (piv == p) {
#pragma unroll
                for (int j = 0; j < k; j++) { const float t = A[k * 6 + j]; A[k * 6 + j] = A[p * 6 + j]; A[p * 6 + j] = t; }
#pragma unroll
                for (int i = p + 1; i < 6; i++) { const float t = A[i * 6 + k]; A[i * 6 + k] = A[i * 6 + p]; A[i * 6 + p] = t; }
                { const float t = A[k * 6 + k]; A[k * 6 + k] = A[p * 6 + p]; A[p * 6 + p] = t; }
#pragma unroll
                for (int i = k + 1; i < p; i++) { const float t = A[i * 6 + k]; A[i * 6 + k] = A[p * 6 + i]; A[p * 6 + i] = t; }
                const int t = perm[k]; perm[k] = perm[p]; perm[p] = t;
            }
        }
        float tmp[6];
#pragma unroll
        for (int j = 0; j < k; j++) tmp[j] = A[j * 6 + j] * A[k * 6 + j];
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < k; j++) s += A[k * 6 + j] * tmp[j];
        A[k * 6 + k] -= s;
#pragma unroll
        for (int i = k + 1; i < 6; i++) {
            float t = 0.f;
#pragma unroll
            for (int j = 0; j < k; j++) t += A[i * 6 + j] * tmp[j];
            A[i * 6 + k] -= t;
        }
        const float akk = A[k * 6 + k];
        if (k == 0 && akk == 0.f) {
#pragma unroll
            for (int i = 0; i < 6; i++) perm[i] = i;
            stopped = true;
        } else if (akk != 0.f) {
#pragma unroll
            for (int i = k + 1; i < 6; i++) A[i * 6 + k] /= akk;
        }
    }
    float y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < 6; j++) v = perm[i] == j ? b[j] : v;
        y[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        float s = y[i];
#pragma unroll
        for (int j = 0; j < i; j++) s -= A[i * 6 + j] * y[j];
        y[i] = s;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        const float d = A[i * 6 + i];
        y[i] = fabsf(d) > 1.17549435e-38f ? y[i] / d : 0.f;
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        float s = y[i];
#pragma unroll
        for (int j = i + 1; j < 6; j++) s -= A[j * 6 + i] * y[j];
        y[i] = s;
    }
#pragma unroll
    for (int j = 0; j < 6; j++) {
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < 6; i++) v = perm[i] == j ? y[i] : v;
        x[j] = v;
    }
}

__device__ __forceinline__ float wmul(double a, double b) { return (float)(a * b); }

// Row gathers for the 7x7 reference / 5x5 current windows: a feature window sits at an
// arbitrary byte offset, so a lane reads whole dwords from the enclosing 4-byte boundary
// and realigns them with v_alignbyte (one 12- / 8-byte buffer load per row instead of
// 7 / 5 scattered byte loads).  Frame pyramids carry >= 64 bytes of tail padding for the
// over-read.
// five bytes at byte offset `off` of a buffer as floats: one 8-byte buffer load from
// the enclosing dword boundary (32-bit offsets: no 64-bit address arithmetic per row)
__device__ __forceinline__ void load_row5_buf(__amdgpu_buffer_rsrc_t rs, uint32_t off, float (&out)[5]) {
    const uint32_t sh = off & 3u;
    const auto d = __builtin_amdgcn_raw_buffer_load_b64(rs, off - sh, 0, 0);
    const uint32_t v0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
    const uint32_t v1 = __builtin_amdgcn_alignbyte(0u, d[1], sh);
#pragma unroll
    for (int b = 0; b < 4; b++) out[b] = (float)((v0 >> (8 * b)) & 0xFFu);
    out[4] = (float)(v1 & 0xFFu);
}

// seven bytes at byte offset `off` of a buffer, packed: one 12-byte buffer load from the
// enclosing dword boundary, realigned
__device__ __forceinline__ void load_row7_packed_buf(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t (&out)[2]) {
    const uint32_t sh = off & 3u;
    const auto d = __builtin_amdgcn_raw_buffer_load_b96(rs, off - sh, 0, 0);
    out[0] = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
    out[1] = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
}

// ------------------------------------------------------------------ sparse align
constexpr int kPA = 16;    // patch_area_
constexpr int kRed = 29;   // 21 (upper H) + 6 (Jres) + chi2 + count

size_t sparse_align_scratch_floats(int n) { return (size_t)n * kPA * 7 + (size_t)n; }

// Single-precision forms of the reference's mixed float/double expressions,
// with identical results:
//  * bilinear weights (1.0 - su) * (1.0 - sv) (SparseImageAlign.cc:84-87,
//    167-170): su, sv are u - floor(u) with u >= 3 (the border test), so
//    1 - su is exact in float and the double product of two 24-bit values is
//    exact; rounding it to float = one correctly rounded float product;
//  * JacobXYZ2Cam's 1. / z and 1.0 + t (SparseImageAlign.h:98,104,110):
//    double has >= 2*24 + 2 bits, so double-then-float rounding of a quotient
//    or sum of floats equals the correctly rounded float operation.
__device__ __forceinline__ float wmulf(float a, float b) { return a * b; }

// JacobXYZ2Cam (SparseImageAlign.h:95-116): translation first, pre-negated.  Recomputed
// where it is used: without the opaque copy the compiler hoists the 12 loop-invariant
// entries and their products out of every level and iteration loop and spills them.
__device__ __forceinline__ void jacob_xyz2cam_ff(float X, float Y, float Z, float fj[12]) {
    asm volatile("" : "+v"(X), "+v"(Y), "+v"(Z));
    const float z_inv = __builtin_amdgcn_rcpf(Z);  // 1 ulp; pose parity is 1e-4 (tests/test_gpu_align.py)
    const float z_inv_2 = z_inv * z_inv;
    fj[0] = -z_inv; fj[1] = 0.f; fj[2] = X * z_inv_2; fj[3] = Y * fj[2];
    fj[4] = -(1.0f + X * fj[2]); fj[5] = Y * z_inv;
    fj[6] = 0.f; fj[7] = -z_inv; fj[8] = Y * z_inv_2; fj[9] = 1.0f + Y * fj[8];
    fj[10] = -fj[3]; fj[11] = -X * z_inv;
}

// One feature's H_f = fs^2 J^T [Sxx Sxy; Sxy Syy] J for its 2x6 frame Jacobian J
// (jacob_xyz2cam_ff: J[0][1] = J[1][0] = 0) as 21 upper-triangle entries, row-major:
// A = fs^2 G J first, then H = J^T A, the structural zeros of J skipped (the sums of
// SparseImageAlign.cc:121-125 regrouped: rounding-level, pose parity 1e-4)
__device__ __forceinline__ void feat_hessian(float X, float Y, float Z, float Sxx, float Sxy, float Syy, float fs2,
                                             float hv[21]) {
#pragma clang fp contract(fast)
    float fj[12];
    jacob_xyz2cam_ff(X, Y, Z, fj);
    const float gxx = Sxx * fs2, gxy = Sxy * fs2, gyy = Syy * fs2;
    float A0[6], A1[6];
    A0[0] = gxx * fj[0];
    A1[0] = gxy * fj[0];
    A0[1] = gxy * fj[7];
    A1[1] = gyy * fj[7];
#pragma unroll
    for (int c = 2; c < 6; c++) {
        A0[c] = gxx * fj[c] + gxy * fj[6 + c];
        A1[c] = gxy * fj[c] + gyy * fj[6 + c];
    }
    int m = 0;
#pragma unroll
    for (int r = 0; r < 6; r++)
#pragma unroll
        for (int c = r; c < 6; c++) {
            if (r == 0) hv[m] = fj[0] * A0[c];
            else if (r == 1) hv[m] = fj[7] * A1[c];
            else hv[m] = fj[r] * A0[c] + fj[6 + r] * A1[c];
            m++;
        }
}

// ---- Levenberg-Marquardt (NLLSSolver::optimizeLevenbergMarquardt,
// NLSSolver_impl.hpp:95-212), the method a SparseImgAlign constructed with
// LevenbergMarquardt runs.  Every residual pass (all features at one pose) feeds
// lm_round, which plays the reference's loop forward to the next pose whose chi2 it
// needs:
//  * the level's first pass is the reference's chi2_ = computeResiduals(model, true)
//    (:104-105; n_meas_ not cleared, so chi2_ divides by the previous count plus this
//    one) and, at the same pose, the first trial's linearisation (:137-141);
//  * a trial damps H (H_ii += H_ii mu, :146), solves (the pivoted LDLT), and asks for
//    the chi2 at T exp(-x) (:154-156); a singular H fails the trial without a pass;
//  * an evaluation pass decides the trial (rho = chi2_ - new_chi2, :157): success
//    updates T, chi2_, stop = |x|max <= eps, mu, nu (:166-170) and ends the iteration;
//    the next iteration's linearisation is at the same pose, so it is this pass; a
//    failure raises mu (mu *= nu, nu *= 2, :184-190) and retries on the cached
//    linearisation, or stops after 5 trials.
// The level ends when stop is set or after 10 iterations (SparseImageAlign.cc:38-44;
// stop_ persists across levels: a later level then runs one trial).  mu_ starts at
// 0.01 per run (reset(), NLSSolver.h:126) and is set to 0.1 per level (:40).
struct LmState {
    SE3 T, Te;           // the model; the pose of the next residual pass
    float mu, nu, chi2;  // mu_, nu_, chi2_
    float x[6];
    float Hc[21], Jc[6];  // the linearisation at T (upper H row-major, Jres)
    int ncl;              // its measurement count
    float H[36];          // H_ as the last trial left it (damped): getFisherInformation
    int nmeas;            // n_meas_ of the last computeResiduals
    int stop, iter, n_trials, brk, rounds;
};
constexpr int kLmMaxRounds = 64;  // a level needs <= 1 + 10 x 5 passes

__device__ __forceinline__ void lm_init(LmState &L, const ygzfe_se3 &T0) {
    for (int i = 0; i < 4; i++) L.T.q[i] = T0.q[i];
    for (int i = 0; i < 3; i++) L.T.t[i] = T0.t[i];
    L.Te = L.T;
    L.mu = 0.01f;
    L.nu = 2.f;
    L.chi2 = 1e10f;
    L.stop = 0;
    L.nmeas = 0;
    for (int i = 0; i < 36; i++) L.H[i] = 0.f;
}

__device__ __forceinline__ void lm_level_start(LmState &L) {
    L.mu = 0.1f;
    L.iter = 0;
    L.brk = 0;
    L.rounds = 0;
    L.Te = L.T;
}

// trials on the cached linearisation until one needs an evaluation pass (L.Te) or the
// level's loop ends (L.brk)
__device__ void lm_trials(LmState &L) {
    for (;;) {
        L.nmeas = L.ncl;  // the trial's computeResiduals(model, true)
        float Hd[36], b[6], x[6];
        for (int r = 0, m = 0; r < 6; r++)
            for (int c = r; c < 6; c++, m++) { Hd[r * 6 + c] = L.Hc[m]; Hd[c * 6 + r] = L.Hc[m]; }
        for (int k = 0; k < 6; k++) Hd[k * 6 + k] += Hd[k * 6 + k] * L.mu;
        for (int k = 0; k < 6; k++) b[k] = L.Jc[k];
        for (int i = 0; i < 36; i++) L.H[i] = Hd[i];
        ldlt_solve6_reg(Hd, b, x);
        if (!isnan(x[0])) {
            for (int k = 0; k < 6; k++) L.x[k] = x[k];
            float mx[6];
            for (int k = 0; k < 6; k++) mx[k] = -x[k];
            SE3 E;
            se3_exp(mx, E);
            se3_mul(L.T, E, L.Te);
            return;
        }
        // singular: rho = -1, a failed trial
        L.mu *= L.nu;
        L.nu *= 2.f;
        if (++L.n_trials >= 5) L.stop = 1;
        if (L.stop) { L.brk = 1; return; }
    }
}

// one residual pass at L.Te: H (upper, 21), Jres, chi2 sum and count
__device__ void lm_round(LmState &L, const float H[21], const float b[6], float chi2sum, int cnt, bool level_first) {
    if (++L.rounds >= kLmMaxRounds) { L.brk = 1; return; }
    if (level_first) {
        L.chi2 = chi2sum / (float)(L.nmeas + cnt);
    } else {
        L.nmeas = cnt;
        const float new_chi2 = chi2sum / (float)cnt;
        const float rho = L.chi2 - new_chi2;
        if (rho > 0) {
            L.T = L.Te;
            L.chi2 = new_chi2;
            float nm = -1.f;
            for (int k = 0; k < 6; k++) nm = fabsf(L.x[k]) > nm ? fabsf(L.x[k]) : nm;
            L.stop = nm <= 0.000001f;
            const double t = 2.0 * (double)rho - 1.0;  // (2 rho - 1)^3 in double (pow(.., 3))
            L.mu = (float)((double)L.mu * fmax(1. / 3., fmin(1. - t * t * t, 2. / 3.)));
            L.nu = 2.f;
            if (L.stop || ++L.iter >= 10) { L.brk = 1; return; }
        } else {
            L.mu *= L.nu;
            L.nu *= 2.f;
            if (++L.n_trials >= 5) L.stop = 1;
            if (L.stop) { L.brk = 1; return; }
            lm_trials(L);  // retry on the cached linearisation
            return;
        }
    }
    // a new iteration: linearised at T (= the pose of this pass)
    for (int k = 0; k < 21; k++) L.Hc[k] = H[k];
    for (int k = 0; k < 6; k++) L.Jc[k] = b[k];
    L.ncl = cnt;
    L.n_trials = 0;
    lm_trials(L);
}

__device__ __forceinline__ void lm_result(const LmState &L, ygzfe_align_result *out) {
    ygzfe_align_result r;
    for (int i = 0; i < 4; i++) r.T_cur_ref.q[i] = L.T.q[i];
    for (int i = 0; i < 3; i++) r.T_cur_ref.t[i] = L.T.t[i];
    r.n_visible = L.nmeas / kPA;
    r.chi2 = L.chi2;
    for (int i = 0; i < 36; i++) r.H[i] = L.H[i];
    *out = r;
}

// Generic path (any n): (feature, pixel) terms strided over the workgroup,
// ref patches and Jacobians cached in a global scratch slab per job.
template <int NT>
__device__ __attribute__((noinline)) void sparse_align_generic(const AlignLevels lv, const ygzfe_camera cam, const AlignJob &job,
                                     float *__restrict__ scratch, ygzfe_align_result *__restrict__ outp) {
    constexpr int NW = NT / 64;
    __shared__ float s_red[NW][kRed];
    __shared__ SE3 s_T, s_old;
    __shared__ float s_chi2, s_H[36];
    __shared__ int s_stop, s_break, s_nmeas;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = job.n;
    float *patch = scratch;
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
    for (int i = tid; i < n; i += NT) vis[i] = 0.f;
    __syncthreads();
    if (n <= 0) {
        if (tid == 0) {
            ygzfe_align_result r;
            for (int i = 0; i < 4; i++) r.T_cur_ref.q[i] = s_T.q[i];
            for (int i = 0; i < 3; i++) r.T_cur_ref.t[i] = s_T.t[i];
            r.n_visible = 0;
            r.chi2 = s_chi2;
            for (int i = 0; i < 36; i++) r.H[i] = 0.f;
            *outp = r;
        }
        return;
    }
    const int border = 3;
    __shared__ LmState s_lm_store;
    LmState *s_lm = &s_lm_store;
    if (job.method == 1 && tid == 0) lm_init(*s_lm, job.T_init);
    for (int level = job.max_level; level >= job.min_level; level--) {
        const int W = lv.w[level], H = lv.h[level];
        const float scale = lv.inv_scale[level];
        const uint8_t *rimg = job.ref_pyr + lv.off[level];
        const uint8_t *cimg = job.cur_pyr + lv.off[level];
        // computeResiduals (SparseImageAlign.cc:130-231) at T: the wave sums of the 21 H
        // terms, Jres, chi2 and the count into s_red (then a barrier)
        auto generic_pass = [&](const SE3 T) {
            float acc[kRed];
            for (int k = 0; k < kRed; k++) acc[k] = 0.f;
            for (int e = tid; e < n * kPA; e += NT) {
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
        };
        // precomputeReferencePatches: (feature, pixel) per thread
        for (int e = tid; e < n * kPA; e += NT) {
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
        if (job.method == 1) {  // Levenberg-Marquardt (lm_round): a residual pass per round
            if (tid == 0) lm_level_start(*s_lm);
            __syncthreads();
            for (int round = 0;; round++) {
                generic_pass(s_lm->Te);
                if (tid == 0) {
                    float r[kRed];
                    for (int k = 0; k < kRed; k++) {
                        float a = 0.f;
                        for (int w = 0; w < NW; w++) a += s_red[w][k];
                        r[k] = a;
                    }
                    lm_round(*s_lm, r, r + 21, r[27], (int)r[28], round == 0);
                }
                __syncthreads();
                if (s_lm->brk) break;
            }
            __syncthreads();
            continue;
        }
        if (tid == 0) s_old = s_T;
        __syncthreads();
        for (int it = 0; it < 10; it++) {
            generic_pass(s_T);
            if (tid == 0) {
                float r[kRed];
                for (int k = 0; k < kRed; k++) {
                    float a = 0.f;
                    for (int w = 0; w < NW; w++) a += s_red[w][k];
                    r[k] = a;
                }
                float Hm[36], b[6], x[6];
                int m = 0;
                for (int rr = 0; rr < 6; rr++)
                    for (int c = rr; c < 6; c++) { Hm[rr * 6 + c] = r[m]; Hm[c * 6 + rr] = r[m]; m++; }
                for (int k = 0; k < 6; k++) b[k] = r[21 + k];
                const int nmeas = (int)r[28];
                const float new_chi2 = r[27] / (float)nmeas;
                for (int k = 0; k < 36; k++) s_H[k] = Hm[k];
                s_nmeas = nmeas;
                ldlt_solve6_reg(Hm, b, x);
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
        if (job.method == 1) {
            lm_result(*s_lm, outp);
            return;
        }
        ygzfe_align_result r;
        for (int i = 0; i < 4; i++) r.T_cur_ref.q[i] = s_T.q[i];
        for (int i = 0; i < 3; i++) r.T_cur_ref.t[i] = s_T.t[i];
        r.n_visible = s_nmeas / kPA;
        r.chi2 = s_chi2;
        for (int i = 0; i < 36; i++) r.H[i] = s_H[i];
        *outp = r;
    }
}

// Register-resident variant (n <= NT features): one thread owns one feature for
// every level and iteration.  Its 4x4 reference patch and the bilinear
// reference gradients (gx, gy) stay in VGPRs, so an iteration reads only the
// 5x5 current-image window of each feature.  Because J_p = (gx_p*Jp0 +
// gy_p*Jp1) * f*scale (SparseImageAlign.cc:123-125), a feature's Jres and H
// contributions are closed forms of the per-feature sums
// Sx = sum gx*res, Sy = sum gy*res, Sxx, Sxy, Syy (same algebra, different
// float association than the reference's per-pixel sums -> 1e-4 pose parity).
// The per-feature sums are reduced by transposing DPP / permlane steps
// (wave_reduce8 / wave_reduce32) and one LDS pass over the waves.  H is the
// level's visible-feature sum less the features projected out of bounds in the
// iteration (SparseImageAlign.cc:160-163 skips them): their H_f is recomputed from
// the level's moments Sxx, Sxy, Syy kept in registers and summed per wave, so LDS
// holds only the reference patches (61 KB).
#ifdef YGZ_STAMPS
// diagnostic build only (lib/libygzfe_diag.so): block 0's timestamps, gathered in LDS
// (an LDS atomic slot + s_memtime: ~100 cycles a stamp, against ~700 for a global
// counter) and copied out by YGZ_STAMP_FLUSH at the solver wave's end
__device__ unsigned long long g_stamps[4096];
__device__ int g_nstamps;
__shared__ unsigned long long s_stamps[1536];
__shared__ unsigned s_nstamps;
#define YGZ_STAMP_AT(tag, who)                                                           \
    do {                                                                                 \
        if (blockIdx.x == 0 && (who)) {                                                  \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();                  \
            const unsigned k_ = atomicAdd(&s_nstamps, 1u);                               \
            if (k_ < 768) { s_stamps[2 * k_] = (unsigned long long)(tag); s_stamps[2 * k_ + 1] = t_; } \
        }                                                                                \
    } while (0)
#define YGZ_STAMP(tag) YGZ_STAMP_AT(tag, threadIdx.x == 0)
#define YGZ_STAMP_INIT() do { if (threadIdx.x == 0) s_nstamps = 0; } while (0)
#define YGZ_STAMP_FLUSH()                                                                \
    do {                                                                                 \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                                       \
            const unsigned n_ = s_nstamps < 768 ? s_nstamps : 768;                       \
            for (unsigned i_ = 0; i_ < 2 * n_; i_++) g_stamps[i_] = s_stamps[i_];        \
            g_nstamps = (int)n_;                                                         \
        }                                                                                \
    } while (0)
extern "C" int ygzfe_diag_stamps(unsigned long long *out, int cap) {
    int n = 0;
    (void)hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_nstamps), sizeof(int));
    n = n * 2 < cap ? n * 2 : cap;
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * n);
    int z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_nstamps), &z, sizeof(int));
    return n / 2;
}
#else
#define YGZ_STAMP(tag) do {} while (0)
#define YGZ_STAMP_AT(tag, who) do {} while (0)
#define YGZ_STAMP_INIT() do {} while (0)
#define YGZ_STAMP_FLUSH() do {} while (0)
#endif

// DPP lane permutation of a float (update_dpp with the old value 0)
#define YGZ_DPP(v, ctrl, rmask) \
    __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, rmask, 0xF, false))

// Transposing wave reductions (every lane active).  A step pairs two values
// and two lane sets: the lanes of one set keep the sum of value x over both
// sets, the other lanes the sum of value y, so each step halves the values a
// lane carries.  Lanes 0-31 | 32-63 by v_permlane32_swap, rows 0,2 | 1,3 by
// v_permlane16_swap, then DPP row_mirror (i <-> 15-i), row_half_mirror
// (i <-> 7-i) and quad_perm [2,3,0,1] inside the rows.
__device__ __forceinline__ float pair_pl32(float x, float y) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float pair_pl16(float x, float y) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
template <int CTRL, int BIT>
__device__ __forceinline__ float pair_dpp(float x, float y, int lane) {
    const bool hi = lane & BIT;
    const float keep = hi ? y : x, send = hi ? x : y;
    return keep + YGZ_DPP(send, CTRL, 0xF);
}
// 32 values -> lane l holds the wave total of value l >> 1
__device__ __forceinline__ float wave_reduce32(float (&v)[32], int lane) {
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = pair_pl32(v[i], v[16 + i]);
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = pair_pl16(v[i], v[8 + i]);
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = pair_dpp<0x140, 8>(v[i], v[4 + i], lane);
#pragma unroll
    for (int i = 0; i < 2; i++) v[i] = pair_dpp<0x141, 4>(v[i], v[2 + i], lane);
    const float t = pair_dpp<0x4E, 2>(v[0], v[1], lane);
    return t + YGZ_DPP(t, 0xB1, 0xF);
}
// 8 values -> lane l holds the wave total of value (l >> 3) & 7
__device__ __forceinline__ float wave_reduce8(float (&v)[8], int lane) {
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = pair_pl32(v[i], v[4 + i]);
#pragma unroll
    for (int i = 0; i < 2; i++) v[i] = pair_pl16(v[i], v[2 + i]);
    float t = pair_dpp<0x140, 8>(v[0], v[1], lane);
    t += YGZ_DPP(t, 0x141, 0xF);
    t += YGZ_DPP(t, 0x4E, 0xF);
    return t + YGZ_DPP(t, 0xB1, 0xF);
}

// ---- pieces of the register kernel: per-pair LDS state, solver-wave steps, and the
// feature threads' level set-up and residual passes

// the per-pair LDS state: partial sums per wave, the level's H over the visible
// features, per-wave H of the features out of bounds this iteration, pose, last H
template <int NW>
struct AlignPairLds {
    float part[NW][32];
    float Hvis[21];
    float opart[NW][24];
    float M[36];  // H_vis^-1 of the level, row-major (ldlt6_inverse_cols)
    SE3 T, old;
    float chi2, Hpk[21];  // H of the last iteration, upper triangle row-major (when hsrc)
    int stop, brk, nmeas;
    int hsrc;    // the last iteration's H: 1 Hpk, 0 Hvis (no feature out of bounds)
    int out_it;  // the iteration (level * 16 + it) whose residual pass saw a feature out of bounds
};

template <int NW>
__device__ __forceinline__ void align_pair_init(AlignPairLds<NW> &P, const AlignJob &job) {
    for (int i = 0; i < 4; i++) P.T.q[i] = job.T_init.q[i];
    for (int i = 0; i < 3; i++) P.T.t[i] = job.T_init.t[i];
    P.chi2 = 1e10f;
    P.stop = 0;
    P.nmeas = 0;
    P.brk = 0;
    P.out_it = -1;
    P.hsrc = 1;
    for (int i = 0; i < 21; i++) P.Hpk[i] = 0.f;
}

template <int NW>
__device__ __forceinline__ void align_pair_result(const AlignPairLds<NW> &P, ygzfe_align_result *out) {
    ygzfe_align_result res;
    for (int i = 0; i < 4; i++) res.T_cur_ref.q[i] = P.T.q[i];
    for (int i = 0; i < 3; i++) res.T_cur_ref.t[i] = P.T.t[i];
    res.n_visible = P.nmeas / kPA;
    res.chi2 = P.chi2;
    const float *Hl = P.hsrc ? P.Hpk : P.Hvis;
    for (int rr = 0, m = 0; rr < 6; rr++)
        for (int c = rr; c < 6; c++, m++) { res.H[rr * 6 + c] = Hl[m]; res.H[c * 6 + rr] = Hl[m]; }
    *out = res;
}

// level start, solver wave: H_vis = the waves' partial sums of the visible features' H
template <int NW>
__device__ __forceinline__ void align_sum_hvis(AlignPairLds<NW> &P, int lane) {
    if (lane < 21) {
        float r = 0.f;
        for (int w = 1; w < NW; w++) r += P.part[w][lane];
        P.Hvis[lane] = r;
    }
}

// level start, solver wave (beside the first residual pass): M = H_vis^-1; returns
// the lane's entry for align_solver_step's product: M[r][c] in lane 8r + c (r, c < 6),
// 0 elsewhere
template <int NW>
__device__ __forceinline__ float align_level_inverse(AlignPairLds<NW> &P, int lane) {
    const float hv = (lane >= 8 && lane < 29) ? P.Hvis[lane - 8] : 0.f;
    ldlt6_inverse_cols(hv, lane, P.M);
    __builtin_amdgcn_wave_barrier();  // one wave: its LDS writes land before its reads
    const int r = lane >> 3, c = lane & 7;
    return (r < 6 && c < 6) ? P.M[r * 6 + c] : 0.f;
}

// the solver wave's copy of the pair's pose state (the same in every lane)
struct SolverRegs {
    SE3 T, old;
    float chi2;
    bool stop;
    float mreg;  // align_level_inverse's entry of M = H_vis^-1
};

// Sophus SE3::exp of a (se3_exp) for the solver wave: the four transcendentals in
// every lane (hardware v_sin/v_cos, no broadcasts) and V a = a_t + c1 (w x a_t) +
// c2 (w (w . a_t) - theta^2 a_t), the closed form of (I + c1 O + c2 O^2) a_t without
// O's zero products (rounding-level, pose parity 1e-4)
__device__ __forceinline__ void se3_exp_solver(const float a[6], SE3 &out) {
#pragma clang fp contract(fast)
    const float eps = 1e-5f;
    const float w0 = a[3], w1 = a[4], w2 = a[5];
    const float theta_sq = w0 * w0 + w1 * w1 + w2 * w2;
    const float theta = __builtin_amdgcn_sqrtf(theta_sq);
    if (theta < eps) {  // wave-uniform: se3_exp's small-angle branch
        const float theta_po4 = theta_sq * theta_sq;
        const float im = 0.5f - (float)(1.0 / 48.0) * theta_sq + (float)(1.0 / 3840.0) * theta_po4;
        const float q[4] = {im * w0, im * w1, im * w2,
                            1.f - 0.5f * theta_sq + (float)(1.0 / 384.0) * theta_po4};
        float V[9];
        quat_to_mat(q, V);
        for (int i = 0; i < 3; i++) out.t[i] = V[i * 3 + 0] * a[0] + V[i * 3 + 1] * a[1] + V[i * 3 + 2] * a[2];
        for (int i = 0; i < 4; i++) out.q[i] = q[i];
        return;
    }
    const float half_theta = 0.5f * theta;
    const float s_half = __sinf(half_theta), c_half = __cosf(half_theta);
    const float s_th = __sinf(theta), c_th = __cosf(theta);
    const float inv_theta = __builtin_amdgcn_rcpf(theta);
    const float imag = s_half * inv_theta;
    const float inv_sq = inv_theta * inv_theta;
    const float c1 = (1.f - c_th) * inv_sq;
    const float c2 = (theta - s_th) * (inv_sq * inv_theta);
    const float v0 = a[0], v1 = a[1], v2 = a[2];
    const float x0 = w1 * v2 - w2 * v1, x1 = w2 * v0 - w0 * v2, x2 = w0 * v1 - w1 * v0;  // w x v
    const float d = w0 * v0 + w1 * v1 + w2 * v2;
    out.t[0] = v0 + c1 * x0 + c2 * (w0 * d - theta_sq * v0);
    out.t[1] = v1 + c1 * x1 + c2 * (w1 * d - theta_sq * v1);
    out.t[2] = v2 + c1 * x2 + c2 * (w2 * d - theta_sq * v2);
    out.q[0] = imag * w0;
    out.q[1] = imag * w1;
    out.q[2] = imag * w2;
    out.q[3] = c_half;
}

// the solver wave's view of a residual pass: lane k (< 8) of *pk8 holds value k's
// total (Jres[6], chi2, count); lanes 8 + hpack6(i, j) of *hr hold H(i, j) = H_vis less
// the out-of-bounds features' H_f when the pass saw any (tag gi)
template <int NW>
__device__ __forceinline__ void align_solver_reduce(AlignPairLds<NW> &P, int gi, int lane, float &pk8, float &hr) {
    {
        const int k8 = lane & 7, w1 = 2 * (lane >> 3) + 1, w2 = w1 + 1;
        pk8 = (w1 < NW ? P.part[w1][k8] : 0.f) + (w2 < NW ? P.part[w2][k8] : 0.f);
        pk8 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(pk8), 0x128, 0xF, 0xF, false));
        pk8 = pair_pl16(pk8, pk8);
        pk8 = pair_pl32(pk8, pk8);
    }
    hr = 0.f;
    if (lane >= 8 && lane < 29) {
        const int k = lane - 8;
        float o = 0.f;
        if (P.out_it == gi) {
#pragma unroll
            for (int w = 1; w < NW; w++) o += P.opart[w][k];
        }
        hr = P.Hvis[k] - o;
    }
}

// one Gauss-Newton step, solver wave (NLSSolver_impl.hpp:18-91): reduce the
// partials, x = M Jres when every feature stayed inside the level (H = H_vis), else
// H = H_vis - the out-of-bounds features' H_f and a fresh LDLT; rollback or
// T <- T exp(-x).  The pose state lives in the wave's registers (S); lane 0 publishes
// the pose and the loop decision.  Returns true when the level's loop ends.
// (Every wave running the step on its own copy, with double-buffered partials and no
// publish barrier, was measured at 0.49 against 0.34 ms per 1,023 pairs: profiles/r05/align.)
template <int NW>
__device__ __forceinline__ bool align_solver_step(AlignPairLds<NW> &P, SolverRegs &S, int it, int gi, int lane,
                                                  const float (*part)[32], const float (*opart)[24],
                                                  const int *out_it, bool writer) {
    const bool fast = *out_it != gi;
    // Jres[6], chi2, n_meas over waves 1..NW-1: lane 8g + k adds waves 2g+1, 2g+2 of
    // value k, then the 8 groups fold (bit 3: DPP row_ror 8; bits 4, 5: permlane16 /
    // permlane32 swaps, no LDS round trip), so every lane holds the total of value k
    float pk8;
    {
        const int k8 = lane & 7, w1 = 2 * (lane >> 3) + 1, w2 = w1 + 1;
        pk8 = (w1 < NW ? part[w1][k8] : 0.f) + (w2 < NW ? part[w2][k8] : 0.f);
        pk8 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(pk8), 0x128, 0xF, 0xF, false));
        pk8 = pair_pl16(pk8, pk8);
        pk8 = pair_pl32(pk8, pk8);
    }
    YGZ_STAMP(6);
    float x[6];
    const int pi = __float_as_int(pk8);
    const int nmeas = (int)__int_as_float(__builtin_amdgcn_readlane(pi, 7));
    const float chi2sum = __int_as_float(__builtin_amdgcn_readlane(pi, 6));
    if (writer && lane == 0) P.nmeas = nmeas;
    YGZ_STAMP(7);
    if (fast) {  // every feature inside the level: H = H_vis, x = H_vis^-1 Jres
#pragma clang fp contract(fast)  // solver wave: fused products (rounding-level, pose parity 1e-4)
        // lane 8r + c: M[r][c] Jres[c], summed over the 8 lanes of row r by DPP
        float pr = (lane & 7) < 6 ? S.mreg * pk8 : 0.f;
        pr += YGZ_DPP(pr, 0xB1, 0xF);   // quad_perm [1,0,3,2]
        pr += YGZ_DPP(pr, 0x4E, 0xF);   // quad_perm [2,3,0,1]
        pr += YGZ_DPP(pr, 0x141, 0xF);  // row_half_mirror
#pragma unroll
        for (int k = 0; k < 6; k++) x[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pr), 8 * k));
        if (writer && lane == 0) P.hsrc = 0;  // H of this iteration (the result's Fisher information) = H_vis
    } else {  // a feature left the level: H = H_vis - the per-wave sums of its H_f, factored afresh
        float r = pk8;
        if (lane >= 8 && lane < 29) {
            const int k = lane - 8;
            float o = 0.f;
#pragma unroll
            for (int w = 1; w < NW; w++) o += opart[w][k];
            r = P.Hvis[k] - o;
            if (writer) P.Hpk[k] = r;
        } else if (lane >= 29) {
            r = 0.f;
        }
        if (writer && lane == 0) P.hsrc = 1;
        ldlt_solve6_nopiv(r, x);
    }
    YGZ_STAMP(8);
    const float new_chi2 = chi2sum / (float)nmeas;
    const bool stop = S.stop || isnan(x[0]);
    const bool rollback = (it > 0 && (double)new_chi2 > 1.2 * (double)S.chi2) || stop;
    if (rollback) {
        S.stop = stop;
        S.T = S.old;
        if (lane == 0) {
            P.T = S.T;
            P.brk = 1;
        }
        return true;
    }
    float mx[6];
#pragma unroll
    for (int k = 0; k < 6; k++) mx[k] = -x[k];
    SE3 E, Tn;
    se3_exp_solver(mx, E);
    se3_mul_fast(S.T, E, Tn);
    YGZ_STAMP(10);
    const float nm = fmaxf(fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))),
                           fmaxf(fabsf(x[4]), fabsf(x[5])));
    const bool brk = nm <= 0.000001f;
    S.old = S.T;
    S.T = Tn;
    S.chi2 = new_chi2;
    if (lane == 0) {
        P.T = Tn;
        P.brk = brk ? 1 : 0;
    }
    return brk;
}

// one reference feature owned by a thread of the feature waves
struct AlignFeat {
    float X, Y, Z, kx, ky;
    bool own, usable;
};
// its data at one level: reference gradients, their moments, visibility so far
struct AlignLevelData {
    float gx[16], gy[16];
    float Sxx, Sxy, Syy;  // the level's gradient moments (H_f of an out-of-bounds feature)
    bool vis;             // visible_fts_ after this level's set-up (never reset between levels)
};

__device__ __forceinline__ void align_feat_load(AlignFeat &F, AlignLevelData &D, const AlignJob &job, int f) {
    F.own = f < job.n;
    F.X = 0.f; F.Y = 0.f; F.Z = 1.f; F.kx = 0.f; F.ky = 0.f;
    F.usable = false;
    if (F.own) {
        F.X = job.xyz[3 * f]; F.Y = job.xyz[3 * f + 1]; F.Z = job.xyz[3 * f + 2];
        F.usable = job.usable[f] != 0;
        F.kx = job.kps[f].x; F.ky = job.kps[f].y;
    }
#pragma unroll
    for (int p = 0; p < 16; p++) { D.gx[p] = 0.f; D.gy[p] = 0.f; }
    D.Sxx = D.Sxy = D.Syy = 0.f;
    D.vis = false;
}

// precomputeReferencePatches (SparseImageAlign.cc:57-128) for the thread's feature at
// `level` into D and its patch column of s_patch (a feature not inside the level keeps
// its previous patch: copied from prev_patch when that is another buffer); the wave's
// partial sums of the visible features' H into part[wave]
template <int NF, int NW>
__device__ __forceinline__ void align_feat_precompute(const AlignFeat &F, bool vis_in, AlignLevelData &D,
                                                      const AlignLevels &lv, const ygzfe_camera &cam,
                                                      const uint8_t *ref_pyr, int level, float (*s_patch)[NF],
                                                      const float (*prev_patch)[NF], int f, float (*part)[32],
                                                      int wave, int lane) {
    const int border = 3;
    const int W = lv.w[level], H = lv.h[level];
    const float scale = lv.inv_scale[level];
    const float fs = cam.fx * scale;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(ref_pyr + lv.off[level]), 0, (int)((uint32_t)W * (uint32_t)H + 64u), 0x00020000);
    bool here = false;
    if (F.own && F.usable) {
        const float u_ref = F.kx * scale, v_ref = F.ky * scale;
        const int ui = (int)floorf(u_ref), vi = (int)floorf(v_ref);
        here = !(ui - border < 0 || vi - border < 0 || ui + border >= W || vi + border >= H);
        if (here) {
            const float su = u_ref - ui, sv = v_ref - vi;
            const float wtl = wmulf(1.f - su, 1.f - sv), wtr = wmulf(su, 1.f - sv);
            const float wbl = wmulf(1.f - su, sv), wbr = wmulf(su, sv);
            // 7x7 window: rows vi-3..vi+3, cols ui-3..ui+3; R[y][x] = ref(vi-3+y, ui-3+x),
            // kept as packed bytes (all 7 rows in flight at once)
            const uint32_t base = (uint32_t)(vi - 3) * (uint32_t)W + (uint32_t)(ui - 3);
            uint32_t R[7][2];
#pragma unroll
            for (int y = 0; y < 7; y++) load_row7_packed_buf(rs, base + (uint32_t)y * (uint32_t)W, R[y]);
            auto rpx = [&](int y, int x) -> float { return (float)((R[y][x >> 2] >> (8 * (x & 3))) & 0xFFu); };
            // J[y][x]: the bilinear sample at (x + su, y + sv) of the window; the
            // reference's patch and central differences are entries of J:
            // patch = J[py+1][px+1], gx = (J[py+1][px+2] - J[py+1][px]) / 2,
            // gy = (J[py+2][px+1] - J[py][px+1]) / 2 -- the expressions of
            // SparseImageAlign.cc:98-125, each evaluated once (the bilinear sums fused:
            // rounding-level, pose parity 1e-4)
            float J0[6], J1[6], J2[6];
            auto jrow = [&](int y, float (&o)[6]) {
#pragma unroll
                for (int x = 0; x < 6; x++)
                    o[x] = __builtin_fmaf(wbr, rpx(y + 1, x + 1),
                                          __builtin_fmaf(wbl, rpx(y + 1, x),
                                                         __builtin_fmaf(wtr, rpx(y, x + 1), wtl * rpx(y, x))));
            };
            jrow(0, J0);
            jrow(1, J1);
#pragma unroll
            for (int py = 0; py < 4; py++) {
                jrow(py + 2, J2);  // rows py, py+1, py+2 in J0, J1, J2
#pragma unroll
                for (int px = 0; px < 4; px++) {
                    const int pi = py * 4 + px;
                    s_patch[pi][f] = J1[px + 1];
                    D.gx[pi] = 0.5f * (J1[px + 2] - J1[px]);
                    D.gy[pi] = 0.5f * (J2[px + 1] - J0[px + 1]);
                }
#pragma unroll
                for (int x = 0; x < 6; x++) { J0[x] = J1[x]; J1[x] = J2[x]; }
            }
        }
    }
    D.vis = vis_in || here;  // visible_fts_ is never reset between levels (SparseImageAlign.cc:34,81)
    if (!here) {  // jacobian_cache_.setZero() per level; the stale ref patch stays
#pragma unroll
        for (int p = 0; p < 16; p++) { D.gx[p] = 0.f; D.gy[p] = 0.f; }
        if (prev_patch != s_patch) {
#pragma unroll
            for (int p = 0; p < 16; p++) s_patch[p][f] = prev_patch[p][f];
        }
    }
    D.Sxx = 0.f, D.Sxy = 0.f, D.Syy = 0.f;
#pragma unroll
    for (int p = 0; p < 16; p++) {
        D.Sxx = __builtin_fmaf(D.gx[p], D.gx[p], D.Sxx);
        D.Sxy = __builtin_fmaf(D.gx[p], D.gy[p], D.Sxy);
        D.Syy = __builtin_fmaf(D.gy[p], D.gy[p], D.Syy);
    }
    float hv[32];
    feat_hessian(F.X, F.Y, F.Z, D.Sxx, D.Sxy, D.Syy, fs * fs, hv);
    const bool counted = F.own && D.vis;
#pragma unroll
    for (int k = 0; k < 21; k++) hv[k] = counted ? hv[k] : 0.f;
#pragma unroll
    for (int k = 21; k < 32; k++) hv[k] = 0.f;
    const float t = wave_reduce32(hv, lane);
    if ((lane & 1) == 0 && (lane >> 1) < 21) part[wave][lane >> 1] = t;
}

// computeResiduals (SparseImageAlign.cc:130-231) for the thread's feature at pose T:
// the wave's partial Jres / chi2 / count into part[wave], and the per-wave H of the
// features projected out of bounds (usually none) into opart[wave]
template <int NF, int NW>
__device__ __forceinline__ void align_feat_residual(const AlignFeat &F, const AlignLevelData &D, const SE3 &T,
                                                    const AlignLevels &lv,
                                                    const ygzfe_camera &cam, const uint8_t *cur_pyr, int level,
                                                    const float (*s_patch)[NF], int f, float (*part)[32],
                                                    float (*opart)[24], int *out_it, int gi, int wave, int lane) {
    const int border = 3;
    const int W = lv.w[level], H = lv.h[level];
    const float scale = lv.inv_scale[level];
    const float fs = cam.fx * scale;
    // the level as a buffer (the pyramid's tail padding covers the 8-byte row reads)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(cur_pyr + lv.off[level]), 0, (int)((uint32_t)W * (uint32_t)H + 64u), 0x00020000);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = 0.f;
    bool out_now = false;
    if (F.own && D.vis) {
        // The residual loop runs in fused multiply-adds and projects with
        // one reciprocal of z: rounding-level differences from the
        // reference's separate products, inside the 1e-4 pose parity of
        // SparseImgAlign (the Jacobian and the bilinear weights keep the
        // reference's values: jacob_xyz2cam_ff, wmulf)
        const float P3[3] = {F.X, F.Y, F.Z};
        float pc3[3];
        se3_act(T, P3, pc3);
        const float izc = __builtin_amdgcn_rcpf(pc3[2]);  // 1 ulp instead of the IEEE division's ~10 VALU
        const float u = __builtin_fmaf(cam.fx * pc3[0], izc, cam.cx) * scale;
        const float v = __builtin_fmaf(cam.fy * pc3[1], izc, cam.cy) * scale;
        const int ui = (int)floorf(u), vi = (int)floorf(v);
        if (ui < 0 || vi < 0 || ui - border < 0 || vi - border < 0 || ui + border >= W || vi + border >= H) {
            out_now = true;
        } else {
            const float su = u - ui, sv = v - vi;
            const float wtl = wmulf(1.f - su, 1.f - sv), wtr = wmulf(su, 1.f - sv);
            const float wbl = wmulf(1.f - su, sv), wbr = wmulf(su, sv);
            float Sx = 0.f, Sy = 0.f, chi2 = 0.f;
            const uint32_t base = (uint32_t)(vi - 2) * (uint32_t)W + (uint32_t)(ui - 2);
            float r0[5];
            load_row5_buf(rs, base, r0);
#pragma unroll
            for (int py = 0; py < 4; py++) {
                float r1[5];
                load_row5_buf(rs, base + (uint32_t)(py + 1) * (uint32_t)W, r1);
#pragma unroll
                for (int px = 0; px < 4; px++) {
                    const int pi = py * 4 + px;
                    const float ic = __builtin_fmaf(
                        wbr, r1[px + 1], __builtin_fmaf(wbl, r1[px], __builtin_fmaf(wtr, r0[px + 1], wtl * r0[px])));
                    const float res = ic - s_patch[pi][f];
                    Sx = __builtin_fmaf(D.gx[pi], res, Sx);
                    Sy = __builtin_fmaf(D.gy[pi], res, Sy);
                    chi2 = __builtin_fmaf(res, res, chi2);
                }
#pragma unroll
                for (int c = 0; c < 5; c++) r0[c] = r1[c];
            }
            // -(J_xyz2cam^T [Sx Sy]) fs (SparseImageAlign.h:95-116 with x = X/Z, y = Y/Z):
            // the twelve products of jacob_xyz2cam_ff collapsed (rounding-level)
            float X = F.X, Y = F.Y, Z = F.Z;
            asm volatile("" : "+v"(X), "+v"(Y), "+v"(Z));  // recomputed here, not hoisted (register pressure)
            const float zi = __builtin_amdgcn_rcpf(Z);
            const float xh = X * zi, yh = Y * zi, xy = xh * yh;
            const float sx = Sx * fs, sy = Sy * fs;
            acc[0] = zi * sx;
            acc[1] = zi * sy;
            acc[2] = -zi * __builtin_fmaf(xh, sx, yh * sy);
            acc[3] = -__builtin_fmaf(xy, sx, __builtin_fmaf(yh * yh, sy, sy));
            acc[4] = __builtin_fmaf(xy, sy, __builtin_fmaf(xh * xh, sx, sx));
            acc[5] = __builtin_fmaf(xh, sy, -(yh * sx));
            acc[6] = chi2;
            acc[7] = 16.f;
        }
    }
    {
        const float t = wave_reduce8(acc, lane);
        if ((lane & 7) == 0) part[wave][lane >> 3] = t;
    }
    // H_f of the features projected out of bounds, summed per wave (usually none)
    if (__ballot(out_now)) {
        float hv[32];
        feat_hessian(F.X, F.Y, F.Z, D.Sxx, D.Sxy, D.Syy, fs * fs, hv);
#pragma unroll
        for (int k = 0; k < 21; k++) hv[k] = out_now ? hv[k] : 0.f;
#pragma unroll
        for (int k = 21; k < 32; k++) hv[k] = 0.f;
        const float t = wave_reduce32(hv, lane);
        if ((lane & 1) == 0 && (lane >> 1) < 21) opart[wave][lane >> 1] = t;
        if (lane == 0) *out_it = gi;  // every wave that saw one writes the same value
    } else if (lane < 21) {
        opart[wave][lane] = 0.f;
    }
}

// One frame pair per workgroup: wave 0 solves, waves 1..NW-1 own one feature per lane.
// The next level's reference patches, gradients and H are set up by the feature waves
// in the first iteration's solver window (between barriers A and B: they depend on the
// reference frame only), into the other half of a double-buffered patch cache, so only
// the first level waits for its set-up.
// (Two pairs per workgroup, ping-ponging the solver wave, was measured at 0.62 ms per
// 1023 pairs against 0.39: the second pair's 40 feature registers spill at 1024
// threads -- profiles/r04_align_pingpong.txt.)
template <int NT, int METHOD>
__global__ __launch_bounds__(NT) void k_sparse_align_reg(AlignLevels lv, ygzfe_camera cam,
                                                         const AlignJob *__restrict__ jobs,
                                                         float *__restrict__ scratch, size_t scratch_per_job,
                                                         ygzfe_align_result *__restrict__ out) {
    constexpr int NW = NT / 64;
    constexpr int NF = NT - 64;  // features are owned by waves 1..NW-1; wave 0 is the solver
    if (jobs[blockIdx.x].n > NF) {  // more features than feature threads: generic path (not inlined)
        sparse_align_generic<NT>(lv, cam, jobs[blockIdx.x], scratch + blockIdx.x * scratch_per_job, out + blockIdx.x);
        return;
    }
    __shared__ AlignPairLds<NW> P;
    __shared__ LmState s_lm[METHOD == 1 ? 1 : 1];  // read by METHOD 1 (Levenberg-Marquardt) only
    __shared__ float s_part_next[NW][32];  // the next level's H partials
    __shared__ float s_patch[2][16][NF];   // ref_patch_cache_ of the owned features, this level / the next
    const AlignJob &job = jobs[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) align_pair_init(P, job);
    YGZ_STAMP_INIT();
    __syncthreads();
    YGZ_STAMP(9);
    if (METHOD == 1 && wave == 0) {  // Levenberg-Marquardt: lm_round decides each pass's pose
        if (lane == 0) lm_init(s_lm[0], job.T_init);
        int gi = 0;
        for (int level = job.max_level; level >= job.min_level; level--, gi += kLmMaxRounds) {
            __syncthreads();  // L0: the level's H partials are in
            if (level == job.max_level) {
                align_sum_hvis(P, lane);
            } else if (lane < 21) {
                float r = 0.f;
                for (int w = 1; w < NW; w++) r += s_part_next[w][lane];
                P.Hvis[lane] = r;
            }
            if (lane == 0) {
                lm_level_start(s_lm[0]);
                P.T = s_lm[0].T;  // the level's first pass is at the model
                P.brk = 0;
            }
            __syncthreads();  // L0b
            for (int round = 0;; round++) {
                __syncthreads();  // A
                float pk8, hr;
                align_solver_reduce(P, gi + round, lane, pk8, hr);
                float Hu[21], b[6];
#pragma unroll
                for (int k = 0; k < 21; k++) Hu[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hr), 8 + k));
#pragma unroll
                for (int k = 0; k < 6; k++) b[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pk8), k));
                const float chi2sum = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pk8), 6));
                const int cnt = (int)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(pk8), 7));
                if (lane == 0) {
                    lm_round(s_lm[0], Hu, b, chi2sum, cnt, round == 0);
                    P.T = s_lm[0].Te;
                    P.brk = s_lm[0].brk;
                }
                __syncthreads();  // B
                if (P.brk) break;
            }
            __syncthreads();  // L1
        }
        if (tid == 0) lm_result(s_lm[0], out + blockIdx.x);
        return;
    }
    if (wave == 0) {
        SolverRegs S;
        for (int i = 0; i < 4; i++) S.T.q[i] = job.T_init.q[i];
        for (int i = 0; i < 3; i++) S.T.t[i] = job.T_init.t[i];
        S.chi2 = 1e10f;
        S.stop = false;
        for (int level = job.max_level; level >= job.min_level; level--) {
            S.old = S.T;
            __syncthreads();  // L0: level start, the level's H partials are in
            YGZ_STAMP(1);
            if (level == job.max_level) {
                align_sum_hvis(P, lane);
            } else if (lane < 21) {
                float r = 0.f;
                for (int w = 1; w < NW; w++) r += s_part_next[w][lane];
                P.Hvis[lane] = r;
            }
            __syncthreads();  // L0b: part free again
            S.mreg = align_level_inverse(P, lane);  // beside the first residual pass
            YGZ_STAMP(2);
            for (int it = 0; it < 10; it++) {
                __syncthreads();  // A: partials written
                YGZ_STAMP(3);
                const bool brk = align_solver_step<NW>(P, S, it, level * 16 + it, lane, P.part, P.opart, &P.out_it,
                                                      true);
                __syncthreads();  // B: pose / decision published
                YGZ_STAMP(4);
                if (brk) break;
            }
            __syncthreads();  // L1: level end
            YGZ_STAMP(5);
        }
        YGZ_STAMP_FLUSH();
        if (tid == 0) {
            P.chi2 = S.chi2;
            align_pair_result(P, out + blockIdx.x);
        }
        return;
    }
    const int f = tid - 64;
    AlignFeat F;
    AlignLevelData D, Dn;
    align_feat_load(F, D, job, f);
#pragma unroll
    for (int p = 0; p < 16; p++) { s_patch[0][p][f] = 0.f; s_patch[1][p][f] = 0.f; }
    int cb = 0;  // the level's half of the patch cache
    if (METHOD == 1) {  // Levenberg-Marquardt: a residual pass per round at the published pose
        int gi = 0;
        for (int level = job.max_level; level >= job.min_level; level--, gi += kLmMaxRounds) {
            if (level == job.max_level) {
                align_feat_precompute<NF, NW>(F, false, D, lv, cam, job.ref_pyr, level, s_patch[cb], s_patch[cb], f,
                                              P.part, wave, lane);
            } else {
                D = Dn;
                cb ^= 1;
            }
            __syncthreads();  // L0
            __syncthreads();  // L0b
            for (int round = 0;; round++) {
                const SE3 T = P.T;
                align_feat_residual<NF, NW>(F, D, T, lv, cam, job.cur_pyr, level, s_patch[cb], f, P.part, P.opart,
                                            &P.out_it, gi + round, wave, lane);
                __syncthreads();  // A
                if (round == 0 && level > job.min_level)
                    align_feat_precompute<NF, NW>(F, D.vis, Dn, lv, cam, job.ref_pyr, level - 1, s_patch[cb ^ 1],
                                                  s_patch[cb], f, s_part_next, wave, lane);
                __syncthreads();  // B
                if (P.brk) break;
            }
            __syncthreads();  // L1
        }
        return;
    }
    for (int level = job.max_level; level >= job.min_level; level--) {
        if (level == job.max_level) {
            align_feat_precompute<NF, NW>(F, false, D, lv, cam, job.ref_pyr, level, s_patch[cb], s_patch[cb], f,
                                          P.part, wave, lane);
        } else {  // set up during the previous level
            D = Dn;
            cb ^= 1;
        }
        __syncthreads();  // L0
        __syncthreads();  // L0b
        for (int it = 0; it < 10; it++) {
            YGZ_STAMP_AT(11, tid == 64);
            const SE3 T = P.T;
            align_feat_residual<NF, NW>(F, D, T, lv, cam, job.cur_pyr, level, s_patch[cb], f, P.part, P.opart,
                                        &P.out_it, level * 16 + it, wave, lane);
            YGZ_STAMP_AT(12, tid == 64);
            YGZ_STAMP_AT(13, tid == 1023);
            __syncthreads();  // A
            if (it == 0 && level > job.min_level)  // the next level, beside the solver's step
                align_feat_precompute<NF, NW>(F, D.vis, Dn, lv, cam, job.ref_pyr, level - 1, s_patch[cb ^ 1],
                                              s_patch[cb], f, s_part_next, wave, lane);
            __syncthreads();  // B
            if (P.brk) break;
        }
        __syncthreads();  // L1
    }
}

int sparse_align_reg_capacity() { return 1024 - 64; }  // one feature per thread of waves 1..15

hipError_t launch_sparse_align(const AlignLevels &lv, const ygzfe_camera &cam, const AlignJob *jobs, int njobs,
                               float *scratch, size_t scratch_per_job, ygzfe_align_result *out, hipStream_t st,
                               int max_n, int method) {
    if (njobs <= 0) return hipSuccess;
    (void)max_n;
    if (method == 1)
        hipLaunchKernelGGL((k_sparse_align_reg<1024, 1>), dim3(njobs), dim3(1024), 0, st, lv, cam, jobs, scratch,
                           scratch_per_job, out);
    else
        hipLaunchKernelGGL((k_sparse_align_reg<1024, 0>), dim3(njobs), dim3(1024), 0, st, lv, cam, jobs, scratch,
                           scratch_per_job, out);
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

// `win` = the pixel (x0, y0) of a window of the w x h level (stride `stride`,
// ww x wh pixels); returns -1 when an iteration would read outside the window
// (the host then re-runs on the whole level).  Whole level: x0 = y0 = 0.
__device__ int align2d_lane(const uint8_t *win, int stride, int w, int h, int x0, int y0, int ww, int wh,
                            const uint8_t *rpb, const uint8_t *rp, int n_iter, float *px) {
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
        if (ur - hp < x0 || vr - hp < y0 || ur + hp >= x0 + ww || vr + hp >= y0 + wh) return -1;
        const float sx = u - ur, sy = v - vr;
        const float wTL = wmul(1.0 - sx, 1.0 - sy), wTR = wmul(sx, 1.0 - sy);
        const float wBL = wmul(1.0 - sx, sy), wBR = wmul(sx, sy);
        float Jr0 = 0.f, Jr1 = 0.f, Jr2 = 0.f;
        for (int y = 0; y < ps; ++y) {
            const uint8_t *it = win + (size_t)(vr + y - hp - y0) * stride + (ur - hp - x0);
            for (int x = 0; x < ps; ++x, ++it) {
                const float sp = wTL * it[0] + wTR * it[1] + wBL * it[stride] + wBR * it[stride + 1];
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
    const int ok = align2d_lane(img, w, w, h, 0, 0, w, h, pwb + (size_t)i * 100, p + (size_t)i * 64, n_iter, q);
    px[2 * i] = q[0];
    px[2 * i + 1] = q[1];
    conv[i] = (uint8_t)ok;
}

// One Align2D on a window of a host level (the drop-in Align2D(const cv::Mat&, ...)),
// by one wave: lane i owns pixel i of the 8x8 patch (its gradient, bilinear
// sample, residual and the three products), and every lane then folds the 64
// products of an iteration in the reference's pixel order (LDS broadcast reads),
// so the sums are the sequential ones of Align.cc:74-96 bit for bit.
// status 0 / 1 = converged flag, -1 = the window was too small.
__global__ __launch_bounds__(64) void k_align2d_window(const uint8_t *__restrict__ win, int stride, int w, int h,
                                                       int x0, int y0, int ww, int wh,
                                                       const uint8_t *__restrict__ pwb,
                                                       const uint8_t *__restrict__ p, int n_iter,
                                                       float *__restrict__ px, int *__restrict__ status) {
    __shared__ float sj[2][64], sp[3][64];
    const int lane = threadIdx.x, y = lane >> 3, x = lane & 7;
    const int hp = 4, step = 10;
    // reference gradients (Align.cc:37-64): 0.5 * central difference in double, to float
    const uint8_t *it = pwb + (y + 1) * step + 1 + x;
    const float J0 = (float)(0.5 * (it[1] - it[-1]));
    const float J1 = (float)(0.5 * (it[step] - it[-step]));
    const float refp = (float)p[lane];
    sj[0][lane] = J0;
    sj[1][lane] = J1;
    __syncthreads();
    float H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 64; i++) {  // H += J J^T in pixel order (Align.cc:58-63)
        const float J[3] = {sj[0][i], sj[1][i], 1.f};
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) H[r * 3 + c] += J[r] * J[c];
    }
    float Hi[9];
    inverse3(H, Hi);
    float mean_diff = 0.f, u = px[0], v = px[1];
    const float min_upd2 = (float)(0.03 * 0.03);
    int converged = 0, st = 0;
    for (int iter = 0; iter < n_iter; ++iter) {
        const int ur = (int)floorf(u), vr = (int)floorf(v);
        if (ur < hp || vr < hp || ur >= w - hp || vr >= h - hp) break;
        if (isnan(u) || isnan(v)) { st = -2; break; }  // Align.cc:63-65: false, estimate untouched
        if (ur - hp < x0 || vr - hp < y0 || ur + hp >= x0 + ww || vr + hp >= y0 + wh) { st = -1; break; }
        const float sx = u - ur, sy = v - vr;
        const float wTL = wmul(1.0 - sx, 1.0 - sy), wTR = wmul(sx, 1.0 - sy);
        const float wBL = wmul(1.0 - sx, sy), wBR = wmul(sx, sy);
        const uint8_t *q = win + (size_t)(vr + y - hp - y0) * stride + (ur - hp - x0) + x;
        const float spx = wTL * q[0] + wTR * q[1] + wBL * q[stride] + wBR * q[stride + 1];
        const float res = spx - refp + mean_diff;
        __syncthreads();  // the previous iteration's folds are done reading sp
        sp[0][lane] = res * J0;
        sp[1][lane] = res * J1;
        sp[2][lane] = res;
        __syncthreads();
        float Jr0 = 0.f, Jr1 = 0.f, Jr2 = 0.f;
        for (int i = 0; i < 64; i++) {
            Jr0 -= sp[0][i];
            Jr1 -= sp[1][i];
            Jr2 -= sp[2][i];
        }
        const float u0 = Hi[0] * Jr0 + Hi[1] * Jr1 + Hi[2] * Jr2;
        const float u1 = Hi[3] * Jr0 + Hi[4] * Jr1 + Hi[5] * Jr2;
        const float u2 = Hi[6] * Jr0 + Hi[7] * Jr1 + Hi[8] * Jr2;
        u += u0;
        v += u1;
        mean_diff += u2;
        if (u0 * u0 + u1 * u1 < min_upd2) { converged = 1; break; }
    }
    if (lane == 0) {
        if (st == 0) {
            px[0] = u;
            px[1] = v;
            st = converged;
        } else if (st == -2) {
            st = 0;
        }
        status[0] = st;
    }
}

// Stream placement probe: one lane waits `us` microseconds on the 100 MHz
// real-time counter (bounded: it always ends), then exits; k_empty does nothing.
__global__ void k_hold_us(int us) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime(), ticks = (uint64_t)us * 100u;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
__global__ void k_empty() {}

hipError_t launch_hold_us(int us, hipStream_t st) {
    hipLaunchKernelGGL(k_hold_us, dim3(1), dim3(64), 0, st, us);
    return hipGetLastError();
}
hipError_t launch_empty(hipStream_t st) {
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    return hipGetLastError();
}

hipError_t launch_align2d_window(const uint8_t *win, int stride, int w, int h, int x0, int y0, int ww, int wh,
                                 const uint8_t *pwb, const uint8_t *p, int n_iter, float *px, int *status,
                                 hipStream_t st) {
    hipLaunchKernelGGL(k_align2d_window, dim3(1), dim3(64), 0, st, win, stride, w, h, x0, y0, ww, wh, pwb, p, n_iter,
                       px, status);
    return hipGetLastError();
}

hipError_t launch_align2d(const uint8_t *img, int w, int h, int n, const uint8_t *pwb, const uint8_t *p,
                          int n_iter, float *px, uint8_t *conv, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_align2d, dim3((n + 255) / 256), dim3(256), 0, st, img, w, h, n, pwb, p, n_iter, px, conv);
    return hipGetLastError();
}

// ------------------------------------------------------------------ FindDirectProjection
// One (map point, keyframe) item: GetWarpAffineMatrix + GetBestSearchLevel +
// WarpAffine 10x10 + Align2D at the search level, by ONE wave: the wave-uniform
// warp set-up, lanes own the 100 warped pixels (2 per lane) and then pixel
// `lane` of the 8x8 patch (gradient, bilinear sample, residual, products), and
// every lane folds the 64 products of an iteration in the reference's pixel order
// (LDS broadcast reads), so H, Jres and the update are Align.cc:8-105's
// sequential float sums bit for bit.  px (level-0 px) in/out, wave-uniform.
struct DirectLds {
    uint8_t pb[112];    // the warped 10x10 patch with its 1-px border (Align.cc:37-64)
    float j[2][64];     // reference gradients in pixel order
    float4 prod[64];    // res * J0, res * J1, res of one iteration, in pixel order
};

__device__ int find_direct_wave(const uint8_t *__restrict__ ref_pyr, const AlignLevels &rlv,
                                const uint8_t *__restrict__ cur_pyr, const AlignLevels &clv, int nlevels,
                                const float *__restrict__ scale, float inv_sigma2_1, const ygzfe_camera &cam,
                                const ygzfe_kp &kp, const float pt[3], const ygzfe_se3 &Tcr, float px[2], int *level,
                                int lane, DirectLds &S) {
    SE3 T;
    for (int k = 0; k < 4; k++) T.q[k] = Tcr.q[k];
    for (int k = 0; k < 3; k++) T.t[k] = Tcr.t[k];
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
    *level = sl;
    // WarpAffine 10x10 (ORBmatcher.cc:1549-1571): pixels lane and lane + 64
    const uint8_t *rimg = ref_pyr + rlv.off[oc];
    const int rw = rlv.w[oc], rh = rlv.h[oc];
    const float det = A0 * A3 - A2 * A1;
    const float inv = 1.f / det;
    const float R00 = A3 * inv, R01 = -A1 * inv, R10 = -A2 * inv, R11 = A0 * inv;
    const float prx = kp.x / scale[oc], pry = kp.y / scale[oc];
    for (int k = lane; k < 100; k += 64) {
        const int y = k / 10, x = k - 10 * (k / 10);
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
        S.pb[k] = val;
    }
    wave_lds_order();
    // Align2D (Align.cc:8-105) at the search level; pixel (y, x) = lane; the patch
    // without border is pb[(y + 1) * 10 + 1 + x] (ORBmatcher.cc:1590-1594)
    const int hp = 4, step = 10, y = lane >> 3, x = lane & 7;
    const uint8_t *it = S.pb + (y + 1) * step + 1 + x;
    const float J0 = (float)(0.5 * (it[1] - it[-1]));
    const float J1 = (float)(0.5 * (it[step] - it[-step]));
    const float refp = (float)it[0];
    S.j[0][lane] = J0;
    S.j[1][lane] = J1;
    wave_lds_order();
    // H += J J^T in pixel order (Align.cc:58-63) with J = (J0, J1, 1): the five distinct
    // sums (H is symmetric term by term, J * 1 is exact, and 64 ones sum to 64 exactly)
    float h00 = 0.f, h01 = 0.f, h02 = 0.f, h11 = 0.f, h12 = 0.f;
    for (int i = 0; i < 64; i++) {
        const float a = S.j[0][i], b = S.j[1][i];
        h00 += a * a;
        h01 += a * b;
        h02 += a;
        h11 += b * b;
        h12 += b;
    }
    const float H[9] = {h00, h01, h02, h01, h11, h12, h02, h12, 64.f};
    float Hi[9];
    inverse3(H, Hi);
    const uint8_t *img = cur_pyr + clv.off[sl];
    const int w = clv.w[sl], h = clv.h[sl];
    const float q0 = px[0] * clv.inv_scale[sl], q1 = px[1] * clv.inv_scale[sl];
    float mean_diff = 0.f, u = q0, v = q1;
    const float min_upd2 = (float)(0.03 * 0.03);
    int converged = 0;
    bool nan_stop = false;
    for (int iter = 0; iter < 10; ++iter) {
        const int ur = (int)floorf(u), vr = (int)floorf(v);
        if (ur < hp || vr < hp || ur >= w - hp || vr >= h - hp) break;
        if (isnan(u) || isnan(v)) { nan_stop = true; break; }  // Align.cc: returns false, estimate untouched
        const float sx = u - ur, sy = v - vr;
        const float wTL = wmul(1.0 - sx, 1.0 - sy), wTR = wmul(sx, 1.0 - sy);
        const float wBL = wmul(1.0 - sx, sy), wBR = wmul(sx, sy);
        const uint8_t *q = img + (size_t)(vr + y - hp) * w + (ur - hp) + x;
        const float spx = wTL * q[0] + wTR * q[1] + wBL * q[w] + wBR * q[w + 1];
        const float res = spx - refp + mean_diff;
        S.prod[lane] = make_float4(res * J0, res * J1, res, 0.f);
        wave_lds_order();
        float Jr0 = 0.f, Jr1 = 0.f, Jr2 = 0.f;
        for (int i = 0; i < 64; i++) {
            const float4 p4 = S.prod[i];
            Jr0 -= p4.x;
            Jr1 -= p4.y;
            Jr2 -= p4.z;
        }
        wave_lds_order();
        const float u0 = Hi[0] * Jr0 + Hi[1] * Jr1 + Hi[2] * Jr2;
        const float u1 = Hi[3] * Jr0 + Hi[4] * Jr1 + Hi[5] * Jr2;
        const float u2 = Hi[6] * Jr0 + Hi[7] * Jr1 + Hi[8] * Jr2;
        u += u0;
        v += u1;
        mean_diff += u2;
        if (u0 * u0 + u1 * u1 < min_upd2) { converged = 1; break; }
    }
    if (nan_stop) {
        u = q0;
        v = q1;
        converged = 0;
    }
    px[0] = u * scale[sl];
    px[1] = v * scale[sl];
    return converged;
}

// one wave per item, four per workgroup
constexpr int kDirectWaves = 4;
__global__ __launch_bounds__(64 * kDirectWaves) void k_find_direct(
    const uint8_t *const *__restrict__ ref_pyrs, AlignLevels rlv, const uint8_t *__restrict__ cur_pyr,
    AlignLevels clv, int nlevels, const float *__restrict__ scale, float inv_sigma2_1, ygzfe_camera cam, int n,
    const int32_t *__restrict__ ref_index, const ygzfe_kp *__restrict__ kps, const float *__restrict__ pts,
    const ygzfe_se3 *__restrict__ Tcr, float *__restrict__ px_io, int32_t *__restrict__ level_out,
    uint8_t *__restrict__ ok_out) {
    __shared__ DirectLds s[kDirectWaves];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int i = blockIdx.x * kDirectWaves + wave;
    if (i >= n) return;
    const float pt[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
    float px[2] = {px_io[2 * i], px_io[2 * i + 1]};
    int sl;
    const int ok = find_direct_wave(ref_pyrs[ref_index[i]], rlv, cur_pyr, clv, nlevels, scale, inv_sigma2_1, cam,
                                    kps[i], pt, Tcr[i], px, &sl, lane, s[wave]);
    if (lane == 0) {
        level_out[i] = sl;
        px_io[2 * i] = px[0];
        px_io[2 * i + 1] = px[1];
        ok_out[i] = (uint8_t)ok;
    }
}

hipError_t launch_find_direct(const uint8_t *const *ref_pyrs, const AlignLevels &ref_lv, const uint8_t *cur_pyr,
                              const AlignLevels &cur_lv, int nlevels, const float *scale, float inv_sigma2_1,
                              const ygzfe_camera &cam, int n, const int32_t *ref_index, const ygzfe_kp *kp_ref,
                              const float *pt_ref, const ygzfe_se3 *T_cr, float *px, int32_t *level, uint8_t *ok,
                              hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_find_direct, dim3((n + kDirectWaves - 1) / kDirectWaves), dim3(64 * kDirectWaves), 0, st,
                       ref_pyrs, ref_lv, cur_pyr, cur_lv, nlevels, scale, inv_sigma2_1, cam, n, ref_index, kp_ref,
                       pt_ref, T_cr, px, level, ok);
    return hipGetLastError();
}

// ------------------------------------------------------------------ SearchLocalPointsDirect
// Tracking::SearchLocalPointsDirect (Tracking.cc:2258-2410) as one speculative
// pass: every (map point, keyframe) item of every point runs FindDirectProjection
// at once (it is a pure function of the point, the keyframe and the current
// frame), then k_direct_select walks each point's items in SelectNearestKeyframe
// order (Tracking.cc:2412-2432) and keeps the first that succeeded and lies
// inside the 20 px border (Tracking.cc:2287-2296 / 2356-2364): the same answer
// the reference's sequential loop with its `break` gives.

__global__ __launch_bounds__(64 * kDirectWaves) void k_direct_items(
    const uint8_t *const *__restrict__ ref_pyrs, AlignLevels lv, const uint8_t *__restrict__ cur_pyr, int nlevels,
    const float *__restrict__ scale, float inv_sigma2_1, ygzfe_camera cam, int n,
    const DirectItem *__restrict__ items, const ygzfe_se3 *__restrict__ tcr_tab, const float *__restrict__ px_proj,
    float *__restrict__ px_out, uint8_t *__restrict__ ok_out) {
    __shared__ DirectLds s[kDirectWaves];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int i = blockIdx.x * kDirectWaves + wave;
    if (i >= n) return;
    const DirectItem it = scalar_load(items + i);
    const ygzfe_se3 Tcr = scalar_load(tcr_tab + it.tcr);
    float px[2] = {px_proj[2 * it.point], px_proj[2 * it.point + 1]};  // (mTrackProjX, mTrackProjY)
    int sl;
    const int ok = find_direct_wave(ref_pyrs[it.ref], lv, cur_pyr, lv, nlevels, scale, inv_sigma2_1, cam, it.kp,
                                    it.pt, Tcr, px, &sl, lane, s[wave]);
    if (lane == 0) {
        px_out[2 * i] = px[0];
        px_out[2 * i + 1] = px[1];
        ok_out[i] = (uint8_t)ok;
    }
}

// Tracking::SearchLocalPointsDirect's sequential part (Tracking.cc:2258-2410) in one
// workgroup, per chunk of 2,048 cache points:
//   A  every point's first converged in-border item, its matched cell mk and its
//      projected cell c (LDS); "pre" = c already marked by an earlier chunk.  A point
//      that could mark a cell (m >= 0, mk >= 0, not pre) enters a per-chunk LDS hash
//      cell -> its earliest such point W(cell);
//   B  a point j is skipped by the reference's loop iff an earlier success marked c_j.
//      W(c_j) >= j: nothing earlier can, j is final.  W(c_j) = i0 < j with i0 itself
//      final (nothing earlier can mark c_{i0}): i0 is a success, j skipped, final.
//      Otherwise j is pending;
//   C  wave 0 resolves the pending points in order (rare: a chain of points in shared
//      cells), each by one ballot scan of [i0, j) for a success that marked c_j;
//   D  statuses out, the chunk's successes marked in the grid bitmap for later chunks.
// The success count decides mnCacheHitTh (:2334-2340); then all 16 waves take the
// local-map points, which have no grid (:2348-2405).
__device__ __forceinline__ int direct_first_item(int i, const int32_t *__restrict__ item_ptr,
                                                 const float *__restrict__ px_item,
                                                 const uint8_t *__restrict__ ok_item, float border, float cols,
                                                 float rows, float &u, float &v) {
    u = 0.f;
    v = 0.f;
    for (int k = item_ptr[i]; k < item_ptr[i + 1]; k++) {
        if (!ok_item[k]) continue;
        const float x = px_item[2 * k], y = px_item[2 * k + 1];
        if (x < border || y < border || x >= cols - border || y >= rows - border) continue;
        // px_ave = sum(matched_pixels) / size() with exactly one pixel (Tracking.cc:2305-2309)
        u = x / 1.0f;
        v = y / 1.0f;
        return k;
    }
    return -1;
}

// static_cast<int>(x / grid_size) per axis, k = gy * grid_cols + gx; -2 when k is outside the grid
__device__ __forceinline__ int direct_cell(float x, float y, int grid_size, int grid_cols, int ncell) {
    const float gs = (float)grid_size;
    const int gx = (int)(x / gs), gy = (int)(y / gs);
    const long k = (long)gy * grid_cols + gx;
    return (k >= 0 && k < ncell) ? (int)k : -2;
}

constexpr int kReplayHashSlots = 4096;  // >= 2 x the chunk's points: load factor <= 1/2

__device__ __forceinline__ uint32_t replay_hash(int cell) { return ((uint32_t)cell * 2654435761u) >> 20; }

// W(cell) = min(W(cell), k): open addressing, keys claimed by CAS (-1 = free)
__device__ __forceinline__ void replay_hash_min(int *hk, int *hv, int cell, int k) {
    uint32_t h = replay_hash(cell);
    while (true) {
        const int prev = atomicCAS(&hk[h], -1, cell);
        if (prev == -1 || prev == cell) {
            atomicMin(&hv[h], k);
            return;
        }
        h = (h + 1) & (kReplayHashSlots - 1);
    }
}

__device__ __forceinline__ int replay_hash_find(const int *hk, const int *hv, int cell) {
    uint32_t h = replay_hash(cell);
    while (true) {
        const int key = hk[h];
        if (key == cell) return hv[h];
        if (key == -1) return 0x7fffffff;
        h = (h + 1) & (kReplayHashSlots - 1);
    }
}

__global__ __launch_bounds__(1024) void k_direct_replay(int n_cache, int n_local, const int32_t *__restrict__ item_ptr,
                                                        const float *__restrict__ px_item,
                                                        const uint8_t *__restrict__ ok_item,
                                                        const float *__restrict__ px_proj, float border, int cols,
                                                        int rows, int grid_size, int grid_cols, int ncell,
                                                        int cache_hit_th, float *__restrict__ px_out,
                                                        int32_t *__restrict__ matched, int32_t *__restrict__ status,
                                                        int32_t *__restrict__ hdr) {
    extern __shared__ uint32_t grid[];
    __shared__ int s_cnt;
    constexpr int kChunk = kReplayHashSlots / 2;
    __shared__ int s_m[kChunk], s_c[kChunk], s_mk[kChunk], s_st[kChunk];
    __shared__ float s_u[kChunk], s_v[kChunk];
    __shared__ int s_hk[kReplayHashSlots], s_hv[kReplayHashSlots];
    const int tid = threadIdx.x, lane = tid & 63;
    const int nwords = (ncell + 31) >> 5;
    for (int w = tid; w < nwords; w += blockDim.x) grid[w] = 0u;
    if (tid == 0) s_cnt = 0;
    const float fc = (float)cols, fr = (float)rows;
    for (int c0 = 0; c0 < n_cache; c0 += kChunk) {
        const int nc = min(kChunk, n_cache - c0);
        for (int h = tid; h < kReplayHashSlots; h += blockDim.x) {
            s_hk[h] = -1;
            s_hv[h] = 0x7fffffff;
        }
        __syncthreads();  // the hash clear; the grid (cleared / the last chunk's marks)
        // A
        for (int k = tid; k < nc; k += blockDim.x) {
            const int i = c0 + k;
            float u, v;
            const int m = direct_first_item(i, item_ptr, px_item, ok_item, border, fc, fr, u, v);
            int mk = -1;
            if (m >= 0) {
                mk = direct_cell(u, v, grid_size, grid_cols, ncell);
                if (mk < 0) mk = -1;  // the reference writes outside its grid; never read back here
            }
            const int c = direct_cell(px_proj[2 * i], px_proj[2 * i + 1], grid_size, grid_cols, ncell);
            const bool pre = c >= 0 && ((grid[c >> 5] >> (c & 31)) & 1u);
            s_m[k] = m;
            s_u[k] = u;
            s_v[k] = v;
            s_c[k] = c;
            s_mk[k] = mk;
            s_st[k] = pre ? 2 : -1;
            if (!pre && m >= 0 && mk >= 0) replay_hash_min(s_hk, s_hv, mk, k);
        }
        __syncthreads();
        // B
        for (int k = tid; k < nc; k += blockDim.x) {
            if (s_st[k] == 2) continue;  // pre-marked: skipped
            const int c = s_c[k];
            int st = s_m[k] >= 0 ? 1 : 0;
            if (c >= 0) {
                const int i0 = replay_hash_find(s_hk, s_hv, c);
                if (i0 < k) {  // i0: not pre, m >= 0, final unless an earlier point can mark c_{i0}
                    const int ci0 = s_c[i0];
                    st = (ci0 >= 0 && replay_hash_find(s_hk, s_hv, ci0) < i0) ? -1 : 2;
                }
            }
            s_st[k] = st;
        }
        __syncthreads();
        // C
        if (tid < 64) {
            for (int base = 0; base < nc; base += 64) {
                uint64_t pend = __ballot(base + lane < nc && s_st[base + lane] == -1);
                while (pend) {
                    const int j = base + (int)__builtin_ctzll(pend);
                    pend &= pend - 1;
                    const int cj = s_c[j];
                    const int i0 = replay_hash_find(s_hk, s_hv, cj);
                    bool hit = false;
                    for (int b = i0; b < j && !hit; b += 64) {
                        const int i = b + lane;
                        hit = __ballot(i < j && s_mk[i] == cj && s_st[i] == 1) != 0;
                    }
                    if (lane == 0) s_st[j] = hit ? 2 : (s_m[j] >= 0 ? 1 : 0);
                    wave_lds_order();
                }
            }
        }
        __syncthreads();
        // D
        int mine = 0;
        for (int k = tid; k < nc; k += blockDim.x) {
            const int i = c0 + k, st = s_st[k], mk = s_mk[k];
            const bool ok = st == 1;
            status[i] = st;
            matched[i] = ok ? s_m[k] : -1;
            px_out[2 * i] = ok ? s_u[k] : 0.f;
            px_out[2 * i + 1] = ok ? s_v[k] : 0.f;
            if (ok && mk >= 0) atomicOr(&grid[mk >> 5], 1u << (mk & 31));
            mine += ok;
        }
        if (mine) atomicAdd(&s_cnt, mine);
        __syncthreads();  // the chunk's LDS arrays are free again
    }
    __syncthreads();
    const int n_success = s_cnt;
    const bool local_ran = !(n_success > cache_hit_th);
    if (tid == 0) {
        hdr[0] = n_success;
        hdr[1] = local_ran ? 1 : 0;
    }
    for (int i = n_cache + tid; i < n_cache + n_local; i += blockDim.x) {
        float u = 0.f, v = 0.f;
        const int m = local_ran ? direct_first_item(i, item_ptr, px_item, ok_item, border, fc, fr, u, v) : -1;
        status[i] = local_ran ? (m >= 0 ? 1 : 0) : 3;
        matched[i] = m;
        px_out[2 * i] = u;
        px_out[2 * i + 1] = v;
    }
}

hipError_t launch_search_direct(const uint8_t *const *ref_pyrs, const AlignLevels &lv, const uint8_t *cur_pyr,
                                int nlevels, const float *scale, float inv_sigma2_1, const ygzfe_camera &cam,
                                int n_cache, int n_local, int n_items, const int32_t *item_ptr, const void *items,
                                const ygzfe_se3 *tcr_tab, const float *px_proj, float *px_item, uint8_t *ok_item, float border, int grid_size,
                                int cache_hit_th, float *px_out, int32_t *matched, int32_t *status, int32_t *hdr,
                                hipStream_t st) {
    const int n_points = n_cache + n_local;
    if (n_items > 0)
        hipLaunchKernelGGL(k_direct_items, dim3((n_items + kDirectWaves - 1) / kDirectWaves), dim3(64 * kDirectWaves), 0,
                           st, ref_pyrs, lv, cur_pyr,
                           nlevels, scale, inv_sigma2_1, cam, n_items, (const DirectItem *)items, tcr_tab, px_proj, px_item,
                           ok_item);
    const int grid_cols = lv.w[0] / grid_size, ncell = (lv.h[0] / grid_size) * grid_cols;
    const size_t lds = (size_t)((ncell + 31) / 32) * 4 + 4;
    hipLaunchKernelGGL(k_direct_replay, dim3(1), dim3(1024), lds, st, n_cache, n_local, item_ptr, px_item, ok_item,
                       px_proj, border, lv.w[0], lv.h[0], grid_size, grid_cols, ncell, cache_hit_th, px_out, matched,
                       status, hdr);
    (void)n_points;
    return hipGetLastError();
}

}  // namespace ygzfe
