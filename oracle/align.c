/*
 * align.c — CPU restatement of SparseImgAlign (SVO inverse-compositional GN on
 * SE3), Align2D and ORBmatcher::FindDirectProjection.
 * TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline); see ygz_oracle.h.
 *
 * Float semantics follow the reference expressions, including the places
 * where a double literal promotes an expression to double (bilinear weights
 * `(1.0 - u) * (1.0 - v)`, JacobXYZ2Cam's `1. / z`, Align2D's `0.5 * (...)`).
 * Sophus SE3f is restated as (unit quaternion, translation) with Eigen's
 * quaternion product/normalise/_transformVector; Eigen's LDLT (diagonal
 * pivoting, zero pivots -> 0) and 3x3/2x2 cofactor inverses are restated.
 */
#include "ygz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------- Sophus SE3f ---------------- */
static void quat_mul(const float a[4], const float b[4], float o[4]) {
    /* Eigen Quaternion product, coeffs (x,y,z,w) */
    float x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    float y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    float z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    float w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}

static void quat_normalize(float q[4]) {
    float n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    float n = sqrtf(n2);
    for (int i = 0; i < 4; i++) q[i] = q[i] / n;
}

static void quat_rotate(const float q[4], const float v[3], float o[3]) {
    /* Eigen QuaternionBase::_transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv */
    float uv0 = q[1] * v[2] - q[2] * v[1];
    float uv1 = q[2] * v[0] - q[0] * v[2];
    float uv2 = q[0] * v[1] - q[1] * v[0];
    uv0 += uv0; uv1 += uv1; uv2 += uv2;
    o[0] = v[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
    o[1] = v[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
    o[2] = v[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
}

void ygzo_se3_act(const ygzo_se3 *T, const float p[3], float out[3]) {
    float r[3];
    quat_rotate(T->q, p, r);
    out[0] = r[0] + T->t[0]; out[1] = r[1] + T->t[1]; out[2] = r[2] + T->t[2];
}

void ygzo_se3_mul(const ygzo_se3 *a, const ygzo_se3 *b, ygzo_se3 *out) {
    /* se3.hpp:160-163,268-271: t += R_a t_b; q = normalize(q_a q_b) */
    float r[3], q[4];
    quat_rotate(a->q, b->t, r);
    float t0 = a->t[0] + r[0], t1 = a->t[1] + r[1], t2 = a->t[2] + r[2];
    quat_mul(a->q, b->q, q);
    quat_normalize(q);
    memcpy(out->q, q, sizeof(q));
    out->t[0] = t0; out->t[1] = t1; out->t[2] = t2;
}

void ygzo_se3_inverse(const ygzo_se3 *T, ygzo_se3 *out) {
    float qi[4] = {-T->q[0], -T->q[1], -T->q[2], T->q[3]};
    float mt[3] = {-T->t[0], -T->t[1], -T->t[2]}, r[3];
    quat_rotate(qi, mt, r);
    memcpy(out->q, qi, sizeof(qi));
    memcpy(out->t, r, sizeof(r));
}

static void quat_to_mat(const float q[4], float R[9]) {
    /* Eigen QuaternionBase::toRotationMatrix */
    const float tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const float twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const float txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const float tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

/* SE3::exp (se3.hpp:407-428) with SO3::expAndTheta (so3.hpp:426-455); tangent
 * order (upsilon, omega); float epsilon 1e-5 (sophus.hpp:56-60). */
void ygzo_se3_exp(const float a[6], ygzo_se3 *out) {
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
        const float s = sinf(half_theta);
        imag = s / theta;
        real = cosf(half_theta);
    }
    float q[4] = {imag * w0, imag * w1, imag * w2, real};
    /* Omega = hat(omega), Omega^2 */
    float O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0}, O2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            O2[i * 3 + j] = O[i * 3 + 0] * O[0 * 3 + j] + O[i * 3 + 1] * O[1 * 3 + j] + O[i * 3 + 2] * O[2 * 3 + j];
    float V[9];
    if (theta < eps) {
        quat_to_mat(q, V); /* "That is an accurate expansion!" — V = R */
    } else {
        const float c1 = (1.f - cosf(theta)) / theta_sq;
        const float c2 = (theta - sinf(theta)) / (theta_sq * theta);
        for (int i = 0; i < 9; i++) V[i] = ((i % 4 == 0) ? 1.f : 0.f) + c1 * O[i] + c2 * O2[i];
    }
    for (int i = 0; i < 3; i++) out->t[i] = V[i * 3 + 0] * a[0] + V[i * 3 + 1] * a[1] + V[i * 3 + 2] * a[2];
    memcpy(out->q, q, sizeof(q));
}

/* Eigen LDLT<Matrix6f> with diagonal pivoting; solve() treats |D_i| <= FLT_MIN as 0. */
static void ldlt_solve6(const float Hin[36], const float b[6], float x[6]) {
    float A[36];
    int perm[6];
    memcpy(A, Hin, sizeof(A));
    for (int i = 0; i < 6; i++) perm[i] = i;
    int trans[6];
    for (int k = 0; k < 6; k++) {
        int piv = k;
        float big = fabsf(A[k * 6 + k]);
        for (int i = k + 1; i < 6; i++)
            if (fabsf(A[i * 6 + i]) > big) { big = fabsf(A[i * 6 + i]); piv = i; }
        trans[k] = piv;
        if (piv != k) {
            /* Eigen LDLT_Traits: transposition restricted to the lower triangle */
            for (int j = 0; j < k; j++) { float t = A[k * 6 + j]; A[k * 6 + j] = A[piv * 6 + j]; A[piv * 6 + j] = t; }
            for (int i = piv + 1; i < 6; i++) { float t = A[i * 6 + k]; A[i * 6 + k] = A[i * 6 + piv]; A[i * 6 + piv] = t; }
            { float t = A[k * 6 + k]; A[k * 6 + k] = A[piv * 6 + piv]; A[piv * 6 + piv] = t; }
            for (int i = k + 1; i < piv; i++) { float t = A[i * 6 + k]; A[i * 6 + k] = A[piv * 6 + i]; A[piv * 6 + i] = t; }
            int t = perm[k]; perm[k] = perm[piv]; perm[piv] = t;
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
        float akk = A[k * 6 + k];
        if (k == 0 && akk == 0.f) { /* whole diagonal zero: Eigen stops, identity transpositions */
            for (int i = 0; i < 6; i++) perm[i] = i;
            break;
        }
        if (akk != 0.f)
            for (int i = k + 1; i < 6; i++) A[i * 6 + k] /= akk;
    }
    (void)trans;
    float y[6];
    for (int i = 0; i < 6; i++) y[i] = b[perm[i]];
    for (int i = 0; i < 6; i++) { /* L y = Pb, unit lower */
        float s = y[i];
        for (int j = 0; j < i; j++) s -= A[i * 6 + j] * y[j];
        y[i] = s;
    }
    for (int i = 0; i < 6; i++) {
        float d = A[i * 6 + i];
        y[i] = fabsf(d) > 1.17549435e-38f ? y[i] / d : 0.f;
    }
    for (int i = 5; i >= 0; i--) { /* L^T */
        float s = y[i];
        for (int j = i + 1; j < 6; j++) s -= A[j * 6 + i] * y[j];
        y[i] = s;
    }
    for (int i = 0; i < 6; i++) x[perm[i]] = y[i];
}

/* JacobXYZ2Cam (SparseImageAlign.h:95-116): translation first, pre-negated. */
static void jacob_xyz2cam(const float p[3], float J[12]) {
    const float x = p[0], y = p[1];
    const float z_inv = (float)(1. / (double)p[2]);
    const float z_inv_2 = z_inv * z_inv;
    J[0] = -z_inv; J[1] = 0.f; J[2] = x * z_inv_2;
    J[3] = y * J[2];
    J[4] = (float)(-(1.0 + (double)(x * J[2])));
    J[5] = y * z_inv;
    J[6] = 0.f; J[7] = -z_inv; J[8] = y * z_inv_2;
    J[9] = (float)(1.0 + (double)(y * J[8]));
    J[10] = -J[3];
    J[11] = -x * z_inv;
}

static inline float wmul(double a, double b) { return (float)(a * b); }

enum { PS = 4, PH = 2, PA = 16 };

/* computeResiduals (SparseImageAlign.cc:130-231) at T over the visible features: returns
 * chi2 (the sum; the caller divides by n_meas_), adds the measurement count to *n_meas,
 * and with linearize the H / Jres terms (unit weights: the robust cost is never enabled) */
static float align_residuals(const uint8_t *cimg, int cw, int chh, float scale, const ygzo_cam *cam,
                             const float *xyz_ref, const uint8_t *vis, const float *patch, const float *jac, int n,
                             const ygzo_se3 *T, int linearize, size_t *n_meas, float H[36], float Jres[6]) {
    const int border = PH + 1, cs = cw;
    float chi2 = 0.f;
    /* the sums live in locals and are written out once: through the (possibly aliasing)
     * pointer parameters every += would be a store + reload, which made this CPU baseline
     * 2.3x slower than the restatement it replaced */
    float h[36], jr[6];
    memcpy(h, H, sizeof(h));
    memcpy(jr, Jres, sizeof(jr));
    size_t nm = *n_meas;
    for (int i = 0; i < n; i++) {
        if (!vis[i]) continue;
        float pc3[3];
        ygzo_se3_act(T, xyz_ref + 3 * (size_t)i, pc3);
        const float u = (cam->fx * pc3[0] / pc3[2] + cam->cx) * scale;
        const float v = (cam->fy * pc3[1] / pc3[2] + cam->cy) * scale;
        const int ui = (int)floorf(u), vi = (int)floorf(v);
        if (ui < 0 || vi < 0 || ui - border < 0 || vi - border < 0 || ui + border >= cw || vi + border >= chh)
            continue;
        const float su = u - ui, sv = v - vi;
        const float wtl = wmul(1.0 - su, 1.0 - sv), wtr = wmul(su, 1.0 - sv);
        const float wbl = wmul(1.0 - su, sv), wbr = wmul(su, sv);
        int pcn = 0;
        for (int y = 0; y < PS; ++y) {
            const uint8_t *p = cimg + (size_t)(vi + y - PH) * cs + (ui - PH);
            for (int xx = 0; xx < PS; ++xx, ++p, ++pcn) {
                const float ic = wtl * p[0] + wtr * p[1] + wbl * p[cs] + wbr * p[cs + 1];
                const float res = ic - patch[(size_t)i * PA + pcn];
                chi2 += res * res * 1.0f;
                nm++;
                if (!linearize) continue;
                const float *J = jac + ((size_t)i * PA + pcn) * 6;
                for (int r = 0; r < 6; r++) {
                    for (int c = 0; c < 6; c++) h[r * 6 + c] += J[r] * J[c] * 1.0f;
                    jr[r] -= J[r] * res * 1.0f;
                }
            }
        }
    }
    *n_meas = nm;
    if (linearize) {
        memcpy(H, h, sizeof(h));
        memcpy(Jres, jr, sizeof(jr));
    }
    return chi2;
}

static float norm_max6(const float x[6]) {
    float nm = -1.f;
    for (int k = 0; k < 6; k++) if (fabsf(x[k]) > nm) nm = fabsf(x[k]);
    return nm;
}

/* update (SparseImageAlign.cc:240-244): T_new = T * exp(-x) */
static void align_update(const ygzo_se3 *T, const float x[6], ygzo_se3 *Tn) {
    float mx[6];
    for (int k = 0; k < 6; k++) mx[k] = -x[k];
    ygzo_se3 E;
    ygzo_se3_exp(mx, &E);
    ygzo_se3_mul(T, &E, Tn);
}

int ygzo_sparse_align_method(uint8_t **ref_levels, uint8_t **cur_levels, const int *lw, const int *lh,
                             const float *inv_scale, const ygzo_cam *cam, const ygzo_kp *kps,
                             const float *xyz_ref, const uint8_t *usable, int n, int max_level,
                             int min_level, const ygzo_se3 *T_init, int method, ygzo_align_out *out) {
    memset(out, 0, sizeof(*out));
    out->T = *T_init;
    if (n <= 0) return 0; /* SparseImageAlign.cc:24-27 */
    float *patch = (float *)calloc((size_t)n * PA, sizeof(float));
    float *jac = (float *)calloc((size_t)n * PA * 6, sizeof(float));
    uint8_t *vis = (uint8_t *)calloc((size_t)n, 1);
    ygzo_se3 T = *T_init;
    /* NLLSSolver::reset (NLSSolver_impl.hpp:289-298): once per run */
    float chi2_ = 1e10f, mu = 0.01f, nu = 2.0f; /* mu_init_ 0.01, nu_init_ 2 (NLSSolver.h:126-129) */
    int stop = 0;
    size_t n_meas = 0;
    float H[36], Jres[6], x[6];
    memset(H, 0, sizeof(H));
    const int border = PH + 1;
    for (int level = max_level; level >= min_level; level--) {
        const int n_iter = 10; /* iterations[] = {10,...}; levels >= 6 read past it (UB) */
        memset(jac, 0, sizeof(float) * (size_t)n * PA * 6);
        /* precomputeReferencePatches (SparseImageAlign.cc:57-128) */
        const uint8_t *rimg = ref_levels[level];
        const int rw = lw[level], rh = lh[level], stride = rw;
        const float scale = inv_scale[level];
        const float focal = cam->fx;
        for (int i = 0; i < n; i++) {
            if (!usable[i]) continue;
            const float u_ref = kps[i].x * scale, v_ref = kps[i].y * scale;
            const int ui = (int)floorf(u_ref), vi = (int)floorf(v_ref);
            if (ui - border < 0 || vi - border < 0 || ui + border >= rw || vi + border >= rh) continue;
            vis[i] = 1;
            float fj[12];
            jacob_xyz2cam(xyz_ref + 3 * (size_t)i, fj);
            const float su = u_ref - ui, sv = v_ref - vi;
            const float wtl = wmul(1.0 - su, 1.0 - sv), wtr = wmul(su, 1.0 - sv);
            const float wbl = wmul(1.0 - su, sv), wbr = wmul(su, sv);
            const float fs = focal * scale;
            int pc = 0;
            for (int y = 0; y < PS; ++y) {
                const uint8_t *p = rimg + (size_t)(vi + y - PH) * stride + (ui - PH);
                for (int xx = 0; xx < PS; ++xx, ++p, ++pc) {
                    patch[(size_t)i * PA + pc] = wtl * p[0] + wtr * p[1] + wbl * p[stride] + wbr * p[stride + 1];
                    float dx = 0.5f * ((wtl * p[1] + wtr * p[2] + wbl * p[stride + 1] + wbr * p[stride + 2]) -
                                       (wtl * p[-1] + wtr * p[0] + wbl * p[stride - 1] + wbr * p[stride]));
                    float dy = 0.5f * ((wtl * p[stride] + wtr * p[1 + stride] + wbl * p[stride * 2] + wbr * p[stride * 2 + 1]) -
                                       (wtl * p[-stride] + wtr * p[1 - stride] + wbl * p[0] + wbr * p[1]));
                    float *J = jac + ((size_t)i * PA + pc) * 6;
                    for (int k = 0; k < 6; k++) J[k] = (dx * fj[k] + dy * fj[6 + k]) * fs;
                }
            }
        }
        const uint8_t *cimg = cur_levels[level];
        const int cw = lw[level], chh = lh[level];
        int it = 0;
        if (method == YGZO_ALIGN_GN) {
            /* optimizeGaussNewton (NLSSolver_impl.hpp:18-91) */
            ygzo_se3 old = T;
            for (it = 0; it < n_iter; ++it) {
                memset(H, 0, sizeof(H));
                memset(Jres, 0, sizeof(Jres));
                n_meas = 0;
                const float chi2 = align_residuals(cimg, cw, chh, scale, cam, xyz_ref, vis, patch, jac, n, &T, 1,
                                                   &n_meas, H, Jres);
                const float new_chi2 = chi2 / (float)n_meas;
                /* solve (SparseImageAlign.cc:233-238) */
                ldlt_solve6(H, Jres, x);
                if (isnan(x[0])) stop = 1;
                if ((it > 0 && new_chi2 > 1.2 * chi2_) || stop) {
                    T = old; /* rollback */
                    break;
                }
                ygzo_se3 Tn;
                align_update(&T, x, &Tn);
                old = T;
                T = Tn;
                chi2_ = new_chi2;
                if (norm_max6(x) <= 0.000001f) { it++; break; }
            }
        } else {
            /* optimizeLevenbergMarquardt (NLSSolver_impl.hpp:95-212); SparseImgAlign::run sets
             * mu_ = 0.1 per level (SparseImageAlign.cc:40), eps_ = 1e-6 (:17).  The level's first
             * computeResiduals neither clears H_ nor n_meas_: chi2_ divides by the count carried
             * over from the previous call plus this one. */
            mu = 0.1f;
            float Hacc[36], Jacc[6];
            memcpy(Hacc, H, sizeof(H));
            memset(Jacc, 0, sizeof(Jacc));
            chi2_ = align_residuals(cimg, cw, chh, scale, cam, xyz_ref, vis, patch, jac, n, &T, 1, &n_meas, Hacc,
                                    Jacc) / (float)n_meas;
            for (it = 0; it < n_iter; ++it) {
                float rho = 0.f;
                int n_trials = 0;
                do {
                    ygzo_se3 Tn = T;
                    float new_chi2 = -1.f;
                    memset(H, 0, sizeof(H));
                    memset(Jres, 0, sizeof(Jres));
                    n_meas = 0;
                    (void)align_residuals(cimg, cw, chh, scale, cam, xyz_ref, vis, patch, jac, n, &T, 1, &n_meas, H,
                                          Jres);
                    for (int k = 0; k < 6; k++) H[k * 6 + k] += H[k * 6 + k] * mu; /* damping (:146) */
                    ldlt_solve6(H, Jres, x);
                    if (!isnan(x[0])) {
                        align_update(&T, x, &Tn);
                        n_meas = 0;
                        float Hd[36] = {0}, Jd[6] = {0};
                        new_chi2 = align_residuals(cimg, cw, chh, scale, cam, xyz_ref, vis, patch, jac, n, &Tn, 0,
                                                   &n_meas, Hd, Jd) / (float)n_meas;
                        rho = chi2_ - new_chi2;
                    } else {
                        rho = -1.f; /* singular */
                    }
                    if (rho > 0) {
                        T = Tn;
                        chi2_ = new_chi2;
                        stop = norm_max6(x) <= 0.000001f;
                        const double r3 = pow(2 * rho - 1, 3);
                        const double f = fmax(1. / 3., fmin(1. - r3, 2. / 3.));
                        mu = (float)((double)mu * f);
                        nu = 2.f;
                    } else {
                        mu *= nu;
                        nu *= 2.f;
                        ++n_trials;
                        if (n_trials >= 5) stop = 1; /* n_trials_max_ (NLSSolver.h:133) */
                    }
                } while (!(rho > 0 || stop));
                if (stop) { it++; break; }
            }
        }
        if (level < YGZO_MAX_LEVELS) out->iters[level] = it;
    }
    out->T = T;
    out->n_visible = (int)(n_meas / PA);
    out->chi2 = chi2_;
    memcpy(out->H, H, sizeof(H));
    free(patch); free(jac); free(vis);
    return out->n_visible;
}

int ygzo_sparse_align(uint8_t **ref_levels, uint8_t **cur_levels, const int *lw, const int *lh,
                      const float *inv_scale, const ygzo_cam *cam, const ygzo_kp *kps,
                      const float *xyz_ref, const uint8_t *usable, int n, int max_level,
                      int min_level, const ygzo_se3 *T_init, ygzo_align_out *out) {
    return ygzo_sparse_align_method(ref_levels, cur_levels, lw, lh, inv_scale, cam, kps, xyz_ref, usable, n,
                                    max_level, min_level, T_init, YGZO_ALIGN_GN, out);
}

/* ---------------- Align2D (Align.cc:8-105) ---------------- */
static void inverse3(const float m[9], float r[9]) {
#define M(i, j) m[(i) * 3 + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    float c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
    float det = c0 * M(0, 0) + c1 * M(1, 0) + c2 * M(2, 0);
    float inv = 1.f / det;
    r[0] = c0 * inv; r[1] = c1 * inv; r[2] = c2 * inv;
    r[3] = COF(0, 1) * inv; r[4] = COF(1, 1) * inv; r[5] = COF(2, 1) * inv;
    r[6] = COF(0, 2) * inv; r[7] = COF(1, 2) * inv; r[8] = COF(2, 2) * inv;
#undef COF
#undef M
}

int ygzo_align2d(const uint8_t *cur, int w, int h, int stride, const uint8_t *rpb,
                 const uint8_t *rp, int n_iter, float *px) {
    const int hp = 4, ps = 8, step = 10;
    float rdx[64], rdy[64], H[9] = {0};
    for (int y = 0; y < ps; ++y) {
        const uint8_t *it = rpb + (y + 1) * step + 1;
        for (int x = 0; x < ps; ++x, ++it) {
            float J0 = (float)(0.5 * (it[1] - it[-1]));
            float J1 = (float)(0.5 * (it[step] - it[-step]));
            float J2 = 1.f;
            rdx[y * 8 + x] = J0;
            rdy[y * 8 + x] = J1;
            float J[3] = {J0, J1, J2};
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) H[r * 3 + c] += J[r] * J[c];
        }
    }
    float Hi[9];
    inverse3(H, Hi);
    float mean_diff = 0.f, u = px[0], v = px[1];
    const float min_upd2 = (float)(0.03 * 0.03);
    int converged = 0;
    for (int iter = 0; iter < n_iter; ++iter) {
        int ur = (int)floorf(u), vr = (int)floorf(v);
        if (ur < hp || vr < hp || ur >= w - hp || vr >= h - hp) break;
        if (isnan(u) || isnan(v)) return 0;
        float sx = u - ur, sy = v - vr;
        float wTL = wmul(1.0 - sx, 1.0 - sy), wTR = wmul(sx, 1.0 - sy);
        float wBL = wmul(1.0 - sx, sy), wBR = wmul(sx, sy);
        float Jr0 = 0.f, Jr1 = 0.f, Jr2 = 0.f;
        for (int y = 0; y < ps; ++y) {
            const uint8_t *it = cur + (size_t)(vr + y - hp) * stride + ur - hp;
            for (int x = 0; x < ps; ++x, ++it) {
                float sp = wTL * it[0] + wTR * it[1] + wBL * it[stride] + wBR * it[stride + 1];
                float res = sp - rp[y * 8 + x] + mean_diff;
                Jr0 -= res * rdx[y * 8 + x];
                Jr1 -= res * rdy[y * 8 + x];
                Jr2 -= res;
            }
        }
        float u0 = Hi[0] * Jr0 + Hi[1] * Jr1 + Hi[2] * Jr2;
        float u1 = Hi[3] * Jr0 + Hi[4] * Jr1 + Hi[5] * Jr2;
        float u2 = Hi[6] * Jr0 + Hi[7] * Jr1 + Hi[8] * Jr2;
        u += u0;
        v += u1;
        mean_diff += u2;
        if (u0 * u0 + u1 * u1 < min_upd2) { converged = 1; break; }
    }
    px[0] = u;
    px[1] = v;
    return converged;
}

/* GetWarpAffineMatrix (ORBmatcher.cc:1525-1547); A stored row-major [a00 a01; a10 a11]. */
void ygzo_warp_affine_matrix(const ygzo_cam *cam, const ygzo_se3 *T_cr, const float pt_ref[3],
                             float px_ref_x, float px_ref_y, float level_scale, float A[4]) {
    const float depth = pt_ref[2];
    const float hps = 4.f;
    float du_x = px_ref_x + hps * level_scale, du_y = px_ref_y + 0.f * level_scale;
    float dv_x = px_ref_x + 0.f * level_scale, dv_y = px_ref_y + hps * level_scale;
    float pdu[3] = {(du_x - cam->cx) * depth / cam->fx, (du_y - cam->cy) * depth / cam->fy, depth};
    float pdv[3] = {(dv_x - cam->cx) * depth / cam->fx, (dv_y - cam->cy) * depth / cam->fy, depth};
    float c[3], cu[3], cv[3];
    ygzo_se3_act(T_cr, pt_ref, c);
    ygzo_se3_act(T_cr, pdu, cu);
    ygzo_se3_act(T_cr, pdv, cv);
    float pc[2] = {cam->fx * c[0] / c[2] + cam->cx, cam->fy * c[1] / c[2] + cam->cy};
    float pu[2] = {cam->fx * cu[0] / cu[2] + cam->cx, cam->fy * cu[1] / cu[2] + cam->cy};
    float pv[2] = {cam->fx * cv[0] / cv[2] + cam->cx, cam->fy * cv[1] / cv[2] + cam->cy};
    A[0] = (pu[0] - pc[0]) / 4; A[2] = (pu[1] - pc[1]) / 4;
    A[1] = (pv[0] - pc[0]) / 4; A[3] = (pv[1] - pc[1]) / 4;
}

/* GetBestSearchLevel (ORBmatcher.h:226-238). */
int ygzo_best_search_level(const float A[4], int max_level, float inv_level_sigma2_1) {
    int lvl = 0;
    float D = A[0] * A[3] - A[2] * A[1];
    while (D > 3.0f && lvl < max_level) { lvl += 1; D *= inv_level_sigma2_1; }
    return lvl;
}

/* WarpAffine (ORBmatcher.cc:1549-1571) with GetBilateralInterpUchar
 * (ORBmatcher.h:241-252; double weights, truncating uchar cast). */
void ygzo_warp_affine(const float A[4], const uint8_t *img, int w, int h, int stride,
                      float px_ref_x, float px_ref_y, float scale_level_ref, float scale_search,
                      int hps, uint8_t *patch) {
    const int ps = hps * 2;
    float det = A[0] * A[3] - A[2] * A[1];
    float inv = 1.f / det;
    float R00 = A[3] * inv, R01 = -A[1] * inv, R10 = -A[2] * inv, R11 = A[0] * inv;
    const float prx = px_ref_x / scale_level_ref, pry = px_ref_y / scale_level_ref;
    uint8_t *o = patch;
    for (int y = 0; y < ps; y++)
        for (int x = 0; x < ps; x++, ++o) {
            float ppx = (float)(x - hps) * scale_search, ppy = (float)(y - hps) * scale_search;
            float qx = (R00 * ppx + R01 * ppy) + prx;
            float qy = (R10 * ppx + R11 * ppy) + pry;
            if (qx < 0 || qy < 0 || qx >= w - 1 || qy >= h - 1) { *o = 0; continue; }
            double X = qx, Y = qy;
            double xx = X - floor(X), yy = Y - floor(Y);
            const uint8_t *d = img + (size_t)(int)Y * stride + (int)X;
            *o = (uint8_t)((1 - xx) * (1 - yy) * d[0] + xx * (1 - yy) * d[1] + (1 - xx) * yy * d[stride] +
                           xx * yy * d[stride + 1]);
        }
}

/* FindDirectProjection (ORBmatcher.cc:1573-1602). */
int ygzo_find_direct_projection(const ygzo_cam *cam, uint8_t **ref_levels, const int *rw,
                                const int *rh, uint8_t **cur_levels, const int *cw, const int *ch,
                                int nlevels, const float *scale, const float *inv_scale,
                                float inv_level_sigma2_1, const ygzo_se3 *T_cr,
                                const float pt_ref[3], const ygzo_kp *kp, float *px_curr,
                                int *search_level) {
    float A[4];
    ygzo_warp_affine_matrix(cam, T_cr, pt_ref, kp->x, kp->y, scale[kp->octave], A);
    int sl = ygzo_best_search_level(A, nlevels - 1, inv_level_sigma2_1);
    *search_level = sl;
    uint8_t pb[100], p[64];
    int oc = kp->octave;
    ygzo_warp_affine(A, ref_levels[oc], rw[oc], rh[oc], rw[oc], kp->x, kp->y, scale[oc], scale[sl], 5, pb);
    for (int y = 1; y < 9; ++y)
        for (int x = 0; x < 8; ++x) p[(y - 1) * 8 + x] = pb[y * 10 + 1 + x];
    float pxs[2] = {px_curr[0] * inv_scale[sl], px_curr[1] * inv_scale[sl]};
    int ok = ygzo_align2d(cur_levels[sl], cw[sl], ch[sl], cw[sl], pb, p, 10, pxs);
    px_curr[0] = pxs[0] * scale[sl];
    px_curr[1] = pxs[1] * scale[sl];
    return ok;
}

/* Tracking::SearchLocalPointsDirect (Tracking.cc:2337-2395), the per-point
 * body of the local-map loop: walk the point's observations in
 * SelectNearestKeyframe order (Tracking.cc:2412-2432; the caller lists them),
 * FindDirectProjection each from (mTrackProjX, mTrackProjY), skip results
 * within `border` px of the level-0 edge (Tracking.cc:2356-2364), keep the
 * first success (`break`), px_ave = that pixel / 1.  ref_levels holds
 * n_ref * nlevels level pointers (keyframe-major). */
void ygzo_search_direct(const ygzo_cam *cam, uint8_t **ref_levels, uint8_t **cur_levels, const int *lw,
                        const int *lh, int nlevels, const float *scale, const float *inv_scale,
                        float inv_level_sigma2_1, int n_points, const int *item_ptr, const int *ref_index,
                        const ygzo_kp *kps, const float *pt_ref, const ygzo_se3 *T_cr, const float *px_proj,
                        float border, float *px_out, int *matched) {
    const int cols = lw[0], rows = lh[0];
    for (int i = 0; i < n_points; i++) {
        int m = -1;
        float ave[2] = {0.f, 0.f};
        for (int k = item_ptr[i]; k < item_ptr[i + 1]; k++) {
            float px[2] = {px_proj[2 * i], px_proj[2 * i + 1]};
            int sl;
            if (ygzo_find_direct_projection(cam, ref_levels + (size_t)ref_index[k] * nlevels, lw, lh, cur_levels, lw,
                                            lh, nlevels, scale, inv_scale, inv_level_sigma2_1, &T_cr[k],
                                            pt_ref + 3 * (size_t)k, &kps[k], px, &sl)) {
                if (px[0] < border || px[1] < border || px[0] >= cols - border || px[1] >= rows - border)
                    continue;
                m = k;
                ave[0] = px[0] / 1.0f;
                ave[1] = px[1] / 1.0f;
                break;
            }
        }
        px_out[2 * i] = ave[0];
        px_out[2 * i + 1] = ave[1];
        matched[i] = m;
    }
}

/* The whole of Tracking::SearchLocalPointsDirect (Tracking.cc:2258-2410) over
 * the points the caller's own filters let through, in the reference's loop order:
 *
 *  - points [0, n_cache): mvpDirectMapPointsCache members that are not bad and
 *    pass isInFrustum (Tracking.cc:2269-2275; the caller erases the others).  A
 *    point whose projection cell (int(mTrackProjX / grid_size),
 *    int(mTrackProjY / grid_size)) of the 5-px coverage grid is already taken is
 *    skipped and stays in the cache (:2277-2284); otherwise its observations are
 *    tried in SelectNearestKeyframe order, the first converged in-border result
 *    is taken (:2286-2303) and the cell of px_ave is marked (:2320-2323); a point
 *    with no result leaves the cache (:2327-2330).
 *  - if the cache gave more than cache_hit_th successes (mnCacheHitTh,
 *    :2334-2340) the local-map points are not searched (status NOT_RUN);
 *    otherwise points [n_cache, n_cache + n_local): mvpLocalMapPoints that are not
 *    in the cache, not bad and in the frustum (:2348-2361), each tried like a
 *    cache point but without the grid (:2363-2405).
 *
 * Grid: grid_rows = rows / grid_size, grid_cols = cols / grid_size of level 0,
 * cell k = gy * grid_cols + gx (:2261-2264, 2277-2279).  A projection on the
 * last partial column aliases into the next row's first cell, as in the
 * reference; an index outside [0, grid_rows * grid_cols) (the reference reads
 * past the vector<bool>) counts as a free cell and is never written.
 *
 * status[i]: 1 matched, 0 no match (cache: erased; local: rejected), 2 grid
 * skip (cache only), 3 not run.  Returns the cache-phase success count;
 * *local_ran = whether the local-map phase ran. */
int ygzo_search_local_points_direct(const ygzo_cam *cam, uint8_t **ref_levels, uint8_t **cur_levels, const int *lw,
                                    const int *lh, int nlevels, const float *scale, const float *inv_scale,
                                    float inv_level_sigma2_1, int n_cache, int n_local, const int *item_ptr,
                                    const int *ref_index, const ygzo_kp *kps, const float *pt_ref,
                                    const ygzo_se3 *T_cr, const float *px_proj, float border, int grid_size,
                                    int cache_hit_th, float *px_out, int *matched, int *status, int *local_ran) {
    const int cols = lw[0], rows = lh[0];
    const int grid_rows = rows / grid_size, grid_cols = cols / grid_size;
    const long ncell = (long)grid_rows * grid_cols;
    uint8_t *grid = (uint8_t *)calloc(ncell > 0 ? (size_t)ncell : 1, 1);
    int cnt_success = 0;
    for (int i = 0; i < n_cache + n_local; i++) {
        const int in_cache = i < n_cache;
        px_out[2 * i] = px_out[2 * i + 1] = 0.f;
        matched[i] = -1;
        if (i == n_cache) {
            *local_ran = !(cnt_success > cache_hit_th);
        }
        if (!in_cache && !*local_ran) { status[i] = 3; continue; }
        if (in_cache) {
            const int gx = (int)(px_proj[2 * i] / grid_size), gy = (int)(px_proj[2 * i + 1] / grid_size);
            const long k = (long)gy * grid_cols + gx;
            if (k >= 0 && k < ncell && grid[k]) { status[i] = 2; continue; }
        }
        int m = -1;
        float ave[2] = {0.f, 0.f};
        for (int it = item_ptr[i]; it < item_ptr[i + 1]; it++) {
            float px[2] = {px_proj[2 * i], px_proj[2 * i + 1]};
            int sl;
            if (ygzo_find_direct_projection(cam, ref_levels + (size_t)ref_index[it] * nlevels, lw, lh, cur_levels, lw,
                                            lh, nlevels, scale, inv_scale, inv_level_sigma2_1, &T_cr[it],
                                            pt_ref + 3 * (size_t)it, &kps[it], px, &sl)) {
                if (px[0] < border || px[1] < border || px[0] >= cols - border || px[1] >= rows - border)
                    continue;
                m = it;
                ave[0] = px[0] / 1.0f;
                ave[1] = px[1] / 1.0f;
                break;
            }
        }
        if (m < 0) { status[i] = 0; continue; }
        status[i] = 1;
        matched[i] = m;
        px_out[2 * i] = ave[0];
        px_out[2 * i + 1] = ave[1];
        if (in_cache) {
            const int gx = (int)(ave[0] / grid_size), gy = (int)(ave[1] / grid_size);
            const long k = (long)gy * grid_cols + gx;
            if (k >= 0 && k < ncell) grid[k] = 1;
            cnt_success++;
        }
    }
    if (n_local == 0) *local_ran = !(cnt_success > cache_hit_th);
    free(grid);
    return cnt_success;
}
