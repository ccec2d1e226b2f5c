/*
 * synth.c — seeded synthetic inputs for tests and bench.py.
 * Not part of the product path.
 *
 *  - ygzs_texture: splitmix64-seeded frame: 600 axis-aligned rectangles (side
 *    U[4,60], intensity U{0..255}, painted in order over a mid-grey field)
 *    plus per-pixel noise U{-3..3}, clamped.
 *  - ygzs_render_plane: a camera (pinhole fx,fy,cx,cy; pose T_cw as unit
 *    quaternion + translation) looking at a textured plane Z_w = plane_z;
 *    bilinear texture lookup in double, plus seeded noise U{-n..n}.
 *  - ygzs_backproject_plane: world point on that plane seen at pixel (u,v);
 *    gives the reference keypoints their MapPoint positions for align tests.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint64_t splitmix64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline int uni(uint64_t *s, int lo, int hi) { /* inclusive */
    return lo + (int)(splitmix64(s) % (uint64_t)(hi - lo + 1));
}

void ygzs_texture(uint64_t seed, int W, int H, uint8_t *out) {
    uint64_t s = seed * 0x2545F4914F6CDD1Dull + 0x1234567ull;
    memset(out, 128, (size_t)W * H);
    /* 600 rectangles per 752x480 of area, at least 600 */
    long nr = 600L * W * H / (752L * 480L);
    if (nr < 600) nr = 600;
    for (long r = 0; r < nr; r++) {
        int x0 = uni(&s, 0, W - 1), y0 = uni(&s, 0, H - 1);
        int w = uni(&s, 4, 60), h = uni(&s, 4, 60), v = uni(&s, 0, 255);
        int x1 = x0 + w > W ? W : x0 + w, y1 = y0 + h > H ? H : y0 + h;
        for (int y = y0; y < y1; y++) memset(out + (size_t)y * W + x0, v, (size_t)(x1 - x0));
    }
    for (size_t i = 0; i < (size_t)W * H; i++) {
        int v = out[i] + uni(&s, -3, 3);
        out[i] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
}

/* rotate v by unit quaternion q (x,y,z,w) in double */
static void qrot(const double q[4], const double v[3], double o[3]) {
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    for (int i = 0; i < 3; i++) uv[i] *= 2;
    double c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    for (int i = 0; i < 3; i++) o[i] = v[i] + q[3] * uv[i] + c[i];
}

/* camera centre and world ray for pixel (u,v) under T_cw */
static int ray_plane(const float cam[4], const float q_cw[4], const float t_cw[3], double u, double v,
                     double plane_z, double P[3]) {
    double qi[4] = {-q_cw[0], -q_cw[1], -q_cw[2], q_cw[3]};
    double mt[3] = {-t_cw[0], -t_cw[1], -t_cw[2]}, C[3];
    qrot(qi, mt, C); /* camera centre in world = -R^T t */
    double dc[3] = {(u - cam[2]) / cam[0], (v - cam[3]) / cam[1], 1.0}, dw[3];
    qrot(qi, dc, dw);
    if (fabs(dw[2]) < 1e-12) return 0;
    double lam = (plane_z - C[2]) / dw[2];
    if (lam <= 0) return 0;
    for (int i = 0; i < 3; i++) P[i] = C[i] + lam * dw[i];
    return 1;
}

void ygzs_render_plane(const uint8_t *tex, int TW, int TH, double texel, double plane_z,
                       const float cam[4], const float q_cw[4], const float t_cw[3], int W, int H,
                       uint64_t noise_seed, int noise_amp, uint8_t *out) {
    uint64_t s = noise_seed * 0x9E3779B97F4A7C15ull + 77;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            double P[3];
            int val = 0;
            if (ray_plane(cam, q_cw, t_cw, x, y, plane_z, P)) {
                double tx = P[0] / texel + TW * 0.5, ty = P[1] / texel + TH * 0.5;
                int ix = (int)floor(tx), iy = (int)floor(ty);
                if (ix >= 0 && iy >= 0 && ix < TW - 1 && iy < TH - 1) {
                    double fx = tx - ix, fy = ty - iy;
                    const uint8_t *p = tex + (size_t)iy * TW + ix;
                    double v = (1 - fx) * (1 - fy) * p[0] + fx * (1 - fy) * p[1] + (1 - fx) * fy * p[TW] +
                               fx * fy * p[TW + 1];
                    val = (int)floor(v + 0.5);
                }
            }
            if (noise_amp > 0) val += uni(&s, -noise_amp, noise_amp);
            out[(size_t)y * W + x] = (uint8_t)(val < 0 ? 0 : (val > 255 ? 255 : val));
        }
}

int ygzs_backproject_plane(const float cam[4], const float q_cw[4], const float t_cw[3], float u,
                           float v, double plane_z, float P_out[3]) {
    double P[3];
    if (!ray_plane(cam, q_cw, t_cw, u, v, plane_z, P)) return 0;
    for (int i = 0; i < 3; i++) P_out[i] = (float)P[i];
    return 1;
}

/* a batch of rendered frames along a smooth trajectory: frame k has pose
 * T_cw(k) = exp(k * xi) with xi = (v, w) per frame (small-angle quaternion). */
void ygzs_trajectory_pose(int k, const float xi[6], float q_out[4], float t_out[3]) {
    double w[3] = {xi[3] * (double)k, xi[4] * (double)k, xi[5] * (double)k};
    double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double s = th > 1e-12 ? sin(th / 2) / th : 0.5;
    q_out[0] = (float)(w[0] * s); q_out[1] = (float)(w[1] * s); q_out[2] = (float)(w[2] * s);
    q_out[3] = (float)cos(th / 2);
    for (int i = 0; i < 3; i++) t_out[i] = (float)(xi[i] * (double)k);
}
