/*
 * bench.c — the CPU baseline of bench.py: the whole per-frame hot path of the
 * restatement (pyramid, ORB extraction, Hamming best/second vs the previous
 * frame, SparseImgAlign 3..1 against the previous frame) driven from C, with
 * no per-stage ctypes hops, on 1 or T host threads (one contiguous chunk of
 * frames per thread, as the GPU ranks shard the sequence).
 * TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg); see ygz_oracle.h.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ygz_oracle.h"

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

typedef struct {
    const uint8_t *frames;
    int first, n, W, H;
    const float *cam, *r3, *cz;
    float plane_z;
    int nfeatures, nlevels, ini, min_th;
    float scale;
    ygzo_bench_stats st;
} job_t;

/* xyz_ref of the previous frame's keypoints on the plane Z_w = plane_z:
 * X_c = lam * d_c, lam = (Z - C_z) / (r3 . d_c) (the bench's map points) */
static void plane_xyz(const float *cam, const float *r3, float cz, float plane_z, const ygzo_kp *k, int n,
                      float *xyz) {
    for (int i = 0; i < n; i++) {
        const float dx = (k[i].x - cam[2]) / cam[0], dy = (k[i].y - cam[3]) / cam[1];
        const float lam = (plane_z - cz) / (r3[0] * dx + r3[1] * dy + r3[2]);
        xyz[3 * i] = dx * lam;
        xyz[3 * i + 1] = dy * lam;
        xyz[3 * i + 2] = lam;
    }
}

static void *run_chunk(void *arg) {
    job_t *J = (job_t *)arg;
    ygzo_orb o;
    ygzo_orb_init(&o, J->nfeatures, J->scale, J->nlevels, J->ini, J->min_th, 0);
    int lw[YGZO_MAX_LEVELS], lh[YGZO_MAX_LEVELS];
    ygzo_level_sizes(&o, J->W, J->H, lw, lh);
    const int cap = 8192;
    uint8_t *lv[2][YGZO_MAX_LEVELS];
    ygzo_kp *kps[2];
    uint8_t *desc[2];
    int nk[2] = {0, 0};
    for (int b = 0; b < 2; b++) {
        for (int l = 0; l < J->nlevels; l++) lv[b][l] = (uint8_t *)malloc((size_t)lw[l] * lh[l]);
        kps[b] = (ygzo_kp *)malloc(sizeof(ygzo_kp) * cap);
        desc[b] = (uint8_t *)malloc((size_t)32 * cap);
    }
    int32_t *bi = (int32_t *)malloc(sizeof(int32_t) * cap * 3);
    float *xyz = (float *)malloc(sizeof(float) * 3 * cap);
    uint8_t *usable = (uint8_t *)malloc(cap);
    memset(usable, 1, cap);
    ygzo_cam cam = {J->cam[0], J->cam[1], J->cam[2], J->cam[3]};
    ygzo_se3 T0 = {{0, 0, 0, 1}, {0, 0, 0}};
    ygzo_align_out ao;
    memset(&J->st, 0, sizeof(J->st));
    for (int i = 0; i < J->n; i++) {
        const int g = J->first + i, b = i & 1, p = b ^ 1;
        double t0 = now_s();
        ygzo_compute_pyramid(&o, J->frames + (size_t)g * J->W * J->H, J->W, J->H, J->W, lv[b]);
        double t1 = now_s();
        nk[b] = ygzo_extract_orbslam(&o, lv[b], lw, lh, NULL, 0, kps[b], desc[b], cap);
        if (nk[b] < 0) nk[b] = 0;
        double t2 = now_s();
        J->st.t_pyr += t1 - t0;
        J->st.t_extract += t2 - t1;
        J->st.keypoints += nk[b];
        J->st.frames++;
        if (i == 0) continue;
        ygzo_hamming_best2(desc[b], nk[b], desc[p], nk[p], bi, bi + cap, bi + 2 * cap);
        double t3 = now_s();
        plane_xyz(J->cam, J->r3 + 3 * (size_t)(g - 1), J->cz[g - 1], J->plane_z, kps[p], nk[p], xyz);
        ygzo_sparse_align(lv[p], lv[b], lw, lh, o.inv_scale, &cam, kps[p], xyz, usable, nk[p], J->nlevels - 1, 1, &T0,
                          &ao);
        double t4 = now_s();
        J->st.t_hamming += t3 - t2;
        J->st.t_align += t4 - t3;
        J->st.pairs++;
        J->st.visible += ao.n_visible;
    }
    for (int b = 0; b < 2; b++) {
        for (int l = 0; l < J->nlevels; l++) free(lv[b][l]);
        free(kps[b]);
        free(desc[b]);
    }
    free(bi);
    free(xyz);
    free(usable);
    return NULL;
}

double ygzo_bench_pipeline(const uint8_t *frames, int n, int W, int H, const float cam[4], float plane_z,
                           const float *r3, const float *cz, int nfeatures, float scale, int nlevels, int ini,
                           int min_th, int threads, ygzo_bench_stats *stats) {
    if (threads < 1) threads = 1;
    if (threads > n) threads = n > 0 ? n : 1;
    job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        const int b = (int)((long long)n * t / threads), e = (int)((long long)n * (t + 1) / threads);
        job_t j = {frames, b, e - b, W, H, cam, r3, cz, plane_z, nfeatures, nlevels, ini, min_th, scale, {0}};
        jobs[t] = j;
    }
    const double t0 = now_s();
    for (int t = 1; t < threads; t++) pthread_create(&tid[t], NULL, run_chunk, &jobs[t]);
    run_chunk(&jobs[0]);
    for (int t = 1; t < threads; t++) pthread_join(tid[t], NULL);
    const double wall = now_s() - t0;
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        for (int t = 0; t < threads; t++) {
            stats->t_pyr += jobs[t].st.t_pyr;
            stats->t_extract += jobs[t].st.t_extract;
            stats->t_hamming += jobs[t].st.t_hamming;
            stats->t_align += jobs[t].st.t_align;
            stats->frames += jobs[t].st.frames;
            stats->pairs += jobs[t].st.pairs;
            stats->keypoints += jobs[t].st.keypoints;
            stats->visible += jobs[t].st.visible;
        }
    }
    free(jobs);
    free(tid);
    return wall;
}

/* The FAST stage alone on one image: cv::FAST(img, th, nonmax) over the
 * 3-px interior (the oracle's FAST_t restatement), for the sanity check
 * against the reference's SSE2 FAST-10.  Returns the
 * corner count; *seconds = mean wall time over reps. */
int ygzo_bench_fast9(const uint8_t *img, int w, int h, int threshold, int reps, double *seconds) {
    int16_t *xs = (int16_t *)malloc(sizeof(int16_t) * (size_t)w * h / 2 + 16);
    int16_t *ys = (int16_t *)malloc(sizeof(int16_t) * (size_t)w * h / 2 + 16);
    uint8_t *sc = (uint8_t *)malloc((size_t)w * h / 2 + 16);
    int n = 0;
    const double t0 = now_s();
    for (int r = 0; r < reps; r++) n = ygzo_fast9_roi(img, w, h, w, threshold, xs, ys, sc, w * h / 2);
    *seconds = (now_s() - t0) / (reps > 0 ? reps : 1);
    free(xs);
    free(ys);
    free(sc);
    return n;
}

/* FAST-10 sanity: the restated Thirdparty/fast pipeline
 * (detect_sse2 + score + 3x3 NMS, ygzo_fast10_detect_score_nms) over one ROI,
 * `reps` times; returns the kept-corner count, *seconds = mean per pipeline. */
int ygzo_bench_fast10(const uint8_t *img, int w, int h, int stride, int barrier, int reps, double *seconds) {
    const size_t cap = (size_t)w * h / 2 + 16;
    int16_t *xs = (int16_t *)malloc(sizeof(int16_t) * cap);
    int16_t *ys = (int16_t *)malloc(sizeof(int16_t) * cap);
    int *sc = (int *)malloc(sizeof(int) * cap);
    int n = 0;
    const double t0 = now_s();
    for (int r = 0; r < reps; r++) n = ygzo_fast10_detect_score_nms(img, w, h, stride, barrier, xs, ys, sc, (int)cap);
    *seconds = (now_s() - t0) / (reps > 0 ? reps : 1);
    free(xs);
    free(ys);
    free(sc);
    return n;
}
