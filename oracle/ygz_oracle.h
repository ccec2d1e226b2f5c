/*
 * ygz_oracle.h — CPU restatement of the ORB-YGZ-SLAM front-end hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path and the timed CPU baseline ("cpu_baseline.kind" = "port") in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product library (libygzfe.so) never links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the Ewenwan/ORB-YGZ-SLAM checkout).  Where the reference delegates to a
 * third-party library that is absent here (OpenCV: unpinned version, see
 * SURVEY.md §8c), the semantics chosen are documented next to the function and
 * in DESIGN.md §Parity.  Parity status:
 *   - FAST-10 (Thirdparty/fast): PINNED against golden vectors produced by the
 *     reference's own sources compiled by oracle/Makefile into oracle/_ref/
 *     (tests/golden/fast10_*.npz, the 167-corner known answer of
 *     Thirdparty/fast/test/test.cpp:332).
 *   - Everything that runs through OpenCV primitives (resize, FAST-9,
 *     GaussianBlur, fastAtan2) and Eigen (LDLT, 3x3 inverse): parity
 *     UNPINNED (no OpenCV/Eigen in the image, no fixtures in the reference);
 *     restated from the published OpenCV/Eigen algorithms named below.
 */
#ifndef YGZ_ORACLE_H_
#define YGZ_ORACLE_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YGZO_MAX_LEVELS 16

/* Same 28-byte layout as cv::KeyPoint {Point2f pt; size; angle; response; octave; class_id}. */
typedef struct ygzo_kp {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} ygzo_kp;

/* Gaussian 7x7 sigma=2 kernel variant. */
enum { YGZO_BLUR_CV4_BITEXACT = 0, YGZO_BLUR_CV3_ROUNDED = 1 };

/* ORBextractor state (ORBextractor.cc:412-470). */
typedef struct ygzo_orb {
    int nfeatures;
    double scale_factor;          /* ORBextractor.h:157 — stored as double */
    int nlevels, ini_th, min_th;
    int blur_variant;
    float scale[YGZO_MAX_LEVELS], inv_scale[YGZO_MAX_LEVELS];
    float sigma2[YGZO_MAX_LEVELS], inv_sigma2[YGZO_MAX_LEVELS];
    int feat_per_level[YGZO_MAX_LEVELS];
    int umax[16];
    int dso_grid;                 /* mnGridSize, -1 initially (ORBextractor.cc:469) */
} ygzo_orb;

void ygzo_orb_init(ygzo_orb *o, int nfeatures, float scale_factor, int nlevels,
                   int ini_th, int min_th, int blur_variant);
/* Level sizes: cvRound(W * inv_scale[l]) (ORBextractor.cc:1131-1132). */
void ygzo_level_sizes(const ygzo_orb *o, int W, int H, int *w, int *h);

/* Pyramid (ORBextractor.cc:1129-1150 + Frame.cc:807-813): levels are tight
 * (stride == width), borderless, like Frame::mvImagePyramid after clone(). */
void ygzo_compute_pyramid(const ygzo_orb *o, const uint8_t *img, int W, int H, int stride,
                          uint8_t **levels);
/* cv::resize INTER_LINEAR (x2 exact -> INTER_AREA fast path). */
void ygzo_resize(const uint8_t *src, int sw, int sh, int sstride, uint8_t *dst, int dw, int dh,
                 int dstride);

/* cv::FAST(roi, kps, th, nonmax=true), TYPE_9_16 on a ROI.  Output corners in
 * raster order: x,y relative to the ROI, score.  Returns count (<= cap). */
int ygzo_fast9_roi(const uint8_t *roi, int w, int h, int stride, int threshold,
                   int16_t *xs, int16_t *ys, uint8_t *scores, int cap);
/* OpenCV cornerScore<16>. */
int ygzo_corner_score16(const uint8_t *ptr, int stride, int threshold);
/* test hook: 1 = scalar segment test only (default: 16-pixel vectors) */
void ygzo_fast9_force_scalar(int on);

/* ComputeKeyPointsOctTree for one level (ORBextractor.cc:725-799), without
 * orientation.  Returns the distributed keypoints in list order. */
int ygzo_octree_level(const ygzo_orb *o, const uint8_t *lvl, int w, int h, int level,
                      ygzo_kp *out, int cap, int *n_candidates);
/* DistributeOctTree (ORBextractor.cc:533-723) on candidate keys (level coords
 * relative to minBorder).  Ties of std::sort on (size, node*) are resolved by
 * node creation order. */
int ygzo_distribute_octree(const ygzo_kp *keys, int n, int minX, int maxX, int minY, int maxY,
                           int N, ygzo_kp *out, int cap);

float ygzo_fast_atan2(float y, float x);
float ygzo_ic_angle(const uint8_t *img, int w, int h, int stride, float x, float y,
                    const int *umax);
void ygzo_gaussian_blur7(const uint8_t *src, int w, int h, int stride, uint8_t *dst,
                         int dstride, int variant);
void ygzo_orb_descriptor(const uint8_t *img, int w, int h, int stride, const ygzo_kp *kp,
                         uint8_t desc[32]);
const int *ygzo_bit_pattern(void);
/* glibc 2.35 sinf / cosf restated (|y| < 120; ORBextractor.cc:109 std::cos(float)). */
void ygzo_sincosf(float y, float *sinp, float *cosp);
/* Test hook: #inputs in float bit range [lo, hi) where ygzo_sincosf != libm. */
int64_t ygzo_sincosf_sweep(uint32_t lo, uint32_t hi);
/* Test hook: the 512 rotated rBRIEF sample offsets for one angle (degrees). */
void ygzo_orb_sample_offsets(float angle_deg, int *dy, int *dx);

/* ORBextractor::operator()(Frame*, kps, desc, ORBSLAM_KEYPOINT, leftEye=true)
 * (ORBextractor.cc:1031-1127) on a prebuilt pyramid.  `existing` (n_existing)
 * are the frame's current keypoints (level-0 coordinates): their descriptor
 * rows come first.  Writes up to cap kps and cap*32 descriptor bytes.
 * Returns the total row count (existing + new) or -1 if cap is too small. */
int ygzo_extract_orbslam(ygzo_orb *o, uint8_t **levels, const int *lw, const int *lh,
                         const ygzo_kp *existing, int n_existing, ygzo_kp *out_kps,
                         uint8_t *out_desc, int cap);

/* ---------------- FAST-10 (Thirdparty/fast) + DSO mode ---------------- */
int ygzo_fast10_is_corner(const uint8_t *p, int stride, int barrier);
/* fast_corner_detect_10 (YGZ variant, full w x h scan: fast_10.cpp:35-42). */
int ygzo_fast10_detect_plain(const uint8_t *img, int w, int h, int stride, int barrier,
                             int16_t *xs, int16_t *ys, int cap);
/* fast_corner_detect_10_sse2 semantics (faster_corner_10_sse.cpp:189-202). */
int ygzo_fast10_detect_sse2(const uint8_t *img, int w, int h, int stride, int barrier,
                            int16_t *xs, int16_t *ys, int cap);
/* detect (SSE2 variant's ROI) + score + 3x3 NMS in one pass: kept corners, raster order */
int ygzo_fast10_detect_score_nms(const uint8_t *img, int w, int h, int stride, int barrier, int16_t *xs,
                                 int16_t *ys, int *scores, int cap);
/* 0: 16-pixel vector FAST-10 test (default), 1: scalar (test hook) */
void ygzo_fast10_force_scalar(int on);
int ygzo_fast10_score(const uint8_t *p, int stride, int threshold);
int ygzo_fast10_nonmax(const int16_t *xs, const int16_t *ys, const int *scores, int n,
                       int *keep);
float ygzo_shi_tomasi(const uint8_t *img, int w, int h, int stride, int u, int v);
/* ComputeKeyPointsDSOSingleLevel (ORBextractor.cc:1275-1386); updates o->dso_grid.
 * exist_kps angles are recomputed in place (ORBextractor.cc:1383-1385). */
int ygzo_dso_single_level(ygzo_orb *o, uint8_t **levels, const int *lw, const int *lh,
                          ygzo_kp *exist, int n_exist, ygzo_kp *out, int cap);
int ygzo_extract_dso(ygzo_orb *o, uint8_t **levels, const int *lw, const int *lh,
                     ygzo_kp *existing, int n_existing, ygzo_kp *out_kps, uint8_t *out_desc,
                     int cap);

/* ---------------- Hamming (ORBmatcher.cc:1507-1523) ---------------- */
int ygzo_descriptor_distance(const uint8_t *a, const uint8_t *b);
/* Dense best/second-best: for every query, best distance (strict <, first
 * index wins), its index, and the second-best distance. */
void ygzo_hamming_best2(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *best_idx,
                        int32_t *best_dist, int32_t *second_dist);

/* ---------------- ORBmatcher tracking-path searches (oracle/match.c) ---------------- */
/* The searched frame: mvKeys (level-0 px), mDescriptors, mvuRight (NULL = none),
 * image bounds mnMinX / mnMaxX / mnMinY / mnMaxY (Frame::ComputeImageBounds). */
typedef struct ygzo_mframe {
    const ygzo_kp *kps;
    const uint8_t *desc;
    const float *u_right;
    int n;
    float min_x, max_x, min_y, max_y;
} ygzo_mframe;
#define YGZO_MQ_VALID 1   /* query takes part (pMP present, not bad / outlier, projected inside) */
#define YGZO_MQ_BLOCKS 2  /* assigning it blocks the keypoint for later queries (Observations() > 0) */
#define YGZO_MQ_STEREO 4  /* the mvuRight test of the projection searches applies */
/* One query: GetFeaturesInArea(u, v, radius, min_level, max_level) window, the
 * stereo u_right, the query keypoint angle (rotation histogram), flags. */
typedef struct ygzo_mquery {
    float u, v, radius, u_right;
    int32_t min_level, max_level;
    float angle;
    int32_t flags;
} ygzo_mquery;
int ygzo_pos_in_grid(const ygzo_mframe *f, float x, float y, int *px, int *py);
int ygzo_features_in_area(const ygzo_mframe *f, float x, float y, float r, int min_level, int max_level, int *out);
void ygzo_compute_three_maxima(const int *histo, int L, int *ind1, int *ind2, int *ind3);
int ygzo_rot_bin(float angle_query, float angle_train);
int ygzo_search_projection_best(const ygzo_mframe *cur, const ygzo_mquery *q, const uint8_t *q_desc, int nq,
                                const uint8_t *train_blocked, int th_dist, int check_ori, int32_t *train_match);
int ygzo_search_projection_ratio(const ygzo_mframe *F, const ygzo_mquery *q, const uint8_t *q_desc, int nq,
                                 const uint8_t *train_blocked, float nnratio, int32_t *train_match);
int ygzo_search_for_initialization(const ygzo_mframe *F1, const ygzo_mframe *F2, float *prev_matched, int window,
                                   float nnratio, int check_ori, int32_t *matches12);
int ygzo_search_by_bow(const ygzo_mframe *kf, const ygzo_mframe *F, const uint8_t *kf_usable, int n_kf_nodes,
                       const int32_t *kf_nodes, const int32_t *kf_ptr, const int32_t *kf_feats, int n_f_nodes,
                       const int32_t *f_nodes, const int32_t *f_ptr, const int32_t *f_feats, float nnratio,
                       int check_ori, int32_t *f_match);

/* ---------------- SparseImgAlign (SparseImageAlign.cc) ---------------- */
typedef struct ygzo_cam { float fx, fy, cx, cy; } ygzo_cam;
/* SE3f as unit quaternion (x,y,z,w) + translation: matches Sophus SE3f. */
typedef struct ygzo_se3 { float q[4]; float t[3]; } ygzo_se3;
typedef struct ygzo_align_out {
    ygzo_se3 T;            /* T_cur_from_ref */
    int n_visible;         /* n_meas_/16 of the last computeResiduals */
    float chi2;            /* chi2_ at exit */
    int iters[YGZO_MAX_LEVELS];
    float H[36];           /* H_ of the last linearisation (LM: damped, as the last trial left it) */
} ygzo_align_out;
/* SparseImgAlign::run (SparseImageAlign.cc:20-49).  Features i = 0..n-1 are the
 * reference frame's keypoints (level-0 px) with usable[i] != 0 when the
 * MapPoint is non-null, not bad, not outlier; xyz_ref = T_ref * P_w. */
int ygzo_sparse_align(uint8_t **ref_levels, uint8_t **cur_levels, const int *lw, const int *lh,
                      const float *inv_scale, const ygzo_cam *cam, const ygzo_kp *kps,
                      const float *xyz_ref, const uint8_t *usable, int n, int max_level,
                      int min_level, const ygzo_se3 *T_init, ygzo_align_out *out);
/* The same with NLLSSolver's method (NLSSolver_impl.hpp:8-13): YGZO_ALIGN_GN =
 * optimizeGaussNewton (:18-91), YGZO_ALIGN_LM = optimizeLevenbergMarquardt (:95-212). */
enum { YGZO_ALIGN_GN = 0, YGZO_ALIGN_LM = 1 };
int ygzo_sparse_align_method(uint8_t **ref_levels, uint8_t **cur_levels, const int *lw, const int *lh,
                             const float *inv_scale, const ygzo_cam *cam, const ygzo_kp *kps,
                             const float *xyz_ref, const uint8_t *usable, int n, int max_level,
                             int min_level, const ygzo_se3 *T_init, int method, ygzo_align_out *out);
void ygzo_se3_mul(const ygzo_se3 *a, const ygzo_se3 *b, ygzo_se3 *out);
void ygzo_se3_exp(const float x[6], ygzo_se3 *out);
void ygzo_se3_act(const ygzo_se3 *T, const float p[3], float out[3]);
void ygzo_se3_inverse(const ygzo_se3 *T, ygzo_se3 *out);

/* ---------------- Align2D + FindDirectProjection ---------------- */
/* Align2D (Align.cc:8-105).  Returns converged flag; px updated in place. */
int ygzo_align2d(const uint8_t *cur, int w, int h, int stride, const uint8_t *ref_patch_with_border,
                 const uint8_t *ref_patch, int n_iter, float *px);
/* WarpAffine (ORBmatcher.cc:1549-1571) of a (2*hps)^2 patch. */
void ygzo_warp_affine(const float A_cr[4], const uint8_t *img_ref, int w, int h, int stride,
                      float px_ref_x, float px_ref_y, float scale_level_ref, float scale_search,
                      int half_patch_size, uint8_t *patch);
/* GetWarpAffineMatrix (ORBmatcher.cc:1525-1547).  T_cr = T_cur * T_ref^-1;
 * pt_ref = T_ref * P_w (float3); px_ref level-0 px of the KF keypoint. */
void ygzo_warp_affine_matrix(const ygzo_cam *cam, const ygzo_se3 *T_cr, const float pt_ref[3],
                             float px_ref_x, float px_ref_y, float level_scale, float A_cr[4]);
int ygzo_best_search_level(const float A_cr[4], int max_level, float inv_level_sigma2_1);
/* FindDirectProjection (ORBmatcher.cc:1573-1602): px_curr (level-0) in/out. */
int ygzo_find_direct_projection(const ygzo_cam *cam, uint8_t **ref_levels, const int *rw,
                                const int *rh, uint8_t **cur_levels, const int *cw, const int *ch,
                                int nlevels, const float *scale, const float *inv_scale,
                                float inv_level_sigma2_1, const ygzo_se3 *T_cr,
                                const float pt_ref[3], const ygzo_kp *kp_ref, float *px_curr,
                                int *search_level);

/* SearchLocalPointsDirect (Tracking.cc:2337-2395) per point: first converged
 * observation inside the border, in the listed (SelectNearestKeyframe) order. */
void ygzo_search_direct(const ygzo_cam *cam, uint8_t **ref_levels, uint8_t **cur_levels, const int *lw,
                        const int *lh, int nlevels, const float *scale, const float *inv_scale,
                        float inv_level_sigma2_1, int n_points, const int *item_ptr, const int *ref_index,
                        const ygzo_kp *kps, const float *pt_ref, const ygzo_se3 *T_cr, const float *px_proj,
                        float border, float *px_out, int *matched);
/* Tracking::SearchLocalPointsDirect (Tracking.cc:2258-2410) whole: the cache
 * phase with the 5-px coverage grid, mnCacheHitTh, then the local-map phase. */
int ygzo_search_local_points_direct(const ygzo_cam *cam, uint8_t **ref_levels, uint8_t **cur_levels, const int *lw,
                                    const int *lh, int nlevels, const float *scale, const float *inv_scale,
                                    float inv_level_sigma2_1, int n_cache, int n_local, const int *item_ptr,
                                    const int *ref_index, const ygzo_kp *kps, const float *pt_ref,
                                    const ygzo_se3 *T_cr, const float *px_proj, float border, int grid_size,
                                    int cache_hit_th, float *px_out, int *matched, int *status, int *local_ran);

/* ---------------- stereo (Frame.cc:509-700) ---------------- */
/* Frame::ComputeStereoMatches (Frame.cc:509-682): left/right pyramids (same
 * level sizes), keypoints (level-0 px) + N x 32 descriptors; mb = baseline,
 * mbf = baseline * fx.  Writes mvuRight / mvDepth (-1 = none) and, if sad_out,
 * the winning SAD per left keypoint (-1 = none).  Returns #depths kept. */
int ygzo_stereo_matches(uint8_t **left_levels, uint8_t **right_levels, const int *lw, const int *lh,
                        int nlevels, const float *scale, const float *inv_scale, const ygzo_kp *kl,
                        const uint8_t *dl, int nl, const ygzo_kp *kr, const uint8_t *dr, int nr, float mb,
                        float mbf, float *uRight, float *depth, int *sad_out);
/* Frame::ComputeStereoFromRGBD (Frame.cc:684-700) */
void ygzo_stereo_from_rgbd(const float *im_depth, int W, int H, int stride, const ygzo_kp *kps, int n, float mbf,
                           float *uRight, float *depth);

/* ---------------- DBoW2 transform (Frame::ComputeBoW, Frame.cc:495-500) ---------------- */
typedef struct ygzo_vocab ygzo_vocab;
/* nodes 0..n-1 as loadFromTextFile leaves them: parent[i] < i for i >= 1,
 * is_leaf / desc (32 B) / weight per node (node 0 = root, unused fields). */
ygzo_vocab *ygzo_vocab_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t *parent,
                              const uint8_t *is_leaf, const uint8_t *desc, const double *weight);
void ygzo_vocab_destroy(ygzo_vocab *v);
/* transform(feature, word_id, weight, &nid, levelsup) (TemplatedVocabulary.h:1241-1281) */
void ygzo_bow_transform_one(const ygzo_vocab *v, const uint8_t *f, int levelsup, int *word, double *weight,
                            int *nid);
/* transform(features, BowVector, FeatureVector, levelsup) (TemplatedVocabulary.h:1150-1212):
 * BowVector as ascending (word, value) arrays, FeatureVector as (node, feature)
 * pairs in map order; all arrays sized n.  Returns #words. */
int ygzo_compute_bow(const ygzo_vocab *v, const uint8_t *desc, int n, int levelsup, int32_t *bow_words,
                     double *bow_values, int *n_words, int32_t *fv_nodes, int32_t *fv_features, int *n_fv);

/* ---------------- undistort (Frame.cc:775-790) ---------------- */
/* cv::initUndistortRectifyMap(K, D, I, K, (W,H), CV_16SC2): map1 [H][W][2]
 * (integer source x, y), map2 [H][W] (5-bit fractions, y*32 + x). */
void ygzo_undistort_map(const float cam[4], const float *dist, int ndist, int W, int H, int16_t *map1,
                        uint16_t *map2);
/* cv::remap(src, dst, map1, map2, INTER_LINEAR), BORDER_CONSTANT 0 */
void ygzo_remap_linear(const uint8_t *src, int W, int H, int sstride, const int16_t *map1, const uint16_t *map2,
                       int DW, int DH, uint8_t *dst, int dstride);
/* the same remap for CV_32F (Frame.cc:799-804, RGB-D depth): float weight table */
void ygzo_remap_linear_f32(const float *src, int W, int H, int sstride, const int16_t *map1, const uint16_t *map2,
                           int DW, int DH, float *dst, int dstride);

/* ---------------- CPU baseline driver (oracle/bench.c, bench.py's cpu_baseline) ---------------- */
typedef struct ygzo_bench_stats {
    double t_pyr, t_extract, t_hamming, t_align; /* summed over threads, seconds */
    int frames, pairs;
    long long keypoints, visible;
} ygzo_bench_stats;
/* pyramid + ORB + Hamming vs previous + SparseImgAlign (nlevels-1 .. 1) per frame of
 * frames[n][H][W] on `threads` threads (contiguous chunks); map points of frame g
 * on the plane Z_w = plane_z through r3[3g], cz[g].  Returns the wall time (s). */
double ygzo_bench_pipeline(const uint8_t *frames, int n, int W, int H, const float cam[4], float plane_z,
                           const float *r3, const float *cz, int nfeatures, float scale, int nlevels, int ini,
                           int min_th, int threads, ygzo_bench_stats *stats);
int ygzo_bench_fast9(const uint8_t *img, int w, int h, int threshold, int reps, double *seconds);

#ifdef __cplusplus
}
#endif
#endif
