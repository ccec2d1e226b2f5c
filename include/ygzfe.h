/*
 * ygzfe.h — C ABI of the MI355X (gfx950) front-end for ORB-YGZ-SLAM.
 *
 * The drop-in boundary of the per-frame hot path: ORB extraction
 * (ORBextractor), Hamming matching (ORBmatcher) and direct alignment
 * (SparseImgAlign, Align2D / FindDirectProjection).  Plain C types only; every
 * entry point names the reference interface it replaces (paths relative to the
 * Ewenwan/ORB-YGZ-SLAM checkout).  INTEGRATION.md shows the C++ adapter
 * (orb-ygz-slam_amd/compat/) that keeps the reference's class signatures so
 * Tracking.cc compiles unchanged.
 *
 * Conventions
 *  - Return value: YGZFE_OK (0) or a negative YGZFE_E* code; ygzfe_last_error()
 *    gives a thread-local message.  The reference never throws; the adapter maps
 *    codes to its "empty result / 0 / false" conventions.
 *  - Host pointers unless the name says `d_` (device pointer, HIP memory of the
 *    handle's device).  `stream` is a hipStream_t passed as void* (NULL = the
 *    handle's own stream).
 *  - Handles are thread-safe across handles, not re-entrant per handle
 *    (the reference extractor is stateful: mvImagePyramid, mnGridSize).
 *  - Results are bit-exact with oracle/ (the CPU restatement) for keypoints and
 *    descriptors; SparseImgAlign poses agree within 1e-4.
 */
#ifndef YGZFE_H_
#define YGZFE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YGZFE_OK 0
#define YGZFE_EINVAL (-1)   /* bad argument / shape */
#define YGZFE_EHIP (-2)     /* HIP runtime failure (no device, launch error) */
#define YGZFE_ECAP (-3)     /* caller buffer too small; *n_out holds the size needed */
#define YGZFE_ENOMEM (-4)
#define YGZFE_ESTATE (-5)   /* call order violated (e.g. extract before pyramid) */

#define YGZFE_MAX_LEVELS 16

/* Same 28-byte layout as cv::KeyPoint {Point2f pt; float size, angle, response;
 * int octave, class_id} so std::vector<cv::KeyPoint>::data() passes straight. */
typedef struct ygzfe_kp {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} ygzfe_kp;

/* ORBextractor::KeyPointMethod (ORBextractor.h:49-51). */
enum ygzfe_method { YGZFE_ORBSLAM_KEYPOINT = 0, YGZFE_FAST_KEYPOINT = 1, YGZFE_DSO_KEYPOINT = 2 };

/* GaussianBlur 7x7 sigma 2 kernel variant: OpenCV >= 3.4.2
 * bit-exact fixed point [18,34,48,56,...] or OpenCV 2.4/3.x cvRound [18,34,49,55,...]. */
enum ygzfe_blur { YGZFE_BLUR_CV4 = 0, YGZFE_BLUR_CV3 = 1 };

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
 * int minThFAST) (ORBextractor.h:53-57, Tracking.cc:255-261). */
typedef struct ygzfe_orb_params {
    int32_t nfeatures;
    float scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
    int32_t blur_variant;
} ygzfe_orb_params;

typedef struct ygzfe_camera { float fx, fy, cx, cy; } ygzfe_camera;   /* Frame::fx.. (Frame.h:178-183) */
typedef struct ygzfe_se3 { float q[4]; float t[3]; } ygzfe_se3;        /* Sophus SE3f: quat (x,y,z,w) + t */

const char *ygzfe_last_error(void);
int ygzfe_device_count(void);

/* ------------------------------------------------------------------------ */
/* ORBextractor (ORBextractor.h:37-192)                                     */
typedef struct ygzfe_extractor ygzfe_extractor;
/* A device-resident frame pyramid: Frame::mvImagePyramid (Frame.h, Frame.cc:807-813). */
typedef struct ygzfe_frame ygzfe_frame;

/* ORBextractor::ORBextractor (ORBextractor.cc:412-470). */
int ygzfe_extractor_create(const ygzfe_orb_params *p, int device, ygzfe_extractor **out);
/* Frames borrow their extractor: destroying it while frames are alive releases it when the
 * last of them is destroyed (any destroy order is safe, e.g. a garbage collector's). */
void ygzfe_extractor_destroy(ygzfe_extractor *ex);
/* GetLevels / GetScaleFactor / GetScaleFactors / GetInverseScaleFactors /
 * GetScaleSigmaSquares / GetInverseScaleSigmaSquares (ORBextractor.h:87-109).
 * Any output pointer may be NULL; arrays hold nlevels floats. */
int ygzfe_extractor_levels(const ygzfe_extractor *ex, int *nlevels, float *scale,
                           float *inv_scale, float *sigma2, float *inv_sigma2);
/* mnFeaturesPerLevel (ORBextractor.cc:434-445). */
int ygzfe_extractor_features_per_level(const ygzfe_extractor *ex, int32_t *out);
/* DSO grid state mnGridSize (ORBextractor.h:191): get / set (-1 = recompute). */
int ygzfe_extractor_dso_grid(ygzfe_extractor *ex, int32_t *get, const int32_t *set);

/* Host-only (no device touched): the extraction plan for a width x height image,
 * i.e. what ORBextractor::operator() derives per call -- level sizes
 * cvRound(W/scale) (ORBextractor.cc:1131-1132), feature budgets (:434-445),
 * umax (:453-467) and the number of FAST cells per level (:728-781).  Arrays
 * hold nlevels entries (umax: 16); any pointer may be NULL. */
int ygzfe_orb_plan(const ygzfe_orb_params *p, int width, int height, int32_t *level_w, int32_t *level_h,
                   int32_t *budget, int32_t *ncells, int32_t *umax);

int ygzfe_frame_create(ygzfe_extractor *ex, int width, int height, ygzfe_frame **out);
void ygzfe_frame_destroy(ygzfe_frame *f);
/* Frame::ComputeImagePyramid -> ORBextractor::ComputePyramid
 * (Frame.cc:807-813, ORBextractor.cc:1129-1150): H2D of the image + pyramid. */
int ygzfe_compute_pyramid(ygzfe_extractor *ex, ygzfe_frame *f, const uint8_t *img, int stride);
/* Same from an image already in device memory. */
int ygzfe_compute_pyramid_device(ygzfe_extractor *ex, ygzfe_frame *f, const uint8_t *d_img,
                                 int stride, void *stream);
/* Host mirror of mvImagePyramid[level] (read at Frame.cc:515,604,618). */
int ygzfe_frame_level(const ygzfe_frame *f, int level, int *w, int *h, uint8_t *dst, int dst_stride);
/* Upload a whole host pyramid (e.g. a Frame deep-copied from elsewhere). */
int ygzfe_frame_set_level(ygzfe_frame *f, int level, const uint8_t *src, int src_stride);
/* Host mirror of levels [first, first + count) in one DMA and one synchronisation:
 * ORBextractor::ComputePyramid's public mvImagePyramid (ORBextractor.cc:1129-1150,
 * ORBextractor.h:114), which Frame::ComputeImagePyramid hands to the Frame
 * (Frame.cc:807-813).  dst[i] / dst_stride[i] receive level first + i. */
int ygzfe_frame_levels(const ygzfe_frame *f, int first, int count, uint8_t *const *dst, const int *dst_stride);
/* Upload levels [first, first + count) of a host pyramid in one DMA (a Frame whose
 * pyramid the device has not seen, e.g. one deep-copied elsewhere, Frame.cc:186-188). */
int ygzfe_frame_set_levels(ygzfe_frame *f, int first, int count, const uint8_t *const *src, const int *src_stride);

/* ORBextractor::operator()(Frame*, keypoints, descriptors, method, leftEye=true)
 * (ORBextractor.cc:1031-1127, called from Frame::ExtractORB Frame.cc:332-348).
 * `kps_io` holds n_existing keypoints (Frame::mvKeys, level-0 coordinates) on
 * entry; on return it holds existing + new keypoints (*n_out rows) and
 * `desc` holds *n_out x 32 descriptor bytes (rows 0..n_existing-1 = existing).
 * DSO mode recomputes the existing keypoints' angles (ORBextractor.cc:1383-1385).
 * cap = capacity of kps_io / desc in rows. */
int ygzfe_extract(ygzfe_extractor *ex, ygzfe_frame *f, int method, ygzfe_kp *kps_io,
                  int n_existing, int cap, uint8_t *desc, int *n_out);
/* ORBextractor::operator()(InputArray image, mask, keypoints, descriptors)
 * (ORBextractor.cc:970-1028): pyramid + octree extraction of one image. */
int ygzfe_detect_and_compute(ygzfe_extractor *ex, ygzfe_frame *f, const uint8_t *img, int stride,
                             ygzfe_kp *kps, int cap, uint8_t *desc, int *n_out);

/* ------------------------------------------------------------------------ */
/* Batched extraction: many frames resident in HBM, one launch per stage.    */
typedef struct ygzfe_batch ygzfe_batch;
int ygzfe_batch_create(const ygzfe_orb_params *p, int device, int width, int height,
                       int max_frames, ygzfe_batch **out);
void ygzfe_batch_destroy(ygzfe_batch *b);
/* Geometry: frame_pitch = bytes of one frame pyramid (frame i level 0 starts at
 * d_frames + i * frame_pitch, stride width), kp_cap = keypoint rows per frame. */
int ygzfe_batch_info(ygzfe_batch *b, size_t *frame_pitch, int *kp_cap, int *nlevels);
/* Device buffer the frame pyramids live in (max_frames x frame_pitch bytes). */
int ygzfe_batch_frames(ygzfe_batch *b, uint8_t **d_frames);
/* Use caller-owned device buffers instead (any may be NULL = keep): pyramids
 * [max_frames * frame_pitch], kps [max_frames * kp_cap], desc
 * [max_frames * kp_cap * 32], counts [max_frames]. */
int ygzfe_batch_bind_buffers(ygzfe_batch *b, uint8_t *d_pyramids, ygzfe_kp *d_kps, uint8_t *d_desc,
                             int32_t *d_counts);
/* H2D of n_frames tight width x height images into the level-0 slots.  Waits
 * for the previous extraction of this batch; work the caller queued on its own
 * streams after that extraction (match, align, ...) must be complete. */
int ygzfe_batch_upload(ygzfe_batch *b, const uint8_t *frames, int n_frames);
/* Pyramid + FAST + octree + orientation + blur + rBRIEF on frames [0, n). */
int ygzfe_batch_extract(ygzfe_batch *b, int n_frames, void *stream);
/* The same extraction split over two streams: work queued on kp_stream after
 * this call sees the keypoint rows (position, octave, size, response; not
 * the angle) and the counts; work queued on desc_stream sees the complete
 * rows and the descriptors.  The blur runs on desc_stream, beside FAST.  A
 * call orders itself after the previous call's descriptor pass (its last
 * reader of the batch buffers), whatever streams the two calls use. */
int ygzfe_batch_extract_split(ygzfe_batch *b, int n_frames, void *kp_stream, void *desc_stream);
/* Synchronise and report kernel-side errors (octree pool overflow). */
int ygzfe_batch_check(ygzfe_batch *b);
/* Dense best/second-best Hamming of frame qframe[p] against tframe[p] for each
 * pair p; outputs [n_pairs][kp_cap] (device pointers). */
int ygzfe_batch_match(ygzfe_batch *b, int n_pairs, const int32_t *d_qframe, const int32_t *d_tframe,
                      int32_t *d_best_idx, int32_t *d_best_dist, int32_t *d_second_dist, void *stream);
/* Results of frame i (same rows as ygzfe_extract with no existing keypoints). */
int ygzfe_batch_result(ygzfe_batch *b, int frame, ygzfe_kp *kps, int cap, uint8_t *desc, int *n_out);
/* Device views: kps [max_frames][kp_cap], desc [max_frames][kp_cap][32], counts [max_frames]. */
int ygzfe_batch_device_results(ygzfe_batch *b, ygzfe_kp **d_kps, uint8_t **d_desc,
                               int32_t **d_counts, int *kp_cap);
/* Per-frame pyramid level view of the batch (device pointer + stride). */
int ygzfe_batch_level(ygzfe_batch *b, int frame, int level, const uint8_t **d_level, int *w,
                      int *h, int *stride);
/* Synchronise and copy level `level` of frame `frame` to the host: the pyramid
 * level (mvImagePyramid, blurred == 0) or its GaussianBlur(7x7, sigma 2) copy
 * that computeDescriptors reads (ORBextractor.cc:1079-1084, blurred != 0). */
int ygzfe_batch_read_level(ygzfe_batch *b, int frame, int level, int blurred, uint8_t *dst, int dst_stride);
/* Synchronise and report per-level work of the last ygzfe_batch_extract over
 * frames [0, n_frames): FAST candidates kept by the cell NMS (the octree input,
 * vToDistributeKeys) and keypoints kept by the octree, each [nlevels] summed
 * over the frames.  For roofline accounting (bytes per launch). */
int ygzfe_batch_stats(ygzfe_batch *b, int n_frames, int64_t *candidates, int64_t *selected);
/* Offline sequence mode: fixed-size per-frame result slots,
 * packed on the device and gathered to rank 0 over RCCL.  Slot layout:
 *   [0, 64)  int32 n_kps, int32 n_visible, f32 q[4] (x,y,z,w), f32 t[3], f32 chi2,
 *            int32 global frame index, int32 has_align, 4 x int32 0;
 *   then kp_cap keypoint rows (ygzfe_kp) and kp_cap x 32 descriptor bytes,
 *   rows >= n_kps zero; zero padding to a 16-B multiple.
 * The align fields of frame f are SparseImgAlign's TCR of the pair (f-1 -> f). */
#define YGZFE_SLOT_HEADER 64
size_t ygzfe_slot_bytes(int kp_cap);
/* Pack batch frames [frame_begin, frame_begin + n_frames) into slots
 * d_slots + k * slot_pitch (slot_pitch >= ygzfe_slot_bytes, multiple of 16);
 * frame f takes d_align[f - 1] (the result of the pair aligning f-1 -> f) when
 * d_align != NULL and f >= 1; global index = global_first + (f - frame_begin).
 * Device pointers, one launch on `stream`. */
int ygzfe_batch_pack_slots(ygzfe_batch *b, int frame_begin, int n_frames, const struct ygzfe_align_result *d_align,
                           int global_first, uint8_t *d_slots, size_t slot_pitch, void *stream);
/* Kernel timing (hipEvents around each stage launch on the batch stream).
 * enable != 0 turns it on; ms[] receives per-stage milliseconds of the last
 * ygzfe_batch_extract; names[] the stage names. Returns stage count. */
int ygzfe_batch_timing(ygzfe_batch *b, int enable, float *ms, const char **names, int cap);
void *ygzfe_batch_stream(ygzfe_batch *b);

/* ------------------------------------------------------------------------ */
/* ORBmatcher (ORBmatcher.h:38-178)                                          */
/* ORBmatcher::DescriptorDistance (ORBmatcher.cc:1507-1523), host scalar. */
int ygzfe_descriptor_distance(const uint8_t *a, const uint8_t *b);
/* Dense best / second-best Hamming search (the inner loops of
 * ORBmatcher::SearchByProjection / SearchForInitialization /
 * SearchByBoW, ORBmatcher.cc:43-126,375-478,1218-1350): for each query, the
 * smallest distance (strict <, first train index wins), its index and the
 * second-smallest distance (257 when absent).  Device pointers. */
int ygzfe_hamming_best2_device(const uint8_t *d_query, int nq, const uint8_t *d_train, int nt,
                               int32_t *d_best_idx, int32_t *d_best_dist, int32_t *d_second_dist,
                               void *stream);
/* Same on host buffers (H2D / D2H on an internal stream of `device`). */
int ygzfe_hamming_best2(int device, const uint8_t *query, int nq, const uint8_t *train, int nt,
                        int32_t *best_idx, int32_t *best_dist, int32_t *second_dist);
/* Windowed search (Frame::GetFeaturesInArea candidate lists, Frame.cc:424-481):
 * CSR candidates; writes the distance of every (query, candidate) pair. */
int ygzfe_hamming_csr(int device, const uint8_t *query, int nq, const uint8_t *train, int nt,
                      const int32_t *row_ptr, const int32_t *cand, int32_t *dist_out);

/* The tracking-path searches, complete with the reference's sequential rules
 * (TH_HIGH / TH_LOW, nnratio, "already matched" skips, the 30-bin rotation
 * histogram and ComputeThreeMaxima), bit-exact with oracle/match.c.
 *
 * A match frame is the searched Frame's state the searches read: mvKeys
 * (level-0 px), mDescriptors, mvuRight (NULL = none) and the image bounds
 * mnMinX / mnMaxX / mnMinY / mnMaxY (Frame.cc:501-507); its 64 x 48 grid
 * (AssignFeaturesToGrid / PosInGrid, Frame.cc:314-330, 483-493) is built on
 * the device.  n <= 65535 keypoints. */
typedef struct ygzfe_bounds { float min_x, max_x, min_y, max_y; } ygzfe_bounds;
typedef struct ygzfe_match_frame ygzfe_match_frame;
int ygzfe_match_frame_create(int device, ygzfe_match_frame **out);
void ygzfe_match_frame_destroy(ygzfe_match_frame *f);
int ygzfe_match_frame_set(ygzfe_match_frame *f, const ygzfe_kp *kps, const uint8_t *desc, int n, const float *u_right,
                          const ygzfe_bounds *bounds);
/* Diagnostics of the last search on this frame: queries re-scanned because the
 * sequential skips exhausted their K best candidates (the result never depends on it). */
int ygzfe_match_frame_stats(const ygzfe_match_frame *f, int *rescans);
/* Passes the parallel resolve of the last search took to reach the sequential
 * result (-1: the serial replay decided: SearchForInitialization, > 4096 queries,
 * or environment YGZFE_MATCH_PASSES=0).  Results are identical either way. */
int ygzfe_match_frame_resolve_stats(const ygzfe_match_frame *f, int *passes);
/* The same from frame `frame` of a batch (device-to-device copy of its rows). */
int ygzfe_match_frame_from_batch(ygzfe_match_frame *f, ygzfe_batch *b, int frame, const ygzfe_bounds *bounds);

#define YGZFE_MQ_VALID 1   /* the query takes part (MapPoint present, not bad / outlier, projected inside) */
#define YGZFE_MQ_BLOCKS 2  /* assigning it makes later queries skip the keypoint (Observations() > 0) */
#define YGZFE_MQ_STEREO 4  /* the projection searches' mvuRight test applies */
/* One query: the GetFeaturesInArea(u, v, radius, min_level, max_level)
 * window (-1 levels as the reference's defaults), the projected right u for
 * the stereo test, the query keypoint's angle (rotation histogram), flags. */
typedef struct ygzfe_match_query {
    float u, v, radius, u_right;
    int32_t min_level, max_level;
    float angle;
    int32_t flags;
} ygzfe_match_query;
enum ygzfe_match_mode { YGZFE_MATCH_BEST = 0, YGZFE_MATCH_RATIO = 1, YGZFE_MATCH_INIT = 2, YGZFE_MATCH_BOW = 3 };

/* SearchByProjection(CurrentFrame, LastFrame, th, bMono, checkLevel)
 * (ORBmatcher.cc:1218-1350), and the relocalisation form
 * SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (:1352-1469):
 * query i = the i-th projected MapPoint (the caller projects with its own pose
 * types; radius = th * mvScaleFactors[octave], levels per bForward / bBackward /
 * checkLevel), q_desc[i] = MapPoint::GetDescriptor().  train_blocked[i2] != 0
 * where CurrentFrame.mvpMapPoints[i2] makes the reference skip i2.  Best only,
 * bestDist <= th_dist (TH_HIGH = 100 / ORBdist), rotation check.  train_match[i2]:
 * -1 untouched, -2 set to NULL by the rotation check, >= 0 the query assigned. */
int ygzfe_search_projection_best(ygzfe_match_frame *cur, const ygzfe_match_query *q, const uint8_t *q_desc, int nq,
                                 const uint8_t *train_blocked, int th_dist, int check_ori, int32_t *train_match,
                                 int *nmatches);
/* SearchByProjection(F, vpMapPoints, th, checkLevel) (ORBmatcher.cc:43-126): best
 * and second best with their octaves, bestDist <= TH_HIGH, the nnratio test when
 * both share an octave.  train_match[idx]: -1 or the query assigned. */
int ygzfe_search_projection_ratio(ygzfe_match_frame *F, const ygzfe_match_query *q, const uint8_t *q_desc, int nq,
                                  const uint8_t *train_blocked, float nnratio, int32_t *train_match, int *nmatches);
/* SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
 * (ORBmatcher.cc:375-478): prev_matched [2 * F1.n] in / out, matches12 [F1.n]. */
int ygzfe_search_for_initialization(ygzfe_match_frame *F1, ygzfe_match_frame *F2, float *prev_matched,
                                    int window_size, float nnratio, int check_ori, int32_t *matches12, int *nmatches);
/* SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.cc:155-263).  The two
 * FeatureVectors (DBoW2, node-sorted) as CSR: node k = nodes[k], features
 * feats[ptr[k] .. ptr[k+1]).  kf_usable[i] = pKF's MapPoint i present and not bad.
 * f_match[F.n]: the KF keypoint index matched to F's keypoint, or -1. */
int ygzfe_search_by_bow(ygzfe_match_frame *kf, ygzfe_match_frame *F, const uint8_t *kf_usable, int n_kf_nodes,
                        const int32_t *kf_nodes, const int32_t *kf_ptr, const int32_t *kf_feats, int n_f_nodes,
                        const int32_t *f_nodes, const int32_t *f_ptr, const int32_t *f_feats, float nnratio,
                        int check_ori, int32_t *f_match, int *nmatches);

/* ------------------------------------------------------------------------ */
/* SparseImgAlign (SparseImageAlign.h:37-60)                                 */
typedef struct ygzfe_align_result {
    ygzfe_se3 T_cur_ref;   /* TCR */
    int32_t n_visible;     /* run() return value: n_meas_/16 */
    float chi2;            /* chi2_ at exit */
    float H[36];           /* H_ of the last linearisation (getFisherInformation() = H/(5e-4*255^2)) */
} ygzfe_align_result;
/* SparseImgAlign(n_levels=max_level, min_level, n_iter=10).run(ref, cur, TCR)
 * (SparseImageAlign.cc:20-49, Tracking.cc:2145-2189).  kps = ref Frame::mvKeys
 * (level-0 px), xyz_ref[3n] = T_ref * MapPoint::GetWorldPos(), usable[n] = map
 * point present && !isBad && !outlier.  T_io: in = T_cur * T_ref^-1 guess,
 * out = TCR.  Returns YGZFE_OK; result->n_visible = run()'s return. */
int ygzfe_sparse_align(const ygzfe_frame *ref, const ygzfe_frame *cur, const ygzfe_camera *cam,
                       const ygzfe_kp *kps, const float *xyz_ref, const uint8_t *usable, int n,
                       int max_level, int min_level, const ygzfe_se3 *T_init,
                       ygzfe_align_result *result);
/* The same split in two, so the alignment of a frame overlaps its own
 * extraction: both need only the frame's pyramid (the reference runs
 * TrackWithSparseAlignment before any extraction, Tracking.cc:471, 2145-2189).
 * _begin stages the inputs and queues the alignment on the extractor's align
 * stream, ordered after the work already queued on the extractor (the
 * pyramids), and returns at once; ygzfe_extract / ygzfe_compute_pyramid may be
 * called meanwhile (a later pyramid rewrite waits for the alignment); _end
 * waits and writes the result.  One alignment in flight per extractor
 * (YGZFE_ESTATE otherwise). */
int ygzfe_sparse_align_begin(const ygzfe_frame *ref, const ygzfe_frame *cur, const ygzfe_camera *cam,
                             const ygzfe_kp *kps, const float *xyz_ref, const uint8_t *usable, int n,
                             int max_level, int min_level, const ygzfe_se3 *T_init);
int ygzfe_sparse_align_end(const ygzfe_frame *cur, ygzfe_align_result *result);
/* NLLSSolver's method (NLSSolver_impl.hpp:8-13): SparseImgAlign(.., n_iter, method).  */
enum ygzfe_align_method { YGZFE_ALIGN_GAUSS_NEWTON = 0, YGZFE_ALIGN_LEVENBERG_MARQUARDT = 1 };
/* ygzfe_sparse_align with the method: Gauss-Newton (optimizeGaussNewton, :18-91, what
 * Tracking.cc:284 constructs) or Levenberg-Marquardt (optimizeLevenbergMarquardt,
 * :95-212: damped H_ii (1 + mu), a trial per chi2 evaluation, mu_ 0.1 per level,
 * SparseImageAlign.cc:40).  For LM, result->H is H_ as the last trial left it (damped). */
int ygzfe_sparse_align_method(const ygzfe_frame *ref, const ygzfe_frame *cur, const ygzfe_camera *cam,
                              const ygzfe_kp *kps, const float *xyz_ref, const uint8_t *usable, int n,
                              int max_level, int min_level, const ygzfe_se3 *T_init, int method,
                              ygzfe_align_result *result);
/* The align stream's hardware-queue placement probe, for audit: streams
 * the probe created (0 before the first alignment) and whether the chosen one passed
 * the probe (1), was taken unprobed (0: probe off, 4 rejections or its 150 ms spent),
 * or no stream exists yet (-1). */
int ygzfe_extractor_align_probe(ygzfe_extractor *ex, int *attempts, int *passed);

/* Batched: pair p aligns frame ref_idx[p] -> cur_idx[p] of a batch, with the
 * ref frame's batch keypoints (level-0 px); d_xyz_ref [n_pairs][kp_cap][3] and
 * d_usable [n_pairs][kp_cap] per ref keypoint row, d_T_init / d_out [n_pairs]. */
int ygzfe_batch_sparse_align(ygzfe_batch *b, int n_pairs, const int32_t *d_ref_idx,
                             const int32_t *d_cur_idx, const float *d_xyz_ref, const uint8_t *d_usable,
                             const ygzfe_camera *cam, int max_level, int min_level,
                             const ygzfe_se3 *d_T_init, ygzfe_align_result *d_out, void *stream);

/* Thirdparty/fast's FAST-10 detector over n_roi ROIs of a host image, the segment
 * test the DSO_KEYPOINT cells run (ORBextractor.cc:1328-1340):
 *   variant 0: fast_corner_detect_10 (fast_10.cpp:8-3154), every pixel of the ROI;
 *   variant 1: fast_corner_detect_10_sse2 (faster_corner_10_sse.cpp:24-202), rows
 *              [3, h-3) x cols [3, w-3); the plain scan when w < 22.
 * rois = (x0, y0, w, h) per ROI; every tested pixel's radius-3 ring must lie in
 * the image (EINVAL otherwise: the reference reads out of bounds there).  Corners
 * in the reference's order (raster), ROI-relative like its fast_xy: xy[r][cap][2];
 * counts[r] = corners found (ECAP if any exceeds cap; the first cap are written). */
int ygzfe_fast10_detect(int device, const uint8_t *img, int width, int height, int stride, const int32_t *rois,
                        int n_roi, int barrier, int variant, int16_t *xy, int cap, int32_t *counts);
/* Debug view of the DSO_KEYPOINT cell kernel itself (ComputeKeyPointsDSOSingleLevel's
 * per-cell FAST-10, ORBextractor.cc:1317-1345): one pass over every g x g cell of the
 * grid of a width x height image (tight rows) at `barrier`, with the cell kernel's own
 * scan region (the whole cell for g < 22, else [3, g-3)).  flags[cell][g * g] = 1 at
 * each corner (cell-relative raster order); border cells, which the kernel skips, are
 * all 0.  (h / g) * (w / g) cells, row-major. */
int ygzfe_debug_dso_cells(int device, const uint8_t *img, int width, int height, int g, int barrier, uint8_t *flags);

/* ------------------------------------------------------------------------ */
/* Align2D / FindDirectProjection (Align.h:20-26, ORBmatcher.cc:1573-1602)   */
/* Align2D(cur_img, ref_patch_with_border 10x10, ref_patch 8x8, n_iter, px)
 * for n independent patches on one level of `cur`; px_io in/out (level px). */
int ygzfe_align2d_batch(const ygzfe_frame *cur, int level, int n, const uint8_t *patches_with_border,
                        const uint8_t *patches, int n_iter, float *px_io, uint8_t *converged);
/* Align2D(const cv::Mat& cur_img, ref_patch_with_border, ref_patch, n_iter,
 * cur_px_estimate) (Align.h:20-26) on a host image (w x h, row stride): the
 * window around the estimate is uploaded (the whole image only if the
 * iterations leave it); px in / out, *converged = the return value. */
int ygzfe_align2d_image(int device, const uint8_t *img, int w, int h, int stride, const uint8_t *patch_with_border,
                        const uint8_t *patch, int n_iter, float *px, uint8_t *converged);
/* FindDirectProjection for n (map point, keyframe) items against `cur`:
 * item i uses keyframe frame ref[ref_index[i]], its keypoint kp_ref[i],
 * pt_ref[3i] = T_ref * P_w, T_cr[i] = T_cur * T_ref^-1, px_io[2i] (level-0 px,
 * in: projection guess, out: aligned); writes search_level[i], ok[i]. */
int ygzfe_find_direct_projection_batch(const ygzfe_frame *const *ref, const ygzfe_frame *cur,
                                       const ygzfe_camera *cam, int n, const int32_t *ref_index,
                                       const ygzfe_kp *kp_ref, const float *pt_ref,
                                       const ygzfe_se3 *T_cr, float *px_io, int32_t *search_level,
                                       uint8_t *ok);

/* Tracking::SearchLocalPointsDirect (Tracking.cc:2258-2410), batched: for
 * n_points map points that passed Frame::isInFrustum (Frame.cc:363-422),
 * point i's candidate observations are items [item_ptr[i], item_ptr[i+1]) in
 * SelectNearestKeyframe order (Tracking.cc:2412-2432, <= 5 keyframes); item k
 * uses keyframe ref[ref_index[k]] with kp_ref[k] = ref->mvKeys[index],
 * pt_ref[3k] = T_ref * P_w, T_cr[k] = T_cur * T_ref^-1.  px_proj[2i] =
 * (mTrackProjX, mTrackProjY).  Every item runs FindDirectProjection
 * (ORBmatcher.cc:1573-1602); per point the first item that converged and lies
 * inside [border, cols - border) x [border, rows - border) of level 0 (border
 * = 20, Tracking.cc:2287-2293) is kept: px_out[2i] = its px, matched_item[i]
 * = its item index, or -1 (px_out (0, 0)) when none did. */
int ygzfe_search_direct_batch(const ygzfe_frame *const *ref, int n_ref, const ygzfe_frame *cur,
                              const ygzfe_camera *cam, int n_points, const int32_t *item_ptr,
                              const int32_t *ref_index, const ygzfe_kp *kp_ref, const float *pt_ref,
                              const ygzfe_se3 *T_cr, const float *px_proj, float border, float *px_out,
                              int32_t *matched_item);

/* The whole of Tracking::SearchLocalPointsDirect (Tracking.cc:2258-2410) in one
 * call, with its sequential rules.  Points [0, n_cache) are the
 * mvpDirectMapPointsCache members in the cache's iteration order that are not
 * bad and pass isInFrustum (Tracking.cc:2269-2275; the caller erases the
 * others); points [n_cache, n_cache + n_local) are mvpLocalMapPoints that are
 * not in the cache, not bad and in the frustum (:2348-2361).  Items, px_proj and
 * border as ygzfe_search_direct_batch.
 *  - cache phase: a point whose projection cell (int(mTrackProjX / grid_size),
 *    int(mTrackProjY / grid_size)) of the coverage grid (grid_size = 5, rows /
 *    grid_size x cols / grid_size cells of level 0) is already marked is skipped
 *    (status GRID_SKIP, it stays in the cache, :2277-2284); a success marks the
 *    cell of its pixel (:2320-2323); a failure leaves the cache (status FAILED).
 *  - if the cache phase had more than cache_hit_th (mnCacheHitTh) successes the
 *    local points are not searched (status NOT_RUN, *local_ran = 0, :2334-2340);
 *    otherwise each is searched without the grid (MATCHED / FAILED).
 * Successes are the rows Tracking appends to mvKeys / mvpMapPoints / mvMatchedFrom
 * in point order.  status may be NULL; *cache_success, *local_ran may be NULL.
 * Cells outside the grid (the reference indexes past its vector<bool>) count as
 * free and are never marked. */
#define YGZFE_DIRECT_FAILED 0
#define YGZFE_DIRECT_MATCHED 1
#define YGZFE_DIRECT_GRID_SKIP 2
#define YGZFE_DIRECT_NOT_RUN 3
int ygzfe_search_local_points_direct(const ygzfe_frame *const *ref, int n_ref, const ygzfe_frame *cur,
                                     const ygzfe_camera *cam, int n_cache, int n_local, const int32_t *item_ptr,
                                     const int32_t *ref_index, const ygzfe_kp *kp_ref, const float *pt_ref,
                                     const ygzfe_se3 *T_cr, const float *px_proj, float border, int grid_size,
                                     int cache_hit_th, float *px_out, int32_t *matched_item, int32_t *status,
                                     int *cache_success, int *local_ran);

/* ------------------------------------------------------------------------ */
/* Stereo (Frame.cc:509-700)                                                 */
/* Frame::ComputeStereoMatches (Frame.cc:509-682): left / right frames (their
 * ORBextractor pyramids, mvImagePyramid), mvKeys + mDescriptors (nl) and
 * mvKeysRight + mDescriptorsRight (nr <= 65535); mb = baseline, mbf = mb * fx
 * (Frame.h).  Writes mvuRight[nl] and mvDepth[nl] (-1 where no match), with
 * the row-band Hamming search, 11x11 SAD sliding window + parabola, and the
 * 1.5 * 1.4 * median SAD outlier cut of the reference. */
int ygzfe_stereo_matches(const ygzfe_frame *left, const ygzfe_frame *right, const ygzfe_kp *kl, const uint8_t *dl,
                         int nl, const ygzfe_kp *kr, const uint8_t *dr, int nr, float mb, float mbf,
                         float *u_right, float *depth);
/* Batched: pair p matches batch frame d_left_idx[p] (left eye) against
 * d_right_idx[p] (right eye), both extracted by ygzfe_batch_extract;
 * d_u_right / d_depth are [n_pairs][kp_cap] rows of the left frame's keypoints. */
int ygzfe_batch_stereo(ygzfe_batch *b, int n_pairs, const int32_t *d_left_idx, const int32_t *d_right_idx,
                       float mb, float mbf, float *d_u_right, float *d_depth, void *stream);
/* Frame::ComputeStereoFromRGBD (Frame.cc:684-700): d = imDepth(int v, int u)
 * (CV_32F metres, row stride in floats); d > 0 -> depth d, uRight = u - mbf/d. */
int ygzfe_stereo_from_rgbd(int device, const float *im_depth, int width, int height, int stride,
                           const ygzfe_kp *kps, int n, float mbf, float *u_right, float *depth);
/* Batched over the first n_frames frames of a batch: depth image f at
 * d_depth_images + f * depth_pitch (floats); outputs [n_frames][kp_cap]. */
int ygzfe_batch_stereo_rgbd(ygzfe_batch *b, int n_frames, const float *d_depth_images, size_t depth_pitch,
                            int stride, float mbf, float *d_u_right, float *d_depth, void *stream);

/* ------------------------------------------------------------------------ */
/* DBoW2 vocabulary / Frame::ComputeBoW (Frame.cc:495-500)                   */
/* TemplatedVocabulary<FORB::TDescriptor, FORB> (Thirdparty/DBoW2) resident in
 * HBM.  scoring: L1_NORM 0, L2_NORM 1, CHI_SQUARE 2, KL 3, BHATTACHARYYA 4,
 * DOT_PRODUCT 5; weighting: TF_IDF 0, TF 1, IDF 2, BINARY 3 (ORBvoc: 0 0). */
typedef struct ygzfe_vocab ygzfe_vocab;
/* From node arrays as loadFromTextFile builds them (TemplatedVocabulary.h:
 * 1362-1448): node 0 = root; node i >= 1 is the next child of parent[i] < i,
 * desc[32 i], weight[i]; is_leaf[i] gives it the next word id. */
int ygzfe_vocab_create(int device, int k, int L, int scoring, int weighting, int n_nodes, const int32_t *parent,
                       const uint8_t *is_leaf, const uint8_t *desc, const double *weight, ygzfe_vocab **out);
/* loadFromTextFile (ORBvoc.txt, TemplatedVocabulary.h:1362) / loadFromBinaryFile (:1478) */
int ygzfe_vocab_load_text(int device, const char *path, ygzfe_vocab **out);
int ygzfe_vocab_load_binary(int device, const char *path, ygzfe_vocab **out);
void ygzfe_vocab_destroy(ygzfe_vocab *v);
int ygzfe_vocab_info(const ygzfe_vocab *v, int *k, int *L, int *scoring, int *weighting, int *n_nodes, int *n_words);
/* transform(feature, word_id, weight, &nid, levelsup) per descriptor (TemplatedVocabulary.h:1241-1281) */
int ygzfe_bow_transform(ygzfe_vocab *v, const uint8_t *desc, int n, int levelsup, int32_t *word, double *weight,
                        int32_t *nid);
/* transform(features, mBowVec, mFeatVec, levelsup) (TemplatedVocabulary.h:1150-1212) for one
 * frame's n <= 8192 descriptors: BowVector = ascending (bow_words, bow_values)[n_words],
 * FeatureVector = (fv_nodes, fv_features)[n_fv] in (node, feature) order; arrays sized n. */
int ygzfe_compute_bow(ygzfe_vocab *v, const uint8_t *desc, int n, int levelsup, int32_t *bow_words,
                      double *bow_values, int *n_words, int32_t *fv_nodes, int32_t *fv_features, int *n_fv);
/* Batched over the first n_frames extracted frames of a batch: outputs [n_frames][kp_cap]
 * rows and per-frame counts, device pointers, on `stream`. */
int ygzfe_batch_compute_bow(ygzfe_batch *b, ygzfe_vocab *v, int n_frames, int levelsup, int32_t *d_bow_words,
                            double *d_bow_values, int *d_n_words, int32_t *d_fv_nodes, int32_t *d_fv_features,
                            int *d_n_fv, void *stream);

/* ------------------------------------------------------------------------ */
/* Undistortion (Frame::ComputeImagePyramid, Frame.cc:775-790):              */
/*   initUndistortRectifyMap(K, D, I, K, size, CV_16SC2, map1, map2) once     */
/*   per camera, remap(img, map1, map2, INTER_LINEAR) per frame.              */
/* K = (fx, fy, cx, cy), D = mDistCoef (Tracking.cc:171-199): ndist 4 or 5   */
/* (k1 k2 p1 p2 [k3]) or 8 (k1 k2 p1 p2 k3 k4 k5 k6), up to 12 (+ s1..s4).   */
typedef struct ygzfe_undistort ygzfe_undistort;
int ygzfe_undistort_create(int device, const ygzfe_camera *K, const float *dist, int ndist, int width, int height,
                           ygzfe_undistort **out);
void ygzfe_undistort_destroy(ygzfe_undistort *u);
/* host copies of the fixed-point maps: map1 = 2*W*H int16 (x, y), map2 = W*H u16 */
int ygzfe_undistort_maps(const ygzfe_undistort *u, int16_t *map1, uint16_t *map2);
/* remap n device images (pitch between images, row stride inside one) */
int ygzfe_undistort_apply_device(const ygzfe_undistort *u, const uint8_t *d_src, size_t src_pitch, int src_stride,
                                 uint8_t *d_dst, size_t dst_pitch, int dst_stride, int n_images, void *stream);
/* The RGB-D depth image's undistortion (Frame.cc:799-804): the same maps, cv::remap
 * INTER_LINEAR on CV_32F (float weight table, BORDER_CONSTANT 0), n_images images of
 * src_stride / dst_stride floats per row, src_pitch / dst_pitch floats apart. */
int ygzfe_undistort_apply_f32_device(const ygzfe_undistort *u, const float *d_src, size_t src_pitch, int src_stride,
                                     float *d_dst, size_t dst_pitch, int dst_stride, int n_images, void *stream);
/* One host image in, its undistorted copy out (the drop-in Frame::ComputeImagePyramid's
 * remaps of mImGray / mImRight, Frame.cc:786-797, and of mImDepth, :799-804); strides in
 * elements. */
int ygzfe_undistort_image(const ygzfe_undistort *u, const uint8_t *src, int src_stride, uint8_t *dst, int dst_stride);
int ygzfe_undistort_depth(const ygzfe_undistort *u, const float *src, int src_stride, float *dst, int dst_stride);
/* ComputeImagePyramid with undistortion: remap(img) -> level 0, then levels */
int ygzfe_compute_pyramid_undistorted(ygzfe_extractor *ex, ygzfe_frame *f, ygzfe_undistort *u, const uint8_t *img,
                                      int stride);
/* batch: raw device frames (W*H each, pitch raw_pitch) -> undistorted
 * level-0 slots of the batch pyramids (run before ygzfe_batch_extract) */
int ygzfe_batch_undistort_device(ygzfe_batch *b, const ygzfe_undistort *u, const uint8_t *d_raw, size_t raw_pitch,
                                 int n_frames, void *stream);
/* batch: host raw frames (W*H each, contiguous) -> staged on the device,
 * undistorted into the level-0 slots */
int ygzfe_batch_upload_undistorted(ygzfe_batch *b, ygzfe_undistort *u, const uint8_t *frames, int n_frames);

#ifdef __cplusplus
}
#endif
#endif
