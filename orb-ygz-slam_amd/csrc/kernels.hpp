// kernels.hpp — host launchers of the gfx950 kernels (defined in *.hip).
#pragma once
#include "common.hpp"

namespace ygzfe {

// extract.hip
hipError_t upload_pattern(const int *pat);
hipError_t run_arith_guard(uint32_t host_fails[2]);  // extract.hip k_arith_guard
hipError_t launch_pyramid(uint8_t *pyr, uint32_t pitch, const Plan &hp, const Plan *dp, const int *dtabs,
                          int nframes, hipStream_t st);
// the batch path of an all-area pyramid: levels 1..K formed by the level-0 blur strips
int pyramid_fusable(const Plan &hp);
hipError_t launch_pyramid_blur0(uint8_t *pyr, uint8_t *blur, uint32_t pitch, const Plan &hp, const Plan *dp,
                                int nframes, hipStream_t st_l0);
hipError_t launch_blur_rest(const uint8_t *pyr, uint8_t *blur, uint32_t pitch, const Plan &hp, const Plan *dp,
                            int nframes, hipStream_t st);
hipError_t launch_blur(const uint8_t *pyr, uint8_t *blur, uint32_t pitch, const Plan &hp, const Plan *dp,
                       int nframes, hipStream_t st);
hipError_t launch_fast(const uint8_t *pyr, uint32_t pitch, const Plan &hp, const Plan *dp, const CellDesc *dcells,
                       uint32_t *cellbuf, int *cellcnt, int nframes, hipStream_t st,
                       const hipStream_t *lvl_streams = nullptr, int n_lvl_streams = 0);
// every level's cells in one launch; clear_flag (nullable) is zeroed by the first lane
hipError_t launch_fast_merged(const uint8_t *pyr, uint32_t pitch, const Plan &hp, const Plan *dp,
                              const CellDesc *dcells, uint32_t *cellbuf, int *cellcnt, int nframes, hipStream_t st,
                              int *clear_flag = nullptr);
// octq: octree stage queues, octree_queue_ints(hp, nframes) ints (counters zeroed here)
hipError_t launch_octree(const Plan &hp, const Plan *dp, const uint32_t *cellbuf, const int *cellcnt,
                         uint32_t *candA, uint32_t *candB, uint32_t *sel, int *selcnt, int *err, int *octq,
                         int nframes, hipStream_t st, const hipStream_t *side = nullptr, int nside = 0,
                         hipEvent_t fork = nullptr, const hipEvent_t *join = nullptr, bool wide = false);
size_t octree_queue_ints(const Plan &hp, int nframes);
// keypoint rows + per-row orientation jobs (uint2 per selection slot: centre byte offset, w | level << 16)
hipError_t launch_emit_kps(const Plan &hp, const Plan *dp, const uint32_t *sel, const int *selcnt,
                           const int *n_existing, ygzfe_kp *kps, int *counts, int row_cap, uint2 *ojobs, int nframes,
                           hipStream_t st);
hipError_t launch_orient_desc(const uint8_t *pyr, const uint8_t *blur, uint32_t pitch, const Plan &hp,
                              const Plan *dp, const uint2 *ojobs, const int *n_existing, ygzfe_kp *kps,
                              uint8_t *desc, int row_cap, int nframes, hipStream_t st);
hipError_t launch_desc_existing(const uint8_t *pyr, const uint8_t *blur, const Plan *dp, ygzfe_kp *kps,
                                uint8_t *desc, int n, int recompute_angle, hipStream_t st);

// dso.hip
hipError_t launch_fast10_rois(const uint8_t *img, int stride, const int *rois, int n_rois, int barrier,
                              int variant, int16_t *out_xy, int cap, int *counts, hipStream_t st);
hipError_t launch_dso_occupancy(const ygzfe_kp *kps, int n, uint8_t *occ, int w, int h, hipStream_t st);
hipError_t launch_dso_pass(const uint8_t *img, int w, int h, int g, const uint8_t *occ, uint32_t *keys, int *cnt,
                           hipStream_t st);
hipError_t launch_dso_finish2(const uint32_t *keys, const int *cnt, int ncells, ygzfe_kp *kps, int row0,
                              int *total, hipStream_t st);
hipError_t launch_dso_cells_debug(const uint8_t *img, int w, int h, int g, int barrier, uint8_t *flags,
                                  hipStream_t st);
constexpr int kDsoMaxGridHost = 96;

// hamming.hip
hipError_t launch_hamming_best2(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *bi, int32_t *bd,
                                int32_t *sd, hipStream_t st);
hipError_t launch_hamming_best2_pairs(const uint8_t *desc, const int32_t *counts, int row_cap, int npairs,
                                      const int32_t *qframe, const int32_t *tframe, int32_t *bi, int32_t *bd,
                                      int32_t *sd, hipStream_t st);
hipError_t launch_hamming_csr(const uint8_t *q, int nq, const uint8_t *t, const int32_t *row_ptr,
                              const int32_t *cand, int32_t *dist, hipStream_t st);

// match.hip: one ORBmatcher search problem (device pointers)
struct MatchJob {
    // the searched frame
    const ygzfe_kp *kps;
    const uint8_t *desc;
    const float *u_right;       // mvuRight or null
    const int32_t *cell;        // PosInGrid: ix << 8 | iy, -1 outside (k_match_cells)
    const int32_t *cend;        // [64 * 48] end of cell ix * 48 + iy in cidx (Frame::mGrid as an index)
    const uint16_t *cidx;       // [n] keypoints by cell
    int n_train;
    float min_x, min_y, inv_w, inv_h;
    // queries in the reference's order
    const ygzfe_match_query *q;
    const uint8_t *qdesc;       // descriptor of query q at qdesc + 32 * (qid ? qid[q] : q)
    const int32_t *qid;         // reported query id (BoW: the KF keypoint index) or null
    int nq;
    const int32_t *cand_ptr;    // BoW: query q's candidates cand[cand_ptr[2q] .. cand_ptr[2q+1]); null = window
    const int32_t *cand;
    const uint8_t *blocked0;    // initial skip state per train keypoint, or null
    // scratch / outputs
    uint64_t *topk;             // [nq][kTopK]
    int32_t *ncand;             // [nq] candidates | valid / blocks bits | listed entries << 24 (k_match_topk)
    float *qangle;              // [nq] query angles (k_match_topk copies them from the query records)
    int32_t *train_out;         // [n_train]
    int32_t *query_out;         // INIT: vnMatches12 [nq]
    int32_t *pushes;            // [nq] rotation-histogram pushes
    int32_t *nmatches;          // [4]: matches, rescans, resolve passes (-1: serial replay), spare
};
hipError_t launch_match_cells(const ygzfe_kp *kps, int n, float min_x, float min_y, float inv_w, float inv_h,
                              int32_t *cell, int32_t *cend, uint16_t *cidx, hipStream_t st);
// max_passes: 0 = serial replay only (k_match_replay); otherwise the parallel resolve
// (k_match_resolve) wherever resolve_fits, INIT always serial
bool resolve_fits(int n_train, int nq);
bool match_resolves(int n_train, int nq, int mode, int max_passes);  // launch_match takes k_match_resolve
hipError_t launch_match(const MatchJob &J, int mode, int th_dist, int check_ori, float nnratio, int max_passes,
                        hipStream_t st);

// align.hip
struct AlignLevels {
    int w[kMaxLevels], h[kMaxLevels];
    uint32_t off[kMaxLevels];
    float inv_scale[kMaxLevels];
};
struct AlignJob {
    const uint8_t *ref_pyr, *cur_pyr;
    const ygzfe_kp *kps;
    const float *xyz;
    const uint8_t *usable;
    int n;
    int max_level, min_level;
    int method;  // NLLSSolver's method (NLSSolver_impl.hpp:8-13): 0 Gauss-Newton, 1 Levenberg-Marquardt
    ygzfe_se3 T_init;
};
// method: 0 Gauss-Newton (every job's method must be 0), 1 Levenberg-Marquardt (every job's 1)
hipError_t launch_sparse_align(const AlignLevels &lv, const ygzfe_camera &cam, const AlignJob *jobs,
                               int njobs, float *scratch, size_t scratch_per_job, ygzfe_align_result *out,
                               hipStream_t st, int max_n, int method = 0);
size_t sparse_align_scratch_floats(int n);
int sparse_align_reg_capacity();  // features the register kernel holds (one per feature-wave thread)
// stream placement probe (ensure_align_stream): a kernel that holds its stream for
// `us` microseconds of wall clock, and an empty one
hipError_t launch_hold_us(int us, hipStream_t st);
hipError_t launch_empty(hipStream_t st);
hipError_t launch_align2d(const uint8_t *img, int w, int h, int n, const uint8_t *pwb, const uint8_t *p,
                          int n_iter, float *px, uint8_t *conv, hipStream_t st);
hipError_t launch_align2d_window(const uint8_t *win, int stride, int w, int h, int x0, int y0, int ww, int wh,
                                 const uint8_t *pwb, const uint8_t *p, int n_iter, float *px, int *status,
                                 hipStream_t st);
hipError_t launch_find_direct(const uint8_t *const *ref_pyrs, const AlignLevels &ref_lv, const uint8_t *cur_pyr,
                              const AlignLevels &cur_lv, int nlevels, const float *scale, float inv_sigma2_1,
                              const ygzfe_camera &cam, int n, const int32_t *ref_index, const ygzfe_kp *kp_ref,
                              const float *pt_ref, const ygzfe_se3 *T_cr, float *px, int32_t *level,
                              uint8_t *ok, hipStream_t st);

// One stereo pair of ComputeStereoMatches (Frame.cc:509-682)
struct StereoJob {
    const uint8_t *left_pyr, *right_pyr;
    const ygzfe_kp *left_kps, *right_kps;
    const uint8_t *left_desc, *right_desc;
    const int *n_left, *n_right;
    float *u_right, *depth;
    int *sad;
};
struct StereoLevels {
    int w[kMaxLevels], h[kMaxLevels];
    uint32_t off[kMaxLevels];
    float scale[kMaxLevels], inv_scale[kMaxLevels];
};
hipError_t launch_stereo(const StereoJob *jobs, int n_pairs, int max_left, const StereoLevels &lv, float mb, float mbf,
                         hipStream_t st);
hipError_t launch_build_stereo_jobs(int n, const uint8_t *pyr, size_t pyr_pitch, const ygzfe_kp *kps,
                                    const uint8_t *desc, const int *counts, int kp_cap, const int32_t *left_idx,
                                    const int32_t *right_idx, float *u_right, float *depth, int *sad,
                                    StereoJob *jobs, hipStream_t st);
hipError_t launch_stereo_rgbd(const float *im_depth, size_t depth_pitch, int W, int H, int stride,
                              const ygzfe_kp *kps, int kp_pitch, const int *n_ptr, int n_max, int n_frames, float mbf,
                              float *u_right, float *depth, hipStream_t st);

// DBoW2 vocabulary in HBM (bow.hip)
constexpr int kBowMaxFeatures = 8192;
struct VocabDev {
    int n_nodes, L;
    const int32_t *child_ptr;   // [n_nodes + 1] CSR slot ranges
    const int32_t *slot_node;   // [n_nodes - 1] child node id per slot
    const uint8_t *slot_desc;   // [n_nodes - 1][32] child descriptor per slot
    const int32_t *word_id;     // [n_nodes]
    const double *weight;       // [n_nodes]
};
hipError_t launch_bow_transform(const VocabDev &V, const uint8_t *desc, size_t desc_pitch, const int *counts,
                                int n_max, int n_frames, int levelsup, int32_t *word, double *weight, int32_t *nid,
                                size_t out_pitch, hipStream_t st);
hipError_t launch_bow_vectors(const int *counts, int n_static, int n_frames, const int32_t *word, const double *weight,
                              const int32_t *nid, size_t in_pitch, int weighting, int scoring, int32_t *bow_words,
                              double *bow_values, int *n_words, int32_t *fv_nodes, int32_t *fv_feats, int *n_fv,
                              size_t out_pitch, hipStream_t st);

// One (map point, keyframe) item of SearchLocalPointsDirect (host-packed, 80 B)
struct DirectItem {
    ygzfe_kp kp;        // ref->mvKeys[index] (28 B)
    float pt[3];        // T_ref * P_w
    int32_t ref;        // keyframe slot
    int32_t point;      // owning map point
    int32_t tcr;        // T_cur * T_ref^-1 in the call's T table (one entry per keyframe when
                        // the items of a keyframe agree, as Tracking's do)
};
static_assert(sizeof(DirectItem) == 52, "DirectItem layout");
// n_cache cache points (5-px coverage grid of grid_size, replayed in order) then
// n_local local-map points (run only if the cache successes <= cache_hit_th);
// hdr[0] = cache successes, hdr[1] = local phase ran
hipError_t launch_search_direct(const uint8_t *const *ref_pyrs, const AlignLevels &lv, const uint8_t *cur_pyr,
                                int nlevels, const float *scale, float inv_sigma2_1, const ygzfe_camera &cam,
                                int n_cache, int n_local, int n_items, const int32_t *item_ptr, const void *items,
                                const ygzfe_se3 *tcr_tab, const float *px_proj, float *px_item, uint8_t *ok_item, float border, int grid_size,
                                int cache_hit_th, float *px_out, int32_t *matched, int32_t *status, int32_t *hdr,
                                hipStream_t st);
constexpr int kDirectMaxGridCells = 65536 * 8 - 64;  // LDS bitmap of k_direct_replay (<= 64 KB)

// slots.hip: offline sequence mode result slots
hipError_t launch_pack_slots(const ygzfe_kp *kps, const uint8_t *desc, const int *counts, int kp_cap,
                             const ygzfe_align_result *align, int frame_begin, int n_frames, int global_first,
                             uint8_t *slots, size_t slot_pitch, hipStream_t st);

hipError_t launch_remap_f32(const float *src, size_t src_pitch, int W, int H, int sstride, const int16_t *map1,
                            const uint16_t *map2, float *dst, size_t dst_pitch, int dstride, int n_images,
                            hipStream_t st);
hipError_t launch_undistort_map(const float cam[4], const float *dist, int ndist, int W, int H, int16_t *map1,
                                uint16_t *map2, hipStream_t st);
int remap_tiles(int W, int H);  // entries of the per-tile source-box table (16 B each: x0, y0, w, h)
hipError_t launch_remap_boxes(int W, int H, const int16_t *map1, void *boxes, hipStream_t st);
hipError_t launch_remap_linear(const uint8_t *src, size_t src_pitch, int W, int H, int sstride, const int16_t *map1,
                               const uint16_t *map2, const void *boxes, int max_box, bool any_large, uint8_t *dst,
                               size_t dst_pitch, int dstride, int n_images, hipStream_t st);

}  // namespace ygzfe
